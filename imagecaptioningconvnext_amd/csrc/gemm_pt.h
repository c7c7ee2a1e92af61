// Stream-tile bf16 GEMM with the epilogue applied from registers -- included by gemm.hip.
//
// The LDS-DMA tiles of gemm_glds.h (64x64 / 128x128, 4 waves) issue 8 MFMAs per wave between
// two barriers, recompute every DMA slot's clamped source address per k-step (8.5 VALU per MFMA
// in the round-4 SQ pass) and stage the fp32 tile through LDS for the epilogue: 0.12 of the
// bf16 peak on the encoder / decoder shapes.  This kernel (round 5) is built around the k-step:
//   * 512-thread blocks (8 waves), each wave owning a 64 x (16*FN) output block: 2 x FM x FN
//     MFMAs per 64-deep k-step (32 at 256x128 / 128x256), 4-12x the old ratio of matrix work per
//     barrier;
//   * one barrier per k-step: the fragments of the next half-step are read from LDS while the
//     current half-step's MFMAs run (two register sets), and the stage a step was read from is
//     refilled right after that step's barrier, so S stages keep S - 1 steps of LDS-DMA in flight;
//   * LDS-DMA by buffer_load ... lds with the per-lane source offset fixed for a tile: a k-step
//     only moves the (scalar) buffer descriptor base, so a DMA piece costs no VALU; rows past the
//     end of an operand read through the descriptor's range check (zeros), M / N tails read a
//     clamped valid row whose outputs are dropped;
//   * persistent: one block per CU walks its tiles (XCD-contiguous slots, banded for L2 reuse),
//     the k-step stream runs across tile boundaries, so the next tile's first steps land while
//     the current tile's epilogue runs;
//   * D^T = B^T A^T on MFMA (v_mfma_f32_16x16x32_bf16, operands swapped): a lane ends with 4
//     consecutive output columns of one row, so the epilogue (alpha, bias, GELU with the
//     pre-activation written, ReLU, dropout, dGELU / ReLU-mask from a saved operand, layer scale,
//     drop-path row scale, residual, beta) runs on the accumulators and leaves as 8-byte stores.
// Waits on the DMA are counted (s_waitcnt vmcnt(N), N = the vector-memory ops this thread issued
// after the awaited step: younger DMA pieces and epilogue stores; the epilogue's operand loads are
// waited for by the compiler inside their own step and need no count) with raw s_barrier.

typedef unsigned pt_u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned pt_u32x4 __attribute__((ext_vector_type(4)));

constexpr uint32_t PT_OOB = 0x80000000u;  // buffer offset past every buffer this kernel addresses

typedef __amdgpu_buffer_rsrc_t pt_rsrc_t;

// s_waitcnt lgkmcnt(0) as the builtin (vmcnt / expcnt fields at their maxima), so that the
// compiler's own wait bookkeeping sees the fragment reads complete: after an inline-asm wait it
// still counted them pending and, once the next half-step's reads were issued, made the MFMAs
// wait for those as well (s_waitcnt lgkmcnt(3..0) ahead of every second MFMA group)
DEV void pt_lgkm0() { __builtin_amdgcn_s_waitcnt(0xC07F); }
// raw buffer descriptor (stride 0, num_records = bytes: offsets at or past it read 0 / drop)
DEV pt_rsrc_t pt_rsrc(const void* base, int64_t bytes) {
  const int n = bytes <= 0 ? 0 : bytes > 0x7fffffffLL ? 0x7fffffff : (int)bytes;
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, n, 0x00020000);
}

DEV pt_u32x2 pt_ld64(pt_rsrc_t rs, uint32_t off) {
  return __builtin_bit_cast(pt_u32x2, __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 0));
}
DEV pt_u32x4 pt_ld128(pt_rsrc_t rs, uint32_t off) {
  return __builtin_bit_cast(pt_u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
}
DEV uint32_t pt_ld32(pt_rsrc_t rs, uint32_t off) { return __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0); }
DEV void pt_st64(pt_rsrc_t rs, uint32_t off, pt_u32x2 v) { __builtin_amdgcn_raw_buffer_store_b64(v, rs, off, 0, 0); }

// s_waitcnt vmcnt(n) for a runtime (uniform) n; n > 63 waits for 63 (stricter: safe)
#define PT_VMW(N) \
  case N:         \
    asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); \
    break;
DEV void pt_vmwait(int n) {
  switch (n) {
    PT_VMW(0) PT_VMW(1) PT_VMW(2) PT_VMW(3) PT_VMW(4) PT_VMW(5) PT_VMW(6) PT_VMW(7) PT_VMW(8) PT_VMW(9)
    PT_VMW(10) PT_VMW(11) PT_VMW(12) PT_VMW(13) PT_VMW(14) PT_VMW(15) PT_VMW(16) PT_VMW(17) PT_VMW(18)
    PT_VMW(19) PT_VMW(20) PT_VMW(21) PT_VMW(22) PT_VMW(23) PT_VMW(24) PT_VMW(25) PT_VMW(26) PT_VMW(27)
    PT_VMW(28) PT_VMW(29) PT_VMW(30) PT_VMW(31) PT_VMW(32) PT_VMW(33) PT_VMW(34) PT_VMW(35) PT_VMW(36)
    PT_VMW(37) PT_VMW(38) PT_VMW(39) PT_VMW(40) PT_VMW(41) PT_VMW(42) PT_VMW(43) PT_VMW(44) PT_VMW(45)
    PT_VMW(46) PT_VMW(47) PT_VMW(48) PT_VMW(49) PT_VMW(50) PT_VMW(51) PT_VMW(52) PT_VMW(53) PT_VMW(54)
    PT_VMW(55) PT_VMW(56) PT_VMW(57) PT_VMW(58) PT_VMW(59) PT_VMW(60) PT_VMW(61) PT_VMW(62)
    default:
      asm volatile("s_waitcnt vmcnt(63)" ::: "memory");
      break;
  }
}
#undef PT_VMW

// One operand's LDS-DMA sources for a tile: per piece j, the lane's byte offset from the k-step's
// descriptor base (gemm_glds.h image layouts: k-major [ROWS][8 slots of 8 k] with slot c of row r
// at c ^ (r & 7); m/n-major [64 k][ROWS/8 slots] with slot c of k-row kr at c ^ tr_swz(kr))
template <int ROWS, bool KMAJ, int NW>
struct PtSrc {
  static constexpr int PER = ROWS * 8 / (NW * 64);
  static_assert(PER >= 1 && PER * NW * 64 == ROWS * 8, "operand tile vs block");
  uint32_t voff[PER];
  DEV void set(long ld, int r0, int R, int w, int lane) {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int p = (j * NW + w) * 64 + lane;
      if constexpr (KMAJ) {
        const int r = p >> 3, c = (p & 7) ^ (r & 7);
        voff[j] = (uint32_t)(((long)min(r0 + r, R - 1) * ld + c * 8) * 2);
      } else {
        constexpr int SL = ROWS / 8;
        const int kr = p / SL, c = (p % SL) ^ (tr_swz(kr) & (SL - 1));
        const int col = min(r0 + c * 8, ((R - 1) >> 3) << 3);
        voff[j] = (uint32_t)(((long)kr * ld + col) * 2);
      }
    }
  }
  // piece j of the k-step whose descriptor is rs into the stage image img (soff: the sub-image's
  // byte offset from the descriptor base, a scalar)
  DEV void issue(int j, pt_rsrc_t rs, char* img, int w, int soff = 0) const {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(img + (j * NW + w) * 1024),
                                             16, voff[j], soff, 0, 0);
  }
};

// zero what this thread's DMA put at k >= K into a k-step's image (the K tail: slots past K of a
// k-major row hold the next row's elements; k-rows past K of m/n-major images read as zeros
// through the range check and are cleared here as well)
template <int ROWS, bool KMAJ, int NW>
DEV void pt_zero_tail(int k0, int K, char* img, int w, int lane) {
  constexpr int PER = ROWS * 8 / (NW * 64);
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int p = (j * NW + w) * 64 + lane;
    uint4* slot = (uint4*)(img + p * 16);
    if constexpr (KMAJ) {
      const int r = p >> 3;
      const int k = k0 + ((p & 7) ^ (r & 7)) * 8;
      if (k >= K) *slot = make_uint4(0u, 0u, 0u, 0u);
      else if (k + 8 > K) *slot = mask_tail<bf16>(*slot, K - k);
    } else {
      if (k0 + p / (ROWS / 8) >= K) *slot = make_uint4(0u, 0u, 0u, 0u);
    }
  }
}

struct PtArgs {
  const bf16* A;
  const bf16* B;
  void* C;
  long lda, ldb, ldc;
  int M, N, K;
  int tiles_n, ntiles, grp;
  imgcap_epilogue ep;
  const uint64_t* seed_ctr;
  int64_t a_bytes, b_bytes;                // operand extents (descriptor range checks)
  uint64_t c_bytes, res_bytes, aux_bytes;  // extents of C, res, aux
  int dbg;  // diagnostic build only (IMGCAP_PT_DBG): bit 1 no MFMAs, bit 2 no DMA after the prologue,
            // bit 3 phase stamps
};
#ifdef IMGCAP_STAMPS
#define PT_DBG(bit) ((a.dbg & (bit)) != 0)
#else
#define PT_DBG(bit) false
#endif

DEV float pt_bf_lo(uint32_t w) { return __uint_as_float(w << 16); }
DEV float pt_bf_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
DEV uint32_t pt_pack(float a, float b) {
  const bf16x2 v = {(bf16)a, (bf16)b};
  return __builtin_bit_cast(uint32_t, v);
}

// tile id -> (tile row, tile column): bands of `grp` tile rows walked column by column
DEV void pt_tile_coords(int L, int tiles_n, int tiles_m, int grp, int& tm, int& tn) {
  const int band = L / (grp * tiles_n), within = L - band * grp * tiles_n;
  const int rows = min(grp, tiles_m - band * grp);
  tm = band * grp + within % rows;
  tn = within / rows;
}

// The kernel argument block, re-read (s_load) where the rarely used fields are needed -- at a
// tile's epilogue and when the DMA stream enters a new tile -- through a pointer the compiler
// cannot see through, so the k-loop does not keep the whole epilogue description in SGPRs (it
// spilled ~100 SGPRs into VGPR lanes when they were kept live)
typedef const __attribute__((address_space(4))) PtArgs* pt_kptr;  // scalar (s_load) reads
DEV pt_kptr pt_kargs() {
  pt_kptr p = (pt_kptr)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(p));
  return p;
}

DEV imgcap_epilogue pt_load_ep(pt_kptr ka) {
  imgcap_epilogue e;
  e.bias = ka->ep.bias;
  e.colscale = ka->ep.colscale;
  e.rowscale = ka->ep.rowscale;
  e.res = ka->ep.res;
  e.aux = ka->ep.aux;
  e.ldr = ka->ep.ldr;
  e.ldaux = ka->ep.ldaux;
  e.drop_ld = ka->ep.drop_ld;
  e.seed = ka->ep.seed;
  e.alpha = ka->ep.alpha;
  e.beta = ka->ep.beta;
  e.drop_p = ka->ep.drop_p;
  e.aux_scale = ka->ep.aux_scale;
  e.act = ka->ep.act;
  e.c_dtype = ka->ep.c_dtype;
  e.rows_per_scale = ka->ep.rows_per_scale;
  e.drop_stream = ka->ep.drop_stream;
  e.split_k = ka->ep.split_k;
  e.c_scale = ka->ep.c_scale;
  return e;
}

// EK: which row x column operands the epilogue may read -- 0 none (bias / scales / GELU with the
// pre-activation written are all allowed), 1 the residual, 2 any (residual, saved operand for
// dGELU / the ReLU mask, old C for beta); fewer live registers for the common forms
// 8-wave blocks run one per CU; 4-wave blocks two per CU (both: two waves per SIMD)
// KS: 64-deep sub-images per stage (a k-step of 64 KS: one barrier and one round of bookkeeping
// per 2 KS half-steps of MFMAs; KS = 2 needs K % 128 == 0)
// WPE: waves per SIMD the registers are sized for -- 2 (<= 256 VGPRs + AGPRs a lane), or 1 for
// the 4-wave blocks with 128-row wave tiles (up to 512, the accumulators in AGPRs)
template <int BM, int BN, int WM, int WN, int S, bool AK, bool BKM, int EK, int KS = 1, int WPE = 2>
__global__ __launch_bounds__(WM* WN * 64, WPE) void gemm_pt_kernel(PtArgs a) {
  constexpr int NW = WM * WN;
  constexpr int TA = BM * 64 * 2, TB = BN * 64 * 2, SUB = TA + TB, STAGE = KS * SUB;
  constexpr int H = 2 * KS;  // 32-deep half-steps per k-step
  constexpr int FM = BM / WM / 16, FN = BN / WN / 16;
  using SrcA = PtSrc<BM, AK, NW>;
  using SrcB = PtSrc<BN, BKM, NW>;
  constexpr int PA = SrcA::PER, PB = SrcB::PER, LPT = KS * (PA + PB);  // DMA pieces per thread per k-step
  constexpr int NST = FM * FN;                                   // 8-byte stores per thread per epilogue
  static_assert(FM >= 1 && FN >= 1 && FM * 16 * WM == BM && FN * 16 * WN == BN, "wave tiles");
  static_assert(S >= 2 && S * STAGE * (NW == 4 && WPE == 2 ? 2 : 1) <= 160 * 1024, "stages");
#ifdef IMGCAP_STAMPS
  // diagnostic build: wave 0's s_memtime per iteration phase (first 64 iterations) kept in LDS
  // behind the stages and copied out at the end (a global store would enter the counted waits)
  constexpr int STAMP_BYTES = 64 * 8 * 8;
#else
  constexpr int STAMP_BYTES = 0;
#endif
  __shared__ __attribute__((aligned(16))) char smem[S * STAGE + STAMP_BYTES];
#ifdef IMGCAP_STAMPS
#define PT_STAMP(k)                                                                                     \
  do {                                                                                                  \
    if ((a.dbg & 8) && threadIdx.x == 0 && g < 64)                                                  \
      ((uint64_t*)(smem + S * STAGE))[g * 8 + (k)] = __builtin_amdgcn_s_memtime();                     \
  } while (0)
#else
#define PT_STAMP(k) \
  do {              \
  } while (0)
#endif

  const int K = a.K;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = w / WN, wn = w % WN;
  const int rb = wm * (BM / WM), cb = wn * (BN / WN);
  const int fr = lane & 15, fq = lane >> 4;

  // this block's tiles: slot, slot + G, ...; the blocks sharing an XCD (b % 8) own consecutive
  // slots, i.e. one rectangle of the output per round
  const int G = gridDim.x, b = blockIdx.x;
  // (XCD x = b % 8 holds G / 8 + (x < G % 8) blocks: a bijection onto 0 .. G - 1 for any G)
  const int xq = G / 8, xr = G % 8, xb = b % 8;
  const int slot = xb * xq + min(xb, xr) + b / 8;
  const int my_tiles = slot < a.ntiles ? (a.ntiles - 1 - slot) / G + 1 : 0;
  const int nk = (K + 64 * KS - 1) / (64 * KS);
  const int total = my_tiles * nk;
  const bool ktail = (K & 63) != 0;
  if (total == 0) return;

  auto coords = [&](pt_kptr ka, int it, int& m0, int& n0) {
    int tm, tn;
    pt_tile_coords(slot + it * G, ka->tiles_n, ka->ntiles / ka->tiles_n, ka->grp, tm, tn);
    m0 = tm * BM;
    n0 = tn * BN;
  };
  // the DMA stream: the next k-step to issue (tile is_it, k-step is_kt) as its descriptor words --
  // base address and range in bytes, advanced by one k-step's stride with scalar adds (a step
  // past the block's last tile gets range 0: its pieces read zeros into a stage no step reads)
  int is_kt = 0, is_it = 0;
  SrcA srcA;
  SrcB srcB;
  auto set_src = [&](int itile) {
    const pt_kptr ka = pt_kargs();
    int m0, n0;
    coords(ka, itile, m0, n0);
    srcA.set(ka->lda, m0, ka->M, w, lane);
    srcB.set(ka->ldb, n0, ka->N, w, lane);
  };
  set_src(0);
  const uint64_t a_base = (uint64_t)a.A, b_base = (uint64_t)a.B;
  const int a_ext = (int)a.a_bytes, b_ext = (int)a.b_bytes;  // host-checked < 2^31
  // bytes between two 64-deep sub-images; a k-step advances KS of them
  const int sa1 = AK ? 128 : 128 * (int)a.lda, sb1 = BKM ? 128 : 128 * (int)a.ldb;
  const int sa = KS * sa1, sb = KS * sb1;
  uint64_t da = a_base, db = b_base;
  int na = a_ext, nb = b_ext;
  // piece q of the pending k-step into the stage image st: sub-image q / (PA + PB), A pieces first
  auto issue_piece = [&](int q, pt_rsrc_t ra, pt_rsrc_t rb_, char* st) {
    constexpr int PU = PA + PB;
    const int u = q / PU, r = q % PU;
    if (r < PA) srcA.issue(r, ra, st + u * SUB, w, u * sa1);
    else srcB.issue(r - PA, rb_, st + u * SUB + TA, w, u * sb1);
  };
  auto advance = [&]() {  // the pending k-step has been issued
    if (++is_kt == nk) {
      is_kt = 0;
      da = a_base;
      db = b_base;
      const bool live = ++is_it < my_tiles;
      na = live ? a_ext : 0;
      nb = live ? b_ext : 0;
      if (live) set_src(is_it);
    } else {
      da += (uint32_t)sa;
      db += (uint32_t)sb;
      na = max(na - sa, 0);
      nb = max(nb - sb, 0);
    }
  };
  auto step_rsrcs = [&](pt_rsrc_t& ra, pt_rsrc_t& rb_) {
    ra = __builtin_amdgcn_make_buffer_rsrc((void*)da, 0, na, 0x00020000);
    rb_ = __builtin_amdgcn_make_buffer_rsrc((void*)db, 0, nb, 0x00020000);
  };
  auto issue_next = [&](char* st) {  // every piece of the pending k-step at once (the prologue)
    pt_rsrc_t ra, rb_;
    step_rsrcs(ra, rb_);
#pragma unroll
    for (int q = 0; q < LPT; ++q) issue_piece(q, ra, rb_, st);
    advance();
  };
  // the dropout seed mixed with the device step counter once, before any DMA is in flight (its
  // load would otherwise be waited for with everything else at the first epilogue)
  uint64_t seed_eff = a.ep.seed;
  if (a.ep.drop_p > 0.f) {
    seed_eff = eff_seed(a.ep.seed, a.seed_ctr);
    uint32_t lo = (uint32_t)seed_eff, hi = (uint32_t)(seed_eff >> 32);
    lo = __builtin_amdgcn_readfirstlane(lo);
    hi = __builtin_amdgcn_readfirstlane(hi);
    asm volatile("" : "+s"(lo), "+s"(hi));
    seed_eff = ((uint64_t)hi << 32) | lo;
  }
  // 8-byte stores per epilogue (x2 with the GELU pre-activation written)
  const int nst = (a.ep.aux != nullptr && a.ep.act == IMGCAP_ACT_GELU) ? 2 * NST : NST;

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragments of half-step kk of the k-step image img (two named register sets, no indexing)
  bf16x8 fa0[FM], fb0[FN], fa1[FM], fb1[FN];
  auto read_frags = [&](const char* img, int kk, bf16x8 (&fa)[FM], bf16x8 (&fb)[FN]) {
#pragma unroll
    for (int j = 0; j < FN; ++j) fb[j] = glds_frag_op<BN, BKM>(img + TA, cb + j * 16, kk, lane);
#pragma unroll
    for (int i = 0; i < FM; ++i) fa[i] = glds_frag_op<BM, AK>(img, rb + i * 16, kk, lane);
  };
  auto mfmas = [&](const bf16x8 (&fa)[FM], const bf16x8 (&fb)[FN]) {
    if (PT_DBG(2)) return;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)  // D^T: rows = output columns (B), columns = output rows (A)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
  };
  // the same MFMAs with the LPT DMA pieces of the pending k-step spread evenly between them (one
  // piece after every FM*FN/LPT MFMAs, order pinned): the texture unit works through the pieces
  // while the matrix pipe runs, instead of every wave stalling on its pieces at once after the
  // barrier (in-kernel stamps: 620 of a 2,640-cycle 256x128 k-step)
  auto mfmas_dma = [&](const bf16x8 (&fa)[FM], const bf16x8 (&fb)[FN], char* st) {
    pt_rsrc_t ra, rb_;
    step_rsrcs(ra, rb_);
    constexpr int NM = FM * FN;
    if (!PT_DBG(4)) {
#pragma unroll
      for (int q = 0; q < LPT; ++q) issue_piece(q, ra, rb_, st);
    }
    mfmas(fa, fb);
    // scheduling groups: (NM / LPT MFMAs, one DMA piece) x LPT, then the remaining MFMAs
#pragma unroll
    for (int q = 0; q < LPT; ++q) {
      __builtin_amdgcn_sched_group_barrier(0x008, NM / LPT, 0);  // MFMA
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);         // VMEM read (the LDS-DMA piece)
    }
    if constexpr (NM % LPT) __builtin_amdgcn_sched_group_barrier(0x008, NM % LPT, 0);
    advance();
  };

  // steps 0 .. S - 1 (an iteration g then always refills with step g + S)
#pragma unroll
  for (int h = 0; h < S; ++h) issue_next(smem + h * STAGE);
  // step 0 in LDS for every wave, its first half-step's fragments in registers
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"((S - 1) * LPT) : "memory");
  if (KS == 1 && ktail && nk == 1) {  // (KS > 1: the host guarantees K % (64 KS) == 0)
    pt_zero_tail<BM, AK, NW>(0, K, smem, w, lane);
    pt_zero_tail<BN, BKM, NW>(0, K, smem + TA, w, lane);
  }
  pt_lgkm0();
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  read_frags(smem, 0, fa0, fb0);

  int e1 = -1000, e2 = -1000;  // the iterations of the two latest epilogues
  int kt = 0, it = 0;
  int cur_off = 0;  // byte offset of step g's stage (the refill target too)
  for (int g = 0; g < total; ++g) {
    char* cur = smem + cur_off;
    const int nxt_off = cur_off == (S - 1) * STAGE ? 0 : cur_off + STAGE;
    const bool last_k = kt == nk - 1;
    PT_STAMP(0);
    // half-step h + 1 of step g from LDS while half-step h's MFMAs run (h = 0 .. H - 2; even
    // half-steps in set 0, odd in set 1)
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int h = 0; h < H - 1; ++h) {
      if (h & 1) {
        read_frags(cur + (h + 1) / 2 * SUB, (h + 1) & 1, fa0, fb0);
        mfmas(fa1, fb1);
      } else {
        read_frags(cur + (h + 1) / 2 * SUB, (h + 1) & 1, fa1, fb1);
        mfmas(fa0, fb0);
      }
    }
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    PT_STAMP(1);
    if (g + 1 < total) {
      // this thread's DMA of step g + 1 has landed once at most N younger ops are outstanding:
      // the pieces of steps g + 2 .. (issued so far) and the stores of epilogues after it
      if (e1 < g + 1 - S) {  // steady state: the S - 2 younger steps, no epilogue stores
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LPT * (S - 2)) : "memory");
      } else {
        pt_vmwait(LPT * (S - 2) + nst * ((e1 >= g + 1 - S) + (e2 >= g + 1 - S)));
      }
      if (KS == 1 && ktail && (kt == nk - 2 || nk == 1)) {  // step g + 1 is a tile's last (K tail) step
        pt_zero_tail<BM, AK, NW>((nk - 1) * 64, K, smem + nxt_off, w, lane);
        pt_zero_tail<BN, BKM, NW>((nk - 1) * 64, K, smem + nxt_off + TA, w, lane);
      }
    }
    PT_STAMP(2);
    pt_lgkm0();
    __builtin_amdgcn_s_barrier();  // step g + 1 in LDS for every wave; every wave is done reading step g
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    PT_STAMP(3);

    // the tile's last step: its epilogue operands are requested before the DMA of step g + S (the
    // compiler's wait for them then leaves that DMA in flight)
    imgcap_epilogue ep;
    int M = 0, N = 0, m0 = 0, n0 = 0;
    bool has_bias = false, has_cs = false, has_rs = false, has_res = false, has_beta = false, aux_out = false,
         aux_in = false;
    pt_rsrc_t rs_c = pt_rsrc(a.A, 0), rs_res = rs_c, rs_aux = rs_c, rs_bias = rs_c, rs_cs = rs_c, rs_rs = rs_c;
    pt_u32x4 bias_v[FN], cs_v[FN];
    pt_u32x2 res_v[EK >= 1 ? FM : 1][FN], aux_v[EK >= 2 ? FM : 1][FN], old_v[EK >= 2 ? FM : 1][FN];
    uint32_t rsc_v[FM];
    // byte offset of this lane's 4 columns of row m in a [.][ld] bf16 matrix (PT_OOB outside)
    auto off = [&](int m, int n, long ld) -> uint32_t {
      return m < M && n < N ? (uint32_t)(((uint64_t)m * ld + n) * 2u) : PT_OOB;
    };
    if (last_k) {
      const pt_kptr ka = pt_kargs();
      ep = pt_load_ep(ka);
      M = ka->M;
      N = ka->N;
      has_bias = ep.bias != nullptr;
      has_cs = ep.colscale != nullptr;
      has_rs = ep.rowscale != nullptr;
      has_res = EK >= 1 && ep.res != nullptr;
      has_beta = EK >= 2 && ep.beta != 0.f;
      aux_out = ep.aux != nullptr && ep.act == IMGCAP_ACT_GELU;
      aux_in = EK >= 2 && ep.aux != nullptr && ep.act != IMGCAP_ACT_GELU;  // dGELU / ReLU mask
      rs_c = pt_rsrc(ka->C, (int64_t)ka->c_bytes);
      rs_res = pt_rsrc(has_res ? ep.res : ka->C, has_res ? (int64_t)ka->res_bytes : 0);
      rs_aux = pt_rsrc(ep.aux ? ep.aux : ka->C, ep.aux ? (int64_t)ka->aux_bytes : 0);
      rs_bias = pt_rsrc(has_bias ? (const void*)ep.bias : ka->C, has_bias ? (int64_t)N * 4 : 0);
      rs_cs = pt_rsrc(has_cs ? (const void*)ep.colscale : ka->C, has_cs ? (int64_t)N * 4 : 0);
      rs_rs = pt_rsrc(has_rs ? (const void*)ep.rowscale : ka->C,
                      has_rs ? (int64_t)((M + ep.rows_per_scale - 1) / ep.rows_per_scale) * 4 : 0);
      coords(ka, it, m0, n0);
      // every load is issued, branch-free (an absent operand reads at an out-of-range offset): a
      // load under a condition left the compiler unsure whether the previous tile's load into the
      // same register was still pending, and it drained every DMA in flight (vmcnt(0)) first
      const long ldc_ = ka->ldc;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = n0 + cb + j * 16 + 4 * fq;
        bias_v[j] = pt_ld128(rs_bias, has_bias && n < N ? (uint32_t)n * 4u : PT_OOB);
        cs_v[j] = pt_ld128(rs_cs, has_cs && n < N ? (uint32_t)n * 4u : PT_OOB);
      }
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int m = m0 + rb + i * 16 + fr;
        rsc_v[i] = pt_ld32(rs_rs, has_rs && m < M ? (uint32_t)(m / ep.rows_per_scale) * 4u : PT_OOB);
        if constexpr (EK >= 1) {
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            const int n = n0 + cb + j * 16 + 4 * fq;
            res_v[i][j] = pt_ld64(rs_res, has_res ? off(m, n, ep.ldr) : PT_OOB);
            if constexpr (EK >= 2) {
              aux_v[i][j] = pt_ld64(rs_aux, aux_in ? off(m, n, ep.ldaux) : PT_OOB);
              old_v[i][j] = pt_ld64(rs_c, has_beta ? off(m, n, ldc_) : PT_OOB);
            }
          }
        }
      }
      // the scalar reads of the argument block done here (s_waitcnt lgkmcnt(0), vm/exp untouched):
      // left pending, the compiler's wait at the join below also held the next fragment reads
      // before the second half-step's MFMAs on every iteration
      __builtin_amdgcn_s_waitcnt(0xC07F);
    }
    // refill the stage step g was read from with step g + S; the first half of step g + 1 from
    // LDS while the second half of step g is multiplied
    PT_STAMP(4);
    if (g + 1 < total) read_frags(smem + nxt_off, 0, fa0, fb0);
    __builtin_amdgcn_s_setprio(1);
    mfmas_dma(fa1, fb1, cur);  // half-step H - 1 with the pieces of step g + S (into the stage step g was read from)
    __builtin_amdgcn_s_setprio(0);
    PT_STAMP(5);

    if (last_k) {
      __builtin_amdgcn_sched_barrier(0);
      const pt_kptr ka = pt_kargs();
      ep.seed = seed_eff;
      const long ldc = ka->ldc;
      // lane: row m = m0 + rb + 16 i + fr, columns n .. n + 3 = n0 + cb + 16 j + 4 fq + (0..3)
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int m = m0 + rb + i * 16 + fr;
        const float rsc = has_rs ? __uint_as_float(rsc_v[i]) : 1.f;
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int n = n0 + cb + j * 16 + 4 * fq;
          float x[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) x[r] = acc[i][j][r] * ep.alpha + (has_bias ? __uint_as_float(bias_v[j][r]) : 0.f);
          if (ep.act == IMGCAP_ACT_GELU) {
            if (aux_out) pt_st64(rs_aux, off(m, n, ep.ldaux), pt_u32x2{pt_pack(x[0], x[1]), pt_pack(x[2], x[3])});
#pragma unroll
            for (int r = 0; r < 4; ++r) x[r] = gelu_sig(x[r]);
          } else if (ep.act == IMGCAP_ACT_RELU) {
#pragma unroll
            for (int r = 0; r < 4; ++r) x[r] = fmaxf(x[r], 0.f);
          }
          if (ep.drop_p > 0.f) {
#pragma unroll
            for (int r = 0; r < 4; ++r)
              x[r] *= dropout_scale(ep.seed, ep.drop_stream, (uint64_t)m * ep.drop_ld + n + r, ep.drop_p);
          }
          if constexpr (EK >= 2) {
            if (aux_in) {
              const float hv[4] = {pt_bf_lo(aux_v[i][j][0]), pt_bf_hi(aux_v[i][j][0]), pt_bf_lo(aux_v[i][j][1]),
                                   pt_bf_hi(aux_v[i][j][1])};
              if (ep.act == IMGCAP_ACT_DGELU) {
#pragma unroll
                for (int r = 0; r < 4; ++r) x[r] *= gelu_grad(hv[r]);
              } else {
#pragma unroll
                for (int r = 0; r < 4; ++r) x[r] = hv[r] > 0.f ? x[r] * ep.aux_scale : 0.f;
              }
            }
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) x[r] *= (has_cs ? __uint_as_float(cs_v[j][r]) : 1.f) * rsc;
          if constexpr (EK >= 1) {
            if (has_res) {
              x[0] += pt_bf_lo(res_v[i][j][0]);
              x[1] += pt_bf_hi(res_v[i][j][0]);
              x[2] += pt_bf_lo(res_v[i][j][1]);
              x[3] += pt_bf_hi(res_v[i][j][1]);
            }
          }
          if constexpr (EK >= 2) {
            if (has_beta) {
              x[0] += ep.beta * pt_bf_lo(old_v[i][j][0]);
              x[1] += ep.beta * pt_bf_hi(old_v[i][j][0]);
              x[2] += ep.beta * pt_bf_lo(old_v[i][j][1]);
              x[3] += ep.beta * pt_bf_hi(old_v[i][j][1]);
            }
          }
          pt_st64(rs_c, off(m, n, ldc), pt_u32x2{pt_pack(x[0], x[1]), pt_pack(x[2], x[3])});
          acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
      e2 = e1;
      e1 = g;
    }
    PT_STAMP(6);
    cur_off = nxt_off;
    if (++kt == nk) {
      kt = 0;
      ++it;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#ifdef IMGCAP_STAMPS
  if ((a.dbg & 8) && threadIdx.x == 0 && g_dev_stamps) {
    const uint64_t* st = (const uint64_t*)(smem + S * STAGE);
    for (int i = 0; i < 64 * 8; ++i) g_dev_stamps[(long)blockIdx.x * 64 * 8 + i] = st[i];
  }
#endif
#undef PT_STAMP
}

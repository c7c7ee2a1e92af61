// Persistent-tile bf16 GEMM with the epilogue applied from registers -- included by gemm.hip.
//
// What bounds the LDS-DMA tiles of gemm_glds.h / gemm256.h on the encoder's and decoder's
// shapes (short K = 384-3072, a few hundred output tiles) is not the k-loop but what every tile
// pays around it (DESIGN.md §3 "What bounds the GEMMs"): the pipeline fill of its first k-step
// (5-8k cycles after launch), the fp32 tile staged through LDS for the epilogue (a 256x256 tile
// took ~20k cycles to leave), and grids that end in a partly filled round.  This kernel:
//   * runs one 512-thread block per CU that walks its tiles (tile ids slot, slot + G, ... with
//     each XCD's concurrent tiles a compact rectangle of the output, so they share A rows and B
//     columns in that XCD's L2);
//   * treats the block's (tile, k-step) sequence as ONE stream of BK = 64 stages: the LDS-DMA of
//     step g + S - 1 is issued while step g is multiplied, across tile boundaries, so the next
//     tile's first operands are already landing while the current tile's epilogue runs (counted
//     s_waitcnt vmcnt + raw s_barrier; the stores of an epilogue are counted too);
//   * computes D^T = B^T A^T on MFMA (v_mfma_f32_16x16x32_bf16 with the operands swapped), so a
//     lane ends with 4 consecutive output columns of one row: the epilogue (alpha, bias, GELU /
//     ReLU / dGELU, dropout, layer scale, drop-path row scale, residual, beta) runs on the
//     accumulators and leaves as 8-byte bf16 buffer stores -- no LDS round trip;
//   * loads the epilogue's operands (bias, scales, residual, saved pre-activation, old C) with
//     inline-asm buffer loads issued before the tile's last DMA, waited for by count, so the
//     compiler does not drain the DMA prefetch with a vmcnt(0) at their first use
//     (cdna_hip_programming.md §5 "Projection GEMM ... item 4(b)").
// Out-of-range rows / columns: operands read a clamped valid row (gemm_glds.h), epilogue loads
// and stores get an out-of-range buffer offset (the hardware drops the store / returns 0), so
// every wave issues the same instruction count and the counted waits stay exact.


typedef int pt_i32x4 __attribute__((ext_vector_type(4)));
typedef unsigned pt_u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned pt_u32x4 __attribute__((ext_vector_type(4)));

constexpr uint32_t PT_OOB = 0x80000000u;  // buffer offset past every buffer this kernel addresses

// raw buffer descriptor (stride 0, num_records = bytes; offsets past it read 0 / drop the store)
typedef __amdgpu_buffer_rsrc_t pt_rsrc_t;
DEV pt_rsrc_t pt_rsrc(const void* base, uint64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, (int)(bytes > 0x7fffffffull ? 0x7fffffffull : bytes),
                                           0x00020000);
}

// the epilogue's loads / stores as compiler-visible buffer ops.  (Inline-asm loads waited for by
// the kernel's own counts were tried first: the compiler takes an asm output as ready when the
// statement ends, and under register pressure it spilled a bias register straight after its
// load was issued -- the stored value was whatever the register held before the load returned.)
// The compiler's own vmcnt before a use counts the LDS-DMA pieces issued after the load, so the
// prefetch stays in flight; the kernel's counted waits below see these ops in the same order.
DEV pt_u32x2 pt_ld64(pt_rsrc_t rs, uint32_t off) {
  return __builtin_bit_cast(pt_u32x2, __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 0));
}
DEV pt_u32x4 pt_ld128(pt_rsrc_t rs, uint32_t off) {
  return __builtin_bit_cast(pt_u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
}
DEV uint32_t pt_ld32(pt_rsrc_t rs, uint32_t off) { return __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0); }
DEV void pt_st64(pt_rsrc_t rs, uint32_t off, pt_u32x2 v) {
  __builtin_amdgcn_raw_buffer_store_b64(v, rs, off, 0, 0);
}

// s_waitcnt vmcnt(n) for a runtime n (uniform): the immediates this kernel needs
#define PT_VMW(N) asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory")
DEV void pt_vmwait(int n) {
  switch (n) {
    case 0: PT_VMW(0); break;
    case 1: PT_VMW(1); break;
    case 2: PT_VMW(2); break;
    case 3: PT_VMW(3); break;
    case 4: PT_VMW(4); break;
    case 5: PT_VMW(5); break;
    case 6: PT_VMW(6); break;
    case 7: PT_VMW(7); break;
    case 8: PT_VMW(8); break;
    case 9: PT_VMW(9); break;
    case 10: PT_VMW(10); break;
    case 11: PT_VMW(11); break;
    case 12: PT_VMW(12); break;
    case 13: PT_VMW(13); break;
    case 14: PT_VMW(14); break;
    case 15: PT_VMW(15); break;
    case 16: PT_VMW(16); break;
    case 17: PT_VMW(17); break;
    case 18: PT_VMW(18); break;
    case 19: PT_VMW(19); break;
    case 20: PT_VMW(20); break;
    case 21: PT_VMW(21); break;
    case 22: PT_VMW(22); break;
    case 23: PT_VMW(23); break;
    case 24: PT_VMW(24); break;
    case 25: PT_VMW(25); break;
    case 26: PT_VMW(26); break;
    case 27: PT_VMW(27); break;
    case 28: PT_VMW(28); break;
    case 29: PT_VMW(29); break;
    case 30: PT_VMW(30); break;
    case 31: PT_VMW(31); break;
    case 32: PT_VMW(32); break;
    case 33: PT_VMW(33); break;
    case 34: PT_VMW(34); break;
    case 35: PT_VMW(35); break;
    case 36: PT_VMW(36); break;
    case 37: PT_VMW(37); break;
    case 38: PT_VMW(38); break;
    case 39: PT_VMW(39); break;
    case 40: PT_VMW(40); break;
    case 41: PT_VMW(41); break;
    case 42: PT_VMW(42); break;
    case 43: PT_VMW(43); break;
    case 44: PT_VMW(44); break;
    case 45: PT_VMW(45); break;
    case 46: PT_VMW(46); break;
    case 47: PT_VMW(47); break;
    default: PT_VMW(48); break;  // callers keep n <= 48 (static_assert in the kernel)
  }
}
#undef PT_VMW

// One operand's 64-deep k-tile -> its LDS image (gemm_glds.h layouts) by NW waves
template <int ROWS, bool KMAJ, int NW>
DEV void pt_issue(const bf16* __restrict__ P, long ld, int r0, int R, int k0, int K, char* img, int w, int lane) {
  constexpr int PER = ROWS * 8 / (NW * 64);
  static_assert(PER >= 1 && PER * NW * 64 == ROWS * 8, "operand tile vs block");
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int p0 = (j * NW + w) * 64;
    const int p = p0 + lane;
    const bf16* src;
    if constexpr (KMAJ) {
      const int r = p >> 3, c = (p & 7) ^ (r & 7);
      src = P + (long)min(r0 + r, R - 1) * ld + min(k0 + c * 8, ((K - 1) >> 3) << 3);
    } else {
      constexpr int SL = ROWS / 8;
      const int kr = p / SL, c = (p % SL) ^ (tr_swz(kr) & (SL - 1));
      const int col = min(r0 + c * 8, ((R - 1) >> 3) << 3);
      src = P + (long)min(k0 + kr, K - 1) * ld + col;
    }
    __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(img + p0 * 16), 16,
                                     0, 0);
  }
}

// Per-lane source of one operand's LDS-DMA pieces, fixed for a tile: the k-step only adds to it
// (the 64-bit row address math of pt_issue, ~14 VALU per piece, is paid once per tile)
template <int ROWS, bool KMAJ, int NW>
struct PtSrc {
  static constexpr int PER = ROWS * 8 / (NW * 64);
  const bf16* base[PER];  // k-major: row start + the slot's k offset; m/n-major: the slot's column
  int koff[PER];          // k-major: slot k offset (clamped per step); m/n-major: k row in the step
  DEV void set(const bf16* __restrict__ P, long ld, int r0, int R, int w, int lane) {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int p = (j * NW + w) * 64 + lane;
      if constexpr (KMAJ) {
        const int r = p >> 3, c = (p & 7) ^ (r & 7);
        base[j] = P + (long)min(r0 + r, R - 1) * ld;
        koff[j] = c * 8;
      } else {
        constexpr int SL = ROWS / 8;
        const int kr = p / SL, c = (p % SL) ^ (tr_swz(kr) & (SL - 1));
        base[j] = P + min(r0 + c * 8, ((R - 1) >> 3) << 3);
        koff[j] = kr;
      }
    }
  }
  // piece j of k-step kt into the stage image img (slots lane-linear per wave-instruction)
  DEV void issue(int j, long ld, int kt, int K, char* img, int w) const {
    const bf16* src;
    if constexpr (KMAJ) {
      src = base[j] + min(kt * 64 + koff[j], ((K - 1) >> 3) << 3);
    } else {
      src = base[j] + (long)min(kt * 64 + koff[j], K - 1) * ld;
    }
    __builtin_amdgcn_global_load_lds((const void*)src,
                                     (__attribute__((address_space(3))) void*)(img + (j * NW + w) * 64 * 16), 16, 0, 0);
  }
};

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
  uint64_t c_bytes, res_bytes, aux_bytes;  // extents of C, res, aux (buffer range checks)
  int dbg;  // diagnostic build only (IMGCAP_PT_DBG): bit 0 skips the MFMAs, 1 the operand DMA, 2 the barrier, 3 the wait
};

// the diagnostic switches exist only in the stamps build: in the product kernel they fold away, so
// the k-step is one basic block the scheduler can interleave (LDS reads of the next fragment group
// above the current MFMAs); a runtime test around each MFMA group had split it into ~20 blocks and
// serialised read -> wait -> MFMA
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

// EK: which row x column operands the epilogue may read -- 0 none (bias / scales / GELU with the
// pre-activation written are all allowed), 1 the residual, 2 any (residual, saved pre-activation
// for dGELU, old C for beta); fewer live registers for the common forms
// diagnostic build only (make diag): per-iteration s_memtime stamps of wave 0, iterations < 64,
// [block][iteration][phase]: 0 top, 1 waited, 2 past barrier, 3 issued, 4 multiplied, 5 end
#ifdef IMGCAP_STAMPS
#define PT_STAMP(k)                                                                                         \
  do {                                                                                                      \
    if (threadIdx.x == 0 && g_dev_stamps && g < 64)                                                         \
      g_dev_stamps[((long)blockIdx.x * 64 + g) * 8 + (k)] = __builtin_amdgcn_s_memtime();                   \
  } while (0)
#else
#define PT_STAMP(k) \
  do {              \
  } while (0)
#endif

template <int BM, int BN, int WM, int WN, int S, bool AK, bool BKM, int EK>
__global__ __launch_bounds__(WM* WN * 64, 1) void gemm_pt_kernel(PtArgs a) {
  constexpr int NW = WM * WN, NT = NW * 64;
  constexpr int TA = BM * 64 * 2, TB = BN * 64 * 2, STAGE = TA + TB;
  constexpr int FM = BM / WM / 16, FN = BN / WN / 16;
  constexpr int LPT = BM * 8 / NT + BN * 8 / NT;  // LDS-DMA instructions per thread per k-step
  constexpr int NST = FM * FN;                    // 8-byte stores per thread per epilogue (x2 with aux)
  static_assert(S >= 3 && S * STAGE <= 160 * 1024, "stages");
  static_assert((S - 2) * LPT + 2 * NST <= 48, "counted waits");
  __shared__ __attribute__((aligned(16))) char smem[S * STAGE];

  imgcap_epilogue ep = a.ep;
  if (ep.drop_p > 0.f) ep.seed = eff_seed(ep.seed, a.seed_ctr);
  const int M = a.M, N = a.N, K = a.K;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = w / WN, wn = w % WN;
  const int rb = wm * (BM / WM), cb = wn * (BN / WN);
  const int fr = lane & 15, fq = lane >> 4;
  const int tiles_n = a.tiles_n, ntiles = a.ntiles, tiles_m = ntiles / tiles_n;

  // this block's tiles: slot, slot + G, ...; the blocks sharing an XCD (b % 8) own consecutive
  // slots, i.e. one rectangle of the output per round
  const int G = gridDim.x, b = blockIdx.x;
  const int slot = (G % 8 == 0) ? (b % 8) * (G / 8) + b / 8 : b;
  const int my_tiles = slot < ntiles ? (ntiles - 1 - slot) / G + 1 : 0;
  const int nk = (K + 63) / 64;
  const int total = my_tiles * nk;

  auto coords = [&](int it, int& m0, int& n0) {  // once per tile (divisions)
    int tm, tn;
    pt_tile_coords(slot + it * G, tiles_n, tiles_m, a.grp, tm, tn);
    m0 = tm * BM;
    n0 = tn * BN;
  };
  // the DMA stream's position (tile, k-step, stage) advanced incrementally: no per-step division
  int is_kt = 0, is_it = 0, is_st = 0;
  PtSrc<BM, AK, NW> srcA;
  PtSrc<BN, BKM, NW> srcB;
  auto set_src = [&](int itile) {
    int m0, n0;
    coords(itile, m0, n0);
    srcA.set(a.A, a.lda, m0, M, w, lane);
    srcB.set(a.B, a.ldb, n0, N, w, lane);
  };
  if (my_tiles > 0) set_src(0);
  constexpr int PA = PtSrc<BM, AK, NW>::PER, PB = PtSrc<BN, BKM, NW>::PER;
  static_assert(PA + PB == LPT, "pieces");
  // piece q (0 .. LPT-1) of the pending k-step (A pieces first)
  auto issue_piece = [&](int q) {
    if (PT_DBG(2)) return;
    char* st = smem + is_st * STAGE;
    if (q < PA) srcA.issue(q, a.lda, is_kt, K, st, w);
    else srcB.issue(q - PA, a.ldb, is_kt, K, st + TA, w);
  };
  auto advance = [&]() {  // the pending k-step has been issued
    is_st = is_st == S - 1 ? 0 : is_st + 1;
    if (++is_kt == nk) {
      is_kt = 0;
      if (++is_it < my_tiles) set_src(is_it);
    }
  };
  auto issue_next = [&]() {
#pragma unroll
    for (int q = 0; q < LPT; ++q) issue_piece(q);
    advance();
  };

  const bool has_bias = ep.bias != nullptr, has_cs = ep.colscale != nullptr, has_rs = ep.rowscale != nullptr;
  const bool has_res = EK >= 1 && ep.res != nullptr, has_beta = EK >= 2 && ep.beta != 0.f;
  const bool aux_out = ep.aux != nullptr && ep.act == IMGCAP_ACT_GELU;            // pre-activation written
  const bool aux_in = EK >= 2 && ep.aux != nullptr && ep.act == IMGCAP_ACT_DGELU;  // saved pre-activation read
  const int nst = aux_out ? 2 * NST : NST;
  const pt_rsrc_t rs_c = pt_rsrc(a.C, a.c_bytes);
  const pt_rsrc_t rs_res = pt_rsrc(has_res ? ep.res : a.C, has_res ? a.res_bytes : 0);
  const pt_rsrc_t rs_aux = pt_rsrc(ep.aux ? ep.aux : a.C, ep.aux ? a.aux_bytes : 0);
  const pt_rsrc_t rs_bias = pt_rsrc(has_bias ? (const void*)ep.bias : a.C, has_bias ? (uint64_t)N * 4 : 0);
  const pt_rsrc_t rs_cs = pt_rsrc(has_cs ? (const void*)ep.colscale : a.C, has_cs ? (uint64_t)N * 4 : 0);
  const pt_rsrc_t rs_rs =
      pt_rsrc(has_rs ? (const void*)ep.rowscale : a.C, has_rs ? (uint64_t)((M + ep.rows_per_scale - 1) / ep.rows_per_scale) * 4 : 0);

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int h = 0; h < S - 1 && h < total; ++h) issue_next();

  int last_epi = -1000;  // iteration of the latest epilogue
  int kt = 0, cur_st = 0, it = 0;
  for (int g = 0; g < total; ++g) {
    PT_STAMP(0);
    // wait for this thread's DMA of step g (ops issued after it may stay in flight)
    const int newer = min(S - 2, total - 1 - g);
    if (g > last_epi + S - 2 && !PT_DBG(8)) {  // (after an epilogue's wait, steps <= last_epi + S - 2 have landed)
      pt_vmwait(newer * LPT + (g == last_epi + S - 1 ? nst : 0));
    }
    PT_STAMP(1);
    char* cur = smem + cur_st * STAGE;
    if ((kt + 1) * 64 > K) {
      pt_zero_tail<BM, AK, NW>(kt * 64, K, cur, w, lane);
      pt_zero_tail<BN, BKM, NW>(kt * 64, K, cur + TA, w, lane);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (!PT_DBG(4)) __builtin_amdgcn_s_barrier();  // step g in LDS for every wave; every wave is past step g - 1
    asm volatile("" ::: "memory");
    PT_STAMP(2);

    const bool last_k = kt == nk - 1;
    int m0 = 0, n0 = 0;
    // epilogue operands of this tile (issued before the next DMA so the counted wait after the
    // MFMAs leaves that DMA in flight)
    pt_u32x4 bias_v[FN], cs_v[FN];
    pt_u32x2 res_v[EK >= 1 ? FM : 1][FN], aux_v[EK >= 2 ? FM : 1][FN], old_v[EK >= 2 ? FM : 1][FN];
    uint32_t rsc_v[FM];
    // byte offset of this lane's 4 columns of row m in a [.][ld] bf16 matrix (PT_OOB outside)
    auto off = [&](int m, int n, long ld) -> uint32_t {
      return m < M && n < N ? (uint32_t)(((uint64_t)m * ld + n) * 2u) : PT_OOB;
    };
    if (last_k) {
      coords(it, m0, n0);
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = n0 + cb + j * 16 + 4 * fq;
        const uint32_t bo = n < N ? (uint32_t)n * 4u : PT_OOB;
        if (has_bias) bias_v[j] = pt_ld128(rs_bias, bo);
        if (has_cs) cs_v[j] = pt_ld128(rs_cs, bo);
      }
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int m = m0 + rb + i * 16 + fr;
        if (has_rs) rsc_v[i] = pt_ld32(rs_rs, m < M ? (uint32_t)(m / ep.rows_per_scale) * 4u : PT_OOB);
        if constexpr (EK >= 1) {
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            const int n = n0 + cb + j * 16 + 4 * fq;
            if (has_res) res_v[i][j] = pt_ld64(rs_res, off(m, n, ep.ldr));
            if constexpr (EK >= 2) {
              if (aux_in) aux_v[i][j] = pt_ld64(rs_aux, off(m, n, ep.ldaux));
              if (has_beta) old_v[i][j] = pt_ld64(rs_c, off(m, n, a.ldc));
            }
          }
        }
      }
    }
    const bool more = g + S - 1 < total;
    PT_STAMP(3);
    // the k-step: 2 x FM groups of FN MFMAs; the LDS-DMA pieces of step g + S - 1 (into the stage
    // step g - 1 used, free since the barrier) are issued one per group, so the texture unit
    // works through them while the matrix pipe runs instead of holding every wave at once
    constexpr int NG = 2 * FM;
    static_assert(LPT <= NG, "one DMA piece per MFMA group at most");
    // one straight-line body per case (DMA pieces or none), no runtime test inside
    auto kstep = [&](auto with_dma) {
      constexpr bool WD = decltype(with_dma)::value;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 af[FM], bfr[FN];
        if (!PT_DBG(1)) {
#pragma unroll
          for (int i = 0; i < FM; ++i) af[i] = glds_frag_op<BM, AK>(cur, rb + i * 16, kk, lane);
#pragma unroll
          for (int j = 0; j < FN; ++j) bfr[j] = glds_frag_op<BN, BKM>(cur + TA, cb + j * 16, kk, lane);
        }
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          if (!PT_DBG(1)) {
#pragma unroll
            for (int j = 0; j < FN; ++j)  // D^T: rows = output columns (B), columns = output rows (A)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
          }
          const int gi = kk * FM + i;  // compile-time after unrolling
          // spread the LPT pieces evenly over the NG groups
          if constexpr (WD) {
            if ((gi * LPT) / NG != ((gi + 1) * LPT) / NG) issue_piece((gi * LPT) / NG);
          }
        }
      }
    };
    if (more) kstep(std::true_type{});
    else kstep(std::false_type{});
    if (more) advance();
    PT_STAMP(4);
    if (last_k) {
      if (more) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LPT) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_sched_barrier(0);
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
            for (int r = 0; r < 4; r += 2) {
              const f32x2 gg = gelu_fast2(f32x2{x[r], x[r + 1]});
              x[r] = gg[0];
              x[r + 1] = gg[1];
            }
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
#pragma unroll
            for (int r = 0; r < 4; ++r) x[r] *= gelu_grad(hv[r]);
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
          pt_st64(rs_c, off(m, n, a.ldc), pt_u32x2{pt_pack(x[0], x[1]), pt_pack(x[2], x[3])});
          acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
      last_epi = g;
    }
    PT_STAMP(5);
    cur_st = cur_st == S - 1 ? 0 : cur_st + 1;
    if (++kt == nk) {
      kt = 0;
      ++it;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}


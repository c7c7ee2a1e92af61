// 128x128x64 bf16 GEMM tile with LDS-DMA staging — included by gemm.hip.
//
// Every operand layout (k-major: nn.Linear forward; m/n-major: the weight-gradient and
// input-gradient forms) with K % 64 == 0 — the bulk of the encoder / decoder projections and
// their backward.  Each k-tile of A and B (128 rows x 64 k = 16 KiB each) is copied
// global -> LDS by global_load_lds_dwordx4 (no VGPR staging, cdna_hip_programming.md §5
// "Async global->LDS copy"), 4 per operand per thread, into a lane-linear image whose 16-byte
// slots are XOR-swizzled on the SOURCE address; fragment reads apply the same involution
// (ds_read_b128 for k-major images, hardware-transposed ds_read_b64_tr_b16 for m/n-major).  Two stages: the DMA of tile k+1 is in
// flight while tile k is multiplied (counted s_waitcnt vmcnt + raw s_barrier, never a
// vmcnt(0) in the loop).  Without staging registers the kernel fits two waves per SIMD, so
// two blocks share a CU and one block's prologue / epilogue hides under the other's MFMAs.
// Rows past M / N read a clamped valid row (their outputs are masked in the epilogue); a K
// tail (K % 64 != 0) is zeroed in LDS after its DMA lands.  With kslice > 0, grid.z walks K
// slices and each block stores its fp32 partial tile into workspace plane z (split-K).

// One operand's 64-deep k-tile -> its LDS image by LDS-DMA, 16-byte slots lane-linear per
// wave-instruction (1 KiB = 64 slots), swizzle applied on the source address:
//   k-major ([rows][K] in memory): image [ROWS][8 slots of 8 k]; slot c of row r at c ^ (r & 7)
//   m/n-major ([K][rows]):          image [64 k][ROWS/8 slots of 8 rows]; slot c of k-row kr at
//                                   c ^ tr_swz(kr), read back transposed by ds_read_b64_tr_b16
DEV int tr_swz(int kr) { return 2 * ((kr & 3) | (((kr >> 3) & 1) << 2)); }

template <int ROWS, bool KMAJ>
DEV void glds_issue_op(const bf16* __restrict__ P, long ld, int r0, int R, int k0, int K, char* img, int w,
                       int lane) {
  constexpr int PER = ROWS * 8 / 256;  // 16-byte slots per thread
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int p0 = (j * 4 + w) * 64;  // first slot of this wave-instruction
    const int p = p0 + lane;
    const bf16* src;
    if constexpr (KMAJ) {
      const int r = p >> 3, c = (p & 7) ^ (r & 7);
      // slots at or past K re-read the last (8-aligned) slot of the row; zeroed after landing
      src = P + (long)min(r0 + r, R - 1) * ld + min(k0 + c * 8, ((K - 1) >> 3) << 3);
    } else {
      constexpr int SL = ROWS / 8;
      const int kr = p / SL, c = (p % SL) ^ (tr_swz(kr) & (SL - 1));
      const int col = min(r0 + c * 8, ((R - 1) >> 3) << 3);  // past-the-end slots re-read a valid one
      src = P + (long)min(k0 + kr, K - 1) * ld + col;
    }
    __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(img + p0 * 16), 16,
                                     0, 0);
  }
}

// Zero what this thread's DMA put past K into a k-tile (K % 64 != 0): whole slots, and for
// k-major images the elements >= K of the slot that straddles K.
template <int ROWS, bool KMAJ>
DEV void glds_zero_tail(int k0, int K, char* img, int w, int lane) {
  constexpr int PER = ROWS * 8 / 256;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int p = (j * 4 + w) * 64 + lane;
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

typedef short glds_v4s16 __attribute__((ext_vector_type(4)));
typedef short glds_v8s16 __attribute__((ext_vector_type(8)));

// A-/B-operand fragment (row row0 + lane&15, k = 32*kk + 8*(lane>>4) + 0..7)
template <int ROWS, bool KMAJ>
DEV bf16x8 glds_frag_op(const char* img, int row0, int kk, int lane) {
  const int fr = lane & 15, fq = lane >> 4;
  if constexpr (KMAJ) {
    const int r = row0 + fr, c = kk * 4 + fq;
    return *(const bf16x8*)(img + ((r << 3) + (c ^ (r & 7))) * 16);
  } else {
    // lane 4q+p of a 16-lane group: k-row 32kk + 8g + q (+4 for the upper half), columns
    // row0 + 4p .. +3; the hardware transpose hands lane i column i of the 4 k-rows
    const int q = fr >> 2, p = fr & 3, g = fq;
    const int kr = kk * 32 + 8 * g + q;
    const int col = row0 + 4 * p;
    constexpr int SM = ROWS / 8 - 1;  // 64-row images have 8 slots per k-row: 3-bit swizzle
    const int byte_lo = kr * (ROWS * 2) + (((col >> 3) ^ (tr_swz(kr) & SM)) << 4) + ((col & 7) << 1);
    const int byte_hi = (kr + 4) * (ROWS * 2) + (((col >> 3) ^ (tr_swz(kr + 4) & SM)) << 4) + ((col & 7) << 1);
    typedef __attribute__((address_space(3))) glds_v4s16 lds_v4s16;
    const glds_v4s16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s16*)(img + byte_lo));
    const glds_v4s16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s16*)(img + byte_hi));
    const glds_v8s16 all = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, all);
  }
}

// One BM x BN output tile (rows m0.., columns n0..) over k-tiles of slice kz (split-K when
// kslice > 0): the body shared by the single-problem and the grouped launch.
template <int BM, int BN, bool AK, bool BKM, int S>
DEV void glds_tile(const bf16* __restrict__ A, long lda, const bf16* __restrict__ B, long ldb, void* __restrict__ C,
                   long ldc, int M, int N, int K, const imgcap_epilogue& ep, int vec_ok, int kslice, int m0, int n0,
                   int kz) {
  constexpr int TILE_A = BM * 64 * 2, TILE_B = BN * 64 * 2, STAGE = TILE_A + TILE_B;
  constexpr int TM = BM / 32, TN = BN / 32;  // 16x16 fragments per wave (2 x 2 waves)
  constexpr int LDT = BN + 4, EPI_ROWS = BM / 2;
  constexpr int LPT = BM * 8 / 256 + BN * 8 / 256;  // LDS-DMA instructions per thread per k-tile
  static_assert(EPI_ROWS * LDT * 4 <= S * STAGE, "epilogue tile fits the stages");
  __shared__ __attribute__((aligned(16))) char smem[S * STAGE];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int rb = wm * (BM / 2), cb = wn * (BN / 2);
  const int fr = lane & 15, fq = lane >> 4;

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // k-tiles [kt0, nk): the whole K, or slice blockIdx.z of a split-K launch (kslice % 64 == 0).
  // S stages: tiles kt+1 .. kt+S-1 are in flight while tile kt is multiplied.
  const int kt0 = kslice ? kz * (kslice / 64) : 0;
  const int nk = kslice ? min((K + 63) / 64, kt0 + kslice / 64) : (K + 63) / 64;
#pragma unroll
  for (int i = 0; i < S - 1; ++i) {
    if (kt0 + i < nk) {
      char* st = smem + i * STAGE;
      glds_issue_op<BM, AK>(A, lda, m0, M, (kt0 + i) * 64, K, st, w, lane);
      glds_issue_op<BN, BKM>(B, ldb, n0, N, (kt0 + i) * 64, K, st + TILE_A, w, lane);
    }
  }
  // (a one-barrier-per-k-tile order -- wait, barrier, refill the stage of tile k-1, multiply --
  // measured slower: C2 GEMM census 687 -> 714 us, C3 17.1k -> 16.6k img/s; removed in round 4)
  for (int kt = kt0; kt < nk; ++kt) {
    const int r = kt - kt0;
    char* cur = smem + (r % S) * STAGE;
    if (kt + S - 1 < nk) {
      char* nxt = smem + ((r + S - 1) % S) * STAGE;
      glds_issue_op<BM, AK>(A, lda, m0, M, (kt + S - 1) * 64, K, nxt, w, lane);
      glds_issue_op<BN, BKM>(B, ldb, n0, N, (kt + S - 1) * 64, K, nxt + TILE_A, w, lane);
    }
    // this thread's copies of tile kt are older than the (newer tiles) x LPT still allowed out
    const int newer = min(S - 1, nk - 1 - kt);
    if (newer == 0) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if ((kt + 1) * 64 > K) {  // K tail: clear the slots past K that this thread's DMA filled
        glds_zero_tail<BM, AK>(kt * 64, K, cur, w, lane);
        glds_zero_tail<BN, BKM>(kt * 64, K, cur + TILE_A, w, lane);
      }
    } else if (newer == 1) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LPT) : "memory");
    } else if (newer == 2) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * LPT) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * LPT) : "memory");
    }
    __builtin_amdgcn_s_barrier();  // every wave's part of tile kt is in LDS
    asm volatile("" ::: "memory");
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = glds_frag_op<BM, AK>(cur, rb + i * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = glds_frag_op<BN, BKM>(cur + TILE_A, cb + j * 16, kk, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // everyone is done reading `cur` before its refill
    asm volatile("" ::: "memory");
  }

  float* tile = (float*)smem;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    if (wm == pass) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) tile[(i * 16 + 4 * fq + r) * LDT + cb + j * 16 + fr] = acc[i][j][r];
    }
    __syncthreads();
    if (kslice)
      partial_from_lds<BN>(tile, LDT, EPI_ROWS, m0 + pass * EPI_ROWS, n0, M, N, (float*)C + (long)kz * M * N);
    else
      epilogue_tile<BN, EPI_ROWS, 256, (EPI_ROWS * BN / 2048 >= 2 ? 2 : 1)>(ep, tile, LDT, m0 + pass * EPI_ROWS, n0, M,
                                                                            N, C, ldc, vec_ok != 0);
    __syncthreads();
  }
}

// Blocks per CU the stages' LDS allows (160 KiB), at most 4: 128x128 x 2 stages two, the
// small-grid 64x64 tile four (2 stages), three (3) or two (4)
template <int BM, int BN, int S>
constexpr int glds_blocks_per_cu() {
  constexpr int lds = S * (BM + BN) * 64 * 2;
  return 160 * 1024 / lds < 4 ? 160 * 1024 / lds : 4;
}

// Block -> output tile.  The hardware deals blocks round-robin over the 8 XCDs (block b on XCD
// b % 8, MI355X_MICROARCH.md "Workgroup dispatch"); each XCD gets a contiguous run of tile ids
// (xcd_remap).  With grp == 0 ids walk the tile grid row-major, so an XCD's run is a band of
// whole tile rows: it reads all of B through its own L2 (the vocab projection: every XCD reads
// the whole 9.7 MB weight).  With grp > 0 ids walk bands of grp tile rows column by column, so
// an XCD's run is a grp x (run / grp) rectangle; grp ~ sqrt(run) balances its A and B bytes.
DEV void glds_tile_order(int grp, int& bx, int& by) {
  xcd_remap(bx, by);
  if (grp <= 0) return;
  const int nx = gridDim.x, ny = gridDim.y;
  const int id = by * nx + bx;
  const int band = id / (grp * nx), within = id - band * grp * nx;
  const int rows = min(grp, ny - band * grp);
  by = band * grp + within % rows;
  bx = within / rows;
}

template <int BM, int BN, bool AK, bool BKM, int S>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(glds_blocks_per_cu<BM, BN, S>(),
                                                                     glds_blocks_per_cu<BM, BN, S>()))) void
gemm_glds_kernel(const bf16* __restrict__ A, long lda, const bf16* __restrict__ B, long ldb, void* __restrict__ C,
                 long ldc, int M, int N, int K, imgcap_epilogue ep, int vec_ok, const uint64_t* seed_ctr,
                 int kslice, int grp) {
  if (ep.drop_p > 0.f) ep.seed = eff_seed(ep.seed, seed_ctr);
  int bx, by;
  glds_tile_order(grp, bx, by);
  glds_tile<BM, BN, AK, BKM, S>(A, lda, B, ldb, C, ldc, M, N, K, ep, vec_ok, kslice, by * BM, bx * BN, blockIdx.z);
}

// ---- grouped launch: many independent fp32-output products in one grid ------------------
// (the weight gradients of a whole backward pass, deferred to its end: hundreds of 128x128
// tiles at once instead of one small grid + split-K + reduce per product).  Block b walks the
// problems' tile prefix; ids are dealt XCD-contiguously so a problem's tiles share an L2.
constexpr int GEMM_GROUP_MAX = 48;
struct GemmGroup {
  int n;
  int first[GEMM_GROUP_MAX + 1];
  imgcap_gemm_problem p[GEMM_GROUP_MAX];
};

template <bool AK, bool BKM>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void gemm_glds_grouped_kernel(
    GemmGroup g) {
  const int nwg = gridDim.x, orig = blockIdx.x;
  int id = orig;
  if (nwg >= 64) {
    const int xcd = orig % 8, q = nwg / 8, r = nwg % 8;
    id = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
  }
  int k = 0;
  while (k + 1 < g.n && id >= g.first[k + 1]) ++k;
  const imgcap_gemm_problem& p = g.p[k];
  const int local = id - g.first[k];
  const int nx = (p.N + 127) / 128;
  imgcap_epilogue ep{};
  ep.alpha = p.alpha;
  ep.beta = p.beta;
  ep.c_dtype = IMGCAP_F32;
  ep.rows_per_scale = 1;
  const int vec_ok = (((uintptr_t)p.C) & 15) == 0 && p.ldc % 8 == 0;
  glds_tile<128, 128, AK, BKM, 2>((const bf16*)p.A, p.lda, (const bf16*)p.B, p.ldb, p.C, p.ldc, p.M, p.N, p.K, ep,
                                  vec_ok, 0, (local / nx) * 128, (local % nx) * 128, 0);
}

// 256x256 bf16 GEMM tile, 8 waves, LDS-DMA staging with an S-deep pipeline — included by
// gemm.hip.
//
// Why a second tile: operand delivery into LDS is what bounds these GEMMs on MI355X.  Measured
// (tools/microbench.py probe): the 128x128 / 4-wave kernel (gemm_glds.h) settles near 500
// TFLOP/s on long grids = ~30 GB/s of LDS-DMA per CU at its 64 FLOP/B; the per-CU fill rate,
// not MFMA issue, is the ceiling, so the tile's FLOP per loaded byte is the lever.  A 256x256
// tile loads 128 FLOP/B.  Each wave owns a 128x64 output block (8 x 4 fragments of 16x16; 12
// fragment reads per 32 MFMAs).  The k-step is BK = 32 deep (32 KiB per stage: A then B
// image) so S = 4 stages fit in 128 KiB and three k-steps of DMA stay in flight while one is
// multiplied -- the DMA latency under load (~1-2 us) is what a 2-stage 64-deep pipeline
// exposes (cdna_hip_programming.md §5, "Pipelining across barriers": counted vmcnt, raw
// s_barrier, never vmcnt(0) in the loop).
// LDS images (lane-linear per wave-instruction, swizzle applied on the source address):
//   k-major [rows][BK]: slot c (8 k) of row r at c ^ swz(r), swz = r&7 (BK 64) / (r>>2)&3 (BK 32)
//     -> each 16-lane ds_read_b128 pass covers all 16 slots of a 256-byte bank row
//   m/n-major [BK][rows]: as gemm_glds.h (tr_swz), read by ds_read_b64_tr_b16.
// Rows past M / N read a clamped valid row (outputs masked), a K tail is zeroed in LDS after
// its DMA lands, the fp32 tile leaves through LDS in four 64-row passes into the shared
// epilogue (bias, activation, dropout, scales, residual, beta).
#ifdef IMGCAP_STAMPS  // diagnostic build only (make diag): per-block s_memtime stamps
__device__ unsigned long long* g_dev_stamps;
#define G256_STAMP(i)                                                                                  \
  do {                                                                                                 \
    if (threadIdx.x == 0 && g_dev_stamps)                                                              \
      g_dev_stamps[(blockIdx.y * gridDim.x + blockIdx.x) * 8 + (i)] = __builtin_amdgcn_s_memtime();    \
  } while (0)
#else
#define G256_STAMP(i) \
  do {                \
  } while (0)
#endif

template <int BK>
DEV int kswz(int r) {
  return BK == 64 ? (r & 7) : ((r >> 2) & 3);
}

template <int ROWS, int BK, bool KMAJ>
DEV void g8_issue(const bf16* __restrict__ P, long ld, int r0, int R, int k0, int K, char* img, int w, int lane) {
  constexpr int PER = ROWS * (BK / 8) / 512;  // 16-byte slots per thread (8 waves)
  constexpr int SPR = BK / 8;                 // slots per k-major row
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int p0 = (j * 8 + w) * 64;
    const int p = p0 + lane;
    const bf16* src;
    if constexpr (KMAJ) {
      const int r = p / SPR, c = (p % SPR) ^ kswz<BK>(r);
      src = P + (long)min(r0 + r, R - 1) * ld + min(k0 + c * 8, ((K - 1) >> 3) << 3);
    } else {
      constexpr int SL = ROWS / 8;
      const int kr = p / SL, c = (p % SL) ^ tr_swz(kr);
      const int col = min(r0 + c * 8, ((R - 1) >> 3) << 3);
      src = P + (long)min(k0 + kr, K - 1) * ld + col;
    }
    __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(img + p0 * 16), 16,
                                     0, 0);
  }
}

template <int ROWS, int BK, bool KMAJ>
DEV void g8_zero_tail(int k0, int K, char* img, int w, int lane) {
  constexpr int PER = ROWS * (BK / 8) / 512;
  constexpr int SPR = BK / 8;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int p = (j * 8 + w) * 64 + lane;
    uint4* slot = (uint4*)(img + p * 16);
    if constexpr (KMAJ) {
      const int r = p / SPR;
      const int k = k0 + ((p % SPR) ^ kswz<BK>(r)) * 8;
      if (k >= K) *slot = make_uint4(0u, 0u, 0u, 0u);
      else if (k + 8 > K) *slot = mask_tail<bf16>(*slot, K - k);
    } else {
      if (k0 + p / (ROWS / 8) >= K) *slot = make_uint4(0u, 0u, 0u, 0u);
    }
  }
}

// fragment (row row0 + lane&15, k = 32*kk + 8*(lane>>4) + 0..7) of a BK-deep image
template <int ROWS, int BK, bool KMAJ>
DEV bf16x8 g8_frag(const char* img, int row0, int kk, int lane) {
  if constexpr (KMAJ) {
    constexpr int SPR = BK / 8;
    const int r = row0 + (lane & 15), c = kk * 4 + (lane >> 4);
    return *(const bf16x8*)(img + (r * SPR + (c ^ kswz<BK>(r))) * 16);
  } else {
    return glds_frag_op<ROWS, false>(img, row0, kk, lane);
  }
}

template <int BK, int S, bool AK, bool BKM>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void gemm256_kernel(
    const bf16* __restrict__ A, long lda, const bf16* __restrict__ B, long ldb, void* __restrict__ C, long ldc,
    int M, int N, int K, imgcap_epilogue ep, int vec_ok, const uint64_t* seed_ctr, int kslice) {
  constexpr int BM = 256, BN = 256;
  constexpr int TILE_A = BM * BK * 2, TILE_B = BN * BK * 2, STAGE = TILE_A + TILE_B;
  constexpr int TM = 8, TN = 4;              // 16x16 fragments per wave: 128 rows x 64 columns
  constexpr int LDT = BN + 4, EPI_ROWS = 128;  // two passes: one per wave row (wm)
  constexpr int LPT = (BM + BN) * (BK / 8) / 512;  // LDS-DMA instructions per thread per k-step
  constexpr int KK = BK / 32;
  constexpr int SMEM = S * STAGE > EPI_ROWS * LDT * 4 ? S * STAGE : EPI_ROWS * LDT * 4;
  static_assert(SMEM <= 160 * 1024, "LDS");
  static_assert(S >= 2 && S <= 4, "stages");
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  G256_STAMP(0);
  if (ep.drop_p > 0.f) ep.seed = eff_seed(ep.seed, seed_ctr);
  int bx, by;
  xcd_remap(bx, by);
  const int m0 = by * BM, n0 = bx * BN;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = w >> 2, wn = w & 3;
  const int rb = wm * 128, cb = wn * 64;
  const int fr = lane & 15, fq = lane >> 4;

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int kt0 = kslice ? blockIdx.z * (kslice / BK) : 0;
  const int nk = kslice ? min((K + BK - 1) / BK, kt0 + kslice / BK) : (K + BK - 1) / BK;
#pragma unroll
  for (int i = 0; i < S - 1; ++i) {
    if (kt0 + i < nk) {
      char* st = smem + i * STAGE;
      g8_issue<BM, BK, AK>(A, lda, m0, M, (kt0 + i) * BK, K, st, w, lane);
      g8_issue<BN, BK, BKM>(B, ldb, n0, N, (kt0 + i) * BK, K, st + TILE_A, w, lane);
    }
  }
  for (int kt = kt0; kt < nk; ++kt) {
    const int r = kt - kt0;
    char* cur = smem + (r % S) * STAGE;
    if (kt + S - 1 < nk) {
      char* nxt = smem + ((r + S - 1) % S) * STAGE;
      g8_issue<BM, BK, AK>(A, lda, m0, M, (kt + S - 1) * BK, K, nxt, w, lane);
      g8_issue<BN, BK, BKM>(B, ldb, n0, N, (kt + S - 1) * BK, K, nxt + TILE_A, w, lane);
    }
    const int newer = min(S - 1, nk - 1 - kt);  // k-steps issued after this one, still allowed out
    if (newer == 0) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if ((kt + 1) * BK > K) {
        g8_zero_tail<BM, BK, AK>(kt * BK, K, cur, w, lane);
        g8_zero_tail<BN, BK, BKM>(kt * BK, K, cur + TILE_A, w, lane);
      }
    } else if (newer == 1) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LPT) : "memory");
    } else if (newer == 2) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * LPT) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * LPT) : "memory");
    }
    __builtin_amdgcn_s_barrier();  // every wave's part of k-step kt is in LDS
    asm volatile("" ::: "memory");
    if (kt == kt0) G256_STAMP(1);
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      bf16x8 bfr[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = g8_frag<BN, BK, BKM>(cur + TILE_A, cb + j * 16, kk, lane);
#pragma unroll
      for (int ih = 0; ih < TM; ih += 4) {  // two halves of the wave's rows: 4 A fragments live at a time
        bf16x8 af[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) af[i] = g8_frag<BM, BK, AK>(cur, rb + (ih + i) * 16, kk, lane);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[ih + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[ih + i][j], 0, 0, 0);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // everyone is done reading `cur` before its refill
    asm volatile("" ::: "memory");
  }

  G256_STAMP(2);
  // two passes; pass p stages fragment rows i in [4p, 4p+4) of EVERY wave (staged row
  // wm*64 + ii*16 + .. -> tile row m0 + wm*128 + p*64 + ..), so each wave's accumulators of
  // pass 0 are dead before pass 1 (no spill while the epilogue runs)
  float* tile = (float*)smem;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    if (pass) __syncthreads();
#pragma unroll
    for (int ii = 0; ii < 4; ++ii)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          tile[(wm * 64 + ii * 16 + 4 * fq + q) * LDT + cb + j * 16 + fr] = acc[pass * 4 + ii][j][q];
    __syncthreads();
    if (kslice) {
#pragma unroll
      for (int h = 0; h < 2; ++h)
        partial_from_lds<BN>(tile + h * 64 * LDT, LDT, 64, m0 + h * 128 + pass * 64, n0, M, N,
                             (float*)C + (long)blockIdx.z * M * N);
    } else {
      epilogue_tile<BN, EPI_ROWS, 512, 2, 64>(ep, tile, LDT, m0 + pass * 64, n0, M, N, C, ldc, vec_ok != 0);
    }
    if (pass == 0) G256_STAMP(3);
  }
  G256_STAMP(4);
#ifdef IMGCAP_STAMPS
  if (threadIdx.x == 0 && g_dev_stamps) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    g_dev_stamps[(blockIdx.y * gridDim.x + blockIdx.x) * 8 + 5] = __builtin_amdgcn_s_memtime();
    g_dev_stamps[(blockIdx.y * gridDim.x + blockIdx.x) * 8 + 6] = __builtin_amdgcn_s_memrealtime();
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    g_dev_stamps[(blockIdx.y * gridDim.x + blockIdx.x) * 8 + 7] = xcc;
  }
#endif
}

// 128x128x128 block-scaled fp8 GEMM tile (MX-FP8) — included by gemm.hip.
//
// C = epilogue(A . B^T) with A [M][K], B [N][K] e4m3fn bytes and E8M0 scales per 32 k
// (As [M][K/32], Bs [N][K/32]): the frozen ConvNeXt Linears of config C5.  Same pipeline as
// gemm_glds_kernel (LDS-DMA staging, XOR-swizzled 16-byte slots, 2 stages, counted vmcnt +
// raw s_barrier), whose 64-deep bf16 k-tile is byte-for-byte a 128-deep fp8 k-tile (128 rows x
// 128 bytes), so the same issue code stages it; the k-tile's scales (4 bytes per row) ride
// along as one 4-byte LDS-DMA per thread.  One v_mfma_scale_f32_16x16x128_f8f6f4 per 16x16
// fragment per k-tile: twice the bf16 MFMA rate at half the operand bytes per flop.
//
// Operand lane map (tools/probe/mfma_mx.hip, exact-integer check): lane l = (r = l%16,
// g = l/16) holds row r's bytes k = 16g..16g+15 (VGPRs 0-3) and 64+16g..64+16g+15 (VGPRs
// 4-7) of the 128-deep step, and its scale operand is the scale of row r's k-block g
// (k = 32g..32g+31) -- blocks are dealt to lanes by index, not by the bytes a lane holds.
typedef int mx_v8i __attribute__((ext_vector_type(8)));

template <int ROWS>
DEV void mx_issue_scales(const uint8_t* __restrict__ S, long lds, int r0, int R, int kt, char* img, int lane) {
  // one 4-byte LDS-DMA per lane: rows r0 + 64*part + lane, k-blocks 4kt..4kt+3
  const int r = min(r0 + lane, R - 1);
  __builtin_amdgcn_global_load_lds((const void*)(S + (long)r * lds + 4 * kt),
                                   (__attribute__((address_space(3))) void*)img, 4, 0, 0);
}

DEV mx_v8i mx_frag(const char* img, int row, int g) {
  const int sw = row & 7;
  const uint4 lo = *(const uint4*)(img + ((row << 3) + (g ^ sw)) * 16);
  const uint4 hi = *(const uint4*)(img + ((row << 3) + ((4 + g) ^ sw)) * 16);
  return mx_v8i{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
}

template <int S>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void gemm_mx_kernel(
    const uint8_t* __restrict__ A, long lda, const uint8_t* __restrict__ As, const uint8_t* __restrict__ B, long ldb,
    const uint8_t* __restrict__ Bs, void* __restrict__ C, long ldc, int M, int N, int K, imgcap_epilogue ep,
    int vec_ok) {
  constexpr int BM = 128, BN = 128;
  constexpr int TILE = BM * 128, SC = BM * 4;         // data bytes / scale bytes per operand
  constexpr int STAGE = 2 * TILE + 2 * SC;
  constexpr int TM = BM / 32, TN = BN / 32;
  constexpr int LDT = BN + 4, EPI_ROWS = BM / 2;
  constexpr int LPT = 4 + 4 + 1;                       // LDS-DMA instructions per thread per k-tile
  static_assert(EPI_ROWS * LDT * 4 <= S * STAGE, "epilogue tile fits the stages");
  __shared__ __attribute__((aligned(16))) char smem[S * STAGE];
  int bx, by;
  xcd_remap(bx, by);
  const int m0 = by * BM, n0 = bx * BN;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int rb = wm * (BM / 2), cb = wn * (BN / 2);
  const int fr = lane & 15, fq = lane >> 4;
  const long kb = K / 32;  // scale row pitch

  // k-tile kt of both operands into stage `st`: bytes as bf16 pairs for the shared issue code
  auto issue = [&](int kt, char* st) {
    glds_issue_op<BM, true>((const bf16*)A, lda / 2, m0, M, kt * 64, K / 2, st, w, lane);
    glds_issue_op<BN, true>((const bf16*)B, ldb / 2, n0, N, kt * 64, K / 2, st + TILE, w, lane);
    if (w < 2) mx_issue_scales<BM>(As, kb, m0 + 64 * w, M, kt, st + 2 * TILE + 256 * w, lane);
    else mx_issue_scales<BN>(Bs, kb, n0 + 64 * (w - 2), N, kt, st + 2 * TILE + SC + 256 * (w - 2), lane);
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / 128;
#pragma unroll
  for (int i = 0; i < S - 1; ++i)
    if (i < nk) issue(i, smem + i * STAGE);
  for (int kt = 0; kt < nk; ++kt) {
    char* cur = smem + (kt % S) * STAGE;
    if (kt + S - 1 < nk) issue(kt + S - 1, smem + ((kt + S - 1) % S) * STAGE);
    const int newer = min(S - 1, nk - 1 - kt);
    if (newer == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (newer == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LPT) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * LPT) : "memory");
    __builtin_amdgcn_s_barrier();  // every wave's part of tile kt is in LDS
    asm volatile("" ::: "memory");
    const uint8_t* sa = (const uint8_t*)(cur + 2 * TILE);
    const uint8_t* sbp = sa + SC;
    mx_v8i af[TM], bfr[TN];
    int xa[TM], xb[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = rb + i * 16 + fr;
      af[i] = mx_frag(cur, row, fq);
      xa[i] = sa[row * 4 + fq];
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int row = cb + j * 16 + fr;
      bfr[j] = mx_frag(cur + TILE, row, fq);
      xb[j] = sbp[row * 4 + fq];
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[i], bfr[j], acc[i][j], 0, 0, 0, xa[i], 0,
                                                                     xb[j]);
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
    epilogue_tile<BN, EPI_ROWS, 256>(ep, tile, LDT, m0 + pass * EPI_ROWS, n0, M, N, C, ldc, vec_ok != 0);
    __syncthreads();
  }
}

// ---- rows -> MX-FP8 (optionally LayerNorm'd first): one wave per row, 8 columns per lane --
template <typename T>
__global__ __launch_bounds__(256) void mx_quant_rows_kernel(int R, int K, const T* __restrict__ x, long ldx,
                                                            const float* __restrict__ lnw,
                                                            const float* __restrict__ lnb, float eps,
                                                            uint8_t* __restrict__ q, uint8_t* __restrict__ s) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= R) return;  // whole waves: the 4-lane groups below stay together
  const T* xr = x + (long)row * ldx;
  float mean = 0.f, rstd = 1.f;
  if (lnw) {
    float sum = 0.f;
    for (int c = lane * 8; c < K; c += 512) {
      float v[8];
      ld_g<T, 8>(xr + c, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) sum += v[j];
    }
    mean = wave_sum(sum) / K;
    float sq = 0.f;
    for (int c = lane * 8; c < K; c += 512) {
      float v[8];
      ld_g<T, 8>(xr + c, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) { const float d = v[j] - mean; sq += d * d; }
    }
    rstd = rsqrtf(wave_sum(sq) / K + eps);
  }
  // every lane runs the same number of iterations (K % 32 == 0 keeps 4-lane groups whole)
  for (int c0 = 0; c0 < K; c0 += 512) {
    const int c = c0 + lane * 8;
    const bool on = c < K;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = 0.f;
    if (on) {
      ld_g<T, 8>(xr + c, v);
      if (lnw) {
        float g[8], b[8];
        ld_g<float, 8>(lnw + c, g);
        ld_g<float, 8>(lnb + c, b);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (v[j] - mean) * rstd * g[j] + b[j];
      }
    }
    mx_store8(v, q + (long)row * K + c, s + (long)row * (K / 32) + c / 32, (lane & 3) == 0, on);
  }
}

// The same with the row held in registers (K <= 512 * NVL): one read of the row instead of three
// (sum, squared deviations, quantise), same summation order -- bitwise the outputs of the loop
// above.  C5's frozen stages quantise 12544 x 768 rows per block: 13.4 us per call before.
template <typename T, int NVL>
__global__ __launch_bounds__(256) void mx_quant_rows_reg_kernel(int R, int K, const T* __restrict__ x, long ldx,
                                                                const float* __restrict__ lnw,
                                                                const float* __restrict__ lnb, float eps,
                                                                uint8_t* __restrict__ q, uint8_t* __restrict__ s) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= R) return;
  const T* xr = x + (long)row * ldx;
  float v[NVL][8];
#pragma unroll
  for (int i = 0; i < NVL; ++i) {
    const int c = i * 512 + lane * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[i][j] = 0.f;
    if (c < K) ld_g<T, 8>(xr + c, v[i]);
  }
  if (lnw) {
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < NVL; ++i)
      if (i * 512 + lane * 8 < K) {
#pragma unroll
        for (int j = 0; j < 8; ++j) sum += v[i][j];
      }
    const float mean = wave_sum(sum) / K;
    float sq = 0.f;
#pragma unroll
    for (int i = 0; i < NVL; ++i)
      if (i * 512 + lane * 8 < K) {
#pragma unroll
        for (int j = 0; j < 8; ++j) { const float d = v[i][j] - mean; sq += d * d; }
      }
    const float rstd = rsqrtf(wave_sum(sq) / K + eps);
#pragma unroll
    for (int i = 0; i < NVL; ++i) {
      const int c = i * 512 + lane * 8;
      if (c < K) {
        float g[8], b[8];
        ld_g<float, 8>(lnw + c, g);
        ld_g<float, 8>(lnb + c, b);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] = (v[i][j] - mean) * rstd * g[j] + b[j];
      }
    }
  }
#pragma unroll
  for (int i = 0; i < NVL; ++i) {
    if (i * 512 >= K) break;  // wave-uniform: the 4-lane groups of mx_store8 stay together
    const int c = i * 512 + lane * 8;
    mx_store8(v[i], q + (long)row * K + c, s + (long)row * (K / 32) + c / 32, (lane & 3) == 0, c < K);
  }
}


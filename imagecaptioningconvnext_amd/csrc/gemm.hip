// MFMA GEMM with fused epilogue for gfx950 (bf16 16x16x32, exact-f32 16x16x4).
//
// One template covers every contraction on the hot path (SURVEY.md §2.2 rows "pointwise
// MLP", "downsample", "projections", "vocab projection" and all their dgrad/wgrad forms):
//   * operand layouts: A k-major ([M][K]) or m-major ([K][M]); B k-major ([N][K], nn.Linear
//     weight) or n-major ([K][N]); m/n-major tiles are transposed while being written to LDS
//   * LDS images are [row][k] with a 16-byte pad, read as one 16-byte fragment per lane
//   * 256 threads = 4 wave64s laid out WM x WN x KS; KS>1 splits each LDS k-tile across wave
//     groups (intra-block split-K for skinny M, e.g. the LSTM recurrence at M = batch) and
//     reduces through LDS, which also makes the epilogue store coalesced
//   * register-staged double buffering: the next k-tile's global loads are in flight while
//     the current tile's MFMAs run
//   * f32 mode feeds the same [row][8 k] fragment to 8 chained 16x16x4 f32 MFMAs (the k
//     order inside a 32-slice is permuted identically for A and B, so the sum is unchanged)
#include "common.h"

namespace imgcap {

template <typename T> struct Frag;
template <> struct Frag<bf16> { bf16x8 v; };
template <> struct Frag<float> { f32x4 lo, hi; };

DEV void mma(f32x4& acc, const Frag<bf16>& a, const Frag<bf16>& b) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.v, b.v, acc, 0, 0, 0);
}
DEV void mma(f32x4& acc, const Frag<float>& a, const Frag<float>& b) {
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.lo[kk], b.lo[kk], acc, 0, 0, 0);
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.hi[kk], b.hi[kk], acc, 0, 0, 0);
}

template <typename T> DEV Frag<T> lds_frag(const T* p);
template <> DEV Frag<bf16> lds_frag<bf16>(const bf16* p) { Frag<bf16> f; f.v = *(const bf16x8*)p; return f; }
template <> DEV Frag<float> lds_frag<float>(const float* p) {
  Frag<float> f; f.lo = *(const f32x4*)p; f.hi = *(const f32x4*)(p + 4); return f;
}

DEV void epi_apply(const imgcap_epilogue& ep, void* C, long cidx, int m, int n, float v) {
  v *= ep.alpha;
  if (ep.bias) v += ep.bias[n];
  if (ep.act == IMGCAP_ACT_GELU) v = gelu_erf(v);
  else if (ep.act == IMGCAP_ACT_RELU) v = fmaxf(v, 0.f);
  if (ep.drop_p > 0.f) v *= dropout_scale(ep.seed, ep.drop_stream, (uint64_t)m * ep.drop_ld + n, ep.drop_p);
  if (ep.aux) v = load_as_f(ep.aux, (long)m * ep.ldaux + n, ep.c_dtype) > 0.f ? v * ep.aux_scale : 0.f;
  if (ep.colscale) v *= ep.colscale[n];
  if (ep.rowscale) v *= ep.rowscale[m / ep.rows_per_scale];
  if (ep.res) v += load_as_f(ep.res, (long)m * ep.ldr + n, ep.c_dtype);
  if (ep.beta != 0.f) v += ep.beta * load_as_f(C, cidx, ep.c_dtype);
  store_from_f(C, cidx, ep.c_dtype, v);
}

template <typename T, int BM, int BN, int WM, int WN, int KS, bool AK, bool BK_>
struct GemmCfg {
  static constexpr int VEC = 16 / sizeof(T);
  static constexpr int BK = 32 * KS;
  static constexpr int LDK = BK + VEC;  // +16 bytes per row
  static constexpr int TM = BM / WM / 16;
  static constexpr int TN = BN / WN / 16;
  static constexpr int A_VECS = BM * BK / VEC / 256;
  static constexpr int B_VECS = BN * BK / VEC / 256;
  static constexpr int STAGE_BYTES = (BM + BN) * LDK * (int)sizeof(T);
  static constexpr int RED_BYTES = KS > 1 ? KS * BM * BN * 4 : 0;
  static constexpr int SMEM = STAGE_BYTES > RED_BYTES ? STAGE_BYTES : RED_BYTES;
  static_assert(WM * WN * KS == 4, "4 waves");
  static_assert(A_VECS >= 1 && B_VECS >= 1, "tile too small for 256 threads");
  static_assert(BM * BK % (VEC * 256) == 0 && BN * BK % (VEC * 256) == 0, "tile/thread mismatch");
};

// Load one operand tile (ROWS x BK) into registers.  KMAJ: element (r,k) at P[r*ld + k].
template <typename T, int ROWS, int BK, int NV, bool KMAJ>
DEV void tile_load(uint4 (&reg)[NV], const T* __restrict__ P, long ld, int r0, int k0, int R, int K) {
  constexpr int VEC = 16 / sizeof(T);
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int v = tid + i * 256;
    int r, k;
    if (KMAJ) { r = v / (BK / VEC); k = (v % (BK / VEC)) * VEC; }
    else      { k = v / (ROWS / VEC); r = (v % (ROWS / VEC)) * VEC; }
    const int gr = r0 + r, gk = k0 + k;
    const bool full = KMAJ ? (gr < R && gk + VEC <= K) : (gk < K && gr + VEC <= R);
    if (full) {
      reg[i] = KMAJ ? *(const uint4*)(P + (long)gr * ld + gk) : *(const uint4*)(P + (long)gk * ld + gr);
    } else {
      T tmp[VEC];
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        const int rr = KMAJ ? gr : gr + j, kk = KMAJ ? gk + j : gk;
        tmp[j] = (rr < R && kk < K) ? (KMAJ ? P[(long)rr * ld + kk] : P[(long)kk * ld + rr]) : from_f<T>(0.f);
      }
      reg[i] = *(uint4*)tmp;
    }
  }
}

template <typename T, int ROWS, int BK, int LDK, int NV, bool KMAJ>
DEV void tile_store(T* S, const uint4 (&reg)[NV]) {
  constexpr int VEC = 16 / sizeof(T);
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int v = tid + i * 256;
    if (KMAJ) {
      const int r = v / (BK / VEC), k = (v % (BK / VEC)) * VEC;
      *(uint4*)(S + r * LDK + k) = reg[i];
    } else {
      const int k = v / (ROWS / VEC), r = (v % (ROWS / VEC)) * VEC;
      const T* t = (const T*)&reg[i];
#pragma unroll
      for (int j = 0; j < VEC; ++j) S[(r + j) * LDK + k] = t[j];
    }
  }
}

template <typename T, int BM, int BN, int WM, int WN, int KS, bool AK, bool BKM>
__global__ __launch_bounds__(256) void gemm_kernel(const T* __restrict__ A, long lda, long sA,
                                                   const T* __restrict__ B, long ldb, long sB,
                                                   void* __restrict__ C, long ldc, long sC,
                                                   int M, int N, int K, imgcap_epilogue ep) {
  using G = GemmCfg<T, BM, BN, WM, WN, KS, AK, BKM>;
  __shared__ __attribute__((aligned(16))) char smem[G::SMEM];
  T* As = (T*)smem;
  T* Bs = As + BM * G::LDK;

  const int bz = blockIdx.z;
  A += bz * sA;
  B += bz * sB;
  const long cbase = (long)bz * sC;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ks = wave / (WM * WN), wmn = wave % (WM * WN);
  const int rb = (wmn / WN) * (BM / WM), cb = (wmn % WN) * (BN / WN);

  f32x4 acc[G::TM][G::TN];
#pragma unroll
  for (int i = 0; i < G::TM; ++i)
#pragma unroll
    for (int j = 0; j < G::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  uint4 ra[G::A_VECS], rbv[G::B_VECS];
  tile_load<T, BM, G::BK, G::A_VECS, AK>(ra, A, lda, m0, 0, M, K);
  tile_load<T, BN, G::BK, G::B_VECS, BKM>(rbv, B, ldb, n0, 0, N, K);
  tile_store<T, BM, G::BK, G::LDK, G::A_VECS, AK>(As, ra);
  tile_store<T, BN, G::BK, G::LDK, G::B_VECS, BKM>(Bs, rbv);
  __syncthreads();

  const int fr = lane & 15, fk = ks * 32 + 8 * (lane >> 4);
  for (int k0 = 0; k0 < K; k0 += G::BK) {
    const bool more = k0 + G::BK < K;
    if (more) {
      tile_load<T, BM, G::BK, G::A_VECS, AK>(ra, A, lda, m0, k0 + G::BK, M, K);
      tile_load<T, BN, G::BK, G::B_VECS, BKM>(rbv, B, ldb, n0, k0 + G::BK, N, K);
    }
    Frag<T> af[G::TM], bfr[G::TN];
#pragma unroll
    for (int i = 0; i < G::TM; ++i) af[i] = lds_frag<T>(As + (rb + i * 16 + fr) * G::LDK + fk);
#pragma unroll
    for (int j = 0; j < G::TN; ++j) bfr[j] = lds_frag<T>(Bs + (cb + j * 16 + fr) * G::LDK + fk);
#pragma unroll
    for (int i = 0; i < G::TM; ++i)
#pragma unroll
      for (int j = 0; j < G::TN; ++j) mma(acc[i][j], af[i], bfr[j]);
    __syncthreads();
    if (more) {
      tile_store<T, BM, G::BK, G::LDK, G::A_VECS, AK>(As, ra);
      tile_store<T, BN, G::BK, G::LDK, G::B_VECS, BKM>(Bs, rbv);
      __syncthreads();
    }
  }

  if (KS == 1) {
#pragma unroll
    for (int i = 0; i < G::TM; ++i)
#pragma unroll
      for (int j = 0; j < G::TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + rb + i * 16 + 4 * (lane >> 4) + r;
          const int n = n0 + cb + j * 16 + fr;
          if (m < M && n < N) epi_apply(ep, C, cbase + (long)m * ldc + n, m, n, acc[i][j][r]);
        }
  } else {
    float* part = (float*)smem;  // [KS][BM][BN]
#pragma unroll
    for (int i = 0; i < G::TM; ++i)
#pragma unroll
      for (int j = 0; j < G::TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          part[(ks * BM + rb + i * 16 + 4 * (lane >> 4) + r) * BN + cb + j * 16 + fr] = acc[i][j][r];
    __syncthreads();
    for (int e = threadIdx.x; e < BM * BN; e += 256) {
      const int r = e / BN, c = e % BN;
      float v = 0.f;
#pragma unroll
      for (int s = 0; s < KS; ++s) v += part[s * BM * BN + e];
      const int m = m0 + r, n = n0 + c;
      if (m < M && n < N) epi_apply(ep, C, cbase + (long)m * ldc + n, m, n, v);
    }
  }
}

template <typename T, int BM, int BN, int WM, int WN, int KS>
static int launch_cfg(int ak, int bk, int M, int N, int K, const void* A, long lda, long sA, const void* B,
                      long ldb, long sB, void* C, long ldc, long sC, int batch, const imgcap_epilogue& ep,
                      hipStream_t st) {
  dim3 grid((N + BN - 1) / BN, (M + BM - 1) / BM, batch);
  const T* a = (const T*)A;
  const T* b = (const T*)B;
#define L_(AKV, BKV) \
  hipLaunchKernelGGL((gemm_kernel<T, BM, BN, WM, WN, KS, AKV, BKV>), grid, dim3(256), 0, st, a, lda, sA, b, ldb, sB, C, ldc, sC, M, N, K, ep)
  if (ak && bk) L_(true, true);
  else if (ak && !bk) L_(true, false);
  else if (!ak && bk) L_(false, true);
  else L_(false, false);
#undef L_
  IMGCAP_CHECK_LAUNCH("imgcap_gemm");
  return 0;
}

template <typename T>
static int gemm_dispatch(int ak, int bk, int M, int N, int K, const void* A, long lda, long sA, const void* B,
                         long ldb, long sB, void* C, long ldc, long sC, int batch, const imgcap_epilogue& ep,
                         hipStream_t st) {
  if (M <= 32)
    return launch_cfg<T, 32, 32, 1, 1, 4>(ak, bk, M, N, K, A, lda, sA, B, ldb, sB, C, ldc, sC, batch, ep, st);
  if (M <= 64)
    return launch_cfg<T, 64, 32, 1, 1, 4>(ak, bk, M, N, K, A, lda, sA, B, ldb, sB, C, ldc, sC, batch, ep, st);
  const long tiles128 = (long)((M + 127) / 128) * ((N + 127) / 128) * batch;
  if (tiles128 < 512)
    return launch_cfg<T, 64, 64, 2, 2, 1>(ak, bk, M, N, K, A, lda, sA, B, ldb, sB, C, ldc, sC, batch, ep, st);
  return launch_cfg<T, 128, 128, 2, 2, 1>(ak, bk, M, N, K, A, lda, sA, B, ldb, sB, C, ldc, sC, batch, ep, st);
}

// bias-gradient style column sums: out[c] = beta*out[c] + sum_r x[r, c]
template <typename T>
__global__ void colsum_kernel(int rows, int cols, const T* __restrict__ x, long ld, float* __restrict__ out,
                              float beta) {
  __shared__ float red[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int w = threadIdx.x >> 6;
  float s = 0.f;
  if (c < cols)
    for (int r = w; r < rows; r += 4) s += to_f(x[(long)r * ld + c]);
  red[w][threadIdx.x & 63] = s;
  __syncthreads();
  if (w == 0 && c < cols) {
    const float t = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    out[c] = (beta != 0.f ? beta * out[c] : 0.f) + t;
  }
}

}  // namespace imgcap

using namespace imgcap;

extern "C" int imgcap_gemm(int dtype, int a_kmajor, int b_kmajor, int M, int N, int K, const void* A, int64_t lda,
                           int64_t strideA, const void* B, int64_t ldb, int64_t strideB, void* C, int64_t ldc,
                           int64_t strideC, int batch, const imgcap_epilogue* epi, void* stream) {
  IMGCAP_REQUIRE(epi != nullptr, "imgcap_gemm: epilogue is NULL");
  IMGCAP_REQUIRE(M >= 0 && N >= 0 && K >= 0 && batch >= 1, "imgcap_gemm: bad sizes");
  if (M == 0 || N == 0) return 0;
  IMGCAP_REQUIRE(dtype == IMGCAP_F32 || dtype == IMGCAP_BF16, "imgcap_gemm: bad dtype");
  const int vec = dtype == IMGCAP_F32 ? 4 : 8;
  IMGCAP_REQUIRE(aligned16(A) && aligned16(B), "imgcap_gemm: A/B must be 16-byte aligned");
  IMGCAP_REQUIRE(lda % vec == 0 && ldb % vec == 0 && strideA % vec == 0 && strideB % vec == 0,
                 "imgcap_gemm: leading dims/strides must be multiples of 16 bytes");
  IMGCAP_REQUIRE(epi->rows_per_scale > 0 || epi->rowscale == nullptr, "imgcap_gemm: rows_per_scale");
  hipStream_t st = (hipStream_t)stream;
  if (K == 0) {  // pure epilogue on zero accumulator is not needed on the path
    return fail(IMGCAP_EINVAL, "imgcap_gemm: K == 0");
  }
  if (dtype == IMGCAP_BF16)
    return gemm_dispatch<bf16>(a_kmajor, b_kmajor, M, N, K, A, lda, strideA, B, ldb, strideB, C, ldc, strideC,
                               batch, *epi, st);
  return gemm_dispatch<float>(a_kmajor, b_kmajor, M, N, K, A, lda, strideA, B, ldb, strideB, C, ldc, strideC,
                              batch, *epi, st);
}

extern "C" int imgcap_colsum(int dtype, int rows, int cols, const void* x, int64_t ldx, float* out, float beta,
                             void* stream) {
  if (cols == 0) return 0;
  dim3 grid((cols + 63) / 64);
  if (dtype == IMGCAP_BF16)
    hipLaunchKernelGGL(colsum_kernel<bf16>, grid, dim3(256), 0, (hipStream_t)stream, rows, cols, (const bf16*)x, ldx,
                       out, beta);
  else
    hipLaunchKernelGGL(colsum_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream, rows, cols, (const float*)x,
                       ldx, out, beta);
  IMGCAP_CHECK_LAUNCH("imgcap_colsum");
  return 0;
}

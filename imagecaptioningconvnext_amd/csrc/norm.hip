// Row LayerNorm of a (dropout-)residual sum: the post-norm blocks of
// nn.TransformerDecoderLayer (transformerDecoder.py:82,104): x = LN(x + dropout(sublayer(x))).
// One wave per row (cols <= 64*16); the row stays in registers between the two variance
// passes, so HBM traffic is one read of each input and one write of s and y.
#include "common.h"

namespace imgcap {

constexpr int LN_MAXV = 16;  // values per lane -> cols <= 1024

template <typename T>
__global__ __launch_bounds__(256) void add_ln_fwd_kernel(int rows, int cols, const T* __restrict__ x,
                                                         const T* __restrict__ r, float p, uint64_t seed,
                                                         uint32_t stream_id, const float* __restrict__ g,
                                                         const float* __restrict__ b, float eps, T* __restrict__ s_out,
                                                         T* __restrict__ y, float* __restrict__ mean_o,
                                                         float* __restrict__ rstd_o) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  float v[LN_MAXV];
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = lane + 64 * i;
    v[i] = 0.f;
    if (c < cols) {
      const long idx = (long)row * cols + c;
      float t = to_f(x[idx]);
      if (r) t += to_f(r[idx]) * dropout_scale(seed, stream_id, idx, p);
      if (s_out) s_out[idx] = from_f<T>(t);
      t = to_f(from_f<T>(t));  // LN sees exactly the stored s (bwd recomputes from it)
      v[i] = t;
      sum += t;
    }
  }
  const float mean = wave_sum(sum) / cols;
  float sq = 0.f;
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = lane + 64 * i;
    if (c < cols) { const float d = v[i] - mean; sq += d * d; }
  }
  const float rstd = rsqrtf(wave_sum(sq) / cols + eps);
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = lane + 64 * i;
    if (c < cols) y[(long)row * cols + c] = from_f<T>((v[i] - mean) * rstd * g[c] + b[c]);
  }
  if (lane == 0) { mean_o[row] = mean; rstd_o[row] = rstd; }
}

template <typename T>
__global__ __launch_bounds__(256) void add_ln_bwd_kernel(int rows, int cols, const T* __restrict__ dy,
                                                         const T* __restrict__ s, const float* __restrict__ mean_i,
                                                         const float* __restrict__ rstd_i, const float* __restrict__ g,
                                                         float p, uint64_t seed, uint32_t stream_id, T* __restrict__ dx,
                                                         T* __restrict__ dr, float* __restrict__ dg,
                                                         float* __restrict__ db, int rows_per_block) {
  // each block: rows_per_block rows, 4 waves; dgamma/dbeta partials reduced in LDS then one
  // atomic per column per block
  __shared__ float pg[1024], pb[1024];
  for (int c = threadIdx.x; c < cols; c += 256) { pg[c] = 0.f; pb[c] = 0.f; }
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float lg[LN_MAXV], lb[LN_MAXV];
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) { lg[i] = 0.f; lb[i] = 0.f; }
  const int r_end = min(rows, (blockIdx.x + 1) * rows_per_block);
  for (int row = blockIdx.x * rows_per_block + w; row < r_end; row += 4) {
    const float mean = mean_i[row], rstd = rstd_i[row];
    float xh[LN_MAXV], gdy[LN_MAXV];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < LN_MAXV; ++i) {
      const int c = lane + 64 * i;
      xh[i] = 0.f; gdy[i] = 0.f;
      if (c < cols) {
        const long idx = (long)row * cols + c;
        const float d = to_f(dy[idx]);
        xh[i] = (to_f(s[idx]) - mean) * rstd;
        gdy[i] = d * g[c];
        lg[i] += d * xh[i];
        lb[i] += d;
        s1 += gdy[i];
        s2 += gdy[i] * xh[i];
      }
    }
    s1 = wave_sum(s1) / cols;
    s2 = wave_sum(s2) / cols;
#pragma unroll
    for (int i = 0; i < LN_MAXV; ++i) {
      const int c = lane + 64 * i;
      if (c < cols) {
        const long idx = (long)row * cols + c;
        const float d = rstd * (gdy[i] - s1 - xh[i] * s2);
        dx[idx] = from_f<T>(d);
        if (dr) dr[idx] = from_f<T>(d * dropout_scale(seed, stream_id, idx, p));
      }
    }
  }
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = lane + 64 * i;
    if (c < cols) { atomicAdd(&pg[c], lg[i]); atomicAdd(&pb[c], lb[i]); }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < cols; c += 256) {
    if (dg) atomicAdd(&dg[c], pg[c]);
    if (db) atomicAdd(&db[c], pb[c]);
  }
}

}  // namespace imgcap

using namespace imgcap;

extern "C" int imgcap_add_layernorm_fwd(int dtype, int rows, int cols, const void* x, const void* r, float drop_p,
                                        uint64_t seed, uint32_t drop_stream, const float* gamma, const float* beta,
                                        float eps, void* s_out, void* y, float* mean, float* rstd, void* stream) {
  IMGCAP_REQUIRE(cols > 0 && cols <= 64 * LN_MAXV, "imgcap_add_layernorm_fwd: cols must be in (0, 1024]");
  if (rows == 0) return 0;
  dim3 grid((rows + 3) / 4);
  if (dtype == IMGCAP_BF16)
    hipLaunchKernelGGL(add_ln_fwd_kernel<bf16>, grid, dim3(256), 0, (hipStream_t)stream, rows, cols, (const bf16*)x,
                       (const bf16*)r, drop_p, seed, drop_stream, gamma, beta, eps, (bf16*)s_out, (bf16*)y, mean, rstd);
  else
    hipLaunchKernelGGL(add_ln_fwd_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream, rows, cols, (const float*)x,
                       (const float*)r, drop_p, seed, drop_stream, gamma, beta, eps, (float*)s_out, (float*)y, mean,
                       rstd);
  IMGCAP_CHECK_LAUNCH("imgcap_add_layernorm_fwd");
  return 0;
}

extern "C" int imgcap_add_layernorm_bwd(int dtype, int rows, int cols, const void* dy, const void* s,
                                        const float* mean, const float* rstd, const float* gamma, float drop_p,
                                        uint64_t seed, uint32_t drop_stream, void* dx, void* dr, float* dgamma,
                                        float* dbeta, void* stream) {
  IMGCAP_REQUIRE(cols > 0 && cols <= 64 * LN_MAXV, "imgcap_add_layernorm_bwd: cols must be in (0, 1024]");
  if (rows == 0) return 0;
  const int rpb = 64;
  dim3 grid((rows + rpb - 1) / rpb);
  if (dtype == IMGCAP_BF16)
    hipLaunchKernelGGL(add_ln_bwd_kernel<bf16>, grid, dim3(256), 0, (hipStream_t)stream, rows, cols, (const bf16*)dy,
                       (const bf16*)s, mean, rstd, gamma, drop_p, seed, drop_stream, (bf16*)dx, (bf16*)dr, dgamma,
                       dbeta, rpb);
  else
    hipLaunchKernelGGL(add_ln_bwd_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream, rows, cols,
                       (const float*)dy, (const float*)s, mean, rstd, gamma, drop_p, seed, drop_stream, (float*)dx,
                       (float*)dr, dgamma, dbeta, rpb);
  IMGCAP_CHECK_LAUNCH("imgcap_add_layernorm_bwd");
  return 0;
}

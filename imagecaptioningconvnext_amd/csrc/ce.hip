// Cross-entropy over vocab rows with fused top-5 hit test.
//   fwd  (train.py:268 / :276 CrossEntropyLoss on packed scores; utils.py:248-250 topk(5)):
//        one pass over the row: online max / sum-exp, plus the count of logits strictly
//        greater than the target's (hit5 = count < 5).
//   bwd: dlogits = (exp(logit - lse) - onehot) * scale, scale read from device memory so the
//        token count never needs a host sync.
#include "common.h"

namespace imgcap {

template <typename T>
__global__ __launch_bounds__(256) void ce_fwd_kernel(int V, const T* __restrict__ logits, long ld,
                                                     const int64_t* __restrict__ tgt, float* __restrict__ lse_o,
                                                     float* __restrict__ loss_o, float* __restrict__ hit_o) {
  __shared__ float red[3][4];
  const int row = blockIdx.x;
  const T* x = logits + (long)row * ld;
  const long t = tgt[row];
  const float xt = (t >= 0 && t < V) ? to_f(x[t]) : 0.f;
  float m = -INFINITY, s = 0.f, cnt = 0.f;
  for (int c = threadIdx.x; c < V; c += 256) {
    const float v = to_f(x[c]);
    if (v > m) { s = s * __expf(m - v) + 1.f; m = v; }
    else s += __expf(v - m);
    cnt += (v > xt) ? 1.f : 0.f;
  }
  // combine (m, s) pairs across the wave then the block
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    const float mn = fmaxf(m, m2);
    s = (m == -INFINITY ? 0.f : s * __expf(m - mn)) + (m2 == -INFINITY ? 0.f : s2 * __expf(m2 - mn));
    m = mn;
  }
  cnt = wave_sum(cnt);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { red[0][w] = m; red[1][w] = s; red[2][w] = cnt; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = red[0][0];
    for (int i = 1; i < 4; ++i) M = fmaxf(M, red[0][i]);
    float S = 0.f, C = 0.f;
    for (int i = 0; i < 4; ++i) { S += red[1][i] * __expf(red[0][i] - M); C += red[2][i]; }
    const float lse = M + logf(S);
    lse_o[row] = lse;
    const bool valid = t >= 0 && t < V;
    if (loss_o) loss_o[row] = valid ? lse - xt : 0.f;
    if (hit_o) hit_o[row] = (valid && C < 5.f) ? 1.f : 0.f;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void ce_bwd_kernel(int V, const T* __restrict__ logits, long ld,
                                                     const int64_t* __restrict__ tgt, const float* __restrict__ lse_i,
                                                     const float* __restrict__ scale_p, T* __restrict__ d, long ldd) {
  const int row = blockIdx.x;
  const long t = tgt[row];
  const T* x = logits + (long)row * ld;
  T* o = d + (long)row * ldd;
  const bool valid = t >= 0 && t < V;
  const float lse = lse_i[row], sc = valid ? *scale_p : 0.f;
  for (int c = threadIdx.x; c < V; c += 256) {
    const float p = __expf(to_f(x[c]) - lse);
    o[c] = from_f<T>(sc * (p - (c == t ? 1.f : 0.f)));
  }
}

// ---- fused forward + backward (the training step: loss, top-5 and dlogits in one pass) ----
// The row is read ONCE into registers (16-byte vectors, NV per thread), reduced (max, then
// sum-exp and the count of logits above the target's), and dlogits = (softmax - onehot) *
// scale written from the same registers: one read and one write of [n, V] instead of the
// fwd + bwd kernels' two reads and one write (element-wise 2-byte loads there).  Padding
// columns [V, ceil(V / VEC) * VEC) of dlogits are written as 0.
template <typename T, int NV>
__global__ __launch_bounds__(256) void ce_fused_kernel(int V, const T* __restrict__ logits, long ld,
                                                       const int64_t* __restrict__ tgt,
                                                       const float* __restrict__ scale_p, float* __restrict__ lse_o,
                                                       float* __restrict__ loss_o, float* __restrict__ hit_o,
                                                       T* __restrict__ d, long ldd) {
  constexpr int VEC = 16 / sizeof(T);
  __shared__ float red[2][4];
  const int row = blockIdx.x, tid = threadIdx.x, w = tid >> 6;
  const T* x = logits + (long)row * ld;
  const long t = tgt[row];
  const bool valid = t >= 0 && t < V;
  const int nvec = (V + VEC - 1) / VEC;
  float v[NV][VEC];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int q = j * 256 + tid;
    if (q < nvec) {
      ld_g<T, VEC>(x + (long)q * VEC, v[j]);
#pragma unroll
      for (int e = 0; e < VEC; ++e)
        if (q * VEC + e >= V) v[j][e] = -INFINITY;
    } else {
#pragma unroll
      for (int e = 0; e < VEC; ++e) v[j][e] = -INFINITY;
    }
  }
  const float xt = valid ? to_f(x[t]) : 0.f;
  float m = -INFINITY;
#pragma unroll
  for (int j = 0; j < NV; ++j)
#pragma unroll
    for (int e = 0; e < VEC; ++e) m = fmaxf(m, v[j][e]);
  m = wave_max(m);
  if ((tid & 63) == 0) red[0][w] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0][0], red[0][1]), fmaxf(red[0][2], red[0][3]));
  float s = 0.f, cnt = 0.f;
#pragma unroll
  for (int j = 0; j < NV; ++j)
#pragma unroll
    for (int e = 0; e < VEC; ++e) {
      s += __expf(v[j][e] - m);  // exp(-inf) = 0 for masked slots
      cnt += (v[j][e] > xt) ? 1.f : 0.f;
    }
  s = wave_sum(s);
  cnt = wave_sum(cnt);
  __syncthreads();  // red[0] read by every thread above
  if ((tid & 63) == 0) { red[0][w] = s; red[1][w] = cnt; }
  __syncthreads();
  const float S = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
  const float C = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
  const float lse = m + logf(S);
  if (tid == 0) {
    lse_o[row] = lse;
    if (loss_o) loss_o[row] = valid ? lse - xt : 0.f;
    if (hit_o) hit_o[row] = (valid && C < 5.f) ? 1.f : 0.f;
  }
  const float sc = valid ? *scale_p : 0.f;
  T* o = d + (long)row * ldd;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int q = j * 256 + tid;
    if (q < nvec) {
      float g[VEC];
#pragma unroll
      for (int e = 0; e < VEC; ++e) {
        const int c = q * VEC + e;
        g[e] = c < V ? sc * (__expf(v[j][e] - lse) - (c == t ? 1.f : 0.f)) : 0.f;
      }
      st_g<T, VEC>(o + (long)q * VEC, g);
    }
  }
}

// 1 / (number of rows with a target): the scale of the fused kernel's dlogits (the same value
// loss_finalize_kernel writes to its out[3] afterwards)
__global__ __launch_bounds__(1024) void ce_scale_kernel(int n, const int64_t* __restrict__ tgt, float* __restrict__ out) {
  __shared__ float red[16];
  float c = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) c += tgt[i] >= 0 ? 1.f : 0.f;
  c = block_sum(c, red);
  if (threadIdx.x == 0) *out = 1.f / (c > 0.f ? c : 1.f);
}

}  // namespace imgcap

namespace imgcap {
// ---- greedy decoding step (decoder.py:150-161, transformerDecoder.py:137-155) -------------
// one block per row; finished rows return at once (their outputs stay as the zeroed buffers)
template <typename T>
__global__ __launch_bounds__(256) void greedy_select_kernel(int V, const T* __restrict__ logits, long ldl, int t,
                                                            int maxlen, int64_t end_id, uint8_t* __restrict__ finished,
                                                            int64_t* __restrict__ next_ids, int64_t* __restrict__ seq,
                                                            float* __restrict__ preds, const float* __restrict__ alpha,
                                                            float* __restrict__ alphas, int P) {
  __shared__ float bv_s[256];
  __shared__ int bi_s[256];
  const int b = blockIdx.x;
  if (finished[b]) return;
  const T* row = logits + (long)b * ldl;
  float* pr = preds + ((long)b * maxlen + t) * V;
  float bv = -INFINITY;
  int bi = 0x7fffffff;
  for (int v = threadIdx.x; v < V; v += 256) {
    const float x = to_f(row[v]);
    pr[v] = x;
    if (x > bv) { bv = x; bi = v; }  // ascending v: the first maximum of this thread's slice
  }
  bv_s[threadIdx.x] = bv;
  bi_s[threadIdx.x] = bi;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      const float ov = bv_s[threadIdx.x + o];
      const int oi = bi_s[threadIdx.x + o];
      if (ov > bv_s[threadIdx.x] || (ov == bv_s[threadIdx.x] && oi < bi_s[threadIdx.x])) {
        bv_s[threadIdx.x] = ov;
        bi_s[threadIdx.x] = oi;
      }
    }
    __syncthreads();
  }
  if (alpha)
    for (int p = threadIdx.x; p < P; p += 256) alphas[((long)b * maxlen + t) * P + p] = alpha[(long)b * P + p];
  if (threadIdx.x == 0) {
    const int id = bi_s[0];
    seq[(long)b * maxlen + t] = id;
    next_ids[b] = id;
    finished[b] = id == end_id ? 1 : 0;
  }
}

}  // namespace imgcap

using namespace imgcap;

extern "C" int imgcap_greedy_select(int dtype, int B, int V, const void* logits, int64_t ldl, int t, int maxlen,
                                    int64_t end_id, uint8_t* finished, int64_t* next_ids, int64_t* sequences,
                                    float* predictions, const float* alpha, float* alphas, int P, void* stream) {
  IMGCAP_REQUIRE(V > 0 && ldl >= V && t >= 0 && t < maxlen, "imgcap_greedy_select: bad V / ldl / t");
  IMGCAP_REQUIRE(!alpha || (alphas && P > 0), "imgcap_greedy_select: alphas");
  if (B == 0) return 0;
  if (dtype == IMGCAP_BF16)
    hipLaunchKernelGGL(greedy_select_kernel<bf16>, dim3(B), dim3(256), 0, (hipStream_t)stream, V, (const bf16*)logits,
                       (long)ldl, t, maxlen, end_id, finished, next_ids, sequences, predictions, alpha, alphas, P);
  else
    hipLaunchKernelGGL(greedy_select_kernel<float>, dim3(B), dim3(256), 0, (hipStream_t)stream, V,
                       (const float*)logits, (long)ldl, t, maxlen, end_id, finished, next_ids, sequences, predictions,
                       alpha, alphas, P);
  IMGCAP_CHECK_LAUNCH("imgcap_greedy_select");
  return 0;
}

extern "C" int imgcap_ce_fwd(int dtype, int n, int V, const void* logits, int64_t ld, const int64_t* targets,
                             float* lse, float* loss, float* hit5, void* stream) {
  if (n == 0) return 0;
  IMGCAP_REQUIRE(V > 0 && ld >= V, "imgcap_ce_fwd: bad V/ld");
  if (dtype == IMGCAP_BF16)
    hipLaunchKernelGGL(ce_fwd_kernel<bf16>, dim3(n), dim3(256), 0, (hipStream_t)stream, V, (const bf16*)logits, ld,
                       targets, lse, loss, hit5);
  else
    hipLaunchKernelGGL(ce_fwd_kernel<float>, dim3(n), dim3(256), 0, (hipStream_t)stream, V, (const float*)logits, ld,
                       targets, lse, loss, hit5);
  IMGCAP_CHECK_LAUNCH("imgcap_ce_fwd");
  return 0;
}

extern "C" int imgcap_ce_bwd(int dtype, int n, int V, const void* logits, int64_t ld, const int64_t* targets,
                             const float* lse, const float* scale, void* dlogits, int64_t ldd, void* stream) {
  if (n == 0) return 0;
  IMGCAP_REQUIRE(V > 0 && ld >= V && ldd >= V, "imgcap_ce_bwd: bad V/ld");
  if (dtype == IMGCAP_BF16)
    hipLaunchKernelGGL(ce_bwd_kernel<bf16>, dim3(n), dim3(256), 0, (hipStream_t)stream, V, (const bf16*)logits, ld,
                       targets, lse, scale, (bf16*)dlogits, ldd);
  else
    hipLaunchKernelGGL(ce_bwd_kernel<float>, dim3(n), dim3(256), 0, (hipStream_t)stream, V, (const float*)logits, ld,
                       targets, lse, scale, (float*)dlogits, ldd);
  IMGCAP_CHECK_LAUNCH("imgcap_ce_bwd");
  return 0;
}

extern "C" int imgcap_ce_fused(int dtype, int n, int V, const void* logits, int64_t ld, const int64_t* targets,
                               float* scale, float* lse, float* loss, float* hit5, void* dlogits, int64_t ldd,
                               void* stream) {
  if (n == 0) return 0;
  IMGCAP_REQUIRE(V > 0 && ld >= V && ldd >= V, "imgcap_ce_fused: bad V / ld / ldd");
  IMGCAP_REQUIRE(scale && lse && dlogits, "imgcap_ce_fused: scale, lse and dlogits required");
  const int vec = dtype == IMGCAP_BF16 ? 8 : 4;
  const int nvec = (V + vec - 1) / vec;
  IMGCAP_REQUIRE(ld % vec == 0 && ldd % vec == 0 && ldd >= (int64_t)nvec * vec && aligned16(logits) &&
                     aligned16(dlogits),
                 "imgcap_ce_fused: 16-byte aligned rows whose pitch covers ceil(V / vec) * vec elements");
  const int per = (nvec + 255) / 256;
  IMGCAP_REQUIRE(per <= 12, "imgcap_ce_fused: V <= 24576 (bf16) / 12288 (fp32)");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(ce_scale_kernel, dim3(1), dim3(1024), 0, st, n, targets, scale);
#define CEF_(T, NV)                                                                                       \
  hipLaunchKernelGGL((ce_fused_kernel<T, NV>), dim3(n), dim3(256), 0, st, V, (const T*)logits, (long)ld, targets, \
                     scale, lse, loss, hit5, (T*)dlogits, (long)ldd)
#define CEF_T(T)                               \
  do {                                         \
    if (per <= 2) CEF_(T, 2);                  \
    else if (per <= 4) CEF_(T, 4);             \
    else if (per <= 6) CEF_(T, 6);             \
    else if (per <= 8) CEF_(T, 8);             \
    else CEF_(T, 12);                          \
  } while (0)
  if (dtype == IMGCAP_BF16) CEF_T(bf16);
  else CEF_T(float);
#undef CEF_T
#undef CEF_
  IMGCAP_CHECK_LAUNCH("imgcap_ce_fused");
  return 0;
}

// Teacher-forced "Show, Attend and Tell" LSTM decoder recurrence (models/decoder.py:104-148)
// and its backward-through-time, driven natively: one C-ABI call enqueues all T steps.
//
// Exact algebraic restructuring of the reference loop (results identical up to fp
// reassociation):
//   * att1 = enc W_ea^T + b_ea (decoder.py:61) is computed ONCE outside the loop (the
//     reference recomputes it every step)
//   * the three GEMMs that read h_{t-1} (decoder_att, f_beta, LSTMCell weight_hh) are one
//     GEMM against W_hcat = [W_da; W_fb; W_hh]
//   * the embedding half of weight_ih (and both LSTM biases) is precomputed for all t (xe);
//     only the attention half (z_t W_ih[:,M:]^T) stays in the loop
//   * fc(dropout(h)) (decoder.py:144) runs once after the loop over all [B*T] rows
//   * rows are never shrunk: rows with t >= decode_length[b] are computed and masked out
//     (alphas = 0 there; the loss never reads their logits; their gradients are zero)
// Per step (forward): GEMM(h->g1) -> attn_fwd (score, softmax_49, context, sigmoid gate) ->
// GEMM(z->g2) -> cell_fwd.  Backward: cell_bwd -> GEMM(dgates->dz) -> attn_bwd ->
// GEMM(dcat->dh).  Weight gradients are batched GEMMs over all B*T rows afterwards (host).
#include "common.h"

namespace imgcap {

constexpr int ATT_THREADS = 256;
constexpr int MAXP = 64;

// ---- forward attention step ------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(ATT_THREADS) void attn_fwd_kernel(imgcap_lstm_desc d, int t) {
  const int b = blockIdx.x;
  const int P = d.P, E = d.E, A = d.A, Tn = d.T;
  const int W3 = A + E + 4 * d.D;
  const bool active = t < d.dl[b];
  const float* g1 = d.g1 + ((long)b * Tn + t) * W3;  // [att2 | gate_pre | hh]
  const T* att1 = (const T*)d.att1 + (long)b * P * A;
  const T* enc = (const T*)d.enc + (long)b * P * E;
  __shared__ float e_s[MAXP];
  __shared__ float red[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // scores e_p = w_f . relu(att1_p + att2)   (full_att bias cancels in the softmax)
  for (int p = w; p < P; p += 4) {
    float s = 0.f;
    for (int a = lane; a < A; a += 64) s += d.w_f[a] * fmaxf(to_f(att1[(long)p * A + a]) + g1[a], 0.f);
    s = wave_sum(s);
    if (lane == 0) e_s[p] = s;
  }
  __syncthreads();
  if (w == 0) {
    const float v = lane < P ? e_s[lane] : -INFINITY;
    const float m = wave_max(v);
    const float ex = lane < P ? __expf(v - m) : 0.f;
    const float sum = wave_sum(ex);
    const float al = ex / sum;
    if (lane < P) {
      e_s[lane] = al;
      d.alphas[((long)b * Tn + t) * P + lane] = active ? al : 0.f;
    }
  }
  __syncthreads();
  T* zs = (T*)d.zs + ((long)b * Tn + t) * E;
  float* awe = d.awe + ((long)b * Tn + t) * E;
  for (int e = threadIdx.x; e < E; e += ATT_THREADS) {
    float s = 0.f;
    for (int p = 0; p < P; ++p) s += e_s[p] * to_f(enc[(long)p * E + e]);
    const float gate = sigmoidf_(g1[A + e]);
    awe[e] = s;
    zs[e] = from_f<T>(gate * s);
  }
}

// ---- forward LSTMCell pointwise (torch gate order i, f, g, o) --------------------------
template <typename T>
__global__ __launch_bounds__(256) void cell_fwd_kernel(imgcap_lstm_desc d, int t) {
  const int D = d.D, Tn = d.T;
  const int W3 = d.A + d.E + 4 * D;
  const long n = (long)d.B * D;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < n; e += (long)gridDim.x * 256) {
    const int b = (int)(e / D), j = (int)(e % D);
    const long bt = (long)b * Tn + t;
    const float* xe = d.xe + bt * 4 * D;
    const float* hh = d.g1 + bt * W3 + d.A + d.E;
    const float* g2 = d.g2 + (long)b * 4 * D;
    const float gi = sigmoidf_(xe[j] + hh[j] + g2[j]);
    const float gf = sigmoidf_(xe[D + j] + hh[D + j] + g2[D + j]);
    const float gg = tanhf(xe[2 * D + j] + hh[2 * D + j] + g2[2 * D + j]);
    const float go = sigmoidf_(xe[3 * D + j] + hh[3 * D + j] + g2[3 * D + j]);
    const float cp = t == 0 ? d.c0[(long)b * D + j] : d.cs[(bt - 1) * D + j];
    const float c = gf * cp + gi * gg;
    const float h = go * tanhf(c);
    float* ga = d.gates + bt * 4 * D;
    ga[j] = gi; ga[D + j] = gf; ga[2 * D + j] = gg; ga[3 * D + j] = go;
    d.cs[bt * D + j] = c;
    ((T*)d.hs)[bt * D + j] = from_f<T>(h);
    if (t + 1 < Tn) ((T*)d.hprev)[(bt + 1) * D + j] = from_f<T>(h);
  }
}

// ---- backward LSTMCell pointwise -----------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void cell_bwd_kernel(imgcap_lstm_desc d, int t) {
  const int D = d.D, Tn = d.T;
  const int W3 = d.A + d.E + 4 * D;
  const long n = (long)d.B * D;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < n; e += (long)gridDim.x * 256) {
    const int b = (int)(e / D), j = (int)(e % D);
    const long bt = (long)b * Tn + t;
    T* dg = (T*)d.dcat + bt * W3 + d.A + d.E;
    if (t >= d.dl[b]) {
      dg[j] = dg[D + j] = dg[2 * D + j] = dg[3 * D + j] = from_f<T>(0.f);
      d.dc[e] = 0.f;
      continue;
    }
    const float dh = to_f(((const T*)d.dhs)[bt * D + j]) + d.dh[e];
    const float* ga = d.gates + bt * 4 * D;
    const float gi = ga[j], gf = ga[D + j], gg = ga[2 * D + j], go = ga[3 * D + j];
    const float c = d.cs[bt * D + j];
    const float cp = t == 0 ? d.c0[e] : d.cs[(bt - 1) * D + j];
    const float tc = tanhf(c);
    const float dct = d.dc[e] + dh * go * (1.f - tc * tc);
    dg[j] = from_f<T>(dct * gg * gi * (1.f - gi));
    dg[D + j] = from_f<T>(dct * cp * gf * (1.f - gf));
    dg[2 * D + j] = from_f<T>(dct * gi * (1.f - gg * gg));
    dg[3 * D + j] = from_f<T>(dh * tc * go * (1.f - go));
    d.dc[e] = dct * gf;
  }
}

// ---- backward attention step -----------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(ATT_THREADS) void attn_bwd_kernel(imgcap_lstm_desc d, int t) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int b = blockIdx.x;
  const int P = d.P, E = d.E, A = d.A, Tn = d.T;
  const int W3 = A + E + 4 * d.D;
  const long bt = (long)b * Tn + t;
  T* dcat = (T*)d.dcat + bt * W3;
  if (t >= d.dl[b]) {
    for (int i = threadIdx.x; i < A + E; i += ATT_THREADS) dcat[i] = from_f<T>(0.f);
    return;
  }
  float* dawe = sm;            // [E]
  float* al = sm + E;          // [MAXP]
  float* dal = al + MAXP;      // [MAXP]
  const float* g1 = d.g1 + bt * W3;
  const float* dz = d.dz + (long)b * E;
  const float* awe = d.awe + bt * E;
  for (int e = threadIdx.x; e < E; e += ATT_THREADS) {
    const float s = sigmoidf_(g1[A + e]);
    dawe[e] = dz[e] * s;
    dcat[A + e] = from_f<T>(dz[e] * awe[e] * s * (1.f - s));
  }
  for (int p = threadIdx.x; p < P; p += ATT_THREADS) al[p] = d.alphas[bt * P + p];
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const T* enc = (const T*)d.enc + (long)b * P * E;
  for (int p = w; p < P; p += 4) {
    float s = 0.f;
    for (int e = lane; e < E; e += 64) s += to_f(enc[(long)p * E + e]) * dawe[e];
    s = wave_sum(s);
    if (lane == 0) dal[p] = s + d.dreg[(long)b * P + p];
  }
  __syncthreads();
  if (w == 0) {
    const float a = lane < P ? al[lane] : 0.f, da = lane < P ? dal[lane] : 0.f;
    const float dot = wave_sum(a * da);
    if (lane < P) dal[lane] = a * (da - dot);  // d score
  }
  __syncthreads();
  const T* att1 = (const T*)d.att1 + (long)b * P * A;
  float* datt1 = d.datt1 + (long)b * P * A;
  float* dwf = d.dwf + (long)b * A;
  for (int a = threadIdx.x; a < A; a += ATT_THREADS) {
    const float wf = d.w_f[a], a2 = g1[a];
    float s_att2 = 0.f, s_wf = 0.f;
    for (int p = 0; p < P; ++p) {
      const float u = to_f(att1[(long)p * A + a]) + a2;
      const float de = dal[p];
      if (u > 0.f) {
        const float du = de * wf;
        s_att2 += du;
        datt1[(long)p * A + a] += du;
        s_wf += de * u;
      }
    }
    dcat[a] = from_f<T>(s_att2);
    dwf[a] += s_wf;
  }
}

// ---- doubly stochastic attention regularisation (train.py:269) --------------------------
//   reg = alphaC * mean_{b,p} (1 - sum_t alpha[b,t,p])^2 ; dreg[b,p] = d reg / d alpha[b,t,p]
__global__ void attn_reg_kernel(int B, int Tn, int P, const float* __restrict__ alphas, float alphaC,
                                float* __restrict__ dreg, float* __restrict__ reg_out) {
  __shared__ float red[16];
  float acc = 0.f;
  for (int e = threadIdx.x; e < B * P; e += blockDim.x) {
    const int b = e / P, p = e % P;
    float s = 0.f;
    for (int t = 0; t < Tn; ++t) s += alphas[((long)b * Tn + t) * P + p];
    acc += (1.f - s) * (1.f - s);
    dreg[e] = alphaC * 2.f * (s - 1.f) / (float)(B * P);
  }
  const float tot = block_sum(acc, red);
  if (threadIdx.x == 0) *reg_out = alphaC * tot / (float)(B * P);
}

static dim3 pw_grid(long n) {
  long b = (n + 255) / 256;
  return dim3((unsigned)(b > 2048 ? 2048 : (b < 1 ? 1 : b)));
}

template <typename T>
static int lstm_fwd_impl(const imgcap_lstm_desc& d, hipStream_t st) {
  const int W3 = d.A + d.E + 4 * d.D;
  const int ct = d.dtype;
  imgcap_epilogue ep{};
  ep.alpha = 1.f;
  ep.c_dtype = IMGCAP_F32;
  ep.rows_per_scale = 1;
  for (int t = 0; t < d.T; ++t) {
    imgcap_epilogue e1 = ep;
    e1.bias = d.b_hcat;
    int rc = imgcap_gemm(ct, 1, 1, d.B, W3, d.D, (const T*)d.hprev + (long)t * d.D, (long)d.T * d.D, 0, d.w_hcat,
                         d.D, 0, d.g1 + (long)t * W3, (long)d.T * W3, 0, 1, &e1, st);
    if (rc) return rc;
    hipLaunchKernelGGL(attn_fwd_kernel<T>, dim3(d.B), dim3(ATT_THREADS), 0, st, d, t);
    IMGCAP_CHECK_LAUNCH("lstm attn_fwd");
    rc = imgcap_gemm(ct, 1, 1, d.B, 4 * d.D, d.E, (const T*)d.zs + (long)t * d.E, (long)d.T * d.E, 0,
                     (const T*)d.w_ih + d.M, d.M + d.E, 0, d.g2, 4 * d.D, 0, 1, &ep, st);
    if (rc) return rc;
    hipLaunchKernelGGL(cell_fwd_kernel<T>, pw_grid((long)d.B * d.D), dim3(256), 0, st, d, t);
    IMGCAP_CHECK_LAUNCH("lstm cell_fwd");
  }
  return 0;
}

template <typename T>
static int lstm_bwd_impl(const imgcap_lstm_desc& d, hipStream_t st) {
  const int W3 = d.A + d.E + 4 * d.D;
  const int ct = d.dtype;
  if (hipMemsetAsync(d.dh, 0, sizeof(float) * d.B * d.D, st) != hipSuccess ||
      hipMemsetAsync(d.dc, 0, sizeof(float) * d.B * d.D, st) != hipSuccess ||
      hipMemsetAsync(d.datt1, 0, sizeof(float) * (size_t)d.B * d.P * d.A, st) != hipSuccess ||
      hipMemsetAsync(d.dwf, 0, sizeof(float) * (size_t)d.B * d.A, st) != hipSuccess)
    return fail(IMGCAP_EINVAL, "lstm bwd: hipMemsetAsync failed");
  imgcap_epilogue ep{};
  ep.alpha = 1.f;
  ep.c_dtype = IMGCAP_F32;
  ep.rows_per_scale = 1;
  const size_t shm = (d.E + 2 * MAXP) * sizeof(float);
  for (int t = d.T - 1; t >= 0; --t) {
    hipLaunchKernelGGL(cell_bwd_kernel<T>, pw_grid((long)d.B * d.D), dim3(256), 0, st, d, t);
    IMGCAP_CHECK_LAUNCH("lstm cell_bwd");
    // dz = dgates_t . W_ih[:, M:]      (W_ih [4D][M+E] read as [K=4D][N=E])
    int rc = imgcap_gemm(ct, 1, 0, d.B, d.E, 4 * d.D, (const T*)d.dcat + (long)t * W3 + d.A + d.E, (long)d.T * W3, 0,
                         (const T*)d.w_ih + d.M, d.M + d.E, 0, d.dz, d.E, 0, 1, &ep, st);
    if (rc) return rc;
    hipLaunchKernelGGL(attn_bwd_kernel<T>, dim3(d.B), dim3(ATT_THREADS), shm, st, d, t);
    IMGCAP_CHECK_LAUNCH("lstm attn_bwd");
    // dh_{t-1} = [d_att2 | d_gate_pre | dgates] . W_hcat   (W_hcat [W3][D] read as [K=W3][N=D])
    rc = imgcap_gemm(ct, 1, 0, d.B, d.D, W3, (const T*)d.dcat + (long)t * W3, (long)d.T * W3, 0, d.w_hcat, d.D, 0,
                     d.dh, d.D, 0, 1, &ep, st);
    if (rc) return rc;
  }
  return 0;
}

static int check_desc(const imgcap_lstm_desc* d) {
  IMGCAP_REQUIRE(d != nullptr, "lstm desc NULL");
  IMGCAP_REQUIRE(d->dtype == IMGCAP_F32 || d->dtype == IMGCAP_BF16, "lstm: dtype");
  IMGCAP_REQUIRE(d->B > 0 && d->T > 0 && d->P > 0 && d->P <= MAXP, "lstm: need 0 < P <= 64");
  IMGCAP_REQUIRE(d->E % 8 == 0 && d->A % 8 == 0 && d->D % 8 == 0 && d->M % 8 == 0, "lstm: dims % 8");
  return 0;
}

}  // namespace imgcap

using namespace imgcap;

extern "C" int imgcap_lstm_tf_fwd(const imgcap_lstm_desc* d, void* stream) {
  if (int rc = check_desc(d)) return rc;
  if (d->dtype == IMGCAP_BF16) return lstm_fwd_impl<bf16>(*d, (hipStream_t)stream);
  return lstm_fwd_impl<float>(*d, (hipStream_t)stream);
}

extern "C" int imgcap_lstm_tf_bwd(const imgcap_lstm_desc* d, void* stream) {
  if (int rc = check_desc(d)) return rc;
  IMGCAP_REQUIRE(d->E + 2 * MAXP <= 16384, "lstm bwd: E too large");
  if (d->dtype == IMGCAP_BF16) return lstm_bwd_impl<bf16>(*d, (hipStream_t)stream);
  return lstm_bwd_impl<float>(*d, (hipStream_t)stream);
}

extern "C" int imgcap_attn_reg(int B, int T, int P, const float* alphas, float alphaC, float* dreg, float* reg_out,
                               void* stream) {
  hipLaunchKernelGGL(attn_reg_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, B, T, P, alphas, alphaC, dreg,
                     reg_out);
  IMGCAP_CHECK_LAUNCH("imgcap_attn_reg");
  return 0;
}

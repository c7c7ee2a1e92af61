// Teacher-forced "Show, Attend and Tell" LSTM decoder recurrence (models/decoder.py:104-148)
// and its backward-through-time, driven natively: one C-ABI call enqueues all T steps.
//
// Exact algebraic restructuring of the reference loop (results identical up to fp
// reassociation):
//   * att1 = enc W_ea^T + b_ea (decoder.py:61) is computed ONCE outside the loop (the
//     reference recomputes it every step)
//   * the three GEMMs that read h_{t-1} (decoder_att, f_beta, LSTMCell weight_hh) are one
//     GEMM against W_hcat = [W_da; W_fb; W_hh]
//   * the embedding half of weight_ih (and bias_ih) is precomputed for all t (xe); only the
//     attention half (z_t W_ih[:,M:]^T) stays in the loop
//   * fc(dropout(h)) (decoder.py:144) runs once after the loop over all [B*T] rows
//   * rows are never shrunk: rows with t >= decode_length[b] are computed and masked out
//     (alphas = 0 there; the loss never reads their logits; their gradients are zero)
//   * backward keeps only the recurrent chain in the loop: the encoder_att / full_att weight
//     gradients are summed over t in ONE pass afterwards (attn_param_grad_kernel), from the
//     saved softmax-input gradients de[b,t,p]
// Per step (forward): skinny GEMM(h->g1) -> attn_fwd -> skinny GEMM(z->g2) -> cell_fwd.
// Backward: cell_bwd -> skinny GEMM(dgates->dz) -> attn_bwd -> skinny GEMM(dcat->dh), with
// the weights pre-transposed (w_ihz_t, w_hcat_t) so every step GEMM is k-major x k-major.
#include "common.h"

namespace imgcap {

constexpr int ATT_THREADS = 1024;
constexpr int ATT_WAVES = ATT_THREADS / 64;
constexpr int MAXP = 64;

template <typename T> DEV void load8(const T* p, float (&v)[8]);
template <> DEV void load8<bf16>(const bf16* p, float (&v)[8]) {
  const bf16x8 x = *(const bf16x8*)p;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (float)x[j];
}
template <> DEV void load8<float>(const float* p, float (&v)[8]) {
  const f32x4 a = *(const f32x4*)p, b = *(const f32x4*)(p + 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) { v[j] = a[j]; v[j + 4] = b[j]; }
}

// ---- forward attention step: one block (16 waves) per batch row ------------------------
template <typename T>
__global__ __launch_bounds__(ATT_THREADS) void attn_fwd_kernel(imgcap_lstm_desc d, int t) {
  const int b = blockIdx.x;
  const int P = d.P, E = d.E, A = d.A, Tn = d.T;
  const int W3 = A + E + 4 * d.D;
  const long bt = (long)b * Tn + t;
  const bool active = t < d.dl[b];
  const float* g1 = d.g1 + bt * W3;  // [att2 | gate_pre | hh]
  const T* att1 = (const T*)d.att1 + (long)b * P * A;
  const T* enc = (const T*)d.enc + (long)b * P * E;
  __shared__ float e_s[MAXP];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // scores e_p = w_f . relu(att1_p + att2)   (full_att bias cancels in the softmax)
  for (int p = w; p < P; p += ATT_WAVES) {
    float s = 0.f;
    for (int a = lane * 8; a < A; a += 512) {
      float x[8];
      load8<T>(att1 + (long)p * A + a, x);
      const f32x4 g0 = *(const f32x4*)(g1 + a), g4 = *(const f32x4*)(g1 + a + 4);
      const f32x4 w0 = *(const f32x4*)(d.w_f + a), w4 = *(const f32x4*)(d.w_f + a + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        s += w0[j] * fmaxf(x[j] + g0[j], 0.f);
        s += w4[j] * fmaxf(x[j + 4] + g4[j], 0.f);
      }
    }
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
      d.alphas[bt * P + lane] = active ? al : 0.f;
    }
  }
  __syncthreads();
  T* zs = (T*)d.zs + bt * E;
  float* awe = d.awe + bt * E;
  for (int e = threadIdx.x; e < E; e += ATT_THREADS) {
    float s = 0.f;
#pragma unroll 7
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
    const bool last = t + 1 >= Tn;  // no carry into the last step
    const float dh = to_f(((const T*)d.dhs)[bt * D + j]) + (last ? 0.f : d.dh[e]);
    const float* ga = d.gates + bt * 4 * D;
    const float gi = ga[j], gf = ga[D + j], gg = ga[2 * D + j], go = ga[3 * D + j];
    const float c = d.cs[bt * D + j];
    const float cp = t == 0 ? d.c0[e] : d.cs[(bt - 1) * D + j];
    const float tc = tanhf(c);
    const float dct = (last ? 0.f : d.dc[e]) + dh * go * (1.f - tc * tc);
    dg[j] = from_f<T>(dct * gg * gi * (1.f - gi));
    dg[D + j] = from_f<T>(dct * cp * gf * (1.f - gf));
    dg[2 * D + j] = from_f<T>(dct * gi * (1.f - gg * gg));
    dg[3 * D + j] = from_f<T>(dh * tc * go * (1.f - go));
    d.dc[e] = dct * gf;
  }
}

// ---- backward attention step: recurrent part only ---------------------------------------
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
    if (threadIdx.x < P) d.de[bt * P + threadIdx.x] = 0.f;
    return;
  }
  float* dawe = sm;              // [E]
  float* al = sm + E;            // [MAXP]
  float* dal = al + MAXP;        // [MAXP]
  float* part = dal + MAXP;      // [2][A]
  const float* g1 = d.g1 + bt * W3;
  const float* dz = d.dz + (long)b * E;
  const float* awe = d.awe + bt * E;
  for (int e = threadIdx.x; e < E; e += ATT_THREADS) {
    const float s = sigmoidf_(g1[A + e]);
    dawe[e] = dz[e] * s;
    dcat[A + e] = from_f<T>(dz[e] * awe[e] * s * (1.f - s));  // d gate_pre
  }
  if (threadIdx.x < P) al[threadIdx.x] = d.alphas[bt * P + threadIdx.x];
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const T* enc = (const T*)d.enc + (long)b * P * E;
  for (int p = w; p < P; p += ATT_WAVES) {  // d alpha_p = enc_p . d awe  (+ reg/upstream term)
    float s = 0.f;
    for (int e = lane * 8; e < E; e += 512) {
      float x[8];
      load8<T>(enc + (long)p * E + e, x);
#pragma unroll
      for (int j = 0; j < 8; ++j) s += x[j] * dawe[e + j];
    }
    s = wave_sum(s);
    if (lane == 0) dal[p] = s + (d.dalpha ? d.dalpha[bt * P + p] : 0.f);
  }
  __syncthreads();
  if (w == 0) {  // softmax backward -> d score
    const float a = lane < P ? al[lane] : 0.f, da = lane < P ? dal[lane] : 0.f;
    const float dot = wave_sum(a * da);
    if (lane < P) {
      const float de = a * (da - dot);
      dal[lane] = de;
      d.de[bt * P + lane] = de;
    }
  }
  __syncthreads();
  // d att2[a] = w_f[a] * sum_p de_p [att1[p,a] + att2[a] > 0]; two halves of p in parallel
  const T* att1 = (const T*)d.att1 + (long)b * P * A;
  const int half = threadIdx.x / 512, tid = threadIdx.x % 512;
  const int p0 = half * ((P + 1) / 2), p1 = min(P, p0 + (P + 1) / 2);
  for (int a = tid; a < A; a += 512) {
    const float a2 = g1[a];
    float s = 0.f;
#pragma unroll 7
    for (int p = p0; p < p1; ++p) s += (to_f(att1[(long)p * A + a]) + a2 > 0.f) ? dal[p] : 0.f;
    part[half * A + a] = s;
  }
  __syncthreads();
  for (int a = threadIdx.x; a < A; a += ATT_THREADS) dcat[a] = from_f<T>((part[a] + part[A + a]) * d.w_f[a]);
}

// ---- attention parameter gradients, summed over all steps at once -----------------------
//   datt1[b,p,a]  = w_f[a] * sum_t de[b,t,p] [att1[b,p,a] + att2[b,t,a] > 0]
//   dwf_part[b,c,a]  = sum_{t, p in chunk c} de[b,t,p] relu(att1[b,p,a] + att2[b,t,a])
//   dbea_part[b,c,a] = sum_{p in chunk c} datt1[b,p,a]
// Block = (chunk of PCH pixels, batch row); thread = attention unit a; the chunk's att1
// values and accumulators stay in registers while t sweeps the saved att2 rows.
constexpr int PCH = 7;
template <typename T>
__global__ __launch_bounds__(512) void attn_param_grad_kernel(imgcap_lstm_desc d) {
  extern __shared__ __attribute__((aligned(16))) float de_s[];  // [T][PCH]
  const int b = blockIdx.y, c = blockIdx.x, nc = gridDim.x;
  const int P = d.P, A = d.A, E = d.E, Tn = d.T;
  const int W3 = A + E + 4 * d.D;
  const int p0 = c * PCH;
  for (int i = threadIdx.x; i < Tn * PCH; i += blockDim.x) {
    const int t = i / PCH, q = i % PCH;
    de_s[i] = p0 + q < P ? d.de[((long)b * Tn + t) * P + p0 + q] : 0.f;
  }
  __syncthreads();
  const T* att1 = (const T*)d.att1 + (long)b * P * A;
  const int tmax = min(Tn, d.dl[b]);
  for (int a = threadIdx.x; a < A; a += blockDim.x) {
    float x1[PCH], acc[PCH];
#pragma unroll
    for (int q = 0; q < PCH; ++q) {
      x1[q] = p0 + q < P ? to_f(att1[(long)(p0 + q) * A + a]) : 0.f;
      acc[q] = 0.f;
    }
    float swf = 0.f;
    const float* a2p = d.g1 + (long)b * Tn * W3 + a;
    for (int t = 0; t < tmax; ++t) {
      const float a2 = a2p[(long)t * W3];
#pragma unroll
      for (int q = 0; q < PCH; ++q) {
        const float u = x1[q] + a2;
        const float g = de_s[t * PCH + q];
        acc[q] += u > 0.f ? g : 0.f;
        swf += g * fmaxf(u, 0.f);
      }
    }
    const float wf = d.w_f[a];
    float sb = 0.f;
    T* out = (T*)d.datt1 + (long)b * P * A + a;
#pragma unroll
    for (int q = 0; q < PCH; ++q) {
      if (p0 + q < P) {
        const float v = acc[q] * wf;
        out[(long)(p0 + q) * A] = from_f<T>(v);
        sb += v;
      }
    }
    d.dwf[((long)b * nc + c) * A + a] = swf;
    d.dbea[((long)b * nc + c) * A + a] = sb;
  }
}

// ---- doubly stochastic attention regularisation (train.py:269) --------------------------
//   reg = alphaC * mean_{b,p} (1 - sum_t alpha[b,t,p])^2
//   dalpha[b,t,p] = d reg / d alpha[b,t,p] for t < dl[b] (the written alphas), else 0
__global__ void attn_reg_kernel(int B, int Tn, int P, const float* __restrict__ alphas, const int32_t* __restrict__ dl,
                                float alphaC, float* __restrict__ dalpha, float* __restrict__ reg_out) {
  __shared__ float red[16];
  float acc = 0.f;
  for (int e = threadIdx.x; e < B * P; e += blockDim.x) {
    const int b = e / P, p = e % P;
    float s = 0.f;
    for (int t = 0; t < Tn; ++t) s += alphas[((long)b * Tn + t) * P + p];
    acc += (1.f - s) * (1.f - s);
    const float g = alphaC * 2.f * (s - 1.f) / (float)(B * P);
    for (int t = 0; t < Tn; ++t) dalpha[((long)b * Tn + t) * P + p] = t < dl[b] ? g : 0.f;
  }
  const float tot = block_sum(acc, red);
  if (threadIdx.x == 0) *reg_out = alphaC * tot / (float)(B * P);
}

static dim3 pw_grid(long n) {
  long b = (n + 255) / 256;
  return dim3((unsigned)(b > 2048 ? 2048 : (b < 1 ? 1 : b)));
}

static imgcap_epilogue f32_epi(const float* bias) {
  imgcap_epilogue ep{};
  ep.alpha = 1.f;
  ep.c_dtype = IMGCAP_F32;
  ep.rows_per_scale = 1;
  ep.bias = bias;
  return ep;
}

template <typename T>
static int lstm_fwd_impl(const imgcap_lstm_desc& d, hipStream_t st) {
  const int W3 = d.A + d.E + 4 * d.D;
  const int ct = d.dtype;
  const imgcap_epilogue e1 = f32_epi(d.b_hcat), e2 = f32_epi(nullptr);
  for (int t = 0; t < d.T; ++t) {
    int rc = imgcap_gemm(ct, 1, 1, d.B, W3, d.D, (const T*)d.hprev + (long)t * d.D, (long)d.T * d.D, 0, d.w_hcat,
                         d.D, 0, d.g1 + (long)t * W3, (long)d.T * W3, 0, 1, &e1, st);
    if (rc) return rc;
    hipLaunchKernelGGL(attn_fwd_kernel<T>, dim3(d.B), dim3(ATT_THREADS), 0, st, d, t);
    IMGCAP_CHECK_LAUNCH("lstm attn_fwd");
    rc = imgcap_gemm(ct, 1, 1, d.B, 4 * d.D, d.E, (const T*)d.zs + (long)t * d.E, (long)d.T * d.E, 0,
                     (const T*)d.w_ih + d.M, d.M + d.E, 0, d.g2, 4 * d.D, 0, 1, &e2, st);
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
  const imgcap_epilogue ep = f32_epi(nullptr);
  const size_t shm = (d.E + 2 * MAXP + 2 * d.A) * sizeof(float);
  for (int t = d.T - 1; t >= 0; --t) {
    hipLaunchKernelGGL(cell_bwd_kernel<T>, pw_grid((long)d.B * d.D), dim3(256), 0, st, d, t);
    IMGCAP_CHECK_LAUNCH("lstm cell_bwd");
    // dz = dgates_t . W_ih[:, M:]      (w_ihz_t = W_ih[:, M:]^T, [E][4D])
    int rc = imgcap_gemm(ct, 1, 1, d.B, d.E, 4 * d.D, (const T*)d.dcat + (long)t * W3 + d.A + d.E, (long)d.T * W3,
                         0, d.w_ihz_t, 4 * d.D, 0, d.dz, d.E, 0, 1, &ep, st);
    if (rc) return rc;
    hipLaunchKernelGGL(attn_bwd_kernel<T>, dim3(d.B), dim3(ATT_THREADS), shm, st, d, t);
    IMGCAP_CHECK_LAUNCH("lstm attn_bwd");
    // dh_{t-1} = [d att2 | d gate_pre | d gates] . W_hcat    (w_hcat_t = W_hcat^T, [D][W3]);
    // at t = 0 this is dL/dh0
    rc = imgcap_gemm(ct, 1, 1, d.B, d.D, W3, (const T*)d.dcat + (long)t * W3, (long)d.T * W3, 0, d.w_hcat_t, W3, 0,
                     d.dh, d.D, 0, 1, &ep, st);
    if (rc) return rc;
  }
  const size_t shm2 = (size_t)d.T * PCH * sizeof(float);
  const int thr = d.A >= 512 ? 512 : ((d.A + 63) / 64) * 64;
  hipLaunchKernelGGL(attn_param_grad_kernel<T>, dim3((d.P + PCH - 1) / PCH, d.B), dim3(thr), shm2, st, d);
  IMGCAP_CHECK_LAUNCH("lstm attn_param_grad");
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
  IMGCAP_REQUIRE((d->E + 2 * MAXP + 2 * d->A) * 4 <= 65536, "lstm bwd: E/A too large for LDS");
  IMGCAP_REQUIRE((size_t)d->T * PCH * 4 <= 65536, "lstm bwd: T too large for LDS");
  IMGCAP_REQUIRE(d->w_ihz_t && d->w_hcat_t && d->de && d->dbea, "lstm bwd: transposed weights / de / dbea needed");
  if (d->dtype == IMGCAP_BF16) return lstm_bwd_impl<bf16>(*d, (hipStream_t)stream);
  return lstm_bwd_impl<float>(*d, (hipStream_t)stream);
}

extern "C" int imgcap_attn_reg(int B, int T, int P, const float* alphas, const int32_t* dl, float alphaC,
                               float* dalpha, float* reg_out, void* stream) {
  hipLaunchKernelGGL(attn_reg_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, B, T, P, alphas, dl, alphaC, dalpha,
                     reg_out);
  IMGCAP_CHECK_LAUNCH("imgcap_attn_reg");
  return 0;
}

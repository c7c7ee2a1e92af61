// Backward of the trainable ConvNeXt children (Encoder.fine_tune, models/encoder.py:29-34;
// train.py:113-114,278-290 train them with their own Adam when fineTuneEncoder).
//
// Per CNBlock  out = x + sd * gamma * (GELU(LN(dwconv7(x)) W1^T + b1) W2^T + b2)  the backward
// is, with dout' = dout * sd (per sample) and a = GELU(h):
//   G      = dout'^T a                  (MFMA GEMM, imgcap_gemm)         [C, 4C] fp32
//   dW2    = gamma * G,  dgamma = sum_k W2 * G + b2 * colsum(dout'),  db2 = gamma * colsum(dout')
//   dh     = dout' (gamma W2) * GELU'(h)  (imgcap_gemm, ACT_DGELU epilogue)
//   dW1    = dh^T LN(z), db1 = colsum(dh), dzn = dh W1   (imgcap_gemm / imgcap_colsum)
//   dz     = LayerNorm backward           (imgcap_add_layernorm_bwd)
//   dx     = dout + dwconv7^T(dz)         (imgcap_dwconv7_bwd_data: flipped taps)
//   dWdw   = sum over pixels dz * shifted x, dbdw = colsum(dz)   (this file)
// This file holds the kernels with no GEMM shape: the depthwise weight gradient, the
// layer-scale gradient, per-sample row scaling, the LayerNorm2d + 2x2 patchify backward of the
// downsample layers, the adaptive-pool backward and the deterministic slice reduction they
// share.  All reductions are fixed-order (no float atomics): results are bit-reproducible.
#include <algorithm>

#include "common.h"

namespace imgcap {

// ---- depthwise 7x7 weight / bias gradient -------------------------------------------------
// Block = 4 waves x 128 channels (2 per lane, one 4-byte bf16 pair or 8-byte f32 pair per load).
// Each wave walks image rows; for each kernel row kh it slides a 7-pixel register window along
// the input row (one new load per output pixel) and accumulates all 49 taps in registers.  The
// 4 waves' sums meet in LDS; the block writes one slice row ws[slice][c][50] (49 taps + bias).
template <typename T>
DEV void ld2(const T* p, float& a, float& b);
template <> DEV void ld2<bf16>(const bf16* p, float& a, float& b) {
  const bf16x2 v = *(const bf16x2*)p;
  a = (float)v[0];
  b = (float)v[1];
}
template <> DEV void ld2<float>(const float* p, float& a, float& b) {
  const f32x2 v = *(const f32x2*)p;
  a = v[0];
  b = v[1];
}

constexpr int WG_CH = 128;  // channels per block
template <typename T>
__global__ __launch_bounds__(256) void dwconv7_wgrad_kernel(int B, int H, int W, int C, const T* __restrict__ dz,
                                                            const T* __restrict__ x, float* __restrict__ ws,
                                                            int rows_per_wave) {
  __shared__ float red[4][WG_CH][51];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = blockIdx.x * WG_CH + 2 * lane;
  const bool cok = c < C;
  const int cc = cok ? c : 0;
  float acc[49][2], accb[2] = {0.f, 0.f};
#pragma unroll
  for (int t = 0; t < 49; ++t) acc[t][0] = acc[t][1] = 0.f;
  const long R = (long)B * H;
  const long r0 = ((long)blockIdx.y * 4 + wv) * rows_per_wave;
  const long r1 = std::min<long>(R, r0 + rows_per_wave);
  for (long r = r0; r < r1; ++r) {
    const int h = (int)(r % H);
    const T* drow = dz + r * W * C + cc;
    for (int w = 0; w < W; ++w) {
      float g0, g1;
      ld2<T>(drow + (long)w * C, g0, g1);
      accb[0] += g0;
      accb[1] += g1;
    }
#pragma unroll
    for (int kh = 0; kh < 7; ++kh) {
      const int ih = h + kh - 3;
      if (ih < 0 || ih >= H) continue;
      const T* xrow = x + (r + kh - 3) * W * C + cc;
      float win[7][2];
#pragma unroll
      for (int q = 0; q < 7; ++q) {
        const int iw = q - 3;
        if (iw >= 0 && iw < W) ld2<T>(xrow + (long)iw * C, win[q][0], win[q][1]);
        else win[q][0] = win[q][1] = 0.f;
      }
      for (int w = 0; w < W; ++w) {
        float g0, g1;
        ld2<T>(drow + (long)w * C, g0, g1);
        float nx0 = 0.f, nx1 = 0.f;
        if (w + 4 < W) ld2<T>(xrow + (long)(w + 4) * C, nx0, nx1);
#pragma unroll
        for (int kw = 0; kw < 7; ++kw) {
          acc[kh * 7 + kw][0] += g0 * win[kw][0];
          acc[kh * 7 + kw][1] += g1 * win[kw][1];
        }
#pragma unroll
        for (int q = 0; q < 6; ++q) { win[q][0] = win[q + 1][0]; win[q][1] = win[q + 1][1]; }
        win[6][0] = nx0;
        win[6][1] = nx1;
      }
    }
  }
#pragma unroll
  for (int t = 0; t < 49; ++t) {
    red[wv][2 * lane][t] = acc[t][0];
    red[wv][2 * lane + 1][t] = acc[t][1];
  }
  red[wv][2 * lane][49] = accb[0];
  red[wv][2 * lane + 1][49] = accb[1];
  __syncthreads();
  (void)cok;
  for (int e = threadIdx.x; e < WG_CH * 50; e += 256) {
    const int cl = e / 50, t = e % 50;
    const int ch = blockIdx.x * WG_CH + cl;
    if (ch < C)
      ws[((long)blockIdx.y * C + ch) * 50 + t] = ((red[0][cl][t] + red[1][cl][t]) + red[2][cl][t]) + red[3][cl][t];
  }
}

// W = 7 (the last stage): a wave's image row is 7 pixels, so the sliding window above spends
// its time waiting on one dependent load pair per output pixel (C5's fine-tuned stage 4: ~107 us
// per call).  Here the row's 7 gradient pixels and the 7 x 7 input window are requested at once
// (fully unrolled: 56 loads in flight per lane) and the 49 taps accumulate from registers; the
// per-tap sums keep the sliding form's order (output pixels w = 0..6 per kernel row, kernel rows
// in order, image rows in order), and the block reduction is the same.
template <typename T>
__global__ __launch_bounds__(256) void dwconv7_wgrad_w7_kernel(int B, int H, int C, const T* __restrict__ dz,
                                                               const T* __restrict__ x, float* __restrict__ ws,
                                                               int rows_per_wave) {
  constexpr int W = 7;
  __shared__ float red[4][WG_CH][51];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = blockIdx.x * WG_CH + 2 * lane;
  const int cc = c < C ? c : 0;
  float acc[49][2], accb[2] = {0.f, 0.f};
#pragma unroll
  for (int t = 0; t < 49; ++t) acc[t][0] = acc[t][1] = 0.f;
  const long R = (long)B * H;
  const long r0 = ((long)blockIdx.y * 4 + wv) * rows_per_wave;
  const long r1 = std::min<long>(R, r0 + rows_per_wave);
  for (long r = r0; r < r1; ++r) {
    const int h = (int)(r % H);
    float g[W][2], xw[7][W][2];
    const T* drow = dz + r * W * C + cc;
#pragma unroll
    for (int w = 0; w < W; ++w) ld2<T>(drow + (long)w * C, g[w][0], g[w][1]);
#pragma unroll
    for (int kh = 0; kh < 7; ++kh) {
      const int ih = h + kh - 3;
      const bool ok = ih >= 0 && ih < H;
      const T* xrow = x + (ok ? r + kh - 3 : r) * W * C + cc;
#pragma unroll
      for (int w = 0; w < W; ++w) {
        ld2<T>(xrow + (long)w * C, xw[kh][w][0], xw[kh][w][1]);
        if (!ok) xw[kh][w][0] = xw[kh][w][1] = 0.f;
      }
    }
#pragma unroll
    for (int w = 0; w < W; ++w) {
      accb[0] += g[w][0];
      accb[1] += g[w][1];
    }
#pragma unroll
    for (int kh = 0; kh < 7; ++kh) {
      if (h + kh - 3 < 0 || h + kh - 3 >= H) continue;  // the sliding form skips these rows too
#pragma unroll
      for (int w = 0; w < W; ++w)
#pragma unroll
        for (int kw = 0; kw < 7; ++kw) {
          const int iw = w + kw - 3;
          const float x0 = (iw >= 0 && iw < W) ? xw[kh][iw][0] : 0.f, x1 = (iw >= 0 && iw < W) ? xw[kh][iw][1] : 0.f;
          acc[kh * 7 + kw][0] += g[w][0] * x0;
          acc[kh * 7 + kw][1] += g[w][1] * x1;
        }
    }
  }
#pragma unroll
  for (int t = 0; t < 49; ++t) {
    red[wv][2 * lane][t] = acc[t][0];
    red[wv][2 * lane + 1][t] = acc[t][1];
  }
  red[wv][2 * lane][49] = accb[0];
  red[wv][2 * lane + 1][49] = accb[1];
  __syncthreads();
  for (int e = threadIdx.x; e < WG_CH * 50; e += 256) {
    const int cl = e / 50, t = e % 50;
    const int ch = blockIdx.x * WG_CH + cl;
    if (ch < C)
      ws[((long)blockIdx.y * C + ch) * 50 + t] = ((red[0][cl][t] + red[1][cl][t]) + red[2][cl][t]) + red[3][cl][t];
  }
}

// t_i = sum_s ws[s * ld + i] for i < n (fixed slice order), stored as
//   split == 0 : out0[i] = beta*out0[i] + t_i
//   split > 0  : i < split -> out0[i], else out1[i - split]   (both with beta)
//   split < 0  : depthwise layout i = c*50 + k -> out0[c*49 + k] (k < 49), out1[c] (k == 49)
__global__ __launch_bounds__(256) void slice_reduce_kernel(long n, int slices, const float* __restrict__ ws, long ld,
                                                           float beta, long split, float* __restrict__ out0,
                                                           float* __restrict__ out1) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  int z = 0;
  for (; z + 4 <= slices; z += 4) {
#pragma unroll
    for (int u = 0; u < 4; ++u) s[u] += ws[(long)(z + u) * ld + i];
  }
  for (; z < slices; ++z) s[0] += ws[(long)z * ld + i];
  const float t = (s[0] + s[1]) + (s[2] + s[3]);
  float* dst;
  if (split < 0) {
    const long c = i / 50, k = i % 50;
    dst = k < 49 ? out0 + c * 49 + k : out1 + c;
  } else {
    dst = (split > 0 && i >= split) ? out1 + (i - split) : out0 + i;
  }
  *dst = (beta != 0.f ? beta * *dst : 0.f) + t;
}

// ---- layer-scale backward (one block per channel row c of W2 [C][4C]) ---------------------
//   dW2[c,:] = gamma[c] * G[c,:];  wg[c,:] = gamma[c] * W2[c,:] (compute dtype, the operand of
//   the d-hidden GEMM);  dgamma[c] = sum_k W2[c,k] G[c,k] + b2[c] cs[c];  db2[c] = gamma[c] cs[c]
template <typename T>
__global__ __launch_bounds__(256) void layer_scale_grad_kernel(int C4, const float* __restrict__ G,
                                                               const float* __restrict__ w2,
                                                               const float* __restrict__ b2,
                                                               const float* __restrict__ gamma,
                                                               const float* __restrict__ cs, float* __restrict__ dw2,
                                                               T* __restrict__ wg, float* __restrict__ dgamma,
                                                               float* __restrict__ db2) {
  __shared__ float red[4];
  const int c = blockIdx.x;
  const float g = gamma[c];
  float dot = 0.f;
  for (int k = threadIdx.x; k < C4; k += 256) {
    const long i = (long)c * C4 + k;
    const float gv = G[i], wv = w2[i];
    dw2[i] = g * gv;
    wg[i] = from_f<T>(g * wv);
    dot += wv * gv;
  }
  dot = block_sum(dot, red);
  if (threadIdx.x == 0) {
    dgamma[c] = dot + b2[c] * cs[c];
    db2[c] = g * cs[c];
  }
}

// y[r, :] = x[r, :] * s[r / rows_per_scale]   (stochastic-depth scale of a block's gradient)
template <typename T>
__global__ __launch_bounds__(256) void rowscale_kernel(long rows, int cols, const T* __restrict__ x,
                                                       const float* __restrict__ s, int rps, T* __restrict__ y) {
  constexpr int G = 16 / sizeof(T);
  const long nv = rows * (cols / G);
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < nv; e += (long)gridDim.x * 256) {
    const long r = e / (cols / G);
    const float f = s[r / rps];
    float v[G];
    ld_g<T, G>(x + e * G, v);
#pragma unroll
    for (int j = 0; j < G; ++j) v[j] *= f;
    st_g<T, G>(y + e * G, v);
  }
}

// ---- LayerNorm2d + 2x2/s2 patchify backward (features[2,4,6]) -----------------------------
// One wave per input pixel (b, ih, iw): its gradient row is the (ih%2, iw%2) quarter of patch
// row (b, ih/2, iw/2); the LayerNorm statistics are recomputed from x.  The block's 4 waves x
// pixels_per_wave pixels sum their dln_w / dln_b contributions and write one slice row
// ws[block][2C] (reduced by slice_reduce_kernel).
template <typename T>
__global__ __launch_bounds__(256) void ln_patchify2_bwd_kernel(int B, int H, int W, int C, const T* __restrict__ x,
                                                               const T* __restrict__ dp,
                                                               const float* __restrict__ lw, T* __restrict__ dx,
                                                               float* __restrict__ ws, int px_per_wave,
                                                               int cmajor) {
  constexpr int MAXV = 24;  // C <= 1536
  extern __shared__ float part[];  // [4][2C]
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float ag[MAXV], ab[MAXV];
#pragma unroll
  for (int j = 0; j < MAXV; ++j) ag[j] = ab[j] = 0.f;
  const long NPX = (long)B * H * W;
  const long p0 = ((long)blockIdx.x * 4 + wv) * px_per_wave;
  for (long px = p0; px < std::min(NPX, p0 + px_per_wave); ++px) {
    const int b = (int)(px / (H * W)), rem = (int)(px % (H * W)), ih = rem / W, iw = rem % W;
    const long prow = ((long)b * (H / 2) + ih / 2) * (W / 2) + iw / 2;
    const int quad = (ih & 1) * 2 + (iw & 1);
    const T* g = dp + prow * 4 * C + (cmajor ? quad : quad * C);
    const int gs = cmajor ? 4 : 1;
    const T* xr = x + px * C;
    float xv[MAXV], gv[MAXV];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < MAXV; ++j) {
      const int c = lane + 64 * j;
      xv[j] = c < C ? to_f(xr[c]) : 0.f;
      gv[j] = c < C ? to_f(g[c * gs]) : 0.f;
      s += xv[j];
    }
    const float mean = wave_sum(s) / C;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < MAXV; ++j)
      if (lane + 64 * j < C) { const float d = xv[j] - mean; q += d * d; }
    const float rstd = rsqrtf(wave_sum(q) / C + 1e-6f);
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < MAXV; ++j) {
      const int c = lane + 64 * j;
      if (c < C) {
        const float xh = (xv[j] - mean) * rstd;
        xv[j] = xh;
        ag[j] += gv[j] * xh;
        ab[j] += gv[j];
        gv[j] *= lw[c];
        s1 += gv[j];
        s2 += gv[j] * xh;
      }
    }
    s1 = wave_sum(s1) / C;
    s2 = wave_sum(s2) / C;
    T* o = dx + px * C;
#pragma unroll
    for (int j = 0; j < MAXV; ++j) {
      const int c = lane + 64 * j;
      if (c < C) o[c] = from_f<T>(rstd * (gv[j] - s1 - xv[j] * s2));
    }
  }
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    const int c = lane + 64 * j;
    if (c < C) { part[wv * 2 * C + c] = ag[j]; part[wv * 2 * C + C + c] = ab[j]; }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < 2 * C; c += 256)
    ws[(long)blockIdx.x * 2 * C + c] = ((part[c] + part[2 * C + c]) + part[4 * C + c]) + part[6 * C + c];
}

// ---- AdaptiveAvgPool2d backward (NHWC): dx[b,ih,iw,c] = sum over the output cells whose
// window [floor(o*H/OH), ceil((o+1)*H/OH)) holds (ih, iw) of dy / window area -----------------
template <typename T>
__global__ __launch_bounds__(256) void adaptive_pool_bwd_kernel(int B, int H, int W, int C, int OH, int OW,
                                                                const T* __restrict__ dy, T* __restrict__ dx) {
  const long n = (long)B * H * W * C;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < n; e += (long)gridDim.x * 256) {
    const int c = (int)(e % C);
    const long px = e / C;
    const int iw = (int)(px % W), ih = (int)((px / W) % H), b = (int)(px / ((long)W * H));
    float s = 0.f;
    const int oh0 = (ih * OH) / H, ow0 = (iw * OW) / W;
    for (int oh = std::max(0, oh0 - 1); oh < OH; ++oh) {
      const int hs = (oh * H) / OH, he = ((oh + 1) * H + OH - 1) / OH;
      if (hs > ih) break;
      if (ih >= he) continue;
      for (int ow = std::max(0, ow0 - 1); ow < OW; ++ow) {
        const int wsx = (ow * W) / OW, we = ((ow + 1) * W + OW - 1) / OW;
        if (wsx > iw) break;
        if (iw >= we) continue;
        s += to_f(dy[(((long)b * OH + oh) * OW + ow) * C + c]) / (float)((he - hs) * (we - wsx));
      }
    }
    dx[e] = from_f<T>(s);
  }
}

}  // namespace imgcap

using namespace imgcap;

namespace {
int grid_for(long n) { return (int)std::min<long>((n + 255) / 256, 4096); }
}  // namespace

extern "C" int imgcap_dwconv7_wgrad(int dtype, int B, int H, int W, int C, const void* dz, const void* x, float* dw,
                                    float* db, void* stream) {
  IMGCAP_REQUIRE(C % 2 == 0, "imgcap_dwconv7_wgrad: C must be even");
  IMGCAP_REQUIRE(dw && db, "imgcap_dwconv7_wgrad: dw and db required");
  const long R = (long)B * H;
  if (R == 0 || C == 0) return 0;
  const int cblocks = (C + WG_CH - 1) / WG_CH;
  // ~2 blocks per CU in total, every wave at least one image row
  const long waves_wanted = std::max<long>(1, std::min<long>(R, (512 / cblocks) * 4));
  const int rpw = (int)((R + waves_wanted - 1) / waves_wanted);
  const int slices = (int)((R + 4L * rpw - 1) / (4L * rpw));
  float* ws = (float*)workspace((size_t)slices * C * 50 * sizeof(float), (hipStream_t)stream);
  if (!ws) return fail(IMGCAP_EWORKSPACE, std::string("imgcap_dwconv7_wgrad: ") + last_error());
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid(cblocks, slices);
  const char* we = getenv("IMGCAP_DW_WGRAD_W7");  // 0: the sliding-window kernel at W = 7 too (A/B)
  const bool w7 = W == 7 && !(we && *we == '0');
  if (w7 && dtype == IMGCAP_BF16)
    hipLaunchKernelGGL(dwconv7_wgrad_w7_kernel<bf16>, grid, dim3(256), 0, st, B, H, C, (const bf16*)dz,
                       (const bf16*)x, ws, rpw);
  else if (w7)
    hipLaunchKernelGGL(dwconv7_wgrad_w7_kernel<float>, grid, dim3(256), 0, st, B, H, C, (const float*)dz,
                       (const float*)x, ws, rpw);
  else if (dtype == IMGCAP_BF16)
    hipLaunchKernelGGL(dwconv7_wgrad_kernel<bf16>, grid, dim3(256), 0, st, B, H, W, C, (const bf16*)dz,
                       (const bf16*)x, ws, rpw);
  else
    hipLaunchKernelGGL(dwconv7_wgrad_kernel<float>, grid, dim3(256), 0, st, B, H, W, C, (const float*)dz,
                       (const float*)x, ws, rpw);
  const long n = (long)C * 50;
  hipLaunchKernelGGL(slice_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, n, slices, ws,
                     (long)C * 50, 0.f, -1L, dw, db);
  IMGCAP_CHECK_LAUNCH("imgcap_dwconv7_wgrad");
  return 0;
}

extern "C" int imgcap_layer_scale_grad(int dtype, int C, int C4, const float* G, const float* w2, const float* b2,
                                       const float* gamma, const float* cs, float* dw2, void* wg, float* dgamma,
                                       float* db2, void* stream) {
  if (C == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == IMGCAP_BF16)
    hipLaunchKernelGGL(layer_scale_grad_kernel<bf16>, dim3(C), dim3(256), 0, st, C4, G, w2, b2, gamma, cs, dw2,
                       (bf16*)wg, dgamma, db2);
  else
    hipLaunchKernelGGL(layer_scale_grad_kernel<float>, dim3(C), dim3(256), 0, st, C4, G, w2, b2, gamma, cs, dw2,
                       (float*)wg, dgamma, db2);
  IMGCAP_CHECK_LAUNCH("imgcap_layer_scale_grad");
  return 0;
}

extern "C" int imgcap_rowscale(int dtype, int64_t rows, int cols, const void* x, const float* s, int rows_per_scale,
                               void* y, void* stream) {
  const int G = dtype == IMGCAP_BF16 ? 8 : 4;
  IMGCAP_REQUIRE(cols % G == 0 && aligned16(x) && aligned16(y) && rows_per_scale > 0,
                 "imgcap_rowscale: cols must fill 16-byte vectors, operands 16-byte aligned");
  const long nv = rows * (cols / G);
  if (nv == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == IMGCAP_BF16)
    hipLaunchKernelGGL(rowscale_kernel<bf16>, dim3(grid_for(nv)), dim3(256), 0, st, (long)rows, cols,
                       (const bf16*)x, s, rows_per_scale, (bf16*)y);
  else
    hipLaunchKernelGGL(rowscale_kernel<float>, dim3(grid_for(nv)), dim3(256), 0, st, (long)rows, cols,
                       (const float*)x, s, rows_per_scale, (float*)y);
  IMGCAP_CHECK_LAUNCH("imgcap_rowscale");
  return 0;
}

extern "C" int imgcap_ln_patchify2_bwd(int dtype, int B, int H, int W, int C, const void* x, const void* dpatches,
                                       const float* ln_w, int cmajor, void* dx, float* dln_w, float* dln_b,
                                       void* stream) {
  IMGCAP_REQUIRE(H % 2 == 0 && W % 2 == 0 && C <= 1536, "imgcap_ln_patchify2_bwd: bad shape");
  const long NPX = (long)B * H * W;
  if (NPX == 0) return 0;
  const int ppw = (int)std::max<long>(1, (NPX + 4 * 512 - 1) / (4 * 512));
  const int blocks = (int)((NPX + 4L * ppw - 1) / (4L * ppw));
  float* ws = (float*)workspace((size_t)blocks * 2 * C * sizeof(float), (hipStream_t)stream);
  if (!ws) return fail(IMGCAP_EWORKSPACE, std::string("imgcap_ln_patchify2_bwd: ") + last_error());
  hipStream_t st = (hipStream_t)stream;
  const size_t shm = (size_t)8 * C * sizeof(float);
  if (dtype == IMGCAP_BF16)
    hipLaunchKernelGGL(ln_patchify2_bwd_kernel<bf16>, dim3(blocks), dim3(256), shm, st, B, H, W, C, (const bf16*)x,
                       (const bf16*)dpatches, ln_w, (bf16*)dx, ws, ppw, cmajor);
  else
    hipLaunchKernelGGL(ln_patchify2_bwd_kernel<float>, dim3(blocks), dim3(256), shm, st, B, H, W, C, (const float*)x,
                       (const float*)dpatches, ln_w, (float*)dx, ws, ppw, cmajor);
  IMGCAP_CHECK_LAUNCH("imgcap_ln_patchify2_bwd");
  imgcap_colsum_item it[2] = {{ws, dln_w, 2L * C, blocks, C, IMGCAP_F32, 0, 0.f},
                              {ws + C, dln_b, 2L * C, blocks, C, IMGCAP_F32, 0, 0.f}};
  return imgcap_colsum_multi(2, it, stream);
}

extern "C" int imgcap_adaptive_pool_bwd_nhwc(int dtype, int B, int H, int W, int C, int OH, int OW, const void* dy,
                                             void* dx, void* stream) {
  const long n = (long)B * H * W * C;
  if (n == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == IMGCAP_BF16)
    hipLaunchKernelGGL(adaptive_pool_bwd_kernel<bf16>, dim3(grid_for(n)), dim3(256), 0, st, B, H, W, C, OH, OW,
                       (const bf16*)dy, (bf16*)dx);
  else
    hipLaunchKernelGGL(adaptive_pool_bwd_kernel<float>, dim3(grid_for(n)), dim3(256), 0, st, B, H, W, C, OH, OW,
                       (const float*)dy, (float*)dx);
  IMGCAP_CHECK_LAUNCH("imgcap_adaptive_pool_bwd_nhwc");
  return 0;
}

extern "C" int imgcap_slice_reduce(int64_t n, int slices, const float* ws, int64_t ld, float beta, int64_t split,
                                   float* out0, float* out1, void* stream) {
  if (n == 0) return 0;
  IMGCAP_REQUIRE(split == 0 || out1, "imgcap_slice_reduce: out1 required when split != 0");
  hipLaunchKernelGGL(slice_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, n,
                     slices, ws, ld, beta, (long)split, out0, out1);
  IMGCAP_CHECK_LAUNCH("imgcap_slice_reduce");
  return 0;
}

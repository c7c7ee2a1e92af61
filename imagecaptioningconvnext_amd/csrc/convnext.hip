// ConvNeXt trunk kernels, NHWC (torchvision ConvNeXt `features`, reached via encoder.py:24).
//   stem       features[0]: Conv2d(3,C0,4,s4,bias) + LayerNorm2d(eps 1e-6), NCHW f32 in
//   dwconv7_ln CNBlock head: depthwise 7x7 (pad 3, bias) + LayerNorm(C, eps 1e-6)
//   ln_patchify2  features[2,4,6] head: LayerNorm2d then 2x2/s2 patch rows for the MFMA GEMM
//   adaptive_pool AdaptiveAvgPool2d (encoder.py:20,25)
// The pointwise Linear pair / downsample conv run on imgcap_gemm (gemm.hip).
#include "common.h"

namespace imgcap {

// ---------------------------------------------------------------------------------------
// stem: one wave per output pixel (looped), lanes own channels c = lane + 64*i (C0 <= 256)
// weights [48][C0] staged in LDS.  48 MACs per output, LN by wave shuffles.
template <typename T>
__global__ __launch_bounds__(256) void stem_kernel(int B, int H, int W, int C0, const float* __restrict__ img,
                                                   const float* __restrict__ w, const float* __restrict__ bias,
                                                   const float* __restrict__ lw, const float* __restrict__ lb,
                                                   T* __restrict__ out, int px_per_block) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* ws = sm;  // [48][C0]
  for (int e = threadIdx.x; e < 48 * C0; e += blockDim.x) {
    const int c = e / 48, k = e % 48;  // torch weight [C0][3][4][4] -> k = ci*16+kh*4+kw
    ws[k * C0 + c] = w[e];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int HO = H / 4, WO = W / 4;
  const long npx = (long)B * HO * WO;
  for (int q = wv; q < px_per_block; q += 4) {
    const long px = (long)blockIdx.x * px_per_block + q;
    if (px >= npx) break;
    const int b = (int)(px / (HO * WO)), rem = (int)(px % (HO * WO)), oh = rem / WO, ow = rem % WO;
    float xv = 0.f;
    if (lane < 48) {
      const int ci = lane >> 4, kh = (lane >> 2) & 3, kw = lane & 3;
      xv = img[(((long)b * 3 + ci) * H + oh * 4 + kh) * W + ow * 4 + kw];
    }
    float xs[48];  // broadcast the 48 patch values to scalar registers
#pragma unroll
    for (int k = 0; k < 48; ++k) xs[k] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(xv), k));
    float acc[4];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = lane + 64 * i;
      acc[i] = 0.f;
      if (c < C0) {
        float a = bias[c];
#pragma unroll
        for (int k = 0; k < 48; ++k) a += xs[k] * ws[k * C0 + c];
        acc[i] = a;
        s += a;
      }
    }
    const float mean = wave_sum(s) / C0;
    float sq = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = lane + 64 * i;
      if (c < C0) { const float d = acc[i] - mean; sq += d * d; }
    }
    const float rstd = rsqrtf(wave_sum(sq) / C0 + 1e-6f);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = lane + 64 * i;
      if (c < C0) out[px * C0 + c] = from_f<T>((acc[i] - mean) * rstd * lw[c] + lb[c]);
    }
  }
}

// ---------------------------------------------------------------------------------------
// dwconv7 + LN.  Thread = 8 channels x PW consecutive output pixels of one row; the 7 input
// rows are walked with a PW+6 wide register window so each input vector is loaded 7x
// (once per kh) instead of 49x.  Threads of one output row cooperate on the LN through LDS.
template <typename T> struct V8;
template <> struct V8<bf16> {
  static DEV void load(const bf16* p, float (&v)[8]) {
    const bf16x8 x = *(const bf16x8*)p;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (float)x[j];
  }
  static DEV void store(bf16* p, const float (&v)[8]) {
    bf16x8 x;
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = (bf16)v[j];
    *(bf16x8*)p = x;
  }
};
template <> struct V8<float> {
  static DEV void load(const float* p, float (&v)[8]) {
    const f32x4 a = *(const f32x4*)p, b = *(const f32x4*)(p + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) { v[j] = a[j]; v[j + 4] = b[j]; }
  }
  static DEV void store(float* p, const float (&v)[8]) {
    *(f32x4*)p = f32x4{v[0], v[1], v[2], v[3]};
    *(f32x4*)(p + 4) = f32x4{v[4], v[5], v[6], v[7]};
  }
};

template <typename T, int PW>
__global__ __launch_bounds__(256) void dwconv7_ln_kernel(int B, int H, int W, int C, const T* __restrict__ x,
                                                         const float* __restrict__ w, const float* __restrict__ bias,
                                                         const float* __restrict__ lw, const float* __restrict__ lb,
                                                         T* __restrict__ out, int rows_per_block) {
  extern __shared__ __attribute__((aligned(16))) float red[];  // [rows_per_block * W][2], then part
  const int CV = C / 8, G = W / PW, tpr = CV * G;
  float* part = red + rows_per_block * W * 2;                    // [blockDim][PW]
  const int t = threadIdx.x;
  const int rl = t / tpr, within = t % tpr, g = within / CV, cv = within % CV;
  const long row = (long)blockIdx.x * rows_per_block + rl;  // (b*H + h)
  const bool active = rl < rows_per_block && row < (long)B * H;
  float acc[PW][8];
  const int c0 = cv * 8, w0 = g * PW;
  int b = 0, h = 0;
  if (active) {
    b = (int)(row / H);
    h = (int)(row % H);
#pragma unroll
    for (int p = 0; p < PW; ++p)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[p][j] = bias[c0 + j];
    for (int kh = 0; kh < 7; ++kh) {
      const int ih = h + kh - 3;
      if (ih < 0 || ih >= H) continue;
      const T* xr = x + (((long)b * H + ih) * W) * C + c0;
      float win[PW + 6][8];
#pragma unroll
      for (int q = 0; q < PW + 6; ++q) {
        const int iw = w0 + q - 3;
        if (iw >= 0 && iw < W) V8<T>::load(xr + (long)iw * C, win[q]);
        else {
#pragma unroll
          for (int j = 0; j < 8; ++j) win[q][j] = 0.f;
        }
      }
#pragma unroll
      for (int kw = 0; kw < 7; ++kw) {
        float wt[8];
        V8<float>::load(w + (kh * 7 + kw) * C + c0, wt);
#pragma unroll
        for (int p = 0; p < PW; ++p)
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[p][j] += win[p + kw][j] * wt[j];
      }
    }
    // per-thread partial sums (fixed-order reduction below keeps results deterministic)
#pragma unroll
    for (int p = 0; p < PW; ++p) {
      float sum = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) sum += acc[p][j];
      part[t * PW + p] = sum;
    }
  }
  __syncthreads();
  const int gbase = t - cv;  // first thread of this (row, pixel group)
  if (active && cv < PW) {
    float sum = 0.f;
    for (int c = 0; c < CV; ++c) sum += part[(gbase + c) * PW + cv];
    red[(rl * W + w0 + cv) * 2] = sum / C;
  }
  __syncthreads();
  float mean[PW];
  if (active) {
#pragma unroll
    for (int p = 0; p < PW; ++p) {
      mean[p] = red[(rl * W + w0 + p) * 2];
      float sq = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) { const float dd = acc[p][j] - mean[p]; sq += dd * dd; }
      part[t * PW + p] = sq;
    }
  }
  __syncthreads();
  if (active && cv < PW) {
    float sq = 0.f;
    for (int c = 0; c < CV; ++c) sq += part[(gbase + c) * PW + cv];
    red[(rl * W + w0 + cv) * 2 + 1] = sq;
  }
  __syncthreads();
  if (active) {
    float g8[8], b8[8];
    V8<float>::load(lw + c0, g8);
    V8<float>::load(lb + c0, b8);
#pragma unroll
    for (int p = 0; p < PW; ++p) {
      const float rstd = rsqrtf(red[(rl * W + w0 + p) * 2 + 1] / C + 1e-6f);
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (acc[p][j] - mean[p]) * rstd * g8[j] + b8[j];
      V8<T>::store(out + (((long)b * H + h) * W + w0 + p) * C + c0, o);
    }
  }
}

// ---------------------------------------------------------------------------------------
// LayerNorm2d + 2x2/s2 patch gather: one wave per input pixel.
template <typename T>
__global__ __launch_bounds__(256) void ln_patchify2_kernel(int B, int H, int W, int C, const T* __restrict__ x,
                                                           const float* __restrict__ lw, const float* __restrict__ lb,
                                                           T* __restrict__ out) {
  const long px = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (px >= (long)B * H * W) return;
  const int b = (int)(px / (H * W)), rem = (int)(px % (H * W)), ih = rem / W, iw = rem % W;
  constexpr int MAXV = 24;  // C <= 1536
  float v[MAXV];
  float s = 0.f;
  const T* xp = x + px * C;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = lane + 64 * i;
    v[i] = c < C ? to_f(xp[c]) : 0.f;
    s += v[i];
  }
  const float mean = wave_sum(s) / C;
  float sq = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = lane + 64 * i;
    if (c < C) { const float d = v[i] - mean; sq += d * d; }
  }
  const float rstd = rsqrtf(wave_sum(sq) / C + 1e-6f);
  const int HO = H / 2, WO = W / 2;
  const int oh = ih / 2, ow = iw / 2, kh = ih & 1, kw = iw & 1;
  T* op = out + (((long)b * HO + oh) * WO + ow) * (4L * C) + (kh * 2 + kw) * C;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = lane + 64 * i;
    if (c < C) op[c] = from_f<T>((v[i] - mean) * rstd * lw[c] + lb[c]);
  }
}

template <typename T>
__global__ void adaptive_pool_kernel(int B, int H, int W, int C, int OH, int OW, const T* __restrict__ x,
                                     T* __restrict__ out) {
  const long total = (long)B * OH * OW * C;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const int c = (int)(e % C);
    long r = e / C;
    const int ow = (int)(r % OW); r /= OW;
    const int oh = (int)(r % OH);
    const int b = (int)(r / OH);
    const int h0 = (oh * H) / OH, h1 = ((oh + 1) * H + OH - 1) / OH;
    const int w0 = (ow * W) / OW, w1 = ((ow + 1) * W + OW - 1) / OW;
    float s = 0.f;
    for (int i = h0; i < h1; ++i)
      for (int j = w0; j < w1; ++j) s += to_f(x[(((long)b * H + i) * W + j) * C + c]);
    out[e] = from_f<T>(s / ((h1 - h0) * (w1 - w0)));
  }
}

template <typename T, int PW>
static int launch_dw(int B, int H, int W, int C, const void* x, const float* w, const float* bias, const float* lw,
                     const float* lb, void* out, hipStream_t st) {
  const int tpr = (C / 8) * (W / PW);
  IMGCAP_REQUIRE(tpr <= 256, "imgcap_dwconv7_ln: C*W too large for one block");
  IMGCAP_REQUIRE(C / 8 >= PW, "imgcap_dwconv7_ln: C must be >= 8*pixels_per_thread");
  const int rpb = 256 / tpr;
  const int threads = ((rpb * tpr + 63) / 64) * 64;
  const long rows = (long)B * H;
  dim3 grid((unsigned)((rows + rpb - 1) / rpb));
  const size_t shm = ((size_t)rpb * W * 2 + (size_t)threads * PW) * sizeof(float);
  hipLaunchKernelGGL((dwconv7_ln_kernel<T, PW>), grid, dim3(threads), shm, st, B, H, W, C, (const T*)x, w, bias, lw,
                     lb, (T*)out, rpb);
  IMGCAP_CHECK_LAUNCH("imgcap_dwconv7_ln");
  return 0;
}

}  // namespace imgcap

using namespace imgcap;

extern "C" int imgcap_convnext_stem(int dtype, int B, int H, int W, int C0, const float* images, const float* w,
                                    const float* bias, const float* ln_w, const float* ln_b, void* out, void* stream) {
  IMGCAP_REQUIRE(H % 4 == 0 && W % 4 == 0 && C0 > 0 && C0 <= 256, "imgcap_convnext_stem: bad shape");
  const long npx = (long)B * (H / 4) * (W / 4);
  if (npx == 0) return 0;
  const int ppb = 32;
  dim3 grid((unsigned)((npx + ppb - 1) / ppb));
  const size_t shm = 48 * C0 * sizeof(float);
  if (dtype == IMGCAP_BF16)
    hipLaunchKernelGGL(stem_kernel<bf16>, grid, dim3(256), shm, (hipStream_t)stream, B, H, W, C0, images, w, bias,
                       ln_w, ln_b, (bf16*)out, ppb);
  else
    hipLaunchKernelGGL(stem_kernel<float>, grid, dim3(256), shm, (hipStream_t)stream, B, H, W, C0, images, w, bias,
                       ln_w, ln_b, (float*)out, ppb);
  IMGCAP_CHECK_LAUNCH("imgcap_convnext_stem");
  return 0;
}

extern "C" int imgcap_dwconv7_ln(int dtype, int B, int H, int W, int C, const void* x, const float* w,
                                 const float* bias, const float* ln_w, const float* ln_b, void* out, void* stream) {
  IMGCAP_REQUIRE(C % 8 == 0, "imgcap_dwconv7_ln: C must be a multiple of 8");
  IMGCAP_REQUIRE(aligned16(x) && aligned16(out) && aligned16(w) && aligned16(ln_w) && aligned16(ln_b),
                 "imgcap_dwconv7_ln: 16-byte alignment");
  IMGCAP_REQUIRE(x != out, "imgcap_dwconv7_ln: in-place not supported");
  if ((long)B * H * W == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == IMGCAP_BF16) {
    if (W % 7 == 0) return launch_dw<bf16, 7>(B, H, W, C, x, w, bias, ln_w, ln_b, out, st);
    if (W % 8 == 0) return launch_dw<bf16, 8>(B, H, W, C, x, w, bias, ln_w, ln_b, out, st);
    return launch_dw<bf16, 1>(B, H, W, C, x, w, bias, ln_w, ln_b, out, st);
  }
  if (W % 7 == 0) return launch_dw<float, 7>(B, H, W, C, x, w, bias, ln_w, ln_b, out, st);
  if (W % 8 == 0) return launch_dw<float, 8>(B, H, W, C, x, w, bias, ln_w, ln_b, out, st);
  return launch_dw<float, 1>(B, H, W, C, x, w, bias, ln_w, ln_b, out, st);
}

extern "C" int imgcap_ln_patchify2(int dtype, int B, int H, int W, int C, const void* x, const float* ln_w,
                                   const float* ln_b, void* out, void* stream) {
  IMGCAP_REQUIRE(H % 2 == 0 && W % 2 == 0 && C <= 1536, "imgcap_ln_patchify2: bad shape");
  const long npx = (long)B * H * W;
  if (npx == 0) return 0;
  dim3 grid((unsigned)((npx + 3) / 4));
  if (dtype == IMGCAP_BF16)
    hipLaunchKernelGGL(ln_patchify2_kernel<bf16>, grid, dim3(256), 0, (hipStream_t)stream, B, H, W, C,
                       (const bf16*)x, ln_w, ln_b, (bf16*)out);
  else
    hipLaunchKernelGGL(ln_patchify2_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream, B, H, W, C,
                       (const float*)x, ln_w, ln_b, (float*)out);
  IMGCAP_CHECK_LAUNCH("imgcap_ln_patchify2");
  return 0;
}

extern "C" int imgcap_adaptive_pool_nhwc(int dtype, int B, int H, int W, int C, int OH, int OW, const void* x,
                                         void* out, void* stream) {
  const long total = (long)B * OH * OW * C;
  if (total == 0) return 0;
  long blocks = (total + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (dtype == IMGCAP_BF16)
    hipLaunchKernelGGL(adaptive_pool_kernel<bf16>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, B, H, W,
                       C, OH, OW, (const bf16*)x, (bf16*)out);
  else
    hipLaunchKernelGGL(adaptive_pool_kernel<float>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, B, H,
                       W, C, OH, OW, (const float*)x, (float*)out);
  IMGCAP_CHECK_LAUNCH("imgcap_adaptive_pool_nhwc");
  return 0;
}

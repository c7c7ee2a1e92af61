// ConvNeXt trunk kernels, NHWC (torchvision ConvNeXt `features`, reached via encoder.py:24).
//   stem       features[0]: Conv2d(3,C0,4,s4,bias) + LayerNorm2d(eps 1e-6), NCHW f32 in
//   dwconv7_ln CNBlock head: depthwise 7x7 (pad 3, bias) + LayerNorm(C, eps 1e-6)
//   ln_patchify2  features[2,4,6] head: LayerNorm2d then 2x2/s2 patch rows for the MFMA GEMM
//   adaptive_pool AdaptiveAvgPool2d (encoder.py:20,25)
// The pointwise Linear pair / downsample conv run on imgcap_gemm (gemm.hip).
#include <type_traits>

#include <algorithm>

#include "common.h"

namespace imgcap {

// ---------------------------------------------------------------------------------------
// stem: block = NPX output pixels; their 4x4x3 patches and the [48][C0] weights are staged in
// LDS; thread = (pixel, 8 output channels): 48x8 MACs, then the per-pixel LayerNorm over C0
// is a fixed-order LDS reduction across the pixel's C0/8 threads.
// TI = uint8_t: raw 0..255 pixels (the reference's HDF5 images, dataLoader.py:43-46), turned into
// the reference's normalised input in the patch load: x = float(u / 255.) (double division, as
// numpy computes it), then (x - mean[c]) / std[c] in fp32 (torchvision Normalize).
template <typename TI> struct StemIn;
template <> struct StemIn<float> {
  static DEV f32x4 load(const float* p, int, const float*, const float*) { return *(const f32x4*)p; }
};
template <> struct StemIn<uint8_t> {
  static DEV f32x4 load(const uint8_t* p, int ci, const float* nmean, const float* nstd) {
    const uchar4 u = *(const uchar4*)p;
    const float m = nmean[ci], sd = nstd[ci];
    auto f = [&](unsigned char c) { return __fdiv_rn((float)((double)c / 255.0) - m, sd); };
    return f32x4{f(u.x), f(u.y), f(u.z), f(u.w)};
  }
};

// Block = npx output pixels (patches) x C0 channels; a thread computes 8 channels of TWO pixels
// (q and q + npx/2), so each weight vector it reads from LDS serves two patches (the kernel is
// LDS-issue bound: per k one patch value per pixel + two 16-byte weight reads).  Patch rows are
// padded to STEM_PS floats (16-byte rows; the pixels of a wave read distinct banks).  Per pixel
// the arithmetic is unchanged: bias, then k = 0..47 in order, LayerNorm sums over j then cv.
constexpr int STEM_PS = 52;
template <typename T, typename TI = float, int PX = 2>
__global__ __launch_bounds__(1024) void stem_kernel(int B, int H, int W, int C0, const TI* __restrict__ img,
                                                    const float* __restrict__ w, const float* __restrict__ bias,
                                                    const float* __restrict__ lw, const float* __restrict__ lb,
                                                    T* __restrict__ out, int npx, const float* __restrict__ nmean,
                                                    const float* __restrict__ nstd) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int CV = C0 / 8;
  float* ws = sm;                       // [48][C0]
  float* patch = ws + 48 * C0;          // [npx][STEM_PS]
  float* red = patch + npx * STEM_PS;   // [npx][CV]
  float* stat = red + npx * CV;         // [npx][2]
  const int HO = H / 4, WO = W / 4;
  const long total = (long)B * HO * WO;
  const long px0 = (long)blockIdx.x * npx;
  for (int e = threadIdx.x; e < 48 * C0; e += blockDim.x) {
    const int c = e / 48, k = e % 48;  // torch weight [C0][3][4][4] -> k = ci*16+kh*4+kw
    ws[k * C0 + c] = w[e];
  }
  for (int e = threadIdx.x; e < npx * 12; e += blockDim.x) {  // 12 float4 rows per patch
    const int q = e / 12, r = e % 12, ci = r / 4, kh = r % 4;
    const long px = px0 + q;
    f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
    if (px < total) {
      const int b = (int)(px / (HO * WO)), rem = (int)(px % (HO * WO)), oh = rem / WO, ow = rem % WO;
      v = StemIn<TI>::load(img + (((long)b * 3 + ci) * H + oh * 4 + kh) * W + ow * 4, ci, nmean, nstd);
    }
    *(f32x4*)(patch + q * STEM_PS + ci * 16 + kh * 4) = v;
  }
  __syncthreads();
  // PX patches per thread (q, q + npx/PX, ...), each weight vector read from LDS serving all PX;
  // the patch values come 4 k at a time (one ds_read_b128 per patch): with PX = 4 a thread reads
  // 48 / 4 * PX + 48 * 2 vectors for 48 * 8 * PX FMAs instead of 48 * 2 scalars + 48 * 2 vectors
  // for 48 * 16 (the kernel is LDS-issue bound)
  const int half = npx / PX;
  const int q = threadIdx.x / CV, cv = threadIdx.x % CV, c0 = cv * 8;
  int qp[PX];
  bool active[PX];
#pragma unroll
  for (int u = 0; u < PX; ++u) {
    qp[u] = q + u * half;
    active[u] = q < half && px0 + qp[u] < total;
  }
  float acc[PX][8];
#pragma unroll
  for (int u = 0; u < PX; ++u)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[u][j] = 0.f;
  if (q < half) {
    const f32x4 b0 = *(const f32x4*)(bias + c0), b1 = *(const f32x4*)(bias + c0 + 4);
#pragma unroll
    for (int u = 0; u < PX; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) { acc[u][j] = b0[j]; acc[u][j + 4] = b1[j]; }
#pragma unroll 2
    for (int k4 = 0; k4 < 48; k4 += 4) {
      f32x4 xp[PX];
#pragma unroll
      for (int u = 0; u < PX; ++u) xp[u] = *(const f32x4*)(patch + qp[u] * STEM_PS + k4);
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const int k = k4 + kk;
        const f32x4 w0 = *(const f32x4*)(ws + k * C0 + c0), w1 = *(const f32x4*)(ws + k * C0 + c0 + 4);
#pragma unroll
        for (int u = 0; u < PX; ++u)
#pragma unroll
          for (int j = 0; j < 4; ++j) { acc[u][j] += xp[u][kk] * w0[j]; acc[u][j + 4] += xp[u][kk] * w1[j]; }
      }
    }
#pragma unroll
    for (int u = 0; u < PX; ++u) {
      if (!active[u]) continue;
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) s += acc[u][j];
      red[qp[u] * CV + cv] = s;
    }
  }
  __syncthreads();
  if (cv == 0) {
#pragma unroll
    for (int u = 0; u < PX; ++u) {
      if (!active[u]) continue;
      float s = 0.f;
      for (int i = 0; i < CV; ++i) s += red[qp[u] * CV + i];
      stat[qp[u] * 2] = s / C0;
    }
  }
  __syncthreads();
  float mean[PX];
#pragma unroll
  for (int u = 0; u < PX; ++u) mean[u] = 0.f;
#pragma unroll
  for (int u = 0; u < PX; ++u) {
    if (!active[u]) continue;
    mean[u] = stat[qp[u] * 2];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) { const float d = acc[u][j] - mean[u]; s += d * d; }
    red[qp[u] * CV + cv] = s;
  }
  __syncthreads();
  if (cv == 0) {
#pragma unroll
    for (int u = 0; u < PX; ++u) {
      if (!active[u]) continue;
      float s = 0.f;
      for (int i = 0; i < CV; ++i) s += red[qp[u] * CV + i];
      stat[qp[u] * 2 + 1] = rsqrtf(s / C0 + 1e-6f);
    }
  }
  __syncthreads();
  if (q < half) {
    const f32x4 g0 = *(const f32x4*)(lw + c0), g1 = *(const f32x4*)(lw + c0 + 4);
    const f32x4 h0 = *(const f32x4*)(lb + c0), h1 = *(const f32x4*)(lb + c0 + 4);
#pragma unroll
    for (int u = 0; u < PX; ++u) {
      if (!active[u]) continue;
      const float rstd = stat[qp[u] * 2 + 1];
      float o[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        o[j] = (acc[u][j] - mean[u]) * rstd * g0[j] + h0[j];
        o[j + 4] = (acc[u][j + 4] - mean[u]) * rstd * g1[j] + h1[j];
      }
      T* op = out + (px0 + qp[u]) * C0 + c0;
      if (sizeof(T) == 2) {
        bf16x8 v;
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (bf16)o[j];
        *(bf16x8*)op = v;
      } else {
        *(f32x4*)op = f32x4{o[0], o[1], o[2], o[3]};
        *(f32x4*)(op + 4) = f32x4{o[4], o[5], o[6], o[7]};
      }
    }
  }
}

// patches per stem thread, pixels per stem block (a multiple of it) and its LDS bytes.  4 patches
// per thread where the channel count gives the block enough threads (tools/gpu/r6_stem.sh, µs at
// 224x224, outputs bitwise equal): C0 = 128 B = 32 56.7 -> 44.6, C0 = 192 B = 64 148 -> 130;
// C0 = 96 (Tiny) keeps 2: 35.3 vs 43.4 at B = 32, 64 vs 72 at B = 64.  IMGCAP_STEM_PX=2/4 overrides.
static int stem_px(int C0) {
  static const int v = [] {
    const char* e = getenv("IMGCAP_STEM_PX");
    return e ? atoi(e) : 0;
  }();
  if (v == 2 || v == 4) return v;
  return C0 >= 128 ? 4 : 2;
}
static int stem_npx(int C0, int px) {
  int npx = px * (1024 / (C0 / 8));
  if (npx > 128) npx = 128;
  return npx / px * px;
}
static size_t stem_lds(int C0, int npx) {
  return (48 * (size_t)C0 + (size_t)npx * STEM_PS + (size_t)npx * (C0 / 8) + (size_t)npx * 2) * sizeof(float);
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

// NC (4 or 8) consecutive channels <-> fp32 (depthwise kernel lanes)
template <typename T, int NC>
DEV void ldc(const T* p, float (&v)[NC]) {
  if constexpr (NC == 8) {
    V8<T>::load(p, v);
  } else if constexpr (sizeof(T) == 2) {
    const bf16x4 x = *(const bf16x4*)p;
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = (float)x[j];
  } else {
    const f32x4 a = *(const f32x4*)p;
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = a[j];
  }
}
template <typename T, int NC>
DEV void stc(T* p, const float (&v)[NC]) {
  if constexpr (NC == 8) {
    V8<T>::store(p, v);
  } else if constexpr (sizeof(T) == 2) {
    bf16x4 x;
#pragma unroll
    for (int j = 0; j < 4; ++j) x[j] = (bf16)v[j];
    *(bf16x4*)p = x;
  } else {
    *(f32x4*)p = f32x4{v[0], v[1], v[2], v[3]};
  }
}

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
// Depthwise 7x7 conv (+bias), no LayerNorm (the consumer normalises: the fused CNBlock MLP
// in its prologue, or add_layernorm for the two-GEMM stages).  Without the cross-channel LN
// the work tiles over channels: block = 4 waves = 32 channels (wave w: channels 8w..8w+7 of
// the tile, so its 49x8 weights are wave-uniform scalar loads) x TR output rows of the
// flattened [B*H] row sequence x the full width; lane = one row x PW consecutive pixels.
// The (TR+6) x (W+6) x 32 input patch (zero halo) is staged once into LDS with 16-byte
// coalesced loads; each lane then slides a PW+6 register window along its row for each of
// the 7 kernel rows (rows of another image than the lane's are skipped: image boundaries
// inside a tile).  fp32 accumulation, packed two channels per FMA.
// LDS layout: 16-byte slots; pixel px of patch row r at slot r*RS + 4*px + px/PW (one gap slot
// after every PW pixels), slot s of the pixel = its channels 8s..8s+7 (fp32: two slots per 8
// channels).  A wave reads slot wv of pixel g*PW + q across its lanes (row lr = lane / GW, group
// g = lane % GW); ds_read_b128 serves a wave in four 16-lane groups ({0-3,12-15,20-27},
// {4-11,16-19,28-31}, {32-35,44-47,52-59}, {36-43,48-51,60-63}; MI355X_MICROARCH.md §LDS), one
// cycle per group when its 16 lanes hit 16 distinct slots of the 256-byte bank row.  The row
// stride RS is searched (dw_row_slots) so that lr * RS + g * (4*PW + 1) is distinct mod 16
// within every group: RS = 8 (mod 16) at GW = 8, 4 at 4, 2 at 2, 1 at 1 for PW = 7 (round 2's
// 16/GW rule gave 2-way conflicts at GW = 8 and 16-way at GW = 1: 6.8 / 34 extra cycles per
// read in profiles/r02_C2_sq.json).
constexpr int DW_CT = 32;  // channels per block
constexpr int kDwGroups[4][16] = {{0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27},
                                  {4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31},
                                  {32, 33, 34, 35, 44, 45, 46, 47, 52, 53, 54, 55, 56, 57, 58, 59},
                                  {36, 37, 38, 39, 40, 41, 42, 43, 48, 49, 50, 51, 60, 61, 62, 63}};
// LDS row stride in 16-byte slots: the smallest >= the row's slots with the fewest bank
// collisions in any ds_read_b128 lane group of the window reads (see above)
__host__ __device__ constexpr int dw_row_slots(int W, int PW, int elem_bytes) {
  const int GW = W / PW;
  const int f = elem_bytes / 2;                       // slots per 8 channels (bf16 1, fp32 2)
  const int base = (4 * (W + 6) + (W + 5) / PW + 1) * f;
  const int gstep = (4 * PW + 1) * f;                 // slot distance between pixel groups
  int best = base, best_m = 1 << 30;
  for (int rs = base; rs < base + 16; ++rs) {
    int worst = 0;
    for (int grp = 0; grp < 4; ++grp) {
      int cnt[16] = {0};
      for (int i = 0; i < 16; ++i) {
        const int l = kDwGroups[grp][i];
        const int sl = ((l / GW) * rs + (l % GW) * gstep) % 16;
        const int c = ++cnt[sl];
        worst = c > worst ? c : worst;
      }
    }
    if (worst < best_m) {
      best_m = worst;
      best = rs;
    }
    if (worst == 1) break;
  }
  return best;
}
// WC: the image width as a compile-time constant (0: runtime W) -- the staging index math
// (patch row / column of each 16-byte load) then folds to multiplies by constants, which at
// the encoder's widths removes about a third of the kernel's vector instructions.
template <typename T, int PW, int WC, int NC>
__global__ __launch_bounds__(64 * DW_CT / NC) void dwconv7_kernel(int B, int H, int W_, int C, const T* __restrict__ x,
                                                      const float* __restrict__ w, const float* __restrict__ bias,
                                                      T* __restrict__ y, int TR_, int RS_,
                                                      const T* res, int flip) {
  extern __shared__ __attribute__((aligned(16))) char dsm[];
  constexpr int VE = 16 / sizeof(T);   // elements per 16-byte vector
  constexpr int NV = DW_CT / VE;       // 16-byte vectors per pixel in the tile (4 bf16, 8 f32)
  constexpr int SPP = DW_CT * 2 / 16;  // 16-byte slots per pixel in the LDS image: bf16 layout
  static_assert(sizeof(T) == 2 || sizeof(T) == 4, "dtype");
  constexpr int NT = 64 * DW_CT / NC;  // threads: one wave per NC channels of the tile
  static_assert(NT % NV == 0, "vector index must be constant per thread");
  const int W = WC ? WC : W_;
  const int TR = WC ? 64 / (WC / PW) : TR_;
  const int RS = WC ? dw_row_slots(WC, PW, (int)sizeof(T)) : RS_;
  const int WP = W + 6;                // padded row width (pixels)
  const long R = (long)B * H;
  const long r0 = (long)blockIdx.x * TR;
  const int cb = blockIdx.y * DW_CT;
  uint4* img = (uint4*)dsm;
  // slot of (patch row r, padded pixel px, 16-byte part s); fp32 pixels use 2x the slots
  auto slot = [&](int r, int px, int s) { return r * RS + (SPP * px + px / PW) * (NV / SPP) + s; };
  // ---- stage the input patch (rows r0-3 .. r0+TR+2 of the flattened sequence) ----
  // batches of 8 loads per thread in flight (clamped address + zero select, no branches around
  // the loads), then their LDS stores: a couple of memory round trips per block.  Load i of the
  // block is (pixel i / NV, vector i % NV); the vector index is the same for all of a thread's
  // loads (256 % NV == 0) and its pixel advances by 256 / NV per load.
  const int npx = (TR + 6) * WP;
  constexpr int BATCH = 8;
  constexpr int PSTEP = NT / NV;
  const int v = threadIdx.x % NV;
  // buffer loads: the zero halo (and the batch tail) comes from the descriptor's range check
  // (an offset past the tensor reads 0), so the loads need no branches or selects
  const auto xr = __builtin_amdgcn_make_buffer_rsrc((void*)x, 0, (int)(R * W * C * (long)sizeof(T)), 0x00020000);
  for (int p0 = threadIdx.x / NV; p0 < npx; p0 += PSTEP * BATCH) {
    uint4 val[BATCH];
#pragma unroll
    for (int u = 0; u < BATCH; ++u) {
      const int px = p0 + u * PSTEP;
      const int pc = px % WP, pr = px / WP;
      const long gr = r0 - 3 + pr;
      const int gw = pc - 3;
      const bool ok = px < npx && gr >= 0 && gr < R && gw >= 0 && gw < W;
      const uint32_t off = ok ? (uint32_t)((((gr * W) + gw) * C + cb + v * VE) * (long)sizeof(T)) : 0x80000000u;
      val[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
    }
#pragma unroll
    for (int u = 0; u < BATCH; ++u) {
      const int px = p0 + u * PSTEP;
      if (px < npx) img[slot(px / WP, px % WP, v)] = val[u];
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c0 = cb + wv * NC;     // this wave's NC channels
  const int GW = W / PW;           // pixel groups per row
  const int lr = lane / GW, g = lane % GW;
  const long orow = r0 + lr;
  if (lr >= TR || orow >= R) return;
  const int h = (int)(orow % H);
  const int w0 = g * PW;
  constexpr int NP = NC / 2;       // channel pairs per lane (packed fp32 FMAs)
  f32x2 acc[PW][NP];
  {
    float b[NC];
#pragma unroll
    for (int j = 0; j < NC; ++j) b[j] = 0.f;
    if (bias) ldc<float, NC>(bias + c0, b);
#pragma unroll
    for (int p = 0; p < PW; ++p)
#pragma unroll
      for (int j = 0; j < NP; ++j) acc[p][j] = f32x2{b[2 * j], b[2 * j + 1]};
  }
  // byte offset of this wave's channels inside a pixel's LDS slots
  const int cofs = wv * NC * (int)sizeof(T);
  const char* imgb = (const char*)img;
  for (int kh = 0; kh < 7; ++kh) {
    const int ih = h + kh - 3;
    // the 7 taps of this kernel row for the wave's channels: wave-uniform, loaded in one batch
    // (scalar loads) ahead of the window, so the taps cost one load round trip per row
    f32x2 wt[7][NP];
#pragma unroll
    for (int kw = 0; kw < 7; ++kw) {
      // flip: the transposed convolution of the backward pass (tap (kh,kw) -> (6-kh,6-kw))
      float t[NC];
      ldc<float, NC>(w + (flip ? 48 - (kh * 7 + kw) : kh * 7 + kw) * C + c0, t);
#pragma unroll
      for (int j = 0; j < NP; ++j) wt[kw][j] = f32x2{t[2 * j], t[2 * j + 1]};
    }
    if (ih < 0 || ih >= H) continue;  // outside this lane's image (zero padding)
    f32x2 win[PW + 6][NP];
#pragma unroll
    for (int q = 0; q < PW + 6; ++q) {
      float v[NC];
      ldc<T, NC>((const T*)(imgb + slot(lr + kh, w0 + q, 0) * 16 + cofs), v);
#pragma unroll
      for (int j = 0; j < NP; ++j) win[q][j] = f32x2{v[2 * j], v[2 * j + 1]};
    }
#pragma unroll
    for (int kw = 0; kw < 7; ++kw)
#pragma unroll
      for (int p = 0; p < PW; ++p)
#pragma unroll
        for (int j = 0; j < NP; ++j) acc[p][j] = win[p + kw][j] * wt[kw][j] + acc[p][j];
  }
  T* out = y + (orow * W + w0) * C + c0;
#pragma unroll
  for (int p = 0; p < PW; ++p) {
    float o[NC];
#pragma unroll
    for (int j = 0; j < NP; ++j) { o[2 * j] = acc[p][j][0]; o[2 * j + 1] = acc[p][j][1]; }
    if (res) {
      float r[NC];
      ldc<T, NC>(res + (orow * W + w0 + p) * C + c0, r);
#pragma unroll
      for (int j = 0; j < NC; ++j) o[j] += r[j];
    }
    stc<T, NC>(out + (long)p * C, o);
  }
}

// Row stride (16-byte slots) of the rolling kernel's image: pixel px at slot sppx*px + px/PW of
// its row (one gap slot after every PW pixels), sppx = 16-byte slots per pixel (DW_CT channels
// of the LDS element type); searched like dw_row_slots for conflict-free window reads.
__host__ __device__ constexpr int dw_roll_row_slots(int W, int PW, int sppx) {
  const int GW = W / PW;
  const int base = sppx * (W + 6) + (W + 5) / PW + 1;
  const int gstep = sppx * PW + 1;
  int best = base, best_m = 1 << 30;
  for (int rs = base; rs < base + 16; ++rs) {
    int worst = 0;
    for (int grp = 0; grp < 4; ++grp) {
      int cnt[16] = {0};
      for (int i = 0; i < 16; ++i) {
        const int l = kDwGroups[grp][i];
        const int c = ++cnt[((l / GW) * rs + (l % GW) * gstep) % 16];
        worst = c > worst ? c : worst;
      }
    }
    if (worst < best_m) {
      best_m = worst;
      best = rs;
    }
    if (worst == 1) break;
  }
  return best;
}

// ---------------------------------------------------------------------------------------
// The same depthwise conv with a compile-time width (the encoder's 56 / 28 / 14 / 7, and 64 / 32
// / 16 / 8): one tile of TR output rows per block, its TR + 6 input rows staged in LDS through
// buffer loads whose range check supplies the zero halo.  Variants measured and removed (round 3,
// tools/microbench.py dw): 2-4 row tiles per block with a ring (halo fetched once; one block per
// CU, 1.2-3x slower) and bf16 staged as fp32 (1.2x slower).
template <typename T, int PW, int WC, int NC>
__global__ __launch_bounds__(64 * DW_CT / NC) void dwconv7_roll_kernel(int B, int H, int C, const T* __restrict__ x,
                                                           const float* __restrict__ w,
                                                           const float* __restrict__ bias, T* __restrict__ y,
                                                           const T* res, int flip) {
  extern __shared__ __attribute__((aligned(16))) char dsm[];
  static_assert(WC > 0, "compile-time width");
  using LT = T;  // LDS element type
  constexpr int VE = 16 / sizeof(T);
  constexpr int NV = DW_CT / VE;
  constexpr int SPPX = DW_CT * (int)sizeof(LT) / 16;  // 16-byte slots per pixel
  constexpr int NT = 64 * DW_CT / NC;
  constexpr int W = WC, GW = W / PW, TR = 64 / GW, WP = W + 6;
  constexpr int RS = dw_roll_row_slots(WC, PW, SPPX);
  constexpr int RING = TR + 6;
  constexpr int PSTEP = NT / NV;                      // pixels per load instruction of the block
  constexpr int NPF = (TR * WP + PSTEP - 1) / PSTEP;  // loads per thread for TR new rows
  const long R = (long)B * H;
  // 1-D grid of (row tile, channel block) slots laid out XCD-contiguously: XCD x = b % 8 runs
  // slots x*q + min(x, r) + 0, 1, ... in dispatch order, so the C / DW_CT channel blocks of one
  // row tile run back to back on one XCD and share its L2 lines (a 32-channel bf16 chunk is half
  // a 128-byte line; with the channel block as blockIdx.y the other half was fetched again
  // ~1/3 of the launch later, through another XCD's L2: 170 MB per C3 stage-1 launch against 77)
  const int ncb = C / DW_CT;
  const int gsz = gridDim.x, b8 = blockIdx.x % 8, g8q = gsz / 8, g8r = gsz % 8;
  const int gslot = b8 * g8q + min(b8, g8r) + blockIdx.x / 8;
  const long rb = (long)(gslot / ncb) * TR;           // the block's first output row
  const int cb = (gslot % ncb) * DW_CT;
  uint4* img = (uint4*)dsm;
  auto slot = [&](int rr, int px, int s) { return rr * RS + SPPX * px + px / PW + s; };
  constexpr int SPV = VE * (int)sizeof(LT) / 16;  // LDS slots per loaded 16-byte vector (1 or 2)
  const int v = threadIdx.x % NV;
  const int p0 = threadIdx.x / NV;
  const auto xr = __builtin_amdgcn_make_buffer_rsrc((void*)x, 0, (int)(R * W * C * (long)sizeof(T)), 0x00020000);
  // TR input rows from relative row i0 (relative row i = global row rb - 3 + i) into registers;
  // the zero halo and rows outside [0, R) come from the descriptor's range check
  auto load_rows = [&](int i0, int nrows, uint4 (&val)[NPF]) {
#pragma unroll
    for (int u = 0; u < NPF; ++u) {
      const int px = p0 + u * PSTEP;
      const int pr = px / WP, pc = px % WP;
      const long gr = rb - 3 + i0 + pr;
      const int gw = pc - 3;
      const bool ok = pr < nrows && gr >= 0 && gr < R && gw >= 0 && gw < W;
      const uint32_t off = ok ? (uint32_t)((((gr * W) + gw) * C + cb + v * VE) * (long)sizeof(T)) : 0x80000000u;
      val[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
    }
  };
  auto store_rows = [&](int i0, int nrows, const uint4 (&val)[NPF]) {
#pragma unroll
    for (int u = 0; u < NPF; ++u) {
      const int px = p0 + u * PSTEP;
      const int pr = px / WP;
      if (pr < nrows) {
        uint4* d = img + slot((i0 + pr) % RING, px % WP, v * SPV);
        if constexpr (SPV == 1) {
          d[0] = val[u];
        } else {  // 8 bf16 -> 8 fp32
          const uint32_t q[4] = {val[u].x, val[u].y, val[u].z, val[u].w};
          d[0] = make_uint4(q[0] << 16, q[0] & 0xFFFF0000u, q[1] << 16, q[1] & 0xFFFF0000u);
          d[1] = make_uint4(q[2] << 16, q[2] & 0xFFFF0000u, q[3] << 16, q[3] & 0xFFFF0000u);
        }
      }
    }
  };
  {  // prologue: the TR + 6 rows of tile 0
    uint4 a[NPF], b[NPF];
    load_rows(0, TR, a);
    load_rows(TR, 6, b);
    store_rows(0, TR, a);
    store_rows(TR, 6, b);
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c0 = cb + wv * NC;
  const int lr = lane / GW, g = lane % GW;
  const int w0 = g * PW;
  constexpr int NP = NC / 2;
  const int cofs = wv * NC * (int)sizeof(LT);
  const char* imgb = (const char*)img;
  float bv[NC];
#pragma unroll
  for (int j = 0; j < NC; ++j) bv[j] = 0.f;
  if (bias) ldc<float, NC>(bias + c0, bv);
  {
    constexpr int k = 0;
    const long orow = rb + lr;
    if (orow < R) {
      const int h = (int)(orow % H);
      f32x2 acc[PW][NP];
#pragma unroll
      for (int p = 0; p < PW; ++p)
#pragma unroll
        for (int j = 0; j < NP; ++j) acc[p][j] = f32x2{bv[2 * j], bv[2 * j + 1]};
      for (int kh = 0; kh < 7; ++kh) {
        const int ih = h + kh - 3;
        f32x2 wt[7][NP];
#pragma unroll
        for (int kw = 0; kw < 7; ++kw) {
          float t[NC];
          ldc<float, NC>(w + (flip ? 48 - (kh * 7 + kw) : kh * 7 + kw) * C + c0, t);
#pragma unroll
          for (int j = 0; j < NP; ++j) wt[kw][j] = f32x2{t[2 * j], t[2 * j + 1]};
        }
        if (ih < 0 || ih >= H) continue;  // outside this lane's image (zero padding)
        const int rr = (k * TR + lr + kh) % RING;
        f32x2 win[PW + 6][NP];
#pragma unroll
        for (int q = 0; q < PW + 6; ++q) {
          float vv[NC];
          ldc<LT, NC>((const LT*)(imgb + slot(rr, w0 + q, 0) * 16 + cofs), vv);
#pragma unroll
          for (int j = 0; j < NP; ++j) win[q][j] = f32x2{vv[2 * j], vv[2 * j + 1]};
        }
#pragma unroll
        for (int kw = 0; kw < 7; ++kw)
#pragma unroll
          for (int p = 0; p < PW; ++p)
#pragma unroll
            for (int j = 0; j < NP; ++j) acc[p][j] = win[p + kw][j] * wt[kw][j] + acc[p][j];
      }
      T* out = y + (orow * W + w0) * C + c0;
#pragma unroll
      for (int p = 0; p < PW; ++p) {
        float o[NC];
#pragma unroll
        for (int j = 0; j < NP; ++j) { o[2 * j] = acc[p][j][0]; o[2 * j + 1] = acc[p][j][1]; }
        if (res) {
          float r[NC];
          ldc<T, NC>(res + (orow * W + w0 + p) * C + c0, r);
#pragma unroll
          for (int j = 0; j < NC; ++j) o[j] += r[j];
        }
        stc<T, NC>(out + (long)p * C, o);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// LayerNorm2d + 2x2/s2 patch gather: one wave per input pixel.
template <typename T>
__global__ __launch_bounds__(256) void ln_patchify2_kernel(int B, int H, int W, int C, const T* __restrict__ x,
                                                           const float* __restrict__ lw, const float* __restrict__ lb,
                                                           T* __restrict__ out, int cmajor) {
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
  // patch row layout: (kh, kw, c) for the repacked frozen weights, or (c, kh, kw) = the torch
  // Conv2d weight layout [2C][C][2][2] used directly when the downsample is trainable
  T* op = out + (((long)b * HO + oh) * WO + ow) * (4L * C) + (cmajor ? kh * 2 + kw : (kh * 2 + kw) * C);
  const int cs = cmajor ? 4 : 1;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = lane + 64 * i;
    if (c < C) op[c * cs] = from_f<T>((v[i] - mean) * rstd * lw[c] + lb[c]);
  }
}

// The same, one 2x2 input patch per V = C / 8 threads: thread = 8 channels of the patch's four
// pixels (16-byte loads; the patch row leaves as 16-byte stores in either layout -- c-major: the
// thread's 8 channels x (kh, kw) are 32 consecutive elements).  The per-pixel mean / variance
// (two passes, as torch) are reduced through LDS: each thread's 8-channel partials, then one
// thread per (patch, pixel) sums the patch's V partials in channel order.  The wave-per-pixel
// form above moved 2-byte elements (one pixel of C = 96 is 1.5 loads per lane) and measured
// 47 us per call at C3 stage 1 -> 2 (77 MB, 1.6 TB/s).
constexpr int LNP_MAXPB = 32;
template <typename T>
__global__ __launch_bounds__(256) void ln_patchify2v_kernel(int B, int H, int W, int C, const T* __restrict__ x,
                                                            const float* __restrict__ lw, const float* __restrict__ lb,
                                                            T* __restrict__ out, int cmajor, int PB) {
  __shared__ float part[256 * 4];            // [thread][pixel] partial sums
  __shared__ float stat[LNP_MAXPB][4][2];    // [patch][pixel] mean, rstd
  const int V = C >> 3;
  const int tid = threadIdx.x, lp = tid / V, v = tid - lp * V;
  const int HO = H >> 1, WO = W >> 1;
  const long np = (long)B * HO * WO;
  const long patch = (long)blockIdx.x * PB + lp;
  const bool on = lp < PB && patch < np;
  float val[4][8];
  if (on) {
    const int b = (int)(patch / (HO * WO)), rem = (int)(patch % (HO * WO));
    const int oh = rem / WO, ow = rem % WO;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const long px = ((long)b * H + 2 * oh + (k >> 1)) * W + 2 * ow + (k & 1);
      ldc<T, 8>(x + px * C + 8 * v, val[k]);
    }
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) val[k][j] = 0.f;
  }
  const float inv_c = 1.f / (float)C;
  float mean[4] = {0.f, 0.f, 0.f, 0.f}, rstd[4] = {1.f, 1.f, 1.f, 1.f};
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = pass == 0 ? val[k][j] : val[k][j] - mean[k];
        s += pass == 0 ? d : d * d;
      }
      part[tid * 4 + k] = s;
    }
    __syncthreads();
    if (lp < PB && v < 4) {  // thread (patch, k = v) reduces pixel k of its patch
      float s = 0.f;
      for (int q = 0; q < V; ++q) s += part[(lp * V + q) * 4 + v];
      stat[lp][v][pass] = pass == 0 ? s * inv_c : rsqrtf(s * inv_c + 1e-6f);
    }
    __syncthreads();
    if (lp < PB) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (pass == 0) mean[k] = stat[lp][k][0];
        else rstd[k] = stat[lp][k][1];
      }
    }
  }
  if (!on) return;
  float g[8], bb[8];
  ldc<float, 8>(lw + 8 * v, g);
  ldc<float, 8>(lb + 8 * v, bb);
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) val[k][j] = (val[k][j] - mean[k]) * rstd[k] * g[j] + bb[j];
  T* op = out + patch * 4L * C;
  if (cmajor) {  // (c, kh, kw): channel 8v + j, pixel k at 32 v + 4 j + k
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = val[e & 3][2 * h + (e >> 2)];
      stc<T, 8>(op + 32 * v + 8 * h, o);
    }
  } else {       // (kh, kw, c)
#pragma unroll
    for (int k = 0; k < 4; ++k) stc<T, 8>(op + (long)k * C + 8 * v, val[k]);
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

__global__ void sd_scales_kernel(int n, int B, const float* __restrict__ probs, uint64_t seed0,
                                 const uint64_t* seed_ctr, uint32_t sid, float* __restrict__ out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  out[i] = dropout_scale(eff_seed(seed0, seed_ctr), sid, (uint64_t)i, probs[i / B]);
}

}  // namespace imgcap

using namespace imgcap;

namespace {
// the rolling kernel's staged rows can exceed the default 64 KB of dynamic LDS: raise the limit
// once per instantiation (first launch, before any capture)
template <typename T, int P, int WC>
void dw_roll_attr() {
  static const bool done = [] {
    (void)hipFuncSetAttribute((const void*)dwconv7_roll_kernel<T, P, WC, 8>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    return true;
  }();
  (void)done;
}

// ---------------------------------------------------------------------------------------
// Depthwise 7x7 for the narrow late stages (W = 14 / 7: stages 3-4), bf16, C % 128 == 0: lane =
// (channel pair, output image row), block = one output row x all C channels (wave g: channels
// 128g .. 128g + 127).  The channel-tiled kernels above stage a patch in LDS and give each lane
// 7 pixels x 8 channels; at these widths their grids are < 1 wave per SIMD and every window value
// is re-unpacked per kernel row (≈ 1.1 VALU per MAC).  Here a lane keeps its channel pair's 49
// weight pairs in registers for the whole row, reads each of the 7 input rows once as coalesced
// 4-byte bf16 pairs (64 lanes = 256 contiguous bytes, the next row requested before the current
// one is used), unpacks it once and applies all 7 taps of that kernel row with packed FMAs
// (≈ 0.7 VALU per MAC), and the grid is B*H rows x C/128 waves.  flip / res: the backward data gradient (taps mirrored, residual added), as dwconv7_kernel.
template <int W, bool LN, int R>
__global__ __launch_bounds__(512) void dwconv7_cp_kernel(int H, int C, const bf16* __restrict__ x,
                                                         const float* __restrict__ w, const float* __restrict__ bias,
                                                         const float* __restrict__ lnw, const float* __restrict__ lnb,
                                                         bf16* __restrict__ y, const bf16* __restrict__ res, int flip) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int HB = (H + R - 1) / R;  // R output rows per block (R = 2: each weight row loaded once for both)
  // (row block, channel group) slots XCD-contiguous: the blocks an XCD runs in dispatch order
  // are consecutive rows, so the 6 input rows two neighbours share come from that XCD's L2 (with
  // row blocks dealt round-robin over the 8 XCDs every input row was fetched ~6 times: 57 MB per
  // C3 stage-3 launch for a 9.6 MB input)
  const int gy = gridDim.y, gsz = gridDim.x * gy;
  const int lin = blockIdx.x + blockIdx.y * gridDim.x, b8 = lin % 8;
  const int gslot = b8 * (gsz / 8) + min(b8, gsz % 8) + lin / 8;
  const long r = gslot / gy;       // b * HB + row block
  const int h = (int)(r % HB) * R;
  const long b = r / HB;
  const int c = ((gslot % gy) * (blockDim.x >> 6) + wv) * 128 + 2 * lane;
  // the 7 weight pairs of kernel row kh (requested with that row's input, one row ahead)
  // buffer loads: per-lane byte offset in a VGPR, the wave-uniform pixel / tap offset in an SGPR
  // (64-bit addresses per load cost two VGPRs each and spilled); rows outside the image read 0
  // through the descriptor's range check
  const auto wr = __builtin_amdgcn_make_buffer_rsrc((void*)w, 0, 49 * C * 4, 0x00020000);
  const auto xr = __builtin_amdgcn_make_buffer_rsrc((void*)x, 0, (int)((b + 1) * H * W * (long)C * 2), 0x00020000);
  auto load_w = [&](int kh, f32x2 (&dst)[7]) {
#pragma unroll
    for (int kw = 0; kw < 7; ++kw) {
      const int t = kh * 7 + kw;
      const auto v = __builtin_amdgcn_raw_buffer_load_b64(wr, c * 4, (flip ? 48 - t : t) * C * 4, 0);
      dst[kw] = __builtin_bit_cast(f32x2, v);
    }
  };
  f32x2 acc[R][W];
  {
    const f32x2 bb = bias ? *(const f32x2*)(bias + c) : f32x2{0.f, 0.f};
#pragma unroll
    for (int rr = 0; rr < R; ++rr)
#pragma unroll
      for (int p = 0; p < W; ++p) acc[rr][p] = bb;
  }
  // input row h + i - 3
  auto load_row = [&](int i, uint32_t (&dst)[W]) {
    const int ih = h + i - 3;
    const bool ok = ih >= 0 && ih < H;
    const uint32_t vo = ok ? (uint32_t)(((b * H + ih) * W * (long)C + c) * 2) : 0x80000000u;
#pragma unroll
    for (int iw = 0; iw < W; ++iw) dst[iw] = __builtin_amdgcn_raw_buffer_load_b32(xr, vo, iw * C * 2, 0);
  };
  auto unpack = [&](const uint32_t (&src)[W], f32x2 (&xin)[W]) {
#pragma unroll
    for (int iw = 0; iw < W; ++iw)
      xin[iw] = f32x2{__uint_as_float(src[iw] << 16), __uint_as_float(src[iw] & 0xFFFF0000u)};
  };
  auto row_fma = [&](f32x2 (&a)[W], const f32x2 (&xin)[W], const f32x2 (&wk)[7]) {
#pragma unroll
    for (int kw = 0; kw < 7; ++kw)
#pragma unroll
      for (int p = 0; p < W; ++p) {
        const int q = p + kw - 3;
        if (q >= 0 && q < W) a[p] = xin[q] * wk[kw] + a[p];
      }
  };
  // rolled loops, one row of loads ahead: fully unrolled, the compiler hoisted later rows' loads
  // to the top (200-255 VGPRs, two waves per SIMD)
  if constexpr (R == 1) {
    uint32_t rb[2][W];
    f32x2 wb[2][7], xin[W];
    load_row(0, rb[0]);
    load_w(0, wb[0]);
#pragma unroll 1
    for (int kh = 0; kh < 6; kh += 2) {
      load_row(kh + 1, rb[1]);
      load_w(kh + 1, wb[1]);
      unpack(rb[0], xin);
      row_fma(acc[0], xin, wb[0]);
      load_row(kh + 2, rb[0]);
      load_w(kh + 2, wb[0]);
      unpack(rb[1], xin);
      row_fma(acc[0], xin, wb[1]);
    }
    unpack(rb[0], xin);
    row_fma(acc[0], xin, wb[0]);
  } else {
    static_assert(R == 2, "one or two output rows per block");
    // input row i feeds output row h with kernel row i and row h + 1 with kernel row i - 1
    uint32_t rc[W], rn[W];
    f32x2 wp[7], wc[7], wn[7], xin[W];
    load_row(0, rc);
    load_w(0, wc);
#pragma unroll 1
    for (int i = 0; i < 8; ++i) {
      if (i < 7) load_row(i + 1, rn);
      if (i < 6) load_w(i + 1, wn);
      unpack(rc, xin);
      if (i < 7) row_fma(acc[0], xin, wc);
      if (i > 0) row_fma(acc[1], xin, wp);
#pragma unroll
      for (int k = 0; k < 7; ++k) {
        wp[k] = wc[k];
        wc[k] = wn[k];
      }
#pragma unroll
      for (int k = 0; k < W; ++k) rc[k] = rn[k];
    }
  }
  const long o0 = (b * H + h) * W * (long)C + c;  // output row h, channel pair c
  if constexpr (LN) {
    // LayerNorm over C of each output pixel (eps 1e-6), two passes, fixed order: the lanes'
    // partials go to LDS [wave][pixel][lane]; wave g reduces pixels g, g + nwv, .. (its lanes sum
    // the waves' partials of one lane column, then a wave sum), the block reads the results back
    constexpr int NP = R * W;
    __shared__ float part[8][NP][64];
    __shared__ float stat[2][NP];
    const int nwv = blockDim.x >> 6;
    float mean[NP];
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        const f32x2 a = acc[p / W][p % W];
        float v;
        if (pass == 0) {
          v = a[0] + a[1];
        } else {
          const float d0 = a[0] - mean[p], d1 = a[1] - mean[p];
          v = d0 * d0 + d1 * d1;
        }
        part[wv][p][lane] = v;
      }
      __syncthreads();
      for (int p = wv; p < NP; p += nwv) {
        float v = 0.f;
        for (int g = 0; g < nwv; ++g) v += part[g][p][lane];
        v = wave_sum(v);
        if (lane == 0) stat[pass][p] = v / C;
      }
      __syncthreads();
      if (pass == 0) {
#pragma unroll
        for (int p = 0; p < NP; ++p) mean[p] = stat[0][p];
      }
    }
    const f32x2 g2 = *(const f32x2*)(lnw + c), b2 = *(const f32x2*)(lnb + c);
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      if (p >= W && h + 1 >= H) break;  // odd H: the last block's second row is outside the image
      const f32x2 a = acc[p / W][p % W];
      const float rstd = rsqrtf(stat[1][p] + 1e-6f);
      const float v0 = (a[0] - mean[p]) * rstd * g2[0] + b2[0], v1 = (a[1] - mean[p]) * rstd * g2[1] + b2[1];
      *(bf16x2*)(y + o0 + (long)p * C) = bf16x2{(bf16)v0, (bf16)v1};
    }
  } else {
#pragma unroll
    for (int p = 0; p < R * W; ++p) {
      if (p >= W && h + 1 >= H) break;
      f32x2 o = acc[p / W][p % W];
      if (res) {
        const uint32_t v = *(const uint32_t*)(res + o0 + (long)p * C);
        o += f32x2{__uint_as_float(v << 16), __uint_as_float(v & 0xFFFF0000u)};
      }
      *(bf16x2*)(y + o0 + (long)p * C) = bf16x2{(bf16)o[0], (bf16)o[1]};
    }
  }
}

bool dw_cp_enabled() {  // IMGCAP_DW_CP=0: the channel-tiled kernels at W = 14 / 7 too (A/B)
  const char* e = getenv("IMGCAP_DW_CP");
  return !(e && *e == '0');
}
// Measured (tools/dw_ln_bench.py, us, vs the channel-tiled kernel): Tiny stage 3 B32 9.0 vs 12.4,
// B64 13.4 vs 17.2; Base stage 3 B32 9.9 vs 13.1; Tiny stage 4 B64 8.9 vs 12.6; Base stage 4 B32
// 8.9 vs 12.5; Large stage 3 B64 (W 14, C 768) 19.3 vs 30.0 (two rows per block, 2-wave channel
// groups; 6-wave blocks with the kernel rows unrolled ran 33.2 vs 30.6: 255 VGPRs, one block per CU).
// LN (imgcap_dwconv7_ln): the LayerNorm in the epilogue (a first form with 2 x W wave sums per
// lane measured 1.1-2.4x slower than this kernel + add_layernorm; the LDS form above reduces each
// pixel once per block).
// C <= 1024 with the LayerNorm (one block holds every channel of a pixel: at most 8 waves);
// without it any C % 128 == 0 (channel-group blocks), e.g. ConvNeXt-Large stage 4, C = 1536
bool dw_cp_fits(int W, int C, bool ln) {
  return dw_cp_enabled() && (W == 7 || W == 14) && C % 128 == 0 && (!ln || C <= 1024);
}

// Output rows per block.  Measured (tools/dw_ln_bench.py, us, one vs two rows): without LN Large
// stage 3 B64 23.7 vs 19.3, B32 14.6 vs 12.9, Tiny stage 4 B64 9.5 vs 8.9, C <= 512 equal; with LN
// Large stage 3 B64 40.5 vs 35.4, Tiny stage 3 B32 14.6 vs 18.5, Base stage 3 15.0 vs 17.2, Base
// stage 4 9.1 vs 10.9 (the LN pass over 2W pixels).  IMGCAP_DW_CP_R=1/2 overrides (A/B).
int dw_cp_rows(int W, int C, bool ln) {
  const char* e = getenv("IMGCAP_DW_CP_R");
  if (e && *e) return *e == '2' ? 2 : 1;
  return C >= 768 && (W == 14 || !ln) ? 2 : 1;
}

int dwconv7_cp_launch(int B, int H, int W, int C, const void* x, const float* w, const float* bias, const float* lnw,
                      const float* lnb, void* y, const void* res, int flip, hipStream_t st) {
  // the LayerNorm form needs every channel of a pixel in one block; without it a block takes 4, 2
  // or 1 waves of 128 channels (blockIdx.y: channel group) so blocks pack a CU's wave slots
  const int nw = C / 128, wpb = lnw ? nw : (nw % 4 == 0 ? 4 : nw % 2 == 0 ? 2 : 1);
  const int R = dw_cp_rows(W, C, lnw != nullptr);
  const dim3 grid((unsigned)((long)B * ((H + R - 1) / R)), (unsigned)(nw / wpb)), block((unsigned)(wpb * 64));
#define CP_(WW, L, RR)                                                                                          \
  hipLaunchKernelGGL((dwconv7_cp_kernel<WW, L, RR>), grid, block, 0, st, H, C, (const bf16*)x, w, bias, lnw, lnb, \
                     (bf16*)y, (const bf16*)res, flip)
#define CP_R(WW, L) \
  if (R == 2) CP_(WW, L, 2); \
  else CP_(WW, L, 1)
  if (W == 14) {
    if (lnw) CP_R(14, true);
    else CP_R(14, false);
  } else {
    if (lnw) CP_R(7, true);
    else CP_R(7, false);
  }
#undef CP_R
#undef CP_
  IMGCAP_CHECK_LAUNCH("imgcap_dwconv7 (channel pairs)");
  return 0;
}

template <typename T>
int dwconv7_launch(int B, int H, int W, int C, const void* x, const float* w, const float* bias, void* y,
                   hipStream_t st, const void* res = nullptr, int flip = 0) {
  if (sizeof(T) == 2 && dw_cp_fits(W, C, false))
    return dwconv7_cp_launch(B, H, W, C, x, w, bias, nullptr, nullptr, y, res, flip, st);
  // pixels per lane: the largest of 7, 8, 4, 2, 1 dividing W; rows per block: 64 lanes / groups.
  // Channels per lane: 8 (4 waves per block); 4 (8 waves) and 1-4 pixels per lane at the 28 / 14 /
  // 7-wide stages measured slower and were removed (round 3, tools/microbench.py dw)
  const int PW = W % 7 == 0 ? 7 : W % 8 == 0 ? 8 : W % 4 == 0 ? 4 : W % 2 == 0 ? 2 : 1;
  const int GW = W / PW, TR = 64 / GW;
  const long R = (long)B * H;
  const int RS = dw_row_slots(W, PW, (int)sizeof(T));
  const size_t shm = (size_t)(TR + 6) * RS * 16;
  dim3 grid((unsigned)((R + TR - 1) / TR), C / DW_CT);
  // the rolling kernel (compile-time widths, 8 channels per lane, bf16 / fp32)
  const long tiles = (R + TR - 1) / TR;
  const int sppx = DW_CT * (int)sizeof(T) / 16;
  const size_t shm_r1 = (size_t)(TR + 6) * dw_roll_row_slots(W, PW, sppx) * 16;
#define DWR_ALL(P, WC)                                                                                      \
  do {                                                                                                     \
    dw_roll_attr<T, P, WC>();                                                                              \
    hipLaunchKernelGGL((dwconv7_roll_kernel<T, P, WC, 8>), dim3((unsigned)(tiles * (C / DW_CT))), dim3(256), shm_r1, \
                       st, B, H, C, (const T*)x, w, bias, (T*)y, (const T*)res, flip);                     \
  } while (0)
  if (W == 56 || W == 28 || W == 14 || W == 7 || W == 64 || W == 32 || W == 16 || W == 8) {
    switch (W) {
      case 56: DWR_ALL(7, 56); break;
      case 28: DWR_ALL(7, 28); break;
      case 14: DWR_ALL(7, 14); break;
      case 7: DWR_ALL(7, 7); break;
      case 64: DWR_ALL(8, 64); break;
      case 32: DWR_ALL(8, 32); break;
      case 16: DWR_ALL(8, 16); break;
      default: DWR_ALL(8, 8); break;
    }
    IMGCAP_CHECK_LAUNCH("imgcap_dwconv7");
    return 0;
  }
#undef DWR_ALL
  // other widths: the runtime-width channel-tiled kernel
#define DW_(P)                                                                                                  \
  hipLaunchKernelGGL((dwconv7_kernel<T, P, 0, 8>), grid, dim3(256), shm, st, B, H, W, C, (const T*)x, w, bias, \
                     (T*)y, TR, RS, (const T*)res, flip)
  switch (PW) {
    case 8: DW_(8); break;
    case 7: DW_(7); break;
    case 4: DW_(4); break;
    case 2: DW_(2); break;
    default: DW_(1); break;
  }
#undef DW_
  IMGCAP_CHECK_LAUNCH("imgcap_dwconv7");
  return 0;
}
}  // namespace

extern "C" int imgcap_dwconv7(int dtype, int B, int H, int W, int C, const void* x, const float* w,
                              const float* bias, void* y, void* stream) {
  IMGCAP_REQUIRE(C % DW_CT == 0, "imgcap_dwconv7: C must be a multiple of 32");
  IMGCAP_REQUIRE((long)B * H * W * C * (dtype == IMGCAP_BF16 ? 2 : 4) < (1L << 31),
                 "imgcap_dwconv7: input must be < 2 GiB (32-bit buffer offsets)");
  IMGCAP_REQUIRE(W >= 1 && W <= 64, "imgcap_dwconv7: W must be in [1, 64]");
  IMGCAP_REQUIRE(aligned16(x) && aligned16(y) && aligned16(w) && aligned16(bias), "imgcap_dwconv7: alignment");
  if ((long)B * H == 0) return 0;
  if (dtype == IMGCAP_BF16) return dwconv7_launch<bf16>(B, H, W, C, x, w, bias, y, (hipStream_t)stream);
  return dwconv7_launch<float>(B, H, W, C, x, w, bias, y, (hipStream_t)stream);
}

extern "C" int imgcap_dwconv7_bwd_data(int dtype, int B, int H, int W, int C, const void* dz, const float* w,
                                       const void* res, void* dx, void* stream) {
  IMGCAP_REQUIRE(C % DW_CT == 0, "imgcap_dwconv7_bwd_data: C must be a multiple of 32");
  IMGCAP_REQUIRE(W >= 1 && W <= 64, "imgcap_dwconv7_bwd_data: W must be in [1, 64]");
  IMGCAP_REQUIRE(aligned16(dz) && aligned16(dx) && aligned16(w) && (!res || aligned16(res)),
                 "imgcap_dwconv7_bwd_data: alignment");
  // res may alias dx (each output element reads its own residual first); dz may not (neighbours)
  IMGCAP_REQUIRE(dz != dx, "imgcap_dwconv7_bwd_data: dz and dx must differ");
  IMGCAP_REQUIRE((long)B * H * W * C * (dtype == IMGCAP_BF16 ? 2 : 4) < (1L << 31),
                 "imgcap_dwconv7_bwd_data: input must be < 2 GiB (32-bit buffer offsets)");
  if ((long)B * H == 0) return 0;
  if (dtype == IMGCAP_BF16)
    return dwconv7_launch<bf16>(B, H, W, C, dz, w, nullptr, dx, (hipStream_t)stream, res, 1);
  return dwconv7_launch<float>(B, H, W, C, dz, w, nullptr, dx, (hipStream_t)stream, res, 1);
}

extern "C" int imgcap_stochastic_depth_scales(int nblocks, int B, const float* probs, uint64_t seed,
                                              uint32_t drop_stream, float* out, void* stream) {
  const int n = nblocks * B;
  if (n == 0) return 0;
  hipLaunchKernelGGL(sd_scales_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, n, B, probs, seed,
                     g_seed_ctr, drop_stream, out);
  IMGCAP_CHECK_LAUNCH("imgcap_stochastic_depth_scales");
  return 0;
}

extern "C" int imgcap_convnext_stem(int dtype, int B, int H, int W, int C0, const float* images, const float* w,
                                    const float* bias, const float* ln_w, const float* ln_b, void* out, void* stream) {
  IMGCAP_REQUIRE(H % 4 == 0 && W % 4 == 0 && C0 % 8 == 0 && C0 <= 1024, "imgcap_convnext_stem: bad shape");
  IMGCAP_REQUIRE(aligned16(images) && aligned16(bias) && aligned16(ln_w) && aligned16(ln_b) && aligned16(out),
                 "imgcap_convnext_stem: alignment");
  const long total = (long)B * (H / 4) * (W / 4);
  if (total == 0) return 0;
  const int CV = C0 / 8;
  const int px = stem_px(C0);
  const int npx = stem_npx(C0, px);
  const int threads = ((npx / px * CV + 63) / 64) * 64;
  dim3 grid((unsigned)((total + npx - 1) / npx));
  const size_t shm = stem_lds(C0, npx);
  IMGCAP_REQUIRE(shm <= 160 * 1024, "imgcap_convnext_stem: LDS");
#define STEM_(T, PXN)                                                                                     \
  hipLaunchKernelGGL((stem_kernel<T, float, PXN>), grid, dim3(threads), shm, (hipStream_t)stream, B, H, W, C0, \
                     images, w, bias, ln_w, ln_b, (T*)out, npx, nullptr, nullptr)
  if (dtype == IMGCAP_BF16) {
    if (px == 4) STEM_(bf16, 4); else STEM_(bf16, 2);
  } else {
    if (px == 4) STEM_(float, 4); else STEM_(float, 2);
  }
#undef STEM_
  IMGCAP_CHECK_LAUNCH("imgcap_convnext_stem");
  return 0;
}

extern "C" int imgcap_convnext_stem_u8(int dtype, int B, int H, int W, int C0, const uint8_t* images,
                                       const float* mean3, const float* std3, const float* w, const float* bias,
                                       const float* ln_w, const float* ln_b, void* out, void* stream) {
  IMGCAP_REQUIRE(H % 4 == 0 && W % 4 == 0 && C0 % 8 == 0 && C0 <= 1024, "imgcap_convnext_stem_u8: bad shape");
  IMGCAP_REQUIRE(((uintptr_t)images & 3) == 0 && aligned16(bias) && aligned16(ln_w) && aligned16(ln_b) &&
                     aligned16(out) && mean3 && std3,
                 "imgcap_convnext_stem_u8: alignment / normalisation constants");
  const long total = (long)B * (H / 4) * (W / 4);
  if (total == 0) return 0;
  const int CV = C0 / 8;
  const int px = stem_px(C0);
  const int npx = stem_npx(C0, px);
  const int threads = ((npx / px * CV + 63) / 64) * 64;
  dim3 grid((unsigned)((total + npx - 1) / npx));
  const size_t shm = stem_lds(C0, npx);
  IMGCAP_REQUIRE(shm <= 160 * 1024, "imgcap_convnext_stem_u8: LDS");
#define STEM_(T, PXN)                                                                                       \
  hipLaunchKernelGGL((stem_kernel<T, uint8_t, PXN>), grid, dim3(threads), shm, (hipStream_t)stream, B, H, W, C0, \
                     images, w, bias, ln_w, ln_b, (T*)out, npx, mean3, std3)
  if (dtype == IMGCAP_BF16) {
    if (px == 4) STEM_(bf16, 4); else STEM_(bf16, 2);
  } else {
    if (px == 4) STEM_(float, 4); else STEM_(float, 2);
  }
#undef STEM_
  IMGCAP_CHECK_LAUNCH("imgcap_convnext_stem_u8");
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
  if (dtype == IMGCAP_BF16 && dw_cp_fits(W, C, true))
    return dwconv7_cp_launch(B, H, W, C, x, w, bias, ln_w, ln_b, out, nullptr, 0, st);
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
                                   const float* ln_b, int cmajor, void* out, void* stream) {
  IMGCAP_REQUIRE(H % 2 == 0 && W % 2 == 0 && C <= 1536, "imgcap_ln_patchify2: bad shape");
  const long npx = (long)B * H * W;
  if (npx == 0) return 0;
  const int V = C / 8;
  if (C % 8 == 0 && V <= 256) {  // ConvNeXt widths: the vectorised patch kernel
    const int PB = std::min(LNP_MAXPB, 256 / V);
    const long np = npx / 4;
    dim3 g((unsigned)((np + PB - 1) / PB));
    if (dtype == IMGCAP_BF16)
      hipLaunchKernelGGL(ln_patchify2v_kernel<bf16>, g, dim3(256), 0, (hipStream_t)stream, B, H, W, C, (const bf16*)x,
                         ln_w, ln_b, (bf16*)out, cmajor, PB);
    else
      hipLaunchKernelGGL(ln_patchify2v_kernel<float>, g, dim3(256), 0, (hipStream_t)stream, B, H, W, C,
                         (const float*)x, ln_w, ln_b, (float*)out, cmajor, PB);
    IMGCAP_CHECK_LAUNCH("imgcap_ln_patchify2");
    return 0;
  }
  dim3 grid((unsigned)((npx + 3) / 4));
  if (dtype == IMGCAP_BF16)
    hipLaunchKernelGGL(ln_patchify2_kernel<bf16>, grid, dim3(256), 0, (hipStream_t)stream, B, H, W, C,
                       (const bf16*)x, ln_w, ln_b, (bf16*)out, cmajor);
  else
    hipLaunchKernelGGL(ln_patchify2_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream, B, H, W, C,
                       (const float*)x, ln_w, ln_b, (float*)out, cmajor);
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

// MFMA GEMM with fused epilogue for gfx950 (bf16 16x16x32, exact-f32 16x16x4).
//
// One code base covers every contraction on the hot path (SURVEY.md §2.2 rows "pointwise
// MLP", "downsample", "projections", "vocab projection" and their dgrad/wgrad forms):
//
// tiled kernel (M > 64): 256 threads = 4 wave64s (2x2), BM x BN x 32 tiles
//   * operand layouts: A k-major ([M][K]) or m-major ([K][M]); B k-major ([N][K], nn.Linear
//     weight) or n-major ([K][N]); m/n-major tiles are transposed while written to LDS
//   * branch-free staging: 16-byte vector loads from clamped addresses, zero-selected when the
//     row/k is out of range (no per-element fallback, so nothing spills); the K tail of the
//     last tile is masked word-wise
//   * register-staged double buffering (next tile's global loads in flight under the MFMAs)
//   * f32 mode feeds the same [row][8 k] fragment to 8 chained 16x16x4 f32 MFMAs (the k order
//     inside a 32-slice is permuted identically for A and B, so the sum is unchanged)
//   * epilogue staged through LDS: each thread finishes 8 consecutive columns of a row
//     (vector bias/scale/residual loads, 16-byte stores)
// skinny kernel (M <= 64, A and B k-major): the LSTM recurrence GEMMs at M = batch.  Each
//   block owns 16 output columns; its 8 waves split K and stream A/B fragments straight from
//   global into registers (no LDS round trip, no barriers in the loop), then reduce in LDS.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "mfma.h"

namespace imgcap {

// ---------------------------------------------------------------------------------------
// epilogue on 8 consecutive columns of one row (n0 .. n0+7), all in range and 16-B aligned
struct EpiFlags {
  bool bias, colscale, rowscale, res, aux, beta, drop;
};

DEV void load8_as_f(const void* p, long i, int dtype, float (&v)[8]) {
  if (dtype == IMGCAP_BF16) {
    const bf16x8 x = *(const bf16x8*)((const bf16*)p + i);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (float)x[j];
  } else {
    const f32x4 a = *(const f32x4*)((const float*)p + i), b = *(const f32x4*)((const float*)p + i + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) { v[j] = a[j]; v[j + 4] = b[j]; }
  }
}
// ACT_GELU with an aux operand: aux[m, n] = the pre-activation (c_dtype), written through
DEV void store_pre8(const imgcap_epilogue& ep, int m, int n0, const float (&v)[8]) {
  const long i = (long)m * ep.ldaux + n0;
  if (ep.c_dtype == IMGCAP_BF16) {
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (bf16)v[j];
    *(bf16x8*)((bf16*)ep.aux + i) = o;
  } else {
    *(f32x4*)((float*)ep.aux + i) = f32x4{v[0], v[1], v[2], v[3]};
    *(f32x4*)((float*)ep.aux + i + 4) = f32x4{v[4], v[5], v[6], v[7]};
  }
}

DEV void epi_vec8(const imgcap_epilogue& ep, const EpiFlags& f, void* C, long cidx, int m, int n0, float (&v)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] *= ep.alpha;
  if (f.bias) {
    const f32x4 b0 = *(const f32x4*)(ep.bias + n0), b1 = *(const f32x4*)(ep.bias + n0 + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) { v[j] += b0[j]; v[j + 4] += b1[j]; }
  }
  if (ep.act == IMGCAP_ACT_GELU) {
    if (f.aux) store_pre8(ep, m, n0, v);  // pre-activation kept for the backward pass
    if (ep.c_dtype != IMGCAP_F32) {  // bf16 / MX out: the sigmoid form (common.h: |error| <= 5.5e-5)
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = gelu_sig(v[j]);
    } else {  // fp32 out: erf by a 1.5e-7-accurate polynomial
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        const f32x2 g = gelu_fast2(f32x2{v[j], v[j + 1]});
        v[j] = g[0];
        v[j + 1] = g[1];
      }
    }
  } else if (ep.act == IMGCAP_ACT_RELU) {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = fmaxf(v[j], 0.f);
  }
  if (f.drop) {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] *= dropout_scale(ep.seed, ep.drop_stream, (uint64_t)m * ep.drop_ld + n0 + j, ep.drop_p);
  }
  if (f.aux && ep.act == IMGCAP_ACT_DGELU) {
    float hv[8];
    load8_as_f(ep.aux, (long)m * ep.ldaux + n0, ep.c_dtype, hv);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] *= gelu_grad(hv[j]);
  } else if (f.aux && ep.act != IMGCAP_ACT_GELU) {
    const long ai = (long)m * ep.ldaux + n0;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = load_as_f(ep.aux, ai + j, ep.c_dtype) > 0.f ? v[j] * ep.aux_scale : 0.f;
  }
  if (f.colscale) {
    const f32x4 s0 = *(const f32x4*)(ep.colscale + n0), s1 = *(const f32x4*)(ep.colscale + n0 + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) { v[j] *= s0[j]; v[j + 4] *= s1[j]; }
  }
  if (f.rowscale) {
    const float s = ep.rowscale[m / ep.rows_per_scale];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] *= s;
  }
  if (ep.c_dtype == IMGCAP_BF16) {
    if (f.res) {
      const bf16x8 r = *(const bf16x8*)((const bf16*)ep.res + (long)m * ep.ldr + n0);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += (float)r[j];
    }
    bf16* cp = (bf16*)C + cidx;
    if (f.beta) {
      const bf16x8 o = *(const bf16x8*)cp;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += ep.beta * (float)o[j];
    }
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (bf16)v[j];
    *(bf16x8*)cp = o;
  } else {
    if (f.res) {
      const float* rp = (const float*)ep.res + (long)m * ep.ldr + n0;
      const f32x4 r0 = *(const f32x4*)rp, r1 = *(const f32x4*)(rp + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) { v[j] += r0[j]; v[j + 4] += r1[j]; }
    }
    float* cp = (float*)C + cidx;
    if (f.beta) {
      const f32x4 o0 = *(const f32x4*)cp, o1 = *(const f32x4*)(cp + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) { v[j] += ep.beta * o0[j]; v[j + 4] += ep.beta * o1[j]; }
    }
    *(f32x4*)cp = f32x4{v[0], v[1], v[2], v[3]};
    *(f32x4*)(cp + 4) = f32x4{v[4], v[5], v[6], v[7]};
  }
}

// scalar epilogue for ragged / unaligned column tails
DEV void epi_scalar(const imgcap_epilogue& ep, void* C, long cidx, int m, int n, float v) {
  v *= ep.alpha;
  if (ep.bias) v += ep.bias[n];
  if (ep.act == IMGCAP_ACT_GELU) {
    if (ep.aux) store_from_f((void*)ep.aux, (long)m * ep.ldaux + n, ep.c_dtype, v);
    v = ep.c_dtype != IMGCAP_F32 ? gelu_sig(v) : gelu_fast(v);
  } else if (ep.act == IMGCAP_ACT_RELU) {
    v = fmaxf(v, 0.f);
  }
  if (ep.drop_p > 0.f) v *= dropout_scale(ep.seed, ep.drop_stream, (uint64_t)m * ep.drop_ld + n, ep.drop_p);
  if (ep.aux && ep.act == IMGCAP_ACT_DGELU) v *= gelu_grad(load_as_f(ep.aux, (long)m * ep.ldaux + n, ep.c_dtype));
  else if (ep.aux && ep.act != IMGCAP_ACT_GELU)
    v = load_as_f(ep.aux, (long)m * ep.ldaux + n, ep.c_dtype) > 0.f ? v * ep.aux_scale : 0.f;
  if (ep.colscale) v *= ep.colscale[n];
  if (ep.rowscale) v *= ep.rowscale[m / ep.rows_per_scale];
  if (ep.res) v += load_as_f(ep.res, (long)m * ep.ldr + n, ep.c_dtype);
  if (ep.beta != 0.f) v += ep.beta * load_as_f(C, cidx, ep.c_dtype);
  store_from_f(C, cidx, ep.c_dtype, v);
}

// Finish a staged f32 tile rows [0, rows) x [0, BN) held in LDS (row stride LDT floats):
// every thread handles 8-column vectors.  vec_ok: ldc, ldr, ldaux multiples of 8 and C/res
// 16-byte aligned (host-checked).
template <int BN>
DEV void epilogue_from_lds(const imgcap_epilogue& ep, const float* tile, int LDT, int rows, int m_base, int n_base,
                           int M, int N, void* C, long ldc, long cbase, bool vec_ok) {
  const EpiFlags f{ep.bias != nullptr, ep.colscale != nullptr, ep.rowscale != nullptr, ep.res != nullptr,
                   ep.aux != nullptr, ep.beta != 0.f, ep.drop_p > 0.f};
  constexpr int NV = BN / 8;
  for (int e = threadIdx.x; e < rows * NV; e += blockDim.x) {
    const int r = e / NV, c8 = (e % NV) * 8;
    const int m = m_base + r, n = n_base + c8;
    if (m >= M || n >= N) continue;
    float v[8];
    const f32x4 a = *(const f32x4*)(tile + r * LDT + c8), b = *(const f32x4*)(tile + r * LDT + c8 + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) { v[j] = a[j]; v[j + 4] = b[j]; }
    const long cidx = cbase + (long)m * ldc + n;
    if (vec_ok && n + 8 <= N) {
      epi_vec8(ep, f, C, cidx, m, n, v);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (n + j < N) epi_scalar(ep, C, cidx + j, m, n + j, v[j]);
    }
  }
}

// 8 values of row m, columns n0..n0+7 (16-byte aligned, in range) of a c_dtype matrix
struct Raw8v { uint4 a, b; };
DEV Raw8v ld_row8(const void* p, long i, int dtype) {
  Raw8v r;
  if (dtype == IMGCAP_BF16) {
    r.a = *(const uint4*)((const bf16*)p + i);
    r.b = r.a;
  } else {
    r.a = *(const uint4*)((const float*)p + i);
    r.b = *(const uint4*)((const float*)p + i + 4);
  }
  return r;
}
DEV void raw8_to_f(const Raw8v& r, int dtype, float (&v)[8]) {
  if (dtype == IMGCAP_BF16) {
    const bf16x8 x = __builtin_bit_cast(bf16x8, r.a);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (float)x[j];
  } else {
    const f32x4 x = __builtin_bit_cast(f32x4, r.a), y = __builtin_bit_cast(f32x4, r.b);
#pragma unroll
    for (int j = 0; j < 4; ++j) { v[j] = x[j]; v[j + 4] = y[j]; }
  }
}

// Fast epilogue of a fp32 tile staged in LDS (rows [0, ROWS) x [0, BN), row stride LDT) by a
// block of NT threads: a thread owns one 8-column group (the same in every pass, so the
// column operands -- bias, layer-scale -- are loaded once per call) and ROWS*BN/(8*NT) rows;
// all of its LDS reads and global operand loads (residual, aux, C for beta, row scales) are
// issued before the first use, so the pass costs one memory round trip instead of one per row.
// Semantics = epi_vec8 / epi_scalar (imgcap_epilogue).
// GAP: staged row r maps to output row m_base + r + (r >= ROWS/2 ? GAP : 0) (two row bands)
// ---- MX-FP8 (OCP e4m3fn + E8M0 block scales of 32) -----------------------------------
// The 8 values a lane holds are 8 consecutive columns; the 4 lanes lane&~3 .. lane|3 hold a
// 32-column block (callers keep all 4 active together).  e = floor(log2(amax)) - 8 so the
// block's largest magnitude lands in [256, 512) and is clamped to e4m3's 448.
DEV void mx_store8(const float (&x)[8], uint8_t* q, uint8_t* s, bool write_scale, bool store = true) {
  float amax = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(x[j]));
  amax = fmaxf(amax, __shfl_xor(amax, 1, 64));
  amax = fmaxf(amax, __shfl_xor(amax, 2, 64));
  const int ex = (int)((__float_as_uint(amax) >> 23) & 0xff);  // biased exponent (0: zero/denormal block)
  const int sb = ex == 0 ? 127 : max(ex - 8, 1);               // scale byte = e + 127
  const float inv = __uint_as_float((uint32_t)(254 - sb) << 23);  // 2^-(sb-127)
  float c[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) c[j] = fminf(fmaxf(x[j] * inv, -448.f), 448.f);
  uint32_t w0 = __builtin_amdgcn_cvt_pk_fp8_f32(c[0], c[1], 0, false);
  w0 = __builtin_amdgcn_cvt_pk_fp8_f32(c[2], c[3], w0, true);
  uint32_t w1 = __builtin_amdgcn_cvt_pk_fp8_f32(c[4], c[5], 0, false);
  w1 = __builtin_amdgcn_cvt_pk_fp8_f32(c[6], c[7], w1, true);
  if (store) *(uint2*)q = make_uint2(w0, w1);
  if (store && write_scale) *s = (uint8_t)sb;
}

template <int BN, int ROWS, int NT, int CH = 2, int GAP = 0>
DEV void epilogue_tile(const imgcap_epilogue& ep, const float* tile, int LDT, int m_base, int n_base, int M, int N,
                       void* C, long ldc, bool vec_ok) {
  constexpr int NV = BN / 8, RPI = NT / NV, IT = ROWS / RPI;
  static_assert(NT % NV == 0 && ROWS % RPI == 0 && IT % CH == 0, "epilogue_tile geometry");
  const int c8 = (threadIdx.x % NV) * 8, rl = threadIdx.x / NV;
  const int n = n_base + c8;
  if (n >= N) return;
  if (!(vec_ok && n + 8 <= N)) {  // ragged / unaligned column group: element-wise
    for (int it = 0; it < IT; ++it) {
      const int r = rl + it * RPI, m = m_base + r + (r >= ROWS / 2 ? GAP : 0);
      if (m >= M) continue;
      for (int j = 0; j < 8 && n + j < N; ++j) epi_scalar(ep, C, (long)m * ldc + n + j, m, n + j, tile[r * LDT + c8 + j]);
    }
    return;
  }
  const bool has_res = ep.res != nullptr, has_aux = ep.aux != nullptr, has_beta = ep.beta != 0.f;
  const bool pre_gelu = has_aux && ep.act == IMGCAP_ACT_GELU;  // aux is an output then
  float bias[8], cs[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { bias[j] = 0.f; cs[j] = 1.f; }
  if (ep.bias) {
    const f32x4 b0 = *(const f32x4*)(ep.bias + n), b1 = *(const f32x4*)(ep.bias + n + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) { bias[j] = b0[j]; bias[j + 4] = b1[j]; }
  }
  if (ep.colscale) {
    const f32x4 s0 = *(const f32x4*)(ep.colscale + n), s1 = *(const f32x4*)(ep.colscale + n + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) { cs[j] = s0[j]; cs[j + 4] = s1[j]; }
  }
#pragma unroll 1
  for (int i0 = 0; i0 < IT; i0 += CH) {
    float v[CH][8];
    Raw8v resv[CH], auxv[CH], cv[CH];
    float rsv[CH];
#pragma unroll
    for (int u = 0; u < CH; ++u) {  // every load of the chunk first
      const int r = rl + (i0 + u) * RPI;
      const int m = min(m_base + r + (r >= ROWS / 2 ? GAP : 0), M - 1);
      const float* t = tile + r * LDT + c8;
      const f32x4 a = *(const f32x4*)t, b = *(const f32x4*)(t + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) { v[u][j] = a[j]; v[u][j + 4] = b[j]; }
      if (has_res) resv[u] = ld_row8(ep.res, (long)m * ep.ldr + n, ep.c_dtype);
      if (has_aux && !pre_gelu) auxv[u] = ld_row8(ep.aux, (long)m * ep.ldaux + n, ep.c_dtype);
      if (has_beta) cv[u] = ld_row8(C, (long)m * ldc + n, ep.c_dtype);
      rsv[u] = ep.rowscale ? ep.rowscale[m / ep.rows_per_scale] : 1.f;
    }
#pragma unroll
    for (int u = 0; u < CH; ++u) {
      const int r = rl + (i0 + u) * RPI;
      const int m = m_base + r + (r >= ROWS / 2 ? GAP : 0);
      if (m >= M) continue;
      float x[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = v[u][j] * ep.alpha + bias[j];
      if (ep.act == IMGCAP_ACT_GELU) {
        if (pre_gelu) store_pre8(ep, m, n, x);
        if (ep.c_dtype != IMGCAP_F32) {  // bf16 / MX out: the sigmoid form (|error| <= 5.5e-5)
#pragma unroll
          for (int j = 0; j < 8; ++j) x[j] = gelu_sig(x[j]);
        } else {
#pragma unroll
          for (int j = 0; j < 8; j += 2) {
            const f32x2 g = gelu_fast2(f32x2{x[j], x[j + 1]});
            x[j] = g[0];
            x[j + 1] = g[1];
          }
        }
      } else if (ep.act == IMGCAP_ACT_RELU) {
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = fmaxf(x[j], 0.f);
      }
      if (ep.drop_p > 0.f) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          x[j] *= dropout_scale(ep.seed, ep.drop_stream, (uint64_t)m * ep.drop_ld + n + j, ep.drop_p);
      }
      if (has_aux && !pre_gelu) {
        float a[8];
        raw8_to_f(auxv[u], ep.c_dtype, a);
        if (ep.act == IMGCAP_ACT_DGELU) {
#pragma unroll
          for (int j = 0; j < 8; ++j) x[j] *= gelu_grad(a[j]);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) x[j] = a[j] > 0.f ? x[j] * ep.aux_scale : 0.f;
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] *= cs[j] * rsv[u];
      if (has_res) {
        float r[8];
        raw8_to_f(resv[u], ep.c_dtype, r);
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] += r[j];
      }
      if (has_beta) {
        float o[8];
        raw8_to_f(cv[u], ep.c_dtype, o);
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] += ep.beta * o[j];
      }
      const long ci = (long)m * ldc + n;
      if (ep.c_dtype == IMGCAP_FP8MX) {  // 4 lanes = one 32-column block: shared E8M0 scale
        mx_store8(x, (uint8_t*)C + ci, ep.c_scale + (long)m * (ldc / 32) + n / 32, (threadIdx.x & 3) == 0);
      } else if (ep.c_dtype == IMGCAP_BF16) {
        bf16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (bf16)x[j];
        *(bf16x8*)((bf16*)C + ci) = o;
      } else {
        float* cp = (float*)C + ci;
        *(f32x4*)cp = f32x4{x[0], x[1], x[2], x[3]};
        *(f32x4*)(cp + 4) = f32x4{x[4], x[5], x[6], x[7]};
      }
    }
  }
}

// split-K partial tile -> its slice of the workspace P[z][M][N] (row pitch N, plain stores)
template <int BN>
DEV void partial_from_lds(const float* tile, int LDT, int rows, int m_base, int n_base, int M, int N,
                          float* P) {
  constexpr int NV = BN / 4;
  const bool vec = (N & 3) == 0;
  for (int e = threadIdx.x; e < rows * NV; e += blockDim.x) {
    const int r = e / NV, c4 = (e % NV) * 4;
    const int m = m_base + r, n = n_base + c4;
    if (m >= M || n >= N) continue;
    const f32x4 v = *(const f32x4*)(tile + r * LDT + c4);
    float* dst = P + (long)m * N + n;
    if (vec) {
      *(f32x4*)dst = v;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (n + j < N) dst[j] = v[j];
    }
  }
}

// C[m, n] = epilogue(sum_z P[z][m][n])  (fixed slice order: deterministic; the full epilogue
// of imgcap_gemm -- bias, activation, dropout, scales, residual, beta -- runs here)
__global__ __launch_bounds__(256) void splitk_reduce_kernel(int M, int N, int S, const float* __restrict__ P,
                                                            void* __restrict__ C, long ldc, imgcap_epilogue ep,
                                                            const uint64_t* seed_ctr) {
  if (ep.drop_p > 0.f) ep.seed = eff_seed(ep.seed, seed_ctr);
  const long total = (long)M * N;
  const long plane = total;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    // slices added in order, loads issued 8 at a time
    float t = 0.f;
    for (int z0 = 0; z0 < S; z0 += 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = z0 + u < S ? P[(z0 + u) * plane + i] : 0.f;
#pragma unroll
      for (int u = 0; u < 8; ++u) t += v[u];
    }
    const int m = (int)(i / N), n = (int)(i % N);
    epi_scalar(ep, C, (long)m * ldc + n, m, n, t);
  }
}

#include "gemm_tiled.h"
#include "gemm_glds.h"
#include "gemm256.h"
#include "gemm_mx.h"
#include "gemm_pt.h"
#include "gemm_ws.h"

// ---------------------------------------------------------------------------------------
// skinny kernel: M <= 16*MT rows, A [M][K] and B [N][K] both k-major.  Block = 16 columns,
// SW waves split K; each wave issues the loads of up to DEPTH k-steps at once (one memory
// round trip per chunk), fragments go straight from global memory to the MFMAs.
template <typename T, int MT, int SW, int DEPTH>
__global__ __launch_bounds__(64 * SW) void gemm_skinny_kernel(const T* __restrict__ A, long lda,
                                                              const T* __restrict__ B, long ldb,
                                                              void* __restrict__ C, long ldc, int M, int N, int K,
                                                              imgcap_epilogue ep, int vec_ok,
                                                              const uint64_t* seed_ctr) {
  if (ep.drop_p > 0.f) ep.seed = eff_seed(ep.seed, seed_ctr);
  __shared__ __attribute__((aligned(16))) float part[SW][MT * 16][SKINNY_LDT];
  const int n0 = blockIdx.x * 16;
  const int n = n0 + (threadIdx.x & 15);
  const bool bok = n < N;
  skinny_tile<T, MT, SW, DEPTH>(A, lda, M, B + (long)(bok ? n : N - 1) * ldb, bok, K, part);
  epilogue_from_lds<16>(ep, &part[0][0][0], SKINNY_LDT, MT * 16, 0, n0, M, N, C, ldc, 0, vec_ok != 0);
}

// Which kernel serves a GEMM (also answered to callers by imgcap_gemm_plan)
struct GemmPlan {
  int kind;   // IMGCAP_GEMM_*
  int split;  // K slices (1 = none)
};

static bool glds_enabled() {
  static const bool on = [] {
    const char* e = getenv("IMGCAP_GEMM_GLDS");  // A/B switch for kernel benchmarks
    return !(e && e[0] == '0');
  }();
  return on;
}

static int glds_stages() {
  static const int s = [] {
    const char* e = getenv("IMGCAP_GLDS_STAGES");  // A/B switch for kernel benchmarks
    const int v = e ? atoi(e) : 2;
    return v >= 2 && v <= 4 ? v : 2;
  }();
  return s;
}

// 64x64 tile stages (IMGCAP_GLDS64_STAGES, 2-4) and the XCD tile order of the LDS-DMA tiles
// (IMGCAP_GEMM_ORDER: 0 row-major bands, 1 grouped rectangles, 2 = auto (default): grouped for
// wide grids, nx >= 1.5 ny; glds_tile_order).  Measured at C2 (tools/gpu/gemm_knobs.sh, 64x64
// tiles): grouped 149x26 (vocab logits) 43.1 -> 35.2 us, 48x25 20.1 -> 18.9; on tall grids
// (6x98, 12x25, 24x98) row-major bands are already the better order (each XCD reads its own
// rows once and the narrow B whole): grouped 19.0 -> 20.3, 23.1 -> 24.0, 22.7 -> 23.1.  More
// 64x64 stages lose: 3 stages 703 -> 734 us over the step's GEMMs, 4 stages 887 us.
static int glds64_stages() {
  static const int s = [] {
    const char* e = getenv("IMGCAP_GLDS64_STAGES");
    const int v = e ? atoi(e) : 2;
    return v >= 2 && v <= 4 ? v : 2;
  }();
  return s;
}
static int gemm_order() {
  static const int o = [] {
    const char* e = getenv("IMGCAP_GEMM_ORDER");
    return e ? atoi(e) : 2;
  }();
  return o;
}
// band height in tile rows for a grid of nx x ny tiles (glds_tile_order): each XCD's run of
// ~nx*ny/8 tiles as a square-ish rectangle; 0 = row-major
static int glds_group(int nx, int ny) {
  const int o = gemm_order();
  if (o == 0 || nx * ny < 64 || (o == 2 && 2 * nx < 3 * ny)) return 0;
  const double run = (double)nx * ny / 8.0;
  int g = (int)(std::sqrt(run) + 0.5);
  return std::max(1, std::min(g, ny));
}

// 256x256 tile (gemm256.h): 0 never, 1 wherever it applies, -1 by shape (default; the
// IMGCAP_GEMM256 environment variable or imgcap_gemm_set_policy override it)
static int g_gemm256_mode = [] {
  const char* e = getenv("IMGCAP_GEMM256");
  return e ? atoi(e) : -1;
}();
static int gemm256_mode() { return g_gemm256_mode; }

static GemmPlan gemm_plan(bool bf16_op, int ak, int bk, int M, int N, int K, long lda, long ldb, int batch, int split) {
  if (M <= 64 && ak && bk && batch == 1) return {IMGCAP_GEMM_SKINNY, 1};
  const int mode = gemm256_mode();
  const bool glds_ok = bf16_op && glds_enabled() && mode != 5 && batch == 1 && lda % 8 == 0 && ldb % 8 == 0 && K >= 64;
  if (glds_ok && split == 1) {
    // the 256 tile wins only with >= ~1.5 rounds of tiles over the CUs and long K (measured:
    // tools/microbench.py probe); below that the 2-blocks-per-CU 128 tile overlaps better
    const long tiles256 = (long)((M + 255) / 256) * ((N + 255) / 256);
    if ((mode >= 1 && mode <= 3) || ((mode < 0 || mode >= 7) && tiles256 >= 384 && K >= 1024)) return {IMGCAP_GEMM_GLDS256, 1};
  }
  const long tiles128 = (long)((M + 127) / 128) * ((N + 127) / 128) * batch;
  const auto auto_split = [&] {
    return (int)std::max(1L, std::min({512 / std::max(tiles128, 1L), (long)(K / 256), 32L}));
  };
  if (glds_ok) {
    // split-K: requested (weight gradients, -1 = auto) or, for grids too small to fill the chip
    // with a long K, chosen here; partial tiles go to scratch and the reduce kernel applies the
    // epilogue.  Auto: ~2 blocks per CU, >= 4 k-tiles per slice.
    int sk = 1;
    // (auto split-K only past K = 4096: below it the unsplit 64x64 tile wins, e.g. 1632x512x2048
    // 14.7 vs 20.1 us, 3136x768x3072 30.6 vs 33.7; at K = 9490 split-K 128 tiles win 41 vs 53)
    const bool long_k_small_grid = split == 1 && tiles128 < 256 && K >= 2048;
    if (split < 0 || (long_k_small_grid && mode != 6 && !(mode < 0 && K <= 4096))) sk = auto_split();
    else if (split > 1) sk = split;
    // 64x64 LDS-DMA tile (4 blocks per CU): small grids (the Transformer decoder's d=512
    // projections at B*L rows) and short-K mid-size grids, where the 128 tile's fixed per-tile
    // latency dominates (tools/microbench.py small: 1.2-1.5x at 104-975 128-tiles with K <= 1536;
    // the 128 tile wins back only on >= ~1000-tile grids with K > 384: at K <= 384 the 64 tile
    // stays ahead on any grid, tools/gemm_modes.py: 12544x1536x384 38.7 vs 42.0 us, 25088x1024x256
    // 39.9 vs 48.1)
    if (sk == 1 && (mode == 6 || (mode < 0 && (tiles128 < 128 || (tiles128 < 1024 && K <= 1536) ||
                                                 (tiles128 < 256 && K <= 4096) || K <= 384))))
      return {IMGCAP_GEMM_GLDS64, 1};
    if (sk > 1 || tiles128 >= 128 || mode == 4) return {IMGCAP_GEMM_GLDS, sk};
    if (mode == 7) return {IMGCAP_GEMM_GLDS128X64, 1};
  }
  if (split != 1) {
    const int sk = split < 0 ? auto_split() : split;
    if (sk > 1) return {IMGCAP_GEMM_TILED128, sk};
  }
  return {tiles128 < 512 ? IMGCAP_GEMM_TILED64 : IMGCAP_GEMM_TILED128, 1};
}

// ---- stream-tile kernel (gemm_pt.h): selection and launch ---------------------------------
// IMGCAP_GEMM_PT / imgcap_gemm_set_pt: -1 by shape (default, pt_by_shape), 0 never, 1 wherever
// eligible (tile by the cost model), 2..7 wherever eligible with tile config 1..6 forced
static int g_gemm_pt_mode = [] {
  const char* e = getenv("IMGCAP_GEMM_PT");
  return e ? atoi(e) : -1;
}();

static int device_cus() {
  static int cus[64] = {0};
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= 64) return 256;
  if (!cus[dev]) {
    hipDeviceProp_t pr;
    cus[dev] = hipGetDeviceProperties(&pr, dev) == hipSuccess && pr.multiProcessorCount > 0 ? pr.multiProcessorCount : 256;
  }
  return cus[dev];
}

// tile configs: 1 = 256x128 (8 waves 4x2, 3 stages), 2 = 128x256 (2x4, 3 stages), 3 = 128x128 (2x4, 4
// stages), 4 = 128x192 (2x4, 3 stages) -- one block per CU; 5 = 128x128 (4 waves 2x2, 2 stages), two
// blocks per CU; 6 = 128x128 (2x4, 2 stages of 128-deep k-steps).  (4-wave blocks with 128-row wave
// tiles at one wave per SIMD -- 256x128 / 256x256 / 128x256 -- spilled and ran 1.5-20x slower.)
constexpr int PT_NCFG = 6;
struct PtCfg { int bm, bn, bpc, ks; };
static PtCfg pt_cfg(int c) {
  switch (c) {
    case 1: return {256, 128, 1, 1};
    case 2: return {128, 256, 1, 1};
    case 3: return {128, 128, 1, 1};
    case 4: return {128, 192, 1, 1};
    case 5: return {128, 128, 2, 1};
    default: return {128, 128, 1, 2};
  }
}

// cycles of the busiest block: its tiles (persistent rounds over the CUs) x (k-steps x max(MFMA,
// operand delivery ~30 B/cycle/CU) + the epilogue's stores at ~8 B/cycle/CU)
static double pt_estimate(int c, int M, int N, int K, int cus) {
  const PtCfg t = pt_cfg(c);
  const long tiles = (long)((M + t.bm - 1) / t.bm) * ((N + t.bn - 1) / t.bn);
  const long rounds = (tiles + cus * t.bpc - 1) / (cus * t.bpc);
  const double nk = (K + 64 * t.ks - 1) / (64 * t.ks);
  const double step = t.ks * std::max((double)t.bm * t.bn / 32.0, (t.bm + t.bn) * 128.0 / 30.0);
  const double epi = t.bm * t.bn * 2.0 / 8.0;
  return rounds * (nk * step + epi);
}

// configs instantiated per (epilogue kind, layout): the 64x64-per-wave tiles hold the general
// epilogue's operands (and the residual of a transposed layout) only by spilling, so those forms
// take the 64x32 / 64x48 wave tiles
// The 256x128 / 128x256 configs (1, 2) never won a shape in the step census (DESIGN §3f') and are
// built only into the diagnostic library (make diag, IMGCAP_STAMPS), with the 128x64 LDS-DMA tile
// (imgcap_gemm_set_policy 7): the product library holds the kernels its plans can pick.
#ifdef IMGCAP_STAMPS
constexpr bool kDiagGemmVariants = true;
#else
constexpr bool kDiagGemmVariants = false;
#endif
static bool pt_allowed(int c, int ek, bool ak, bool bk, int K) {
  if (c <= 2 && !kDiagGemmVariants) return false;
  if (pt_cfg(c).ks > 1 && K % (64 * pt_cfg(c).ks)) return false;  // 128-deep k-steps: no K tail
  if (c == 6) return ek == 0 || (ek == 1 && ak && bk);
  if (ek == 2) return c == 3;
  if (ek == 1 && !(ak && bk)) return c == 3 || c == 4;
  if (c == 5) return ek <= 1 && ak && bk;
  return true;
}
static int pt_ek(const imgcap_epilogue* ep) {
  if (!ep) return 0;
  return ((ep->aux && ep->act != IMGCAP_ACT_GELU) || ep->beta != 0.f) ? 2 : ep->res ? 1 : 0;
}

static int pt_choose(int M, int N, int K, int ek, bool ak, bool bk) {
  const int cus = device_cus();
  int best = 0;
  double bt = 0;
  for (int c = 1; c <= PT_NCFG; ++c) {
    if (!pt_allowed(c, ek, ak, bk, K)) continue;
    const double t = pt_estimate(c, M, N, K, cus);
    if (!best || t < bt) { best = c; bt = t; }
  }
  return best;
}

// the default plan: the stream tile only where a step census (tools/gemm_census.py, C3 / C4 steps,
// every call timed under each config) measured it ahead of the LDS-staged 64x64 plan -- the
// forward pointwise / downsample products of the encoder (A, B both k-major, no saved-operand
// epilogue):
//   N = 384 (128x192: two column tiles, no N tail), M >= 8192:         12544x384x1536 28.2 vs 31.7 us
//   N = 256 (128x128, two blocks a CU), M >= 8192:                     25088x256x1024 26.2 vs 29.0
//   N = 512, K >= 1024, M >= 4096 (128x128, 128-deep k-steps):         6272x512x2048  25.4 vs 29.9
//   N >= 1024 and M >= 20000, or N >= 4096 and K >= 1024 (128x128 x2):  25088x1024x256 37.6 vs 43.4,
//                                                                     1568x4096x1024 24.2 vs 27.9
// everything else (decoder products, grids under a round of 128x128 tiles, the deep-K stage-4
// second Linear, the backward's transposed layouts) stays on the 64x64 plan, which was as fast or
// faster there
static int pt_by_shape(int M, int N, int K, int ek, bool ak, bool bk) {
  if (!(ak && bk) || ek > 1) return 0;
  int c = 0;
  // (round 6: Tiny's stage-4 first Linear 3136x3072x768 on 128x192 and Base's stage-3 first Linear
  // 6272x2048x512 on 128x128 two a CU ran 30.1 / 30.3 µs against 32.8 / 32.1 alone, but the steps
  // fell: C4 8,396 / 8,346 -> 8,232 / 8,221, C3 19,871 / 19,838 -> 19,742 / 19,749 img/s on one box,
  // tools/gpu/r6_ptrule.sh -- the census rule above holds)
  if (N == 384 && M >= 8192) c = 4;
  else if (N == 256 && M >= 8192) c = 5;
  else if (N == 512 && K >= 1024 && M >= 4096) c = 6;
  else if ((N >= 1024 && M >= 20000) || (N >= 4096 && K >= 1024)) c = 5;
  return c && pt_allowed(c, ek, ak, bk, K) ? c : 0;
}

// bytes from an operand's base to the end of its last 16-byte slot: the descriptor's range check is
// per dword, so an extent ending inside a slot would zero the valid elements of a partial dword
// (the pitch is a multiple of 8 elements >= the row, so the rounded extent stays inside the rows)
static int64_t pt_extent(bool kmaj, int rows, int K, long ld) {
  const auto r8 = [](int64_t x) { return (x + 7) / 8 * 8; };
  return kmaj ? ((int64_t)(rows - 1) * ld + r8(K)) * 2 : ((int64_t)(K - 1) * ld + r8(rows)) * 2;
}

// which stream-tile config serves this call (0: none) -- the epilogue forms the kernel implements
static int pt_plan(int ak, int bk, int M, int N, int K, long lda, long ldb, int batch, int split,
                   const imgcap_epilogue* ep, bool vec_ok) {
  const int mode = g_gemm_pt_mode;
  if (mode == 0 || batch != 1 || split != 1 || lda % 8 || ldb % 8 || N % 4 || K < 64) return 0;
  if (pt_extent(ak, M, K, lda) > 0x7fffffffLL || pt_extent(bk, N, K, ldb) > 0x7fffffffLL) return 0;
  if (ep) {
    if (!vec_ok || ep->c_dtype != IMGCAP_BF16) return 0;
    if (ep->rowscale && ep->rows_per_scale <= 0) return 0;
  }
  const int ek = pt_ek(ep);
  if (mode >= 2 && mode <= PT_NCFG + 1) return pt_allowed(mode - 1, ek, ak, bk, K) ? mode - 1 : pt_choose(M, N, K, ek, ak, bk);
  if (mode < 0) return pt_by_shape(M, N, K, ek, ak, bk);
  return pt_choose(M, N, K, ek, ak, bk);
}

// explicit instantiations of the stream-tile kernels pt_allowed admits (the host stubs of kernel
// templates first named inside the launcher template were otherwise left undefined)
#ifdef IMGCAP_STAMPS
template __global__ void gemm_pt_kernel<256, 128, 4, 2, 3, true, true, 0>(PtArgs);
template __global__ void gemm_pt_kernel<256, 128, 4, 2, 3, true, true, 1>(PtArgs);
template __global__ void gemm_pt_kernel<256, 128, 4, 2, 3, true, false, 0>(PtArgs);
template __global__ void gemm_pt_kernel<256, 128, 4, 2, 3, false, true, 0>(PtArgs);
template __global__ void gemm_pt_kernel<256, 128, 4, 2, 3, false, false, 0>(PtArgs);
template __global__ void gemm_pt_kernel<128, 256, 2, 4, 3, true, true, 0>(PtArgs);
template __global__ void gemm_pt_kernel<128, 256, 2, 4, 3, true, true, 1>(PtArgs);
template __global__ void gemm_pt_kernel<128, 256, 2, 4, 3, true, false, 0>(PtArgs);
template __global__ void gemm_pt_kernel<128, 256, 2, 4, 3, false, true, 0>(PtArgs);
template __global__ void gemm_pt_kernel<128, 256, 2, 4, 3, false, false, 0>(PtArgs);
#endif
template __global__ void gemm_pt_kernel<128, 128, 2, 4, 4, true, true, 0>(PtArgs);
template __global__ void gemm_pt_kernel<128, 128, 2, 4, 4, true, true, 1>(PtArgs);
template __global__ void gemm_pt_kernel<128, 128, 2, 4, 4, true, true, 2>(PtArgs);
template __global__ void gemm_pt_kernel<128, 128, 2, 4, 4, true, false, 0>(PtArgs);
template __global__ void gemm_pt_kernel<128, 128, 2, 4, 4, true, false, 1>(PtArgs);
template __global__ void gemm_pt_kernel<128, 128, 2, 4, 4, true, false, 2>(PtArgs);
template __global__ void gemm_pt_kernel<128, 128, 2, 4, 4, false, true, 0>(PtArgs);
template __global__ void gemm_pt_kernel<128, 128, 2, 4, 4, false, true, 1>(PtArgs);
template __global__ void gemm_pt_kernel<128, 128, 2, 4, 4, false, true, 2>(PtArgs);
template __global__ void gemm_pt_kernel<128, 128, 2, 4, 4, false, false, 0>(PtArgs);
template __global__ void gemm_pt_kernel<128, 128, 2, 4, 4, false, false, 1>(PtArgs);
template __global__ void gemm_pt_kernel<128, 128, 2, 4, 4, false, false, 2>(PtArgs);
template __global__ void gemm_pt_kernel<128, 192, 2, 4, 3, true, true, 0>(PtArgs);
template __global__ void gemm_pt_kernel<128, 192, 2, 4, 3, true, true, 1>(PtArgs);
template __global__ void gemm_pt_kernel<128, 192, 2, 4, 3, true, false, 0>(PtArgs);
template __global__ void gemm_pt_kernel<128, 192, 2, 4, 3, true, false, 1>(PtArgs);
template __global__ void gemm_pt_kernel<128, 192, 2, 4, 3, false, true, 0>(PtArgs);
template __global__ void gemm_pt_kernel<128, 192, 2, 4, 3, false, true, 1>(PtArgs);
template __global__ void gemm_pt_kernel<128, 192, 2, 4, 3, false, false, 0>(PtArgs);
template __global__ void gemm_pt_kernel<128, 192, 2, 4, 3, false, false, 1>(PtArgs);
template __global__ void gemm_pt_kernel<128, 128, 2, 2, 2, true, true, 0>(PtArgs);
template __global__ void gemm_pt_kernel<128, 128, 2, 2, 2, true, true, 1>(PtArgs);
template __global__ void gemm_pt_kernel<128, 128, 2, 4, 2, true, true, 0, 2>(PtArgs);
template __global__ void gemm_pt_kernel<128, 128, 2, 4, 2, true, true, 1, 2>(PtArgs);
template __global__ void gemm_pt_kernel<128, 128, 2, 4, 2, true, false, 0, 2>(PtArgs);
template __global__ void gemm_pt_kernel<128, 128, 2, 4, 2, false, true, 0, 2>(PtArgs);
template __global__ void gemm_pt_kernel<128, 128, 2, 4, 2, false, false, 0, 2>(PtArgs);

// only the (config, epilogue kind, layout) combinations pt_allowed admits are instantiated
template <bool AKV, bool BKV>
void pt_launch_t(int cfg, int ek, int G, const PtArgs& a, hipStream_t st) {
#define PT_L(BM_, BN_, WM_, WN_, S_, EK_) \
  hipLaunchKernelGGL((gemm_pt_kernel<BM_, BN_, WM_, WN_, S_, AKV, BKV, EK_>), dim3(G), dim3(WM_ * WN_ * 64), 0, st, a)
  if (cfg == 3) {
    if (ek == 0) PT_L(128, 128, 2, 4, 4, 0);
    else if (ek == 1) PT_L(128, 128, 2, 4, 4, 1);
    else PT_L(128, 128, 2, 4, 4, 2);
  } else if (cfg == 4) {
    if (ek == 0) PT_L(128, 192, 2, 4, 3, 0);
    else PT_L(128, 192, 2, 4, 3, 1);
  } else if (cfg == 6) {
    if (ek == 0) hipLaunchKernelGGL((gemm_pt_kernel<128, 128, 2, 4, 2, AKV, BKV, 0, 2>), dim3(G), dim3(512), 0, st, a);
    else if constexpr (AKV && BKV)
      hipLaunchKernelGGL((gemm_pt_kernel<128, 128, 2, 4, 2, AKV, BKV, 1, 2>), dim3(G), dim3(512), 0, st, a);
  } else if (cfg == 5) {
    if constexpr (AKV && BKV) {
      if (ek == 0) PT_L(128, 128, 2, 2, 2, 0);
      else PT_L(128, 128, 2, 2, 2, 1);
    }
  } else if constexpr (kDiagGemmVariants) {
    if (cfg == 1) {
      if (ek == 0) PT_L(256, 128, 4, 2, 3, 0);
      else if constexpr (AKV && BKV) PT_L(256, 128, 4, 2, 3, 1);
    } else {
      if (ek == 0) PT_L(128, 256, 2, 4, 3, 0);
      else if constexpr (AKV && BKV) PT_L(128, 256, 2, 4, 3, 1);
    }
  }
#undef PT_L
}

static int pt_launch(int cfg, int ak, int bk, int M, int N, int K, const bf16* A, long lda, const bf16* B, long ldb,
                     void* C, long ldc, const imgcap_epilogue& ep, hipStream_t st) {
  const PtCfg t = pt_cfg(cfg);
  PtArgs a;
  a.A = A;
  a.B = B;
  a.C = C;
  a.lda = lda;
  a.ldb = ldb;
  a.ldc = ldc;
  a.M = M;
  a.N = N;
  a.K = K;
  const int tm = (M + t.bm - 1) / t.bm;
  a.tiles_n = (N + t.bn - 1) / t.bn;
  a.ntiles = tm * a.tiles_n;
  const int cus = device_cus();
  const int G = a.ntiles < cus * t.bpc ? a.ntiles : cus * t.bpc;
  // each XCD's concurrent tiles (G / 8 of them) as a rectangle of grp tile rows balancing its
  // A and B bytes: rows ~ sqrt(run * BN / BM)
  const double run = std::max(1.0, G / 8.0);
  a.grp = std::max(1, std::min(tm, (int)(std::sqrt(run * t.bn / t.bm) + 0.5)));
  a.ep = ep;
  a.seed_ctr = g_seed_ctr;
  a.a_bytes = pt_extent(ak, M, K, lda);
  a.b_bytes = pt_extent(bk, N, K, ldb);
  a.c_bytes = ((uint64_t)(M - 1) * ldc + N) * 2;
  a.res_bytes = ep.res ? ((uint64_t)(M - 1) * ep.ldr + N) * 2 : 0;
  a.aux_bytes = ep.aux ? ((uint64_t)(M - 1) * ep.ldaux + N) * 2 : 0;
  static const int dbg = [] {  // diagnostic build switches (gemm_pt.h PT_DBG)
    const char* e = getenv("IMGCAP_PT_DBG");
    return e ? atoi(e) : 0;
  }();
  a.dbg = dbg;
  if (a.c_bytes > 0x7fffffffull || a.res_bytes > 0x7fffffffull || a.aux_bytes > 0x7fffffffull)
    return fail(IMGCAP_EUNSUPPORTED, "imgcap_gemm(stream tile): operand over 2 GiB");
  const int ek = pt_ek(&ep);
  if (!pt_allowed(cfg, ek, ak, bk, K)) return fail(IMGCAP_EINVAL, "imgcap_gemm(stream tile): config not built for this epilogue");
  if (ak && bk) pt_launch_t<true, true>(cfg, ek, G, a, st);
  else if (ak) pt_launch_t<true, false>(cfg, ek, G, a, st);
  else if (bk) pt_launch_t<false, true>(cfg, ek, G, a, st);
  else pt_launch_t<false, false>(cfg, ek, G, a, st);
  IMGCAP_CHECK_LAUNCH("imgcap_gemm(stream tile)");
  return 0;
}

// ---- weight-stationary short-K kernel (gemm_ws.h): selection and launch ------------------------
// IMGCAP_GEMM_WS / imgcap_gemm_set_ws: -1 by shape (default), 0 never, 1 wherever eligible (blocks
// of 8 waves), 2 wherever eligible (blocks of 4 waves, two per CU)
static int g_gemm_ws_mode = [] {
  const char* e = getenv("IMGCAP_GEMM_WS");
  return e ? atoi(e) : -1;
}();

// 0: not eligible / not chosen; 1: 8-wave blocks (256 columns); 2: 4-wave blocks (128 columns)
static int ws_plan(int ak, int bk, int M, int N, int K, long lda, long ldb, long ldc, const void* C, int batch,
                   int split, const imgcap_epilogue* ep) {
  const int mode = g_gemm_ws_mode;
  if (mode == 0 || !ak || !bk || batch != 1 || split != 1 || (K != 384 && K != 512) || M < 64) return 0;
  if (lda % 8 || ldb % 8 || ldc % 4 || N % 4 || ((uintptr_t)C & 7)) return 0;
  if (ep) {
    if (ep->c_dtype != IMGCAP_BF16 || ep->res || ep->aux || ep->beta != 0.f || ep->rowscale) return 0;
    if (ep->act != IMGCAP_ACT_NONE && ep->act != IMGCAP_ACT_GELU && ep->act != IMGCAP_ACT_RELU) return 0;
  }
  if ((int64_t)(M - 1) * ldc + N > 0x3fffffffLL || (int64_t)(N - 1) * ldb + K > 0x3fffffffLL) return 0;
  if (mode == 1 || mode == 2) return mode;
  // by shape (tools/ws_bench.py, round 6, us per launch against the plan without this kernel):
  // 12544x1536x384 +GELU 32.2 vs 39.9 (4-wave blocks), 25088x1536x384 50.0 vs 64.5, 50176x192x384
  // 18.8 vs 21.7, 3136x6144x512 (the decoder's stacked memory K/V) 32.4 vs 40.2 (8-wave blocks);
  // with the sigmoid-form GELU in both epilogues also C2's 6272x1536x384 +GELU 20.0 vs 22.4.
  // Elsewhere -- the decoder's 3328-row d = 512 products, C4's 6272x2048x512 -- the per-block weight
  // slice load (the kernel's fixed cost, ~8-10 us) is not amortised and the 64x64 LDS tile stays.
  if (N % 8 != 0 || (ep && ep->colscale)) return 0;
  if (K == 384 && M >= 4096 && (N >= 1024 || N == 192)) return 2;
  if (K == 512 && N >= 4096 && M >= 2048) return 1;
  return 0;
}

#ifdef IMGCAP_STAMPS
template <int KS, int NW, int S>
void wsp_go(const WsArgs& a, int act, dim3 grid, hipStream_t st) {
  if (act == IMGCAP_ACT_GELU) hipLaunchKernelGGL((gemm_wsp_kernel<KS, NW, S, 1>), grid, dim3(NW * 64), 0, st, a);
  else if (act == IMGCAP_ACT_RELU) hipLaunchKernelGGL((gemm_wsp_kernel<KS, NW, S, 2>), grid, dim3(NW * 64), 0, st, a);
  else hipLaunchKernelGGL((gemm_wsp_kernel<KS, NW, S, 0>), grid, dim3(NW * 64), 0, st, a);
}
#endif

template <int KS, int NW, int S, bool STG = false>
void ws_go(const WsArgs& a, int act, dim3 grid, hipStream_t st) {
  if (act == IMGCAP_ACT_GELU) hipLaunchKernelGGL((gemm_ws_kernel<KS, NW, S, 1, STG>), grid, dim3(NW * 64), 0, st, a);
  else if (act == IMGCAP_ACT_RELU) hipLaunchKernelGGL((gemm_ws_kernel<KS, NW, S, 2, STG>), grid, dim3(NW * 64), 0, st, a);
  else hipLaunchKernelGGL((gemm_ws_kernel<KS, NW, S, 0, STG>), grid, dim3(NW * 64), 0, st, a);
}

static int ws_launch(int cfg, int M, int N, int K, const bf16* A, long lda, const bf16* B, long ldb, void* C, long ldc,
                     const imgcap_epilogue& ep, hipStream_t st) {
  const int NW = cfg == 1 ? 8 : 4, bpc = cfg == 1 ? 1 : 2;
  WsArgs a;
  a.A = A;
  a.B = B;
  a.C = C;
  a.lda = lda;
  a.ldb = ldb;
  a.ldc = ldc;
  a.M = M;
  a.N = N;
  a.slices = (N + 32 * NW - 1) / (32 * NW);
  const int nchunks = (M + 31) / 32;
  const int want = std::max(1, device_cus() * bpc / a.slices);
  a.chunks_per = (nchunks + want - 1) / want;
  a.row_groups = (nchunks + a.chunks_per - 1) / a.chunks_per;
  a.ep = ep;
  a.seed_ctr = g_seed_ctr;
  a.b_bytes = ((int64_t)(N - 1) * ldb + K) * 2;
  a.c_bytes = ((int64_t)(M - 1) * ldc + N) * 2;
  const dim3 grid(a.slices * a.row_groups);
  static const int stg = [] {  // output tile staged through LDS (default; IMGCAP_WS_STG=0: 8-byte stores)
    const char* e = getenv("IMGCAP_WS_STG");
    return e ? atoi(e) : 1;
  }();
#ifdef IMGCAP_STAMPS  // diagnostic build: the measured-slower forms (gemm_ws.h)
  static const int deep = [] {  // deeper A-chunk rings (IMGCAP_WS_DEEP=1)
    const char* e = getenv("IMGCAP_WS_DEEP");
    return e ? atoi(e) : 0;
  }();
  static const int pipe = [] {  // the software-pipelined form (IMGCAP_WS_PIPE=1)
    const char* e = getenv("IMGCAP_WS_PIPE");
    return e ? atoi(e) : 0;
  }();
#else
  constexpr int deep = 0, pipe = 0;
#endif
  if (pipe && !ep.colscale) {
#ifdef IMGCAP_STAMPS
    if (K == 384) {
      if (NW == 8) wsp_go<24, 8, 4>(a, ep.act, grid, st);
      else wsp_go<24, 4, 3>(a, ep.act, grid, st);
    } else {
      if (NW == 8) wsp_go<32, 8, 3>(a, ep.act, grid, st);
      else wsp_go<32, 4, 2>(a, ep.act, grid, st);
    }
#endif
  } else if (stg && N % 8 == 0) {
    if (K == 384) {
      if (NW == 8) ws_go<24, 8, 5, true>(a, ep.act, grid, st);
      else ws_go<24, 4, 2, true>(a, ep.act, grid, st);
    } else {
      if (NW == 8) ws_go<32, 8, 4, true>(a, ep.act, grid, st);
      else ws_go<32, 4, 2, true>(a, ep.act, grid, st);
    }
  } else if (K == 384) {
    if (NW == 8) {
#ifdef IMGCAP_STAMPS
      if (deep) ws_go<24, 8, 6>(a, ep.act, grid, st);
      else
#endif
        ws_go<24, 8, 3>(a, ep.act, grid, st);
    } else {
      ws_go<24, 4, 3>(a, ep.act, grid, st);
    }
  } else {
    if (NW == 8) {
#ifdef IMGCAP_STAMPS
      if (deep) ws_go<32, 8, 4>(a, ep.act, grid, st);
      else
#endif
        ws_go<32, 8, 3>(a, ep.act, grid, st);
    } else {
      ws_go<32, 4, 2>(a, ep.act, grid, st);
    }
  }
  IMGCAP_CHECK_LAUNCH("imgcap_gemm(weight-stationary)");
  return 0;
}

template <typename T>
static int gemm_dispatch(int ak, int bk, int M, int N, int K, const void* A, long lda, long sA, const void* B,
                         long ldb, long sB, void* C, long ldc, long sC, int batch, const imgcap_epilogue& ep,
                         int vec_ok, hipStream_t st, int split) {
  if constexpr (sizeof(T) == 2) {
    const int wc = ws_plan(ak, bk, M, N, K, lda, ldb, ldc, C, batch, split, &ep);
    if (wc) return ws_launch(wc, M, N, K, (const bf16*)A, lda, (const bf16*)B, ldb, C, ldc, ep, st);
    const int pc = pt_plan(ak, bk, M, N, K, lda, ldb, batch, split, &ep, vec_ok != 0);
    if (pc) return pt_launch(pc, ak, bk, M, N, K, (const bf16*)A, lda, (const bf16*)B, ldb, C, ldc, ep, st);
  }
  const GemmPlan plan = gemm_plan(sizeof(T) == 2, ak, bk, M, N, K, lda, ldb, batch, split);
  if (plan.kind == IMGCAP_GEMM_SKINNY) {
    const int blocks = (N + 15) / 16;
    const bool wide = blocks < 96;  // few column blocks: split K over 16 waves instead of 8
    const T* a = (const T*)A;
    const T* b = (const T*)B;
#define SK_(MT, SW, DEPTH)                                                                                   \
  hipLaunchKernelGGL((gemm_skinny_kernel<T, MT, SW, DEPTH>), dim3(blocks), dim3(64 * SW), 0, st, a, lda, b, ldb, C, \
                     ldc, M, N, K, ep, vec_ok, g_seed_ctr)
    // DEPTH = the wave's k-step count rounded up to a power of two (all loads of a wave in one
    // round trip); capped by registers (fp32 fragments are twice as wide)
    const int per = ((K + 31) / 32 + (wide ? 16 : 8) - 1) / (wide ? 16 : 8);
    const int depth = per <= 1 ? 1 : per <= 2 ? 2 : per <= 4 ? 4 : 8;
    constexpr bool F32 = sizeof(T) == 4;
#define SK_W(MT, SW)                                              \
  do {                                                            \
    if (depth <= 1) SK_(MT, SW, 1);                               \
    else if (F32 || depth <= 2) SK_(MT, SW, 2);                   \
    else if (depth <= 4 || MT == 4) SK_(MT, SW, (F32 ? 2 : 4));   \
    else SK_(MT, SW, (F32 || MT == 4 ? 2 : 8));                   \
  } while (0)
    if (M <= 32) {
      if (wide) SK_W(2, 16); else SK_W(2, 8);
    } else {
      if (wide) SK_W(4, 16); else SK_W(4, 8);
    }
#undef SK_W
#undef SK_
    IMGCAP_CHECK_LAUNCH("imgcap_gemm(skinny)");
    return 0;
  }
  if constexpr (sizeof(T) == 2) {
    if (plan.kind == IMGCAP_GEMM_GLDS256) {
      dim3 grid((N + 255) / 256, (M + 255) / 256);
      const bf16* a = (const bf16*)A;
      const bf16* b = (const bf16*)B;
      const int var = gemm256_mode() >= 1 && gemm256_mode() <= 3 ? gemm256_mode() : 1;  // 1: BK 64 x 2 stages, 2: BK 32 x 4, 3: BK 32 x 3
#define G256_V(AKV, BKV, BKT, SV)                                                                               \
  hipLaunchKernelGGL((gemm256_kernel<BKT, SV, AKV, BKV>), grid, dim3(512), 0, st, a, lda, b, ldb, C, ldc, M, N, K, \
                     ep, vec_ok, g_seed_ctr, 0)
#define G256_(AKV, BKV)                       \
  do {                                        \
    if (var == 1) G256_V(AKV, BKV, 64, 2);    \
    else if (var == 3) G256_V(AKV, BKV, 32, 3); \
    else G256_V(AKV, BKV, 32, 4);             \
  } while (0)
      if (ak && bk) G256_(true, true);
      else if (ak) G256_(true, false);
      else if (bk) G256_(false, true);
      else G256_(false, false);
#undef G256_
#undef G256_V
      IMGCAP_CHECK_LAUNCH("imgcap_gemm(glds256)");
      return 0;
    }
    if (plan.kind == IMGCAP_GEMM_GLDS64 || plan.kind == IMGCAP_GEMM_GLDS128X64) {
      const bool sq = plan.kind == IMGCAP_GEMM_GLDS64;
      dim3 grid((N + 63) / 64, sq ? (M + 63) / 64 : (M + 127) / 128);
      const bf16* a = (const bf16*)A;
      const bf16* b = (const bf16*)B;
      const int grp = glds_group(grid.x, grid.y), S64 = glds64_stages();
#define GS_S(AKV, BKV, SV)                                                                                            \
  hipLaunchKernelGGL((gemm_glds_kernel<64, 64, AKV, BKV, SV>), grid, dim3(256), 0, st, a, lda, b, ldb, C, ldc, M, N, K, \
                     ep, vec_ok, g_seed_ctr, 0, grp)
#define GS_(AKV, BKV)                                                                                                 \
  do {                                                                                                             \
    if (sq) {                                                                                                      \
      if (S64 == 4) GS_S(AKV, BKV, 4);                                                                             \
      else if (S64 == 3) GS_S(AKV, BKV, 3);                                                                        \
      else GS_S(AKV, BKV, 2);                                                                                      \
    } else if constexpr (kDiagGemmVariants) {                                                                       \
      hipLaunchKernelGGL((gemm_glds_kernel<128, 64, AKV, BKV, 2>), grid, dim3(256), 0, st, a, lda, b, ldb, C, ldc, M, \
                         N, K, ep, vec_ok, g_seed_ctr, 0, grp);                                                    \
    }                                                                                                              \
  } while (0)
      if (ak && bk) GS_(true, true);
      else if (ak) GS_(true, false);
      else if (bk) GS_(false, true);
      else GS_(false, false);
#undef GS_
#undef GS_S
      IMGCAP_CHECK_LAUNCH("imgcap_gemm(glds small)");
      return 0;
    }
    if (plan.kind == IMGCAP_GEMM_GLDS) {
      const int sk = plan.split;
      const int kslice = sk > 1 ? ((K + sk - 1) / sk + 63) / 64 * 64 : 0;
      const int zdim = sk > 1 ? (K + kslice - 1) / kslice : 1;
      void* Cdst = C;
      if (sk > 1) {
        Cdst = workspace((size_t)zdim * M * N * sizeof(float), st);
        if (!Cdst) return fail(IMGCAP_EWORKSPACE, std::string("imgcap_gemm: split-K ") + last_error());
      }
      dim3 grid((N + 127) / 128, (M + 127) / 128, zdim);
      const bf16* a = (const bf16*)A;
      const bf16* b = (const bf16*)B;
      const int S = glds_stages();
      const int grp = glds_group(grid.x, grid.y);
#define GL_S(AKV, BKV, SV)                                                                                           \
  hipLaunchKernelGGL((gemm_glds_kernel<128, 128, AKV, BKV, SV>), grid, dim3(256), 0, st, a, lda, b, ldb, Cdst, ldc, M, \
                     N, K, ep, vec_ok, g_seed_ctr, kslice, grp)
#define GL_(AKV, BKV)              \
  do {                             \
    if (S == 4) GL_S(AKV, BKV, 4);  \
    else if (S == 3) GL_S(AKV, BKV, 3); \
    else GL_S(AKV, BKV, 2);        \
  } while (0)
      if (ak && bk) GL_(true, true);
      else if (ak) GL_(true, false);
      else if (bk) GL_(false, true);
      else GL_(false, false);
#undef GL_
#undef GL_S
      if (sk > 1) {
        const long total = (long)M * N;
        const int blocks = (int)std::min<long>((total + 255) / 256, 2048);
        hipLaunchKernelGGL(splitk_reduce_kernel, dim3(blocks), dim3(256), 0, st, M, N, zdim, (const float*)Cdst, C,
                           ldc, ep, g_seed_ctr);
      }
      IMGCAP_CHECK_LAUNCH("imgcap_gemm(glds)");
      return 0;
    }
  }
  if (plan.kind == IMGCAP_GEMM_TILED128 && plan.split > 1)
    return launch_tiled<T, 128, 128, 64>(ak, bk, M, N, K, A, lda, sA, B, ldb, sB, C, ldc, sC, 1, ep, vec_ok, st,
                                         plan.split);
  if (plan.kind == IMGCAP_GEMM_TILED64)
    return launch_tiled<T, 64, 64, 64>(ak, bk, M, N, K, A, lda, sA, B, ldb, sB, C, ldc, sC, batch, ep, vec_ok, st);
  return launch_tiled<T, 128, 128, 64>(ak, bk, M, N, K, A, lda, sA, B, ldb, sB, C, ldc, sC, batch, ep, vec_ok, st);
}

// bias-gradient style column sums: out[c] = beta*out[c] + sum_r x[r, c].
// Block = 64 columns (8 vectors of 8) x 32 row lanes over the row slice blockIdx.y of
// gridDim.y; fixed-order LDS reduction.  With one slice the block writes out directly; with
// several, each writes its partial row of ws and colsum_reduce_kernel adds the slices in
// order — deterministic either way, and enough blocks to fill the chip for narrow outputs.
template <typename T>
__global__ __launch_bounds__(256) void colsum_kernel(int rows, int cols, const T* __restrict__ x, long ld,
                                                     float* __restrict__ out, float beta, int vec_ok,
                                                     int rows_per_slice) {
  __shared__ float red[32][65];
  const int cv = threadIdx.x & 7, rl = threadIdx.x >> 3;
  const int c0 = blockIdx.x * 64 + cv * 8;
  const int r_beg = blockIdx.y * rows_per_slice, r_end = min(rows, r_beg + rows_per_slice);
  float s[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = 0.f;
  if (vec_ok && c0 + 8 <= cols) {
    for (int r = r_beg + rl; r < r_end; r += 32) {
      float v[8];
      ld_g<T, 16 / sizeof(T)>(x + (long)r * ld + c0, *(float(*)[16 / sizeof(T)])v);
      if constexpr (sizeof(T) == 4) ld_g<T, 4>(x + (long)r * ld + c0 + 4, *(float(*)[4])(v + 4));
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += v[j];
    }
  } else {
    for (int r = r_beg + rl; r < r_end; r += 32)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (c0 + j < cols) s[j] += to_f(x[(long)r * ld + c0 + j]);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[rl][cv * 8 + j] = s[j];
  __syncthreads();
  if (threadIdx.x < 64) {
    const int c = blockIdx.x * 64 + threadIdx.x;
    float t = 0.f;
    for (int i = 0; i < 32; ++i) t += red[i][threadIdx.x];
    if (c < cols) {
      if (gridDim.y == 1) out[c] = (beta != 0.f ? beta * out[c] : 0.f) + t;
      else out[(long)blockIdx.y * cols + c] = t;
    }
  }
}

// Block = 32 columns x 8 slice groups: each thread adds the slices y = g, g+8, .. (loads issued
// together, <= 8 per thread for <= 64 slices), then the 8 group sums of a column are added in
// LDS in a fixed order.
__global__ __launch_bounds__(256) void colsum_reduce_kernel(int cols, int slices, const float* __restrict__ ws,
                                                            float* __restrict__ out, float beta) {
  __shared__ float red[8][33];
  const int cl = threadIdx.x & 31, g = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + cl;
  const int cc = c < cols ? c : 0;
  float v[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int y = g + 8 * u;
    v[u] = y < slices ? ws[(long)y * cols + cc] : 0.f;
  }
  float t = 0.f;
#pragma unroll
  for (int u = 0; u < 8; ++u) t += v[u];
  red[g][cl] = t;
  __syncthreads();
  if (g == 0 && c < cols) {
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) s += red[q][cl];
    out[c] = (beta != 0.f ? beta * out[c] : 0.f) + s;
  }
}

// ---- many column sums in one launch (the bias gradients of a whole backward pass) ----------
// A block = (item, 64-column group), 256 threads = 32 row lanes x 8 column vectors: each lane
// walks its rows with 8 rows' 16-byte loads in flight per trip, then a fixed-order LDS sum over
// the row lanes: out = beta*out + sum (deterministic, no library scratch -- the LSTM engine runs
// these sums on a side stream beside scratch users).  The round-4 kernel (1024-thread blocks,
// 128 row lanes) spilled its fp32 path to scratch memory and took ~250 us for C3's bias sums.
constexpr int COLSUM_MAX_ITEMS = 48;
struct ColsumBatch {
  int n;
  int first_block[COLSUM_MAX_ITEMS + 1];
  imgcap_colsum_item it[COLSUM_MAX_ITEMS];
};

__global__ __launch_bounds__(256) void colsum_multi_kernel(ColsumBatch b) {
  __shared__ float red[32][65];
  int k = 0;
  while (k + 1 < b.n && (int)blockIdx.x >= b.first_block[k + 1]) ++k;
  const imgcap_colsum_item& item = b.it[k];
  const int cg = blockIdx.x - b.first_block[k];
  const int cv = threadIdx.x & 7, rl = threadIdx.x >> 3;
  const int c0 = cg * 64 + cv * 8;
  const bool vec = item.vec_ok && c0 + 8 <= item.cols;
  const int rows = item.rows;
  const long ld = item.ld;
  float s[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = 0.f;
  if (c0 < item.cols) {
    constexpr int U = 8;  // rows in flight per lane
    int r = rl;
    if (item.dtype == IMGCAP_BF16) {
      const bf16* x = (const bf16*)item.x + c0;
      if (vec) {
        for (; r + 32 * (U - 1) < rows; r += 32 * U) {
          bf16x8 v[U];
#pragma unroll
          for (int u = 0; u < U; ++u) v[u] = *(const bf16x8*)(x + (long)(r + 32 * u) * ld);
#pragma unroll
          for (int u = 0; u < U; ++u)
#pragma unroll
            for (int j = 0; j < 8; ++j) s[j] += (float)v[u][j];
        }
        for (; r < rows; r += 32) {
          const bf16x8 v = *(const bf16x8*)(x + (long)r * ld);
#pragma unroll
          for (int j = 0; j < 8; ++j) s[j] += (float)v[j];
        }
      } else {
        for (; r < rows; r += 32)
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (c0 + j < item.cols) s[j] += (float)x[(long)r * ld + j];
      }
    } else {
      const float* x = (const float*)item.x + c0;
      if (vec) {
        for (; r + 32 * (U - 1) < rows; r += 32 * U) {
          f32x4 v[U][2];
#pragma unroll
          for (int u = 0; u < U; ++u) {
            v[u][0] = *(const f32x4*)(x + (long)(r + 32 * u) * ld);
            v[u][1] = *(const f32x4*)(x + (long)(r + 32 * u) * ld + 4);
          }
#pragma unroll
          for (int u = 0; u < U; ++u)
#pragma unroll
            for (int j = 0; j < 4; ++j) { s[j] += v[u][0][j]; s[j + 4] += v[u][1][j]; }
        }
        for (; r < rows; r += 32) {
          const f32x4 v0 = *(const f32x4*)(x + (long)r * ld), v1 = *(const f32x4*)(x + (long)r * ld + 4);
#pragma unroll
          for (int j = 0; j < 4; ++j) { s[j] += v0[j]; s[j + 4] += v1[j]; }
        }
      } else {
        for (; r < rows; r += 32)
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (c0 + j < item.cols) s[j] += x[(long)r * ld + j];
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[rl][cv * 8 + j] = s[j];
  __syncthreads();
  if (threadIdx.x < 64) {
    const int c = cg * 64 + threadIdx.x;
    float t = 0.f;
#pragma unroll 8
    for (int i = 0; i < 32; ++i) t += red[i][threadIdx.x];
    if (c < item.cols) item.out[c] = (item.beta != 0.f ? item.beta * item.out[c] : 0.f) + t;
  }
}

// Two-pass form with caller-owned scratch (imgcap_colsum_multi_part): phase 1 blocks = (item,
// 64-column group, 256-row chunk), every load of a block in flight at once, partial sums to
// part[chunk][cols]; phase 2 adds an item's chunk partials in order.  Thousands of one-trip
// blocks instead of ~900 blocks walking up to 3,328 rows each.
constexpr int COLSUM_RC = 256;
struct ColsumBatch2 {
  int n;
  int first_block[COLSUM_MAX_ITEMS + 1];
  int first_col[COLSUM_MAX_ITEMS + 1];
  long part_off[COLSUM_MAX_ITEMS];
  imgcap_colsum_item it[COLSUM_MAX_ITEMS];
  float* part;
};

__global__ __launch_bounds__(256) void colsum_part_kernel(ColsumBatch2 b) {
  __shared__ float red[32][65];
  int k = 0;
  while (k + 1 < b.n && (int)blockIdx.x >= b.first_block[k + 1]) ++k;
  const imgcap_colsum_item& item = b.it[k];
  const int ngrp = (item.cols + 63) / 64;
  const int lb = blockIdx.x - b.first_block[k];
  const int cg = lb % ngrp, ch = lb / ngrp;
  const int cv = threadIdx.x & 7, rl = threadIdx.x >> 3;
  const int c0 = cg * 64 + cv * 8;
  const int r0 = ch * COLSUM_RC + rl;
  const int rend = min(item.rows, (ch + 1) * COLSUM_RC);
  const bool vec = item.vec_ok && c0 + 8 <= item.cols;
  const long ld = item.ld;
  float s[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = 0.f;
  if (c0 < item.cols) {
    constexpr int U = COLSUM_RC / 32;  // rows per lane, all in flight
    if (item.dtype == IMGCAP_BF16) {
      const bf16* x = (const bf16*)item.x + c0;
      if (vec) {
        bf16x8 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int r = r0 + 32 * u;
          v[u] = r < rend ? *(const bf16x8*)(x + (long)r * ld) : bf16x8{};
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int j = 0; j < 8; ++j) s[j] += (float)v[u][j];
      } else {
        for (int r = r0; r < rend; r += 32)
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (c0 + j < item.cols) s[j] += (float)x[(long)r * ld + j];
      }
    } else {
      const float* x = (const float*)item.x + c0;
      if (vec) {
        f32x4 v[U][2];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int r = r0 + 32 * u;
          v[u][0] = r < rend ? *(const f32x4*)(x + (long)r * ld) : f32x4{};
          v[u][1] = r < rend ? *(const f32x4*)(x + (long)r * ld + 4) : f32x4{};
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int j = 0; j < 4; ++j) { s[j] += v[u][0][j]; s[j + 4] += v[u][1][j]; }
      } else {
        for (int r = r0; r < rend; r += 32)
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (c0 + j < item.cols) s[j] += x[(long)r * ld + j];
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[rl][cv * 8 + j] = s[j];
  __syncthreads();
  if (threadIdx.x < 64) {
    const int c = cg * 64 + threadIdx.x;
    float t = 0.f;
#pragma unroll 8
    for (int i = 0; i < 32; ++i) t += red[i][threadIdx.x];
    if (c < item.cols) b.part[b.part_off[k] + (long)ch * item.cols + c] = t;
  }
}

__global__ __launch_bounds__(256) void colsum_fin_kernel(ColsumBatch2 b) {
  const int g = blockIdx.x * 256 + threadIdx.x;
  if (g >= b.first_col[b.n]) return;
  int k = 0;
  while (k + 1 < b.n && g >= b.first_col[k + 1]) ++k;
  const imgcap_colsum_item& item = b.it[k];
  const int c = g - b.first_col[k];
  const int nch = (item.rows + COLSUM_RC - 1) / COLSUM_RC;
  const float* p = b.part + b.part_off[k] + c;
  float t = 0.f;
  for (int i = 0; i < nch; ++i) t += p[(long)i * item.cols];
  item.out[c] = (item.beta != 0.f ? item.beta * item.out[c] : 0.f) + t;
}

// out[c][r] = in[r][c] (2-D transpose through an LDS tile; weights -> k-major copies)
template <typename T>
__global__ __launch_bounds__(256) void transpose_kernel(int rows, int cols, const T* __restrict__ in, long ldi,
                                                        T* __restrict__ out, long ldo) {
  __shared__ T tile[64][65];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  for (int e = threadIdx.x; e < 64 * 64; e += 256) {
    const int r = e / 64, c = e % 64;
    if (r0 + r < rows && c0 + c < cols) tile[r][c] = in[(long)(r0 + r) * ldi + c0 + c];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < 64 * 64; e += 256) {
    const int c = e / 64, r = e % 64;
    if (r0 + r < rows && c0 + c < cols) out[(long)(c0 + c) * ldo + r0 + r] = tile[r][c];
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
  IMGCAP_REQUIRE(K > 0, "imgcap_gemm: K == 0");
  IMGCAP_REQUIRE(dtype == IMGCAP_F32 || dtype == IMGCAP_BF16, "imgcap_gemm: bad dtype");
  const int vec = dtype == IMGCAP_F32 ? 4 : 8;
  IMGCAP_REQUIRE(aligned16(A) && aligned16(B), "imgcap_gemm: A/B must be 16-byte aligned");
  IMGCAP_REQUIRE(lda % vec == 0 && ldb % vec == 0 && strideA % vec == 0 && strideB % vec == 0,
                 "imgcap_gemm: leading dims/strides must be multiples of 16 bytes");
  IMGCAP_REQUIRE(epi->rows_per_scale > 0 || epi->rowscale == nullptr, "imgcap_gemm: rows_per_scale");
  IMGCAP_REQUIRE(epi->bias == nullptr || aligned16(epi->bias), "imgcap_gemm: bias alignment");
  IMGCAP_REQUIRE(epi->colscale == nullptr || aligned16(epi->colscale), "imgcap_gemm: colscale alignment");
  // leading dims of the stored operands must cover the logical extent (loads may read a full
  // 16-byte vector from the last valid row/column)
  IMGCAP_REQUIRE(a_kmajor ? lda >= K : lda >= M, "imgcap_gemm: lda too small");
  IMGCAP_REQUIRE(b_kmajor ? ldb >= K : ldb >= N, "imgcap_gemm: ldb too small");
  const bool vec_ok = aligned16(C) && ldc % 8 == 0 && strideC % 8 == 0 &&
                      (epi->res == nullptr || (aligned16(epi->res) && epi->ldr % 8 == 0)) &&
                      (epi->aux == nullptr || (aligned16(epi->aux) && epi->ldaux % 8 == 0));
  int split = 1;
  if (epi->split_k != 0 && epi->split_k != 1) {
    IMGCAP_REQUIRE(epi->c_dtype == IMGCAP_F32 && batch == 1 && !epi->bias && !epi->colscale && !epi->rowscale &&
                       !epi->res && !epi->aux && epi->act == IMGCAP_ACT_NONE && epi->drop_p == 0.f,
                   "imgcap_gemm: split_k needs an fp32 C = alpha*A.B + beta*C (no other epilogue, batch 1)");
    split = epi->split_k;
  }
  hipStream_t st = (hipStream_t)stream;
  if (dtype == IMGCAP_BF16)
    return gemm_dispatch<bf16>(a_kmajor, b_kmajor, M, N, K, A, lda, strideA, B, ldb, strideB, C, ldc, strideC,
                               batch, *epi, vec_ok, st, split);
  return gemm_dispatch<float>(a_kmajor, b_kmajor, M, N, K, A, lda, strideA, B, ldb, strideB, C, ldc, strideC,
                              batch, *epi, vec_ok, st, split);
}

extern "C" int imgcap_gemm_plan(int dtype, int a_kmajor, int b_kmajor, int M, int N, int K, int64_t lda, int64_t ldb,
                                int batch, int split_k, int* splits) {
  const GemmPlan p = gemm_plan(dtype == IMGCAP_BF16, a_kmajor, b_kmajor, M, N, K, lda, ldb, batch,
                               (split_k == 0 || split_k == 1) ? 1 : split_k);
  if (splits) *splits = p.split;
  return p.kind;
}

extern "C" int imgcap_colsum(int dtype, int rows, int cols, const void* x, int64_t ldx, float* out, float beta,
                             void* stream) {
  if (cols == 0) return 0;
  const int cblocks = (cols + 63) / 64;
  // slices: ~512 blocks in total, >= 64 rows each, at most 64 slices
  int slices = std::min(std::min(64, (512 + cblocks - 1) / cblocks), std::max(1, rows / 64));
  const int rps = (rows + slices - 1) / std::max(slices, 1);
  slices = rows > 0 ? (rows + rps - 1) / rps : 1;
  float* dst = out;
  if (slices > 1) {
    dst = (float*)workspace((size_t)slices * cols * sizeof(float), (hipStream_t)stream);
    if (!dst) return fail(IMGCAP_EWORKSPACE, std::string("imgcap_colsum: ") + last_error());
  }
  const dim3 grid(cblocks, slices);
  const int vec_ok = aligned16(x) && ldx % 8 == 0;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == IMGCAP_BF16)
    hipLaunchKernelGGL(colsum_kernel<bf16>, grid, dim3(256), 0, st, rows, cols, (const bf16*)x, ldx, dst, beta,
                       vec_ok, std::max(rps, 1));
  else
    hipLaunchKernelGGL(colsum_kernel<float>, grid, dim3(256), 0, st, rows, cols, (const float*)x, ldx, dst, beta,
                       vec_ok, std::max(rps, 1));
  if (slices > 1)
    hipLaunchKernelGGL(colsum_reduce_kernel, dim3((cols + 31) / 32), dim3(256), 0, st, cols, slices, dst, out, beta);
  IMGCAP_CHECK_LAUNCH("imgcap_colsum");
  return 0;
}

extern "C" int imgcap_transpose(int dtype, int rows, int cols, const void* in, int64_t ldi, void* out, int64_t ldo,
                                void* stream) {
  if (rows == 0 || cols == 0) return 0;
  dim3 grid((cols + 63) / 64, (rows + 63) / 64);
  if (dtype == IMGCAP_BF16)
    hipLaunchKernelGGL(transpose_kernel<bf16>, grid, dim3(256), 0, (hipStream_t)stream, rows, cols, (const bf16*)in,
                       ldi, (bf16*)out, ldo);
  else
    hipLaunchKernelGGL(transpose_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream, rows, cols,
                       (const float*)in, ldi, (float*)out, ldo);
  IMGCAP_CHECK_LAUNCH("imgcap_transpose");
  return 0;
}

extern "C" int imgcap_gemm_set_pt(int mode) {
  IMGCAP_REQUIRE(mode >= -1 && mode <= PT_NCFG + 1, "imgcap_gemm_set_pt: -1..7");
  if ((mode == 2 || mode == 3) && !kDiagGemmVariants)
    return fail(IMGCAP_EUNSUPPORTED, "imgcap_gemm_set_pt(2|3): the 256x128 / 128x256 tiles are in the diagnostic build only");
  g_gemm_pt_mode = mode;
  return 0;
}

extern "C" int imgcap_gemm_get_pt(void) { return g_gemm_pt_mode; }

extern "C" int imgcap_gemm_set_ws(int mode) {
  IMGCAP_REQUIRE(mode >= -1 && mode <= 2, "imgcap_gemm_set_ws: -1..2");
  g_gemm_ws_mode = mode;
  return 0;
}

extern "C" int imgcap_gemm_get_ws(void) { return g_gemm_ws_mode; }

extern "C" int imgcap_gemm_plan_ep(int dtype, int a_kmajor, int b_kmajor, int M, int N, int K, int64_t lda,
                                   int64_t ldb, int batch, const imgcap_epilogue* epi, int* splits) {
  const int split = (epi == nullptr || epi->split_k == 0 || epi->split_k == 1) ? 1 : epi->split_k;
  if (dtype == IMGCAP_BF16) {
    // (the C pointer / ldc of the call are not known here: an aligned C with ldc = N is assumed)
    const int wc = ws_plan(a_kmajor, b_kmajor, M, N, K, lda, ldb, (N + 3) / 4 * 4, nullptr, batch, split, epi);
    if (wc) {
      if (splits) *splits = 1;
      return IMGCAP_GEMM_WS + wc - 1;
    }
    const int pc = pt_plan(a_kmajor, b_kmajor, M, N, K, lda, ldb, batch, split, epi, true);
    if (pc) {
      if (splits) *splits = 1;
      return IMGCAP_GEMM_PT + pc - 1;
    }
  }
  const GemmPlan p = gemm_plan(dtype == IMGCAP_BF16, a_kmajor, b_kmajor, M, N, K, lda, ldb, batch, split);
  if (splits) *splits = p.split;
  return p.kind;
}

extern "C" int imgcap_gemm_set_policy(int glds256) {
  IMGCAP_REQUIRE(glds256 >= -1 && glds256 <= 8, "imgcap_gemm_set_policy: -1..8");
  if (glds256 == 7 && !kDiagGemmVariants)
    return fail(IMGCAP_EUNSUPPORTED, "imgcap_gemm_set_policy(7): the 128x64 tile is in the diagnostic build only");
  g_gemm256_mode = glds256;
  return 0;
}

#ifdef IMGCAP_STAMPS
extern "C" int imgcap_debug_stamps(void* p) {
  unsigned long long* v = (unsigned long long*)p;
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_dev_stamps), &v, sizeof(v));
}
#endif

extern "C" int imgcap_colsum_multi(int n, const imgcap_colsum_item* items, void* stream) {
  IMGCAP_REQUIRE(n >= 0 && n <= COLSUM_MAX_ITEMS, "imgcap_colsum_multi: at most 48 items per call");
  if (n == 0) return 0;
  ColsumBatch b{};
  b.n = n;
  int blocks = 0;
  for (int i = 0; i < n; ++i) {
    IMGCAP_REQUIRE(items[i].rows >= 0 && items[i].cols >= 0, "imgcap_colsum_multi: negative extent");
    b.it[i] = items[i];
    b.it[i].vec_ok = aligned16(items[i].x) && (items[i].dtype == IMGCAP_BF16 ? items[i].ld % 8 == 0
                                                                               : items[i].ld % 4 == 0);
    b.first_block[i] = blocks;
    blocks += (items[i].cols + 63) / 64;
  }
  b.first_block[n] = blocks;
  if (blocks == 0) return 0;
  hipLaunchKernelGGL(colsum_multi_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, b);
  IMGCAP_CHECK_LAUNCH("imgcap_colsum_multi");
  return 0;
}

extern "C" int imgcap_colsum_multi_part(int n, const imgcap_colsum_item* items, float* part, int64_t part_floats,
                                        void* stream) {
  IMGCAP_REQUIRE(n >= 0 && n <= COLSUM_MAX_ITEMS, "imgcap_colsum_multi_part: at most 48 items per call");
  if (n == 0) return 0;
  ColsumBatch2 b{};
  b.n = n;
  int blocks = 0, cols = 0;
  long off = 0;
  for (int i = 0; i < n; ++i) {
    IMGCAP_REQUIRE(items[i].rows >= 0 && items[i].cols >= 0, "imgcap_colsum_multi_part: negative extent");
    b.it[i] = items[i];
    b.it[i].vec_ok = aligned16(items[i].x) && (items[i].dtype == IMGCAP_BF16 ? items[i].ld % 8 == 0
                                                                               : items[i].ld % 4 == 0);
    b.first_block[i] = blocks;
    b.first_col[i] = cols;
    b.part_off[i] = off;
    const int nch = (items[i].rows + COLSUM_RC - 1) / COLSUM_RC;
    blocks += ((items[i].cols + 63) / 64) * nch;
    cols += items[i].cols;
    off += (long)nch * items[i].cols;
  }
  b.first_block[n] = blocks;
  b.first_col[n] = cols;
  IMGCAP_REQUIRE(off <= part_floats && (off == 0 || part), "imgcap_colsum_multi_part: partials buffer too small");
  if (cols == 0) return 0;
  b.part = part;
  hipStream_t st = (hipStream_t)stream;
  if (blocks > 0) hipLaunchKernelGGL(colsum_part_kernel, dim3(blocks), dim3(256), 0, st, b);
  hipLaunchKernelGGL(colsum_fin_kernel, dim3((cols + 255) / 256), dim3(256), 0, st, b);
  IMGCAP_CHECK_LAUNCH("imgcap_colsum_multi_part");
  return 0;
}

extern "C" int imgcap_gemm_grouped(int a_kmajor, int b_kmajor, int n, const imgcap_gemm_problem* probs,
                                   void* stream) {
  IMGCAP_REQUIRE(n >= 0 && n <= GEMM_GROUP_MAX, "imgcap_gemm_grouped: at most 48 problems per call");
  if (n == 0) return 0;
  GemmGroup g{};
  int tiles = 0, m = 0;
  for (int i = 0; i < n; ++i) {
    const imgcap_gemm_problem& p = probs[i];
    IMGCAP_REQUIRE(p.M >= 0 && p.N >= 0 && p.K > 0, "imgcap_gemm_grouped: bad sizes");
    if (p.M == 0 || p.N == 0) continue;
    IMGCAP_REQUIRE(aligned16(p.A) && aligned16(p.B) && p.lda % 8 == 0 && p.ldb % 8 == 0,
                   "imgcap_gemm_grouped: operands 16-byte aligned, leading dims multiples of 8");
    IMGCAP_REQUIRE(a_kmajor ? p.lda >= p.K : p.lda >= p.M, "imgcap_gemm_grouped: lda too small");
    IMGCAP_REQUIRE(b_kmajor ? p.ldb >= p.K : p.ldb >= p.N, "imgcap_gemm_grouped: ldb too small");
    g.p[m] = p;
    g.first[m] = tiles;
    tiles += ((p.M + 127) / 128) * ((p.N + 127) / 128);
    ++m;
  }
  g.n = m;
  g.first[m] = tiles;
  if (tiles == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
#define GG_(AKV, BKV) hipLaunchKernelGGL((gemm_glds_grouped_kernel<AKV, BKV>), dim3(tiles), dim3(256), 0, st, g)
  if (a_kmajor && b_kmajor) GG_(true, true);
  else if (a_kmajor) GG_(true, false);
  else if (b_kmajor) GG_(false, true);
  else GG_(false, false);
#undef GG_
  IMGCAP_CHECK_LAUNCH("imgcap_gemm_grouped");
  return 0;
}

extern "C" int imgcap_gemm_mx(int M, int N, int K, const void* A, int64_t lda, const uint8_t* As, const void* B,
                              int64_t ldb, const uint8_t* Bs, void* C, int64_t ldc, const imgcap_epilogue* epi,
                              void* stream) {
  IMGCAP_REQUIRE(M >= 0 && N >= 0 && K > 0 && K % 128 == 0, "imgcap_gemm_mx: K must be a positive multiple of 128");
  if (M == 0 || N == 0) return 0;
  IMGCAP_REQUIRE(aligned16(A) && aligned16(B) && lda % 16 == 0 && ldb % 16 == 0 && lda >= K && ldb >= K,
                 "imgcap_gemm_mx: operands 16-byte aligned, row pitches >= K and multiples of 16 bytes");
  IMGCAP_REQUIRE(((uintptr_t)As & 3) == 0 && ((uintptr_t)Bs & 3) == 0, "imgcap_gemm_mx: scales 4-byte aligned");
  imgcap_epilogue ep{};
  if (epi) ep = *epi;
  else { ep.alpha = 1.f; ep.c_dtype = IMGCAP_BF16; ep.rows_per_scale = 1; }
  if (ep.rows_per_scale <= 0) ep.rows_per_scale = 1;
  IMGCAP_REQUIRE(ep.drop_p == 0.f && ep.aux == nullptr && ep.beta == 0.f && ep.split_k <= 1,
                 "imgcap_gemm_mx: no dropout, aux, beta or split-K in this epilogue");
  const int esz = ep.c_dtype == IMGCAP_F32 ? 4 : ep.c_dtype == IMGCAP_BF16 ? 2 : 1;
  const bool vec_ok = aligned16(C) && (ldc * esz) % 16 == 0 && (!ep.res || (aligned16(ep.res) && ep.ldr % 8 == 0)) &&
                      (!ep.bias || aligned16(ep.bias)) && (!ep.colscale || aligned16(ep.colscale));
  if (ep.c_dtype == IMGCAP_FP8MX)
    IMGCAP_REQUIRE(vec_ok && N % 32 == 0 && ldc % 32 == 0 && ep.c_scale && ep.res == nullptr,
                   "imgcap_gemm_mx: MX-FP8 output needs N, ldc % 32 == 0, 16-byte aligned C, c_scale, no res");
  hipStream_t st = (hipStream_t)stream;
  // 128x128 tile, two blocks per CU.  Measured and removed (round 3, tools/gpu/r3_mx.sh): a
  // 256x256 tile (one block per CU; C5 5.05k vs 5.11k img/s with the 128 tile everywhere) and
  // 3 / 4 stages for the 128 tile (1.4-1.6x slower at the stage-3 shapes).
  dim3 grid((N + 127) / 128, (M + 127) / 128);
  hipLaunchKernelGGL((gemm_mx_kernel<2>), grid, dim3(256), 0, st, (const uint8_t*)A, (long)lda, As,
                     (const uint8_t*)B, (long)ldb, Bs, C, (long)ldc, M, N, K, ep, vec_ok ? 1 : 0);
  IMGCAP_CHECK_LAUNCH("imgcap_gemm_mx");
  return 0;
}

extern "C" int imgcap_mx_quant_rows(int dtype, int R, int K, const void* x, int64_t ldx, const float* ln_w,
                                    const float* ln_b, float eps, uint8_t* q, uint8_t* s, void* stream) {
  IMGCAP_REQUIRE(R >= 0 && K > 0 && K % 32 == 0, "imgcap_mx_quant_rows: K must be a positive multiple of 32");
  IMGCAP_REQUIRE((ln_w == nullptr) == (ln_b == nullptr), "imgcap_mx_quant_rows: ln_w and ln_b together");
  IMGCAP_REQUIRE(((uintptr_t)q & 7) == 0, "imgcap_mx_quant_rows: q 8-byte aligned");
  if (dtype == IMGCAP_BF16)
    IMGCAP_REQUIRE(aligned16(x) && ldx % 8 == 0, "imgcap_mx_quant_rows: bf16 rows 16-byte aligned");
  if (R == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  dim3 grid((R + 3) / 4);
  if (dtype == IMGCAP_BF16 && K <= 2048) {  // the row in registers
#define MXQ_(N)                                                                                                    \
  hipLaunchKernelGGL((mx_quant_rows_reg_kernel<bf16, N>), grid, dim3(256), 0, st, R, K, (const bf16*)x, (long)ldx, \
                     ln_w, ln_b, eps, q, s)
    if (K <= 512) MXQ_(1);
    else if (K <= 1024) MXQ_(2);
    else if (K <= 1536) MXQ_(3);
    else MXQ_(4);
#undef MXQ_
  } else if (dtype == IMGCAP_BF16)
    hipLaunchKernelGGL((mx_quant_rows_kernel<bf16>), grid, dim3(256), 0, st, R, K, (const bf16*)x, (long)ldx, ln_w,
                       ln_b, eps, q, s);
  else
    hipLaunchKernelGGL((mx_quant_rows_kernel<float>), grid, dim3(256), 0, st, R, K, (const float*)x, (long)ldx, ln_w,
                       ln_b, eps, q, s);
  IMGCAP_CHECK_LAUNCH("imgcap_mx_quant_rows");
  return 0;
}

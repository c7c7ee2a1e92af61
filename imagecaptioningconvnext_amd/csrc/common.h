// Shared device/host helpers for the imgcap HIP library (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cmath>
#include <string>

#include "../../include/imgcap_abi.h"

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

#define DEV __device__ __forceinline__

namespace imgcap {

// ---- error plumbing (host) -------------------------------------------------------------
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);
// device scratch of at least `bytes` from the calling thread's current slot on the current
// device (NULL when the caller-attached buffer is too small or an allocation fails; callers
// return IMGCAP_EWORKSPACE before launching anything, so the call can simply be retried after
// imgcap_workspace_attach); abi.cpp
void* workspace(size_t bytes, hipStream_t stream);
std::string last_error();
// zero `bytes` (a multiple of 16, 16-byte aligned) with a kernel on `stream` -- a kernel node
// when captured, not a memset node (elementwise.hip; DESIGN.md §2b: the captured split step
// faulted with the runtime's graph packet capture on while a memset node sat in the first half)
hipError_t zero_async(void* p, size_t bytes, hipStream_t stream);

#define IMGCAP_CHECK_LAUNCH(what)                                                   \
  do {                                                                             \
    hipError_t _e = hipGetLastError();                                             \
    if (_e != hipSuccess) return ::imgcap::fail((int)_e, std::string(what) + ": " + \
                                                hipGetErrorString(_e));            \
  } while (0)

#define IMGCAP_REQUIRE(cond, msg)                                      \
  do {                                                                 \
    if (!(cond)) return ::imgcap::fail(IMGCAP_EINVAL, std::string(msg)); \
  } while (0)

inline bool aligned16(const void* p) { return (((uintptr_t)p) & 15) == 0; }

// ---- scalar conversions -------------------------------------------------------------------
DEV float to_f(float x) { return x; }
DEV float to_f(bf16 x) { return (float)x; }
template <typename T> DEV T from_f(float x);
template <> DEV float from_f<float>(float x) { return x; }
template <> DEV bf16 from_f<bf16>(float x) { return (bf16)x; }

DEV float load_as_f(const void* p, long i, int dtype) {
  return dtype == IMGCAP_F32 ? ((const float*)p)[i] : (float)((const bf16*)p)[i];
}
DEV void store_from_f(void* p, long i, int dtype, float v) {
  if (dtype == IMGCAP_F32) ((float*)p)[i] = v; else ((bf16*)p)[i] = (bf16)v;
}

// G consecutive elements as floats; one 16-byte access when G*sizeof(T) == 16 (caller
// guarantees alignment), element-wise otherwise.
template <typename T, int G>
DEV void ld_g(const T* __restrict__ p, float (&v)[G]) {
  if constexpr (G * sizeof(T) == 16) {
    const uint4 u = *(const uint4*)p;
    const T* e = (const T*)&u;
#pragma unroll
    for (int j = 0; j < G; ++j) v[j] = to_f(e[j]);
  } else {
#pragma unroll
    for (int j = 0; j < G; ++j) v[j] = to_f(p[j]);
  }
}
template <typename T, int G>
DEV void st_g(T* __restrict__ p, const float (&v)[G]) {
  if constexpr (G * sizeof(T) == 16) {
    uint4 u;
    T* e = (T*)&u;
#pragma unroll
    for (int j = 0; j < G; ++j) e[j] = from_f<T>(v[j]);
    *(uint4*)p = u;
  } else {
#pragma unroll
    for (int j = 0; j < G; ++j) p[j] = from_f<T>(v[j]);
  }
}

// ---- wave / block reductions (wave64) --------------------------------------------------
DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Sum over the whole block; `red` must hold blockDim.x/64 floats.  All threads get the result.
DEV float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
  for (int i = 0; i < nw; ++i) s += red[i];
  return s;
}

// ---- counter-based RNG for dropout / stochastic depth -------------------------------------
// A mask element is a pure function of (seed, stream, index), so the backward kernels
// recompute it instead of storing it.
// 32-bit arithmetic: the key (seed, stream) is uniform across a launch and folds once; per
// element, the counter times an odd constant XOR the key through murmur3's fmix32 -- a bijection
// of the counter for a fixed key, ~11 VALU operations (the round-4 64-bit mix cost ~30, 1.3-1.5 us
// per attention / add+LayerNorm launch at dropout 0.1).  The key goes in twice: XORed into the
// counter, and its own fmix32 image after the first multiply, so two sites' masks are not the
// same function of XOR-shifted counters.  Trade-off, kept deliberately: 2^32 key
// streams, so over ~2^16 (site, step) pairs two may draw the same mask (birthday bound); dropout
// needs independent-looking masks per site, not cryptographic separation.
DEV uint32_t fmix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x85EBCA6Bu;
  x ^= x >> 13;
  x *= 0xC2B2AE35u;
  return x ^ (x >> 16);
}
DEV uint32_t hash3(uint64_t seed, uint32_t stream, uint64_t idx) {
  const uint32_t key = (uint32_t)seed ^ ((uint32_t)(seed >> 32) * 0x85EBCA6Bu) ^ ((stream + 1u) * 0x9E3779B9u);
  const uint32_t key2 = fmix32(key ^ 0x5BD1E995u);  // launch-uniform: hoisted out of element loops
  uint32_t x = ((uint32_t)idx * 0xCC9E2D51u) ^ ((uint32_t)(idx >> 32) * 0x1B873593u) ^ key;
  x ^= x >> 16;
  x *= 0x85EBCA6Bu;
  x ^= key2;
  x ^= x >> 13;
  x *= 0xC2B2AE35u;
  x ^= x >> 16;
  return x;
}
// Optional device-resident step counter (imgcap_set_seed_counter).  When set, every mask seed
// is mixed with *ctr at kernel run time, so a captured HIP graph draws fresh masks on each
// replay while the seeds baked into its kernel arguments stay fixed.
extern const uint64_t* g_seed_ctr;
DEV uint64_t eff_seed(uint64_t seed, const uint64_t* ctr) {
  return ctr ? seed ^ ((*ctr + 1) * 0x2545F4914F6CDD1Dull) : seed;
}
// keep iff u >= p ; returns scale 1/(1-p) or 0
DEV float dropout_scale(uint64_t seed, uint32_t stream, uint64_t idx, float p) {
  if (p <= 0.f) return 1.f;
  const float u = (hash3(seed, stream, idx) >> 8) * (1.0f / 16777216.0f);
  return u >= p ? 1.f / (1.f - p) : 0.f;
}

DEV float gelu_erf(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }
// d/dx of the erf-form GELU: Phi(x) + x phi(x)
DEV float gelu_grad(float x) {
  return 0.5f * (1.f + erff(x * 0.70710678118654752f)) + x * 0.39894228040143268f * __expf(-0.5f * x * x);
}
// erf-form GELU on two values at once, erf from Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7,
// far below the bf16 rounding of the result): packed-math polynomial (v_pk_fma_f32), native
// v_rcp_f32 / v_exp_f32 -- roughly a third of the instructions of two library erff calls
DEV f32x2 gelu_fast2(f32x2 x) {
  const f32x2 u = f32x2{fabsf(x[0]), fabsf(x[1])} * 0.70710678118654752f;
  const f32x2 den = u * 0.3275911f + 1.f;
  const f32x2 t = f32x2{__builtin_amdgcn_rcpf(den[0]), __builtin_amdgcn_rcpf(den[1])};
  f32x2 p = t * 1.061405429f + -1.453152027f;
  p = p * t + 1.421413741f;
  p = p * t + -0.284496736f;
  p = p * t + 0.254829592f;
  p = p * t;
  const f32x2 q = u * u * -1.44269504088896341f;  // -u^2 log2(e)
  const f32x2 ex = f32x2{__builtin_amdgcn_exp2f(q[0]), __builtin_amdgcn_exp2f(q[1])};
  const f32x2 e = 1.f - p * ex;                        // erf(|x| / sqrt 2)
  const f32x2 se = f32x2{copysignf(e[0], x[0]), copysignf(e[1], x[1])};
  return 0.5f * x * (1.f + se);
}
DEV float gelu_fast(float x) { return gelu_fast2(f32x2{x, 0.f})[0]; }
// erf-form GELU as x * sigmoid(x p(min(x^2, 25))): p is the weighted minimax fit (degree 2 in x^2
// over |x| <= 5) of logit(Phi(x)) / x; |GELU error| <= 5.5e-5 over all of R (fp32, checked
// against the exact form on 6e5 points in [-30, 30]; the tails saturate to x / -0), i.e. far
// below the bf16 rounding of a stored hidden value.  Seven plain VALU operations + v_exp_f32 +
// v_rcp_f32 (~40 issue cycles) against ~70 for the polynomial-erf form -- the VALU side of the
// fused MLP is what bounds it (cnblock_mlp.hip).  Kept scalar: packed f32 VALU issues slower
// beside MFMAs.  The coefficients carry the -log2(e) of the sigmoid's exp.
DEV float gelu_sig(float x) {
  const float s = fminf(x * x, 25.f);
  const float p = fmaf(fmaf(s, 9.117902926e-04f, -1.061791434e-01f), s, -2.301726884e+00f);
  return x * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(x * p));
}
DEV float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }

}  // namespace imgcap

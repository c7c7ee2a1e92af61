// MFMA fragment types and register-level operand loads shared by the GEMM kernels
// (gemm.hip) and the fused LSTM step kernels (lstm.hip).  gfx950: bf16 16x16x32, and exact
// fp32 as 8 chained 16x16x4 MFMAs over the same 8-k fragment.
#pragma once
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

template <typename T> DEV Frag<T> frag_from(const uint4& lo, const uint4& hi);
template <> DEV Frag<bf16> frag_from<bf16>(const uint4& lo, const uint4&) {
  Frag<bf16> f;
  f.v = __builtin_bit_cast(bf16x8, lo);
  return f;
}
template <> DEV Frag<float> frag_from<float>(const uint4& lo, const uint4& hi) {
  Frag<float> f;
  f.lo = __builtin_bit_cast(f32x4, lo);
  f.hi = __builtin_bit_cast(f32x4, hi);
  return f;
}

template <typename T> DEV Frag<T> lds_frag(const T* p);
template <> DEV Frag<bf16> lds_frag<bf16>(const bf16* p) { Frag<bf16> f; f.v = *(const bf16x8*)p; return f; }
template <> DEV Frag<float> lds_frag<float>(const float* p) {
  Frag<float> f; f.lo = *(const f32x4*)p; f.hi = *(const f32x4*)(p + 4); return f;
}

// zero the elements of a 16-byte vector whose index >= nvalid (0..VEC); word-wise, in registers
template <typename T>
DEV uint4 mask_tail(uint4 v, int nvalid) {
  constexpr int EPW = 4 / sizeof(T);  // elements per 32-bit word
  uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int e0 = i * EPW;
    if (EPW == 1) {
      if (e0 >= nvalid) w[i] = 0u;
    } else {
      if (e0 >= nvalid) w[i] = 0u;
      else if (e0 + 1 >= nvalid) w[i] &= 0xFFFFu;
    }
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// ---------------------------------------------------------------------------------------
// skinny operand loads (M <= 64 rows, both operands k-major): one 8-k fragment of one row per
// lane straight from global memory, clamped + zero-selected (branch-free)
template <typename T> struct SkinnyLd {
  static constexpr int H = sizeof(T) == 4 ? 2 : 1;  // 16-byte vectors per 8-element fragment
};

template <typename T>
DEV void skinny_load(uint4 (&dst)[SkinnyLd<T>::H], const T* row, int k0, int K, bool row_ok) {
  constexpr int H = SkinnyLd<T>::H;
  const uint4 zero = make_uint4(0u, 0u, 0u, 0u);
  const bool kin = row_ok && k0 < K;
  const int ck = kin ? k0 : 0;
  dst[0] = *(const uint4*)(row + ck);
  if (H == 2) dst[H - 1] = (ck + 4 < K) ? *(const uint4*)(row + ck + 4) : zero;
  if (!kin) {
#pragma unroll
    for (int h = 0; h < H; ++h) dst[h] = zero;
  } else if (k0 + 8 > K) {
    dst[0] = mask_tail<T>(dst[0], K - k0);
    if (H == 2) dst[H - 1] = mask_tail<T>(dst[H - 1], K - k0 - 4);
  }
}


// Block-cooperative skinny tile: part[0] <- A[0:16*MT, :] . Bcols^T for this block's 16 output
// columns.  `brow` is the lane's B row (column lane&15 of the block; bok false -> zeros), A is
// k-major with M valid rows.  The block's SW waves split the K steps (32 k each) evenly; each
// wave issues all loads of up to DEPTH steps before its first MFMA (one memory round trip per
// DEPTH steps; loads are unconditional -- out-of-range steps read a valid address and are
// zero-selected -- so the compiler never serialises them behind per-load branches).  The SW
// partial tiles are summed in LDS in a fixed order.  part: [SW][16*MT][20] floats.
constexpr int SKINNY_LDT = 16 + 4;
template <typename T, int MT, int SW, int DEPTH>
DEV void skinny_tile(const T* __restrict__ A, long lda, int M, const T* __restrict__ brow, bool bok, int K,
                     float (*part)[MT * 16][SKINNY_LDT]) {
  constexpr int H = SkinnyLd<T>::H;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int fr = lane & 15, fk = 8 * (lane >> 4);
  const int nks = (K + 31) / 32;
  const int per = (nks + SW - 1) / SW;
  const int ks0 = w * per, ks1 = min(nks, ks0 + per);
  const int kend = min(K, ks1 * 32);  // this wave's k range is [ks0*32, kend)
  const T* arow[MT];
  bool aok[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) {
    const int m = t * 16 + fr;
    aok[t] = m < M;
    arow[t] = A + (long)(aok[t] ? m : 0) * lda;
  }
  f32x4 acc[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int base = ks0; base < ks1; base += DEPTH) {
    uint4 ar[DEPTH][MT][H], br[DEPTH][H];
#pragma unroll
    for (int i = 0; i < DEPTH; ++i) {
      const int k0 = (base + i) * 32 + fk;
      skinny_load<T>(br[i], brow, k0, kend, bok);
#pragma unroll
      for (int t = 0; t < MT; ++t) skinny_load<T>(ar[i][t], arow[t], k0, kend, aok[t]);
    }
#pragma unroll
    for (int i = 0; i < DEPTH; ++i) {
      const Frag<T> fb = frag_from<T>(br[i][0], br[i][H - 1]);
#pragma unroll
      for (int t = 0; t < MT; ++t) mma(acc[t], frag_from<T>(ar[i][t][0], ar[i][t][H - 1]), fb);
    }
  }
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) part[w][t * 16 + 4 * (lane >> 4) + r][fr] = acc[t][r];
  __syncthreads();
  for (int e = threadIdx.x; e < MT * 16 * 16; e += 64 * SW) {
    const int r = e / 16, c = e % 16;
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < SW; ++q) s += part[q][r][c];
    part[0][r][c] = s;
  }
  __syncthreads();
}

}  // namespace imgcap

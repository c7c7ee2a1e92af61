// Masked multi-head attention of nn.TransformerDecoderLayer (transformerDecoder.py:82,104):
// self-attention (causal + key padding) and cross-attention over the 49 encoder pixels,
// with attention-probability dropout, forward and backward.
//
// Captions are <= 52 tokens and the memory is 49 pixels, so one workgroup owns one
// (batch, head) pair and keeps the whole problem on-chip: Q/K/V (and dO) tiles padded to 64
// rows in LDS, S = Q K^T, the masked softmax and P V on MFMA (bf16 16x16x32 or exact-f32
// 16x16x4); each of the 4 waves owns 16 query rows.  The forward saves the row
// log-sum-exp; the backward recomputes P from it (no N^2 storage):
//   dP~ = dO V^T,  dP = dP~ * mask/(1-p),  dS = P (dP - rowsum(P dP)),
//   dV = P~^T dO,  dQ = scale dS K,  dK = scale dS^T Q.
// Every MFMA operand is read k-contiguous from LDS; transposed images are written once.
#include "common.h"

namespace imgcap {

constexpr int HD = 64;   // head dim
constexpr int LP = 64;   // padded sequence length

template <typename T> struct MFrag;
template <> struct MFrag<bf16> { bf16x8 v; };
template <> struct MFrag<float> { f32x4 lo, hi; };
DEV void mfma16(f32x4& acc, const MFrag<bf16>& a, const MFrag<bf16>& b) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.v, b.v, acc, 0, 0, 0);
}
DEV void mfma16(f32x4& acc, const MFrag<float>& a, const MFrag<float>& b) {
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.lo[kk], b.lo[kk], acc, 0, 0, 0);
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.hi[kk], b.hi[kk], acc, 0, 0, 0);
}
template <typename T> DEV MFrag<T> mfrag(const T* p);
template <> DEV MFrag<bf16> mfrag<bf16>(const bf16* p) { MFrag<bf16> f; f.v = *(const bf16x8*)p; return f; }
template <> DEV MFrag<float> mfrag<float>(const float* p) {
  MFrag<float> f; f.lo = *(const f32x4*)p; f.hi = *(const f32x4*)(p + 4); return f;
}

template <typename T> struct Img {
  static constexpr int LD = HD + 16 / (int)sizeof(T);  // +16 bytes per row
  static constexpr int ELEMS = LP * LD;
};

// C[16 rows of this wave][64 cols] = sum_k A[row][k] * B[col][k]   (both k-contiguous, K = 64)
template <typename T>
DEV void wave_mm(f32x4 (&acc)[4], const T* A, const T* Bm, int row0, int lane) {
  constexpr int LD = Img<T>::LD;
  const int fr = lane & 15, fk = 8 * (lane >> 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < HD; ks += 32) {
    const MFrag<T> a = mfrag<T>(A + (row0 + fr) * LD + ks + fk);
#pragma unroll
    for (int j = 0; j < 4; ++j) mfma16(acc[j], a, mfrag<T>(Bm + (j * 16 + fr) * LD + ks + fk));
  }
}

// Staging of a [L][HD] head slice (row stride ld) into an LDS image, rows >= L zero.  Split in
// two so a kernel issues the global loads of ALL its slices (and its mask / lse reads) before
// the first LDS store: one memory round trip instead of one per slice and loop trip.  256
// threads, 16-byte vectors: 2 per thread per slice (bf16), 4 (fp32).
template <typename T> struct RowVecs {
  static constexpr int VEC = 16 / sizeof(T), NV = HD / VEC, PER = LP * NV / 256;
  uint4 v[PER];
};
template <typename T>
DEV void load_rows(RowVecs<T>& rv, const T* src, long ld, int L) {
  using R = RowVecs<T>;
#pragma unroll
  for (int i = 0; i < R::PER; ++i) {
    const int e = threadIdx.x + i * 256;
    const int r = e / R::NV, c = (e % R::NV) * R::VEC;
    rv.v[i] = r < L ? *(const uint4*)(src + (long)r * ld + c) : make_uint4(0u, 0u, 0u, 0u);
  }
}
template <typename T>
DEV void store_rows(T* img, const RowVecs<T>& rv) {
  using R = RowVecs<T>;
  constexpr int LD = Img<T>::LD;
#pragma unroll
  for (int i = 0; i < R::PER; ++i) {
    const int e = threadIdx.x + i * 256;
    *(uint4*)(img + (e / R::NV) * LD + (e % R::NV) * R::VEC) = rv.v[i];
  }
}
// transposed image: img[c][r] = row r, column c
template <typename T>
DEV void store_rows_t(T* img, const RowVecs<T>& rv) {
  using R = RowVecs<T>;
  constexpr int LD = Img<T>::LD;
#pragma unroll
  for (int i = 0; i < R::PER; ++i) {
    const int e = threadIdx.x + i * 256;
    const int r = e / R::NV, c = (e % R::NV) * R::VEC;
    const T* x = (const T*)&rv.v[i];
#pragma unroll
    for (int k = 0; k < R::VEC; ++k) img[(c + k) * LD + r] = x[k];
  }
}
// key-padding flags of batch row b (1 = masked) for the block's LDS copy
DEV unsigned char key_pad_flag(const imgcap_mha_desc& d, int b, int j) {
  return (j < d.Lk && d.key_ids && d.key_ids[(long)b * d.Lk + j] == d.pad_id) ? 1 : 0;
}
// transpose an LDS image
template <typename T>
DEV void lds_transpose(T* dst, const T* src) {
  constexpr int LD = Img<T>::LD;
  for (int e = threadIdx.x; e < LP * HD; e += blockDim.x) {
    const int r = e / HD, c = e % HD;
    dst[c * LD + r] = src[r * LD + c];
  }
}

DEV float row_max16(float v) {
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
DEV float row_sum16(float v) {
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o, 64);
  return v;
}

DEV bool key_masked(const imgcap_mha_desc& d, const unsigned char* kpad, int i, int j) {
  if (j >= d.Lk) return true;
  if (d.causal && j > i) return true;
  return kpad[j] != 0;
}

// ------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void mha_fwd_kernel(imgcap_mha_desc d, const uint64_t* seed_ctr) {
  if (d.drop_p > 0.f) d.seed = eff_seed(d.seed, seed_ctr);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int LD = Img<T>::LD;
  T* Qs = (T*)smem;
  T* Ks = Qs + Img<T>::ELEMS;   // reused for P~ after S is done
  T* Vt = Ks + Img<T>::ELEMS;
  const int bh = blockIdx.x, b = bh / d.H, h = bh % d.H;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long kvr = d.kv_rows ? d.kv_rows : d.Lk;  // batch stride of k / v in rows
  const T* q = (const T*)d.q + (long)b * d.Lq * d.ldq + h * HD;
  const T* k = (const T*)d.k + (long)b * kvr * d.ldk + h * HD;
  const T* v = (const T*)d.v + (long)b * kvr * d.ldv + h * HD;
  __shared__ unsigned char kpad[LP];
  {
    RowVecs<T> qv, kv, vv;
    load_rows<T>(qv, q, d.ldq, d.Lq);
    load_rows<T>(kv, k, d.ldk, d.Lk);
    load_rows<T>(vv, v, d.ldv, d.Lk);
    const unsigned char kp = threadIdx.x < LP ? key_pad_flag(d, b, threadIdx.x) : 0;
    store_rows<T>(Qs, qv);
    store_rows<T>(Ks, kv);
    store_rows_t<T>(Vt, vv);
    if (threadIdx.x < LP) kpad[threadIdx.x] = kp;
  }
  __syncthreads();
  f32x4 s[4];
  const int row0 = w * 16;
  wave_mm<T>(s, Qs, Ks, row0, lane);
  // masked, scaled, row softmax in registers: lane holds rows row0+4*(lane>>4)+r, cols j*16+(lane&15)
  float lse_r[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = row0 + 4 * (lane >> 4) + r;
    float m = -INFINITY;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = j * 16 + (lane & 15);
      const float x = key_masked(d, kpad, i, col) ? -INFINITY : s[j][r] * d.scale;
      s[j][r] = x;
      m = fmaxf(m, x);
    }
    m = row_max16(m);
    if (m == -INFINITY) m = 0.f;
    float sum = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float e = __expf(s[j][r] - m);
      s[j][r] = e;
      sum += e;
    }
    sum = row_sum16(sum);
    const float inv = sum > 0.f ? 1.f / sum : 0.f;
    lse_r[r] = m + logf(sum > 0.f ? sum : 1.f);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = j * 16 + (lane & 15);
      float p = s[j][r] * inv;
      if (d.drop_p > 0.f && i < d.Lq && col < d.Lk)
        p *= dropout_scale(d.seed, d.drop_stream, (((uint64_t)bh * d.Lq + i) * d.Lk + col), d.drop_p);
      s[j][r] = p;
      if (d.probs && i < d.Lq && col < d.Lk) d.probs[((long)bh * d.Lq + i) * d.Lk + col] = p;
    }
  }
  __syncthreads();  // everyone is done reading Ks: reuse it for P~
  T* Ps = Ks;
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int j = 0; j < 4; ++j) Ps[(row0 + 4 * (lane >> 4) + r) * LD + j * 16 + (lane & 15)] = from_f<T>(s[j][r]);
  __syncthreads();
  f32x4 o[4];
  wave_mm<T>(o, Ps, Vt, row0, lane);
  T* out = (T*)d.o + (long)b * d.Lq * d.ldo + h * HD;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = row0 + 4 * (lane >> 4) + r;
    if (i < d.Lq) {
#pragma unroll
      for (int j = 0; j < 4; ++j) out[(long)i * d.ldo + j * 16 + (lane & 15)] = from_f<T>(o[j][r]);
      if ((lane & 15) == 0) d.lse[(long)bh * d.Lq + i] = lse_r[r];
    }
  }
}

// ------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void mha_bwd_kernel(imgcap_mha_desc d, const uint64_t* seed_ctr) {
  if (d.drop_p > 0.f) d.seed = eff_seed(d.seed, seed_ctr);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int LD = Img<T>::LD;
  constexpr int NE = Img<T>::ELEMS;
  T* Qs = (T*)smem;
  T* Ks = Qs + NE;
  T* Vs = Ks + NE;
  T* dOs = Vs + NE;
  T* X1 = dOs + NE;
  T* X2 = X1 + NE;
  const int bh = blockIdx.x, b = bh / d.H, h = bh % d.H;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const T* q = (const T*)d.q + (long)b * d.Lq * d.ldq + h * HD;
  const T* k = (const T*)d.k + (long)b * d.Lk * d.ldk + h * HD;
  const T* v = (const T*)d.v + (long)b * d.Lk * d.ldv + h * HD;
  const T* dO = (const T*)d.dout + (long)b * d.Lq * d.lddo + h * HD;
  __shared__ unsigned char kpad[LP];
  const int row0 = w * 16;
  float lse_r[4];
  {
    RowVecs<T> qv, kv, vv, ov;
    load_rows<T>(qv, q, d.ldq, d.Lq);
    load_rows<T>(kv, k, d.ldk, d.Lk);
    load_rows<T>(vv, v, d.ldv, d.Lk);
    load_rows<T>(ov, dO, d.lddo, d.Lq);
    const unsigned char kp = threadIdx.x < LP ? key_pad_flag(d, b, threadIdx.x) : 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = row0 + 4 * (lane >> 4) + r;
      lse_r[r] = i < d.Lq ? d.lse[(long)bh * d.Lq + i] : 0.f;
    }
    store_rows<T>(Qs, qv);
    store_rows<T>(Ks, kv);
    store_rows<T>(Vs, vv);
    store_rows<T>(dOs, ov);
    if (threadIdx.x < LP) kpad[threadIdx.x] = kp;
  }
  __syncthreads();
  f32x4 p[4], dp[4];
  wave_mm<T>(p, Qs, Ks, row0, lane);    // S
  wave_mm<T>(dp, dOs, Vs, row0, lane);  // dP~ = dO V^T
  // P from the saved lse; P~ = P * mask; dP = dP~ * mask; dS = P (dP - rowsum(P dP))
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = row0 + 4 * (lane >> 4) + r;
    const float lse = lse_r[r];
    float dot = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = j * 16 + (lane & 15);
      const bool masked = i >= d.Lq || key_masked(d, kpad, i, col);
      const float pr = masked ? 0.f : __expf(p[j][r] * d.scale - lse);
      const float ms = (d.drop_p > 0.f && !masked)
                           ? dropout_scale(d.seed, d.drop_stream, (((uint64_t)bh * d.Lq + i) * d.Lk + col), d.drop_p)
                           : 1.f;
      const float dpv = dp[j][r] * ms;
      dot += pr * dpv;
      p[j][r] = pr;         // P (pre-dropout) for now
      dp[j][r] = dpv;       // dP
    }
    dot = row_sum16(dot);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = j * 16 + (lane & 15);
      const float pr = p[j][r];
      dp[j][r] = pr * (dp[j][r] - dot);  // dS
      const bool masked = i >= d.Lq || key_masked(d, kpad, i, col);
      const float ms = (d.drop_p > 0.f && !masked)
                           ? dropout_scale(d.seed, d.drop_stream, (((uint64_t)bh * d.Lq + i) * d.Lk + col), d.drop_p)
                           : 1.f;
      p[j][r] = pr * ms;                 // P~
    }
  }
  // ---- dV = P~^T dO ----
  // X1[j][i] = P~[i][j]; X2[c][i] = dO[i][c]
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int j = 0; j < 4; ++j) X1[(j * 16 + (lane & 15)) * LD + row0 + 4 * (lane >> 4) + r] = from_f<T>(p[j][r]);
  lds_transpose<T>(X2, dOs);
  __syncthreads();
  f32x4 acc[4];
  wave_mm<T>(acc, X1, X2, row0, lane);
  {
    T* dv = (T*)d.dv + (long)b * d.Lk * d.lddv + h * HD;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = row0 + 4 * (lane >> 4) + r;
      if (j < d.Lk)
#pragma unroll
        for (int c = 0; c < 4; ++c) dv[(long)j * d.lddv + c * 16 + (lane & 15)] = from_f<T>(acc[c][r]);
    }
  }
  __syncthreads();
  // ---- dK = scale dS^T Q ----
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int j = 0; j < 4; ++j) X1[(j * 16 + (lane & 15)) * LD + row0 + 4 * (lane >> 4) + r] = from_f<T>(dp[j][r]);
  lds_transpose<T>(X2, Qs);
  __syncthreads();
  wave_mm<T>(acc, X1, X2, row0, lane);
  {
    T* dk = (T*)d.dk + (long)b * d.Lk * d.lddk + h * HD;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = row0 + 4 * (lane >> 4) + r;
      if (j < d.Lk)
#pragma unroll
        for (int c = 0; c < 4; ++c) dk[(long)j * d.lddk + c * 16 + (lane & 15)] = from_f<T>(acc[c][r] * d.scale);
    }
  }
  __syncthreads();
  // ---- dQ = scale dS K ----
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int j = 0; j < 4; ++j) X1[(row0 + 4 * (lane >> 4) + r) * LD + j * 16 + (lane & 15)] = from_f<T>(dp[j][r]);
  lds_transpose<T>(X2, Ks);
  __syncthreads();
  wave_mm<T>(acc, X1, X2, row0, lane);
  {
    T* dq = (T*)d.dq + (long)b * d.Lq * d.lddq + h * HD;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = row0 + 4 * (lane >> 4) + r;
      if (i < d.Lq)
#pragma unroll
        for (int c = 0; c < 4; ++c) dq[(long)i * d.lddq + c * 16 + (lane & 15)] = from_f<T>(acc[c][r] * d.scale);
    }
  }
}

// ---- bf16: natural row images, transposed operands read by ds_read_b64_tr_b16 ----------------
// Every head slice sits in LDS as it is in memory, [64 rows][64 columns] (128-byte rows), its
// 16-byte slots XOR-swizzled by row bits 1 and 3: both operand reads are then conflict-free
// (k-contiguous fragments by ds_read_b128: 4 LDS cycles a wave-instruction; fragments whose k
// runs down the image by ds_read_b64_tr_b16: 2).  No transposed copies (the round-4 kernels
// built 1 (fwd) / 3 (bwd) by 2-byte element moves at 2.4-3 conflict cycles per LDS instruction)
// and one (fwd) / two (bwd) barriers.  MFMAs run as D^T = B^T A^T, so a lane ends with one row
// and 4 consecutive columns: softmax row sums over 4 lanes, 8-byte stores of P / dS / outputs.
typedef short mi_v4s16 __attribute__((ext_vector_type(4)));
typedef short mi_v8s16 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) mi_v4s16 mi_lds_v4s16;
constexpr int MI_IMG = LP * HD * 2;  // bytes of one image

DEV int mi_swz(int r) { return (((r >> 1) & 1) * 2) ^ (((r >> 3) & 1) * 4); }
DEV int mi_off(int r, int c) { return r * 128 + (((c >> 3) ^ mi_swz(r)) << 4) + ((c & 7) << 1); }

// operand rows row0 + (lane & 15), k = 32 kk + 8 (lane >> 4) + 0..7, from an image whose rows are
// the operand's rows
DEV bf16x8 mi_frag_k(const char* img, int row0, int kk, int lane) {
  const int r = row0 + (lane & 15);
  return *(const bf16x8*)(img + r * 128 + (((4 * kk + (lane >> 4)) ^ mi_swz(r)) << 4));
}
// the same fragment from an image whose COLUMNS are the operand's rows (k down the image): lane
// 4q+p of a 16-lane group reads 4 columns of image row 8g+q (+4), the hardware transpose hands
// lane i column col0 + i
DEV bf16x8 mi_frag_t(const char* img, int col0, int kk, int lane) {
  const int fr = lane & 15, g = lane >> 4;
  const int kr = kk * 32 + 8 * g + (fr >> 2), col = col0 + 4 * (fr & 3);
  const mi_v4s16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((mi_lds_v4s16*)(img + mi_off(kr, col)));
  const mi_v4s16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((mi_lds_v4s16*)(img + mi_off(kr + 4, col)));
  const mi_v8s16 all = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, all);
}
DEV void mi_store(char* img, const RowVecs<bf16>& rv) {
#pragma unroll
  for (int i = 0; i < RowVecs<bf16>::PER; ++i) {
    const int e = threadIdx.x + i * 256, r = e >> 3;
    *(uint4*)(img + r * 128 + (((e & 7) ^ mi_swz(r)) << 4)) = rv.v[i];
  }
}
// D^T[xrows][yrows] over k = 0..63: acc[cb] = sum_k X[16 cb + ..][k] Y[y0 + ..][k] for the 4
// 16-row blocks of X (both given as fragment readers)
#define MI_MM(acc, XFRAG, YFRAG)                                                   \
  do {                                                                             \
    _Pragma("unroll") for (int j_ = 0; j_ < 4; ++j_) acc[j_] = f32x4{0.f, 0.f, 0.f, 0.f}; \
    _Pragma("unroll") for (int kk_ = 0; kk_ < 2; ++kk_) {                          \
      const bf16x8 y_ = YFRAG(kk_);                                                \
      _Pragma("unroll") for (int j_ = 0; j_ < 4; ++j_)                             \
        acc[j_] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(XFRAG(j_, kk_), y_, acc[j_], 0, 0, 0); \
    }                                                                              \
  } while (0)
// The probability / dS images (P~ in the forward; P~ and dS in the backward) are written by the
// MFMA epilogue, one 8-byte piece (4 columns) of 16 different rows per 16-lane group: in the row
// images above those 16 pieces fall on 4 bank pairs (ds_write_b64 banks by (a/4) mod 32), a 4-way
// conflict (SQ: 0.87 / 0.92 conflict cycles per LDS instruction, round 6).  These images swizzle
// both the 16-byte slot (by row bits 0, 1, 3) and the 8-byte half inside it (by row bit 2): the
// 16 rows of a write group land on 16 distinct 8-byte positions of the 128-byte bank window, and
// the k-contiguous (ds_read_b128, aligned slot, halves swapped back in registers) and transposed
// (ds_read_b64_tr_b16) operand reads stay conflict-free (bank model: tools/lds_bank_model.py).
DEV int mp_sa(int r) { return (r & 3) | ((r >> 1) & 4); }
DEV int mp_sb(int r) { return (r >> 2) & 1; }
DEV int mp_off(int r, int c) { return r * 128 + (((c >> 3) ^ mp_sa(r)) << 4) + ((((c >> 2) & 1) ^ mp_sb(r)) << 3) + ((c & 3) << 1); }
DEV bf16x8 mp_frag_k(const char* img, int row0, int kk, int lane) {
  const int r = row0 + (lane & 15);
  const uint4 v = *(const uint4*)(img + r * 128 + (((4 * kk + (lane >> 4)) ^ mp_sa(r)) << 4));
  const uint4 w = mp_sb(r) ? make_uint4(v.z, v.w, v.x, v.y) : v;
  return __builtin_bit_cast(bf16x8, w);
}
DEV bf16x8 mp_frag_t(const char* img, int col0, int kk, int lane) {
  const int fr = lane & 15, g = lane >> 4;
  const int kr = kk * 32 + 8 * g + (fr >> 2), col = col0 + 4 * (fr & 3);
  const mi_v4s16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((mi_lds_v4s16*)(img + mp_off(kr, col)));
  const mi_v4s16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((mi_lds_v4s16*)(img + mp_off(kr + 4, col)));
  const mi_v8s16 all = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, all);
}
DEV uint2 mi_pack4(float a, float b, float c, float e) {
  const bf16x2 lo = {(bf16)a, (bf16)b}, hi = {(bf16)c, (bf16)e};
  return make_uint2(__builtin_bit_cast(uint32_t, lo), __builtin_bit_cast(uint32_t, hi));
}
DEV float mi_row_max(float v) { return fmaxf(fmaxf(v, __shfl_xor(v, 16, 64)), fmaxf(__shfl_xor(v, 32, 64), __shfl_xor(v, 48, 64))); }
DEV float mi_row_sum(float v) {
  v += __shfl_xor(v, 16, 64);
  return v + __shfl_xor(v, 32, 64);
}

__global__ __launch_bounds__(256) void mha_fwd_bf16_kernel(imgcap_mha_desc d, const uint64_t* seed_ctr) {
  if (d.drop_p > 0.f) d.seed = eff_seed(d.seed, seed_ctr);
  __shared__ __attribute__((aligned(16))) char sm[4 * MI_IMG];
  __shared__ unsigned char kpad[LP];
  char* Qs = sm;
  char* Ks = sm + MI_IMG;
  char* Vs = sm + 2 * MI_IMG;
  char* Ps = sm + 3 * MI_IMG;
  const int bh = blockIdx.x, b = bh / d.H, h = bh % d.H;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, fr = lane & 15, fq = lane >> 4;
  const long kvr = d.kv_rows ? d.kv_rows : d.Lk;
  const bf16* q = (const bf16*)d.q + (long)b * d.Lq * d.ldq + h * HD;
  const bf16* k = (const bf16*)d.k + (long)b * kvr * d.ldk + h * HD;
  const bf16* v = (const bf16*)d.v + (long)b * kvr * d.ldv + h * HD;
  {
    RowVecs<bf16> qv, kv, vv;
    load_rows<bf16>(qv, q, d.ldq, d.Lq);
    load_rows<bf16>(kv, k, d.ldk, d.Lk);
    load_rows<bf16>(vv, v, d.ldv, d.Lk);
    const unsigned char kp = threadIdx.x < LP ? key_pad_flag(d, b, threadIdx.x) : 0;
    mi_store(Qs, qv);
    mi_store(Ks, kv);
    mi_store(Vs, vv);
    if (threadIdx.x < LP) kpad[threadIdx.x] = kp;
  }
  __syncthreads();
  const int row0 = 16 * w, i = row0 + fr;  // this lane's query row; keys j = 16 jb + 4 fq + r
  f32x4 s[4];
#define XK(jb, kk) mi_frag_k(Ks, 16 * (jb), kk, lane)
#define YQ(kk) mi_frag_k(Qs, row0, kk, lane)
  MI_MM(s, XK, YQ);
#undef XK
#undef YQ
  float m = -INFINITY;
#pragma unroll
  for (int jb = 0; jb < 4; ++jb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = 16 * jb + 4 * fq + r;
      const float x = key_masked(d, kpad, i, j) ? -INFINITY : s[jb][r] * d.scale;
      s[jb][r] = x;
      m = fmaxf(m, x);
    }
  m = mi_row_max(m);
  if (m == -INFINITY) m = 0.f;
  float sum = 0.f;
#pragma unroll
  for (int jb = 0; jb < 4; ++jb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float e = __expf(s[jb][r] - m);
      s[jb][r] = e;
      sum += e;
    }
  sum = mi_row_sum(sum);
  const float inv = sum > 0.f ? 1.f / sum : 0.f;
  const float lse = m + logf(sum > 0.f ? sum : 1.f);
#pragma unroll
  for (int jb = 0; jb < 4; ++jb) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = 16 * jb + 4 * fq + r;
      float pv = s[jb][r] * inv;
      if (d.drop_p > 0.f && i < d.Lq && j < d.Lk)
        pv *= dropout_scale(d.seed, d.drop_stream, (((uint64_t)bh * d.Lq + i) * d.Lk + j), d.drop_p);
      s[jb][r] = pv;
      if (d.probs && i < d.Lq && j < d.Lk) d.probs[((long)bh * d.Lq + i) * d.Lk + j] = pv;
    }
    *(uint2*)(Ps + mp_off(i, 16 * jb + 4 * fq)) = mi_pack4(s[jb][0], s[jb][1], s[jb][2], s[jb][3]);
  }
  // a wave reads back only its own 16 rows of P~: LDS operations of one wave complete in order
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
  f32x4 o[4];
#define XV(cb, kk) mi_frag_t(Vs, 16 * (cb), kk, lane)
#define YP(kk) mp_frag_k(Ps, row0, kk, lane)
  MI_MM(o, XV, YP);
#undef XV
#undef YP
  if (i < d.Lq) {
    bf16* out = (bf16*)d.o + ((long)b * d.Lq + i) * d.ldo + h * HD;
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) *(uint2*)(out + 16 * cb + 4 * fq) = mi_pack4(o[cb][0], o[cb][1], o[cb][2], o[cb][3]);
    if (fq == 0) d.lse[(long)bh * d.Lq + i] = lse;
  }
}

__global__ __launch_bounds__(256) void mha_bwd_bf16_kernel(imgcap_mha_desc d, const uint64_t* seed_ctr) {
  if (d.drop_p > 0.f) d.seed = eff_seed(d.seed, seed_ctr);
  __shared__ __attribute__((aligned(16))) char sm[6 * MI_IMG];
  __shared__ unsigned char kpad[LP];
  char* Qs = sm;
  char* Ks = sm + MI_IMG;
  char* Vs = sm + 2 * MI_IMG;
  char* dOs = sm + 3 * MI_IMG;
  char* Pt = sm + 4 * MI_IMG;   // P~ (dropped-out probabilities)
  char* dSs = sm + 5 * MI_IMG;  // dS (unscaled)
  const int bh = blockIdx.x, b = bh / d.H, h = bh % d.H;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, fr = lane & 15, fq = lane >> 4;
  const bf16* q = (const bf16*)d.q + (long)b * d.Lq * d.ldq + h * HD;
  const bf16* k = (const bf16*)d.k + (long)b * d.Lk * d.ldk + h * HD;
  const bf16* v = (const bf16*)d.v + (long)b * d.Lk * d.ldv + h * HD;
  const bf16* dO = (const bf16*)d.dout + (long)b * d.Lq * d.lddo + h * HD;
  const int row0 = 16 * w, i = row0 + fr;  // query row of the S / dP phase
  float lse;
  {
    RowVecs<bf16> qv, kv, vv, ov;
    load_rows<bf16>(qv, q, d.ldq, d.Lq);
    load_rows<bf16>(kv, k, d.ldk, d.Lk);
    load_rows<bf16>(vv, v, d.ldv, d.Lk);
    load_rows<bf16>(ov, dO, d.lddo, d.Lq);
    const unsigned char kp = threadIdx.x < LP ? key_pad_flag(d, b, threadIdx.x) : 0;
    lse = i < d.Lq ? d.lse[(long)bh * d.Lq + i] : 0.f;
    mi_store(Qs, qv);
    mi_store(Ks, kv);
    mi_store(Vs, vv);
    mi_store(dOs, ov);
    if (threadIdx.x < LP) kpad[threadIdx.x] = kp;
  }
  __syncthreads();
  f32x4 p[4], dp[4];
#define XK(jb, kk) mi_frag_k(Ks, 16 * (jb), kk, lane)
#define XV(jb, kk) mi_frag_k(Vs, 16 * (jb), kk, lane)
#define YQ(kk) mi_frag_k(Qs, row0, kk, lane)
#define YO(kk) mi_frag_k(dOs, row0, kk, lane)
  MI_MM(p, XK, YQ);   // S
  MI_MM(dp, XV, YO);  // dP~ = dO V^T
#undef XK
#undef XV
#undef YQ
#undef YO
  // P from the saved lse; P~ = P * mask; dP = dP~ * mask; dS = P (dP - rowsum(P dP))
  float ms[4][4];
  float dot = 0.f;
#pragma unroll
  for (int jb = 0; jb < 4; ++jb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = 16 * jb + 4 * fq + r;
      const bool masked = i >= d.Lq || key_masked(d, kpad, i, j);
      const float pr = masked ? 0.f : __expf(p[jb][r] * d.scale - lse);
      ms[jb][r] = (d.drop_p > 0.f && !masked)
                      ? dropout_scale(d.seed, d.drop_stream, (((uint64_t)bh * d.Lq + i) * d.Lk + j), d.drop_p)
                      : 1.f;
      const float dpv = dp[jb][r] * ms[jb][r];
      dot += pr * dpv;
      p[jb][r] = pr;
      dp[jb][r] = dpv;
    }
  dot = mi_row_sum(dot);
#pragma unroll
  for (int jb = 0; jb < 4; ++jb) {
    float ds[4], pt[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      ds[r] = p[jb][r] * (dp[jb][r] - dot);
      pt[r] = p[jb][r] * ms[jb][r];
    }
    *(uint2*)(Pt + mp_off(i, 16 * jb + 4 * fq)) = mi_pack4(pt[0], pt[1], pt[2], pt[3]);
    *(uint2*)(dSs + mp_off(i, 16 * jb + 4 * fq)) = mi_pack4(ds[0], ds[1], ds[2], ds[3]);
  }
  __syncthreads();  // dV / dK sum over every wave's query rows
  const int j = row0 + fr;  // key row of the dV / dK phase
  f32x4 acc[4];
  // dV[j][c] = sum_i P~[i][j] dO[i][c]
#define XO(cb, kk) mi_frag_t(dOs, 16 * (cb), kk, lane)
#define YP(kk) mp_frag_t(Pt, row0, kk, lane)
  MI_MM(acc, XO, YP);
#undef XO
#undef YP
  if (j < d.Lk) {
    bf16* dv = (bf16*)d.dv + ((long)b * d.Lk + j) * d.lddv + h * HD;
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) *(uint2*)(dv + 16 * cb + 4 * fq) = mi_pack4(acc[cb][0], acc[cb][1], acc[cb][2], acc[cb][3]);
  }
  // dK[j][c] = scale sum_i dS[i][j] Q[i][c]
#define XQ(cb, kk) mi_frag_t(Qs, 16 * (cb), kk, lane)
#define YS(kk) mp_frag_t(dSs, row0, kk, lane)
  MI_MM(acc, XQ, YS);
#undef XQ
#undef YS
  if (j < d.Lk) {
    bf16* dk = (bf16*)d.dk + ((long)b * d.Lk + j) * d.lddk + h * HD;
    const float sc = d.scale;
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
      *(uint2*)(dk + 16 * cb + 4 * fq) = mi_pack4(acc[cb][0] * sc, acc[cb][1] * sc, acc[cb][2] * sc, acc[cb][3] * sc);
  }
  // dQ[i][c] = scale sum_j dS[i][j] K[j][c]
#define XKT(cb, kk) mi_frag_t(Ks, 16 * (cb), kk, lane)
#define YS(kk) mp_frag_k(dSs, row0, kk, lane)
  MI_MM(acc, XKT, YS);
#undef XKT
#undef YS
  if (i < d.Lq) {
    bf16* dq = (bf16*)d.dq + ((long)b * d.Lq + i) * d.lddq + h * HD;
    const float sc = d.scale;
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
      *(uint2*)(dq + 16 * cb + 4 * fq) = mi_pack4(acc[cb][0] * sc, acc[cb][1] * sc, acc[cb][2] * sc, acc[cb][3] * sc);
  }
}
#undef MI_MM

static int check(const imgcap_mha_desc* d) {
  IMGCAP_REQUIRE(d != nullptr, "mha desc NULL");
  IMGCAP_REQUIRE(d->dh == HD, "mha: head dim must be 64");
  IMGCAP_REQUIRE(d->Lq > 0 && d->Lq <= LP && d->Lk > 0 && d->Lk <= LP, "mha: sequence lengths must be in [1, 64]");
  IMGCAP_REQUIRE(d->kv_rows == 0 || d->kv_rows >= d->Lk, "mha: kv_rows must be 0 or >= Lk");
  const int vec = d->dtype == IMGCAP_F32 ? 4 : 8;
  IMGCAP_REQUIRE(d->ldq % vec == 0 && d->ldk % vec == 0 && d->ldv % vec == 0 && aligned16(d->q) && aligned16(d->k) &&
                     aligned16(d->v),
                 "mha: q/k/v must be 16-byte aligned with 16-byte row strides");
  return 0;
}
// the bf16 kernels write 4 consecutive outputs per lane as one 8-byte store
static bool out_ok(int dtype, const void* p, long ld) {
  return dtype != IMGCAP_BF16 || (((uintptr_t)p & 7) == 0 && ld % 4 == 0);
}

}  // namespace imgcap

using namespace imgcap;

extern "C" int imgcap_mha_fwd(const imgcap_mha_desc* d, void* stream) {
  if (int rc = check(d)) return rc;
  IMGCAP_REQUIRE(out_ok(d->dtype, d->o, d->ldo), "mha fwd: bf16 o must be 8-byte aligned with ldo % 4 == 0");
  const dim3 grid(d->B * d->H);
  if (d->dtype == IMGCAP_BF16)
    hipLaunchKernelGGL(mha_fwd_bf16_kernel, grid, dim3(256), 0, (hipStream_t)stream, *d, g_seed_ctr);
  else
    hipLaunchKernelGGL(mha_fwd_kernel<float>, grid, dim3(256), 3 * Img<float>::ELEMS * sizeof(float),
                       (hipStream_t)stream, *d, g_seed_ctr);
  IMGCAP_CHECK_LAUNCH("imgcap_mha_fwd");
  return 0;
}

extern "C" int imgcap_mha_bwd(const imgcap_mha_desc* d, void* stream) {
  if (int rc = check(d)) return rc;
  IMGCAP_REQUIRE(d->kv_rows == 0 || d->kv_rows == d->Lk, "mha bwd: kv_rows (key/value cache stride) is fwd-only");
  const int vec = d->dtype == IMGCAP_F32 ? 4 : 8;
  IMGCAP_REQUIRE(d->lddo % vec == 0 && aligned16(d->dout), "mha bwd: dout alignment");
  IMGCAP_REQUIRE(out_ok(d->dtype, d->dq, d->lddq) && out_ok(d->dtype, d->dk, d->lddk) && out_ok(d->dtype, d->dv, d->lddv),
                 "mha bwd: bf16 dq / dk / dv must be 8-byte aligned with pitches % 4 == 0");
  const dim3 grid(d->B * d->H);
  static bool attr_set = false;
  if (!attr_set) {  // the f32 backward needs > 64 KiB of dynamic LDS
    if (hipFuncSetAttribute((const void*)mha_bwd_kernel<float>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            6 * Img<float>::ELEMS * sizeof(float)) != hipSuccess)
      return fail(IMGCAP_EINVAL, "mha bwd: cannot raise the LDS limit");
    attr_set = true;
  }
  if (d->dtype == IMGCAP_BF16)
    hipLaunchKernelGGL(mha_bwd_bf16_kernel, grid, dim3(256), 0, (hipStream_t)stream, *d, g_seed_ctr);
  else
    hipLaunchKernelGGL(mha_bwd_kernel<float>, grid, dim3(256), 6 * Img<float>::ELEMS * sizeof(float),
                       (hipStream_t)stream, *d, g_seed_ctr);
  IMGCAP_CHECK_LAUNCH("imgcap_mha_bwd");
  return 0;
}

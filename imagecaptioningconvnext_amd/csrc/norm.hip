// Row LayerNorm of a (dropout-)residual sum: the post-norm blocks of
// nn.TransformerDecoderLayer (transformerDecoder.py:82,104): x = LN(x + dropout(sublayer(x))).
// One wave per row (cols <= 1024); a lane owns granules of G consecutive columns (16-byte
// accesses when the row pitch allows), and the row stays in registers between the mean and
// variance passes, so HBM traffic is one read of each input and one write of s and y.
#include <algorithm>
#include <initializer_list>

#include "common.h"

namespace imgcap {

constexpr int LN_MAXC = 2048;

template <typename T, int G, int MAXC>
__global__ __launch_bounds__(256) void add_ln_fwd_kernel(int rows, int cols, const T* __restrict__ x,
                                                         const T* __restrict__ r, float p, uint64_t seed0,
                                                         const uint64_t* seed_ctr, uint32_t stream_id,
                                                         const float* __restrict__ g, const float* __restrict__ b,
                                                         float eps, T* __restrict__ s_out, T* __restrict__ y,
                                                         float* __restrict__ mean_o, float* __restrict__ rstd_o) {
  constexpr int MAXJ = MAXC / (64 * G);
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const uint64_t seed = (r && p > 0.f) ? eff_seed(seed0, seed_ctr) : seed0;
  float v[MAXJ][G];
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) {
    const int c0 = G * (lane + 64 * j);
#pragma unroll
    for (int e = 0; e < G; ++e) v[j][e] = 0.f;
    if (c0 < cols) {
      const long idx = (long)row * cols + c0;
      float xv[G];
      ld_g<T, G>(x + idx, xv);
      if (r) {
        float rv[G];
        ld_g<T, G>(r + idx, rv);
#pragma unroll
        for (int e = 0; e < G; ++e) xv[e] += rv[e] * dropout_scale(seed, stream_id, idx + e, p);
      }
      if (s_out) st_g<T, G>(s_out + idx, xv);
#pragma unroll
      for (int e = 0; e < G; ++e) {
        v[j][e] = to_f(from_f<T>(xv[e]));  // LN sees exactly the stored s (bwd recomputes from it)
        sum += v[j][e];
      }
    }
  }
  const float mean = wave_sum(sum) / cols;
  float sq = 0.f;
#pragma unroll
  for (int j = 0; j < MAXJ; ++j)
    if (G * (lane + 64 * j) < cols)
#pragma unroll
      for (int e = 0; e < G; ++e) { const float d = v[j][e] - mean; sq += d * d; }
  const float rstd = rsqrtf(wave_sum(sq) / cols + eps);
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) {
    const int c0 = G * (lane + 64 * j);
    if (c0 < cols) {
      float o[G];
#pragma unroll
      for (int e = 0; e < G; ++e) o[e] = (v[j][e] - mean) * rstd * g[c0 + e] + b[c0 + e];
      st_g<T, G>(y + (long)row * cols + c0, o);
    }
  }
  if (lane == 0) { mean_o[row] = mean; rstd_o[row] = rstd; }
}

// dS = LN backward of dy; dx = dS; dr = dS * dropmask.  Each wave walks rows_per_wave rows;
// dgamma/dbeta partials are summed over the block's waves in LDS in a fixed order and written
// as the block's slice row ws[block][2][cols]; imgcap_slice_reduce adds the slices in order
// (deterministic; no same-address atomics, which serialised ~500 blocks per column before).
template <typename T, int G, int MAXC>
__global__ __launch_bounds__(256) void add_ln_bwd_kernel(int rows, int cols, const T* __restrict__ dy,
                                                         const T* __restrict__ s, const float* __restrict__ mean_i,
                                                         const float* __restrict__ rstd_i, const float* __restrict__ g,
                                                         float p, uint64_t seed0, const uint64_t* seed_ctr,
                                                         uint32_t stream_id, T* __restrict__ dx, T* __restrict__ dr,
                                                         float* __restrict__ ws, int rows_per_wave) {
  constexpr int MAXJ = MAXC / (64 * G);
  __shared__ float part[2][4][MAXC];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t seed = (dr && p > 0.f) ? eff_seed(seed0, seed_ctr) : seed0;
  float lg[MAXJ][G], lb[MAXJ][G];
#pragma unroll
  for (int j = 0; j < MAXJ; ++j)
#pragma unroll
    for (int e = 0; e < G; ++e) { lg[j][e] = 0.f; lb[j][e] = 0.f; }
  const int r0 = (blockIdx.x * 4 + w) * rows_per_wave;
  const int r_end = min(rows, r0 + rows_per_wave);
  for (int row = r0; row < r_end; ++row) {
    const float mean = mean_i[row], rstd = rstd_i[row];
    float xh[MAXJ][G], gdy[MAXJ][G];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) {
      const int c0 = G * (lane + 64 * j);
#pragma unroll
      for (int e = 0; e < G; ++e) { xh[j][e] = 0.f; gdy[j][e] = 0.f; }
      if (c0 < cols) {
        const long idx = (long)row * cols + c0;
        float dv[G], sv[G];
        ld_g<T, G>(dy + idx, dv);
        ld_g<T, G>(s + idx, sv);
#pragma unroll
        for (int e = 0; e < G; ++e) {
          xh[j][e] = (sv[e] - mean) * rstd;
          gdy[j][e] = dv[e] * g[c0 + e];
          lg[j][e] += dv[e] * xh[j][e];
          lb[j][e] += dv[e];
          s1 += gdy[j][e];
          s2 += gdy[j][e] * xh[j][e];
        }
      }
    }
    s1 = wave_sum(s1) / cols;
    s2 = wave_sum(s2) / cols;
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) {
      const int c0 = G * (lane + 64 * j);
      if (c0 < cols) {
        const long idx = (long)row * cols + c0;
        float d[G];
#pragma unroll
        for (int e = 0; e < G; ++e) d[e] = rstd * (gdy[j][e] - s1 - xh[j][e] * s2);
        st_g<T, G>(dx + idx, d);
        if (dr) {
#pragma unroll
          for (int e = 0; e < G; ++e) d[e] *= dropout_scale(seed, stream_id, idx + e, p);
          st_g<T, G>(dr + idx, d);
        }
      }
    }
  }
  if (!ws) return;
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) {
    const int c0 = G * (lane + 64 * j);
    if (c0 < cols)
#pragma unroll
      for (int e = 0; e < G; ++e) { part[0][w][c0 + e] = lg[j][e]; part[1][w][c0 + e] = lb[j][e]; }
  }
  __syncthreads();
  float* out = ws + (long)blockIdx.x * 2 * cols;
  for (int c = threadIdx.x; c < cols; c += 256) {
    out[c] = ((part[0][0][c] + part[0][1][c]) + part[0][2][c]) + part[0][3][c];
    out[cols + c] = ((part[1][0][c] + part[1][1][c]) + part[1][2][c]) + part[1][3][c];
  }
}

}  // namespace imgcap

using namespace imgcap;

namespace {
// granule: 16-byte accesses when the row pitch and every operand allow it, else scalar
template <typename T>
bool vec_rows(int cols, std::initializer_list<const void*> ptrs) {
  if ((cols * sizeof(T)) % 16 != 0) return false;
  for (const void* q : ptrs)
    if (q && !aligned16(q)) return false;
  return true;
}
}  // namespace

extern "C" int imgcap_add_layernorm_fwd(int dtype, int rows, int cols, const void* x, const void* r, float drop_p,
                                        uint64_t seed, uint32_t drop_stream, const float* gamma, const float* beta,
                                        float eps, void* s_out, void* y, float* mean, float* rstd, void* stream) {
  IMGCAP_REQUIRE(cols > 0 && cols <= LN_MAXC, "imgcap_add_layernorm_fwd: cols must be in (0, 2048]");
  if (rows == 0) return 0;
  dim3 grid((rows + 3) / 4);
  hipStream_t st = (hipStream_t)stream;
#define LNF_(T, G)                                                                                              \
  do {                                                                                                          \
    if (cols <= 512) { LNF2_(T, G, 512); } else if (cols <= 1024) { LNF2_(T, G, 1024); } else { LNF2_(T, G, 2048); } \
  } while (0)
#define LNF2_(T, G, MC)                                                                                         \
  hipLaunchKernelGGL((add_ln_fwd_kernel<T, G, MC>), grid, dim3(256), 0, st, rows, cols, (const T*)x, (const T*)r,    \
                     drop_p, seed, g_seed_ctr, drop_stream, gamma, beta, eps, (T*)s_out, (T*)y, mean, rstd)
  if (dtype == IMGCAP_BF16) {
    if (vec_rows<bf16>(cols, {x, r, s_out, y})) LNF_(bf16, 8); else LNF_(bf16, 1);
  } else {
    if (vec_rows<float>(cols, {x, r, s_out, y})) LNF_(float, 4); else LNF_(float, 1);
  }
#undef LNF_
#undef LNF2_
  IMGCAP_CHECK_LAUNCH("imgcap_add_layernorm_fwd");
  return 0;
}

// rows per wave and blocks of the LN backward: ~512 blocks of 4 waves
static int lnb_rpw(int rows) { return std::max(1, (rows + 4 * 512 - 1) / (4 * 512)); }
extern "C" int imgcap_add_layernorm_bwd_blocks(int rows) {
  if (rows <= 0) return 0;
  const int rpw = lnb_rpw(rows);
  return (rows + 4 * rpw - 1) / (4 * rpw);
}

extern "C" int imgcap_add_layernorm_bwd(int dtype, int rows, int cols, const void* dy, const void* s,
                                        const float* mean, const float* rstd, const float* gamma, float drop_p,
                                        uint64_t seed, uint32_t drop_stream, void* dx, void* dr, float* dgamma,
                                        float* dbeta, float* part, void* stream) {
  IMGCAP_REQUIRE(!part || (!dgamma && !dbeta), "imgcap_add_layernorm_bwd: part replaces dgamma/dbeta");
  IMGCAP_REQUIRE(cols > 0 && cols <= LN_MAXC, "imgcap_add_layernorm_bwd: cols must be in (0, 2048]");
  if (rows == 0) return 0;
  const int rpw = lnb_rpw(rows);
  const int nblk = imgcap_add_layernorm_bwd_blocks(rows);
  dim3 grid(nblk);
  hipStream_t st = (hipStream_t)stream;
  float* ws = part;  // the caller's [nblk][2][cols] partials (its deferred column sums), or ours
  if (dgamma || dbeta) {
    ws = (float*)workspace((size_t)nblk * 2 * cols * sizeof(float), st);
    if (!ws) return fail(IMGCAP_EWORKSPACE, std::string("imgcap_add_layernorm_bwd: ") + last_error());
  }
#define LNB_(T, G)                                                                                              \
  do {                                                                                                          \
    if (cols <= 512) { LNB2_(T, G, 512); } else if (cols <= 1024) { LNB2_(T, G, 1024); } else { LNB2_(T, G, 2048); } \
  } while (0)
#define LNB2_(T, G, MC)                                                                                         \
  hipLaunchKernelGGL((add_ln_bwd_kernel<T, G, MC>), grid, dim3(256), 0, st, rows, cols, (const T*)dy, (const T*)s,   \
                     mean, rstd, gamma, drop_p, seed, g_seed_ctr, drop_stream, (T*)dx, (T*)dr, ws, rpw)
  if (dtype == IMGCAP_BF16) {
    if (vec_rows<bf16>(cols, {dy, s, dx, dr})) LNB_(bf16, 8); else LNB_(bf16, 1);
  } else {
    if (vec_rows<float>(cols, {dy, s, dx, dr})) LNB_(float, 4); else LNB_(float, 1);
  }
#undef LNB_
#undef LNB2_
  IMGCAP_CHECK_LAUNCH("imgcap_add_layernorm_bwd");
  // the [nblk][2][cols] partials are column-summed by the multi-colsum kernel (rows in
  // parallel; a per-column serial walk over ~500 slices cost ~30 us)
  if (part) return 0;
  imgcap_colsum_item it[2];
  int n = 0;
  if (dgamma) it[n++] = imgcap_colsum_item{ws, dgamma, 2L * cols, nblk, cols, IMGCAP_F32, 0, 1.f};
  if (dbeta) it[n++] = imgcap_colsum_item{ws + cols, dbeta, 2L * cols, nblk, cols, IMGCAP_F32, 0, 1.f};
  return imgcap_colsum_multi(n, it, stream);
}

// HBM-bound elementwise kernels of the step: fused clip+Adam over the flat parameter
// buffer, token embedding (+dropout +positional encoding) and its scatter-add backward,
// casts and fills.
#include "common.h"

namespace imgcap {

// utils.py:183-192 clamp_(-clip, clip) then torch.optim.Adam (train.py:110, .step at :291),
// same formula as torch's single-tensor Adam:
//   m = b1 m + (1-b1) g ; v = b2 v + (1-b2) g^2
//   p -= (lr / (1-b1^t)) * m / (sqrt(v)/sqrt(1-b2^t) + eps)
__global__ __launch_bounds__(256) void clamp_adam_kernel(long n, float* __restrict__ p, const float* __restrict__ g,
                                                         float* __restrict__ m, float* __restrict__ v,
                                                         bf16* __restrict__ shadow, float lr, float b1, float b2,
                                                         float eps, float step_size, float bc2_sqrt, float clip,
                                                         float inv_div, const float* __restrict__ skip) {
  // a step whose persistent LSTM hand-off timed out (its metrics' error word) leaves the
  // parameters and moments untouched: its gradients are invalid
  if (skip && *skip != 0.f) return;
  const long n4 = n / 4;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    f32x4 gg = ((const f32x4*)g)[i], mm = ((f32x4*)m)[i], vv = ((f32x4*)v)[i], pp = ((f32x4*)p)[i];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float gj = fminf(fmaxf(gg[j] * inv_div, -clip), clip);
      mm[j] = b1 * mm[j] + (1.f - b1) * gj;
      vv[j] = b2 * vv[j] + (1.f - b2) * gj * gj;
      const float denom = sqrtf(vv[j]) / bc2_sqrt + eps;
      pp[j] = pp[j] - step_size * (mm[j] / denom);
    }
    ((f32x4*)m)[i] = mm;
    ((f32x4*)v)[i] = vv;
    ((f32x4*)p)[i] = pp;
    if (shadow) {
      bf16x4 s = {(bf16)pp[0], (bf16)pp[1], (bf16)pp[2], (bf16)pp[3]};
      ((bf16x4*)shadow)[i] = s;
    }
  }
  // tail
  for (long i = n4 * 4 + blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    float gj = fminf(fmaxf(g[i] * inv_div, -clip), clip);
    m[i] = b1 * m[i] + (1.f - b1) * gj;
    v[i] = b2 * v[i] + (1.f - b2) * gj * gj;
    p[i] = p[i] - step_size * (m[i] / (sqrtf(v[i]) / bc2_sqrt + eps));
    if (shadow) shadow[i] = (bf16)p[i];
  }
}

template <typename T>
__global__ __launch_bounds__(256) void embedding_fwd_kernel(int n, int dim, const int64_t* __restrict__ ids,
                                                            const float* __restrict__ table,
                                                            const float* __restrict__ pe, int L, float p,
                                                            uint64_t seed0, const uint64_t* seed_ctr, uint32_t sid,
                                                            T* __restrict__ out) {
  const uint64_t seed = p > 0.f ? eff_seed(seed0, seed_ctr) : seed0;
  const long total = (long)n * dim;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const long r = e / dim;
    const int c = (int)(e % dim);
    float v = table[ids[r] * (long)dim + c] * dropout_scale(seed, sid, e, p);
    if (pe) v += pe[(r % L) * dim + c];
    out[e] = from_f<T>(v);
  }
}

// dim % 8 == 0: one thread per 8 columns of a position -- the id read once, the table / pe rows
// as 16-byte loads, 32-bit index math (the element form divides a 64-bit index per element);
// the same per-element arithmetic (table * dropout scale of element e, then + pe)
template <typename T>
__global__ __launch_bounds__(256) void embedding_fwd8_kernel(int n, int dim, const int64_t* __restrict__ ids,
                                                             const float* __restrict__ table,
                                                             const float* __restrict__ pe, int L, float p,
                                                             uint64_t seed0, const uint64_t* seed_ctr, uint32_t sid,
                                                             T* __restrict__ out) {
  const uint64_t seed = p > 0.f ? eff_seed(seed0, seed_ctr) : seed0;
  const unsigned d8 = (unsigned)dim >> 3, total = (unsigned)n * d8;
  for (unsigned g = blockIdx.x * 256u + threadIdx.x; g < total; g += gridDim.x * 256u) {
    const unsigned r = g / d8, c = (g - r * d8) * 8;
    const float* tp = table + ids[r] * (long)dim + c;
    const f32x4 a = *(const f32x4*)tp, b = *(const f32x4*)(tp + 4);
    float v[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
    const long e0 = (long)r * dim + c;
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] *= dropout_scale(seed, sid, e0 + k, p);
    if (pe) {
      const float* pp = pe + (long)(r % (unsigned)L) * dim + c;
      const f32x4 pa = *(const f32x4*)pp, pb = *(const f32x4*)(pp + 4);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        v[k] += pa[k];
        v[k + 4] += pb[k];
      }
    }
    st_g<T, 8>(out + e0, v);
  }
}

// Deterministic embedding backward (nn.Embedding, decoder.py:84 / transformerDecoder.py:94):
// dtable[id] += sum over the positions r with ids[r] == id, IN POSITION ORDER, of dout[r]
// (times the dropout mask of the Transformer path).  No float atomics, so the result is
// bitwise the same on every run.  Three launches after zeroing the rank words:
//   emb_rank:    rank of position i in the (id, position) order, counted against one chunk of
//                EMB_CHUNK ids per workgroup (chunk in LDS, broadcast reads); the chunk counts
//                are summed with integer atomics (exact, order-free)
//   emb_scatter: sorted position / id at that rank
//   emb_segsum:  one wave per sorted index; a run's first index reads the run's positions a
//                window of EMB_CH at a time and sums their rows in order
constexpr int EMB_CHUNK = 128;  // ids per rank workgroup: many small workgroups fill the chip
constexpr int EMB_MAXN = 1 << 20;
__global__ __launch_bounds__(256) void emb_rank_kernel(int n, const int64_t* __restrict__ ids,
                                                       int* __restrict__ rank) {
  __shared__ __attribute__((aligned(16))) int chunk[EMB_CHUNK];
  const int c0 = blockIdx.y * EMB_CHUNK, cn = min(EMB_CHUNK, n - c0);
  // pad the chunk with INT_MAX (never < id, never == id: ids < 2^31 - 1)
  for (int k = threadIdx.x; k < EMB_CHUNK; k += 256) chunk[k] = k < cn ? (int)ids[c0 + k] : 0x7fffffff;
  __syncthreads();
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int id = (int)ids[i];
  const int before = i - c0;  // chunk entries k < before precede position i
  int cnt = 0;
  const int4* c4 = (const int4*)chunk;
#pragma unroll
  for (int q = 0; q < EMB_CHUNK / 4; ++q) {  // broadcast 16-byte LDS reads, 4 ids each
    const int4 v = c4[q];
    const int k = 4 * q;
    cnt += (v.x < id) | ((v.x == id) & (k < before));
    cnt += (v.y < id) | ((v.y == id) & (k + 1 < before));
    cnt += (v.z < id) | ((v.z == id) & (k + 2 < before));
    cnt += (v.w < id) | ((v.w == id) & (k + 3 < before));
  }
  if (cnt) atomicAdd(rank + i, cnt);
}

__global__ __launch_bounds__(256) void emb_scatter_kernel(int n, const int64_t* __restrict__ ids,
                                                          const int* __restrict__ rank, int* __restrict__ spos,
                                                          int* __restrict__ sid) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int r = rank[i];
  spos[r] = i;
  sid[r] = (int)ids[i];
}

constexpr int EMB_MAXDIM = 2048;  // columns: 8 per lane, at most 4 passes of 512
// sorted indices per chunk (one wave's share of a long run).  16, not 64: the bench's captions all
// start with <start>, a 64-position run that one wave summed in 8 dependent load rounds (55.8 us
// per launch in the C3 step, rocprof round 6); as 4 pieces the rounds run on 4 waves
constexpr int EMB_CH = 16;
// The rows of each id summed in position order, in chunks of the sorted index array aligned to
// EMB_CH: a wave owns a chunk's piece of a run (the run's head, or the chunk's first index when
// the run started in an earlier chunk).  A run inside one chunk is added to the table directly; a
// run crossing chunk boundaries leaves its pieces in ws[chunk][0 = continuation, 1 = head] and
// emb_combine_kernel adds them in chunk order -- a fixed summation order whatever the schedule,
// and a long run (the padding id of captions padded to L: thousands of positions) is spread over
// run / EMB_CH waves instead of one.
template <typename T>
__global__ __launch_bounds__(256) void emb_segsum_kernel(int n, int dim, const int* __restrict__ spos,
                                                         const int* __restrict__ sid, const T* __restrict__ dout,
                                                         float p, uint64_t seed0, const uint64_t* seed_ctr,
                                                         uint32_t stream_id, float* __restrict__ dtable,
                                                         float* __restrict__ ws) {
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (i >= n) return;
  // the neighbours' ids and this index's position in one round trip
  const int id = sid[i];
  const int prev = i > 0 ? sid[i - 1] : -1, next = i + 1 < n ? sid[i + 1] : -1;
  const int pos0 = spos[i];
  const bool head = prev != id;          // the run starts here
  if (!head && i % EMB_CH) return;       // inside a chunk piece owned by another wave
  const uint64_t seed = p > 0.f ? eff_seed(seed0, seed_ctr) : seed0;
  const bool vec = (dim % 8) == 0;
  constexpr int NC = EMB_MAXDIM / 512;
  if (head && next != id && vec) {
    // a one-position run (most ids of a batch): its row and the table row requested together,
    // the same single addition as the general loop (0 + x * scale, then table += that)
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int c0 = c * 512 + lane * 8;
      if (c0 >= dim) continue;
      float x[8], t[8];
      ld_g<T, 8>(dout + (long)pos0 * dim + c0, x);
      float* tp = dtable + (long)id * dim + c0;
      *(f32x4*)t = *(const f32x4*)tp;
      *(f32x4*)(t + 4) = *(const f32x4*)(tp + 4);
#pragma unroll
      for (int k = 0; k < 8; ++k) t[k] += 0.f + x[k] * dropout_scale(seed, stream_id, (long)pos0 * dim + c0 + k, p);
      *(f32x4*)tp = *(const f32x4*)t;
      *(f32x4*)(tp + 4) = *(const f32x4*)(t + 4);
    }
    return;
  }
  float acc[NC][8];
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[c][k] = 0.f;
  // this piece: indices [i, lim) of the run, lim = the chunk's end; its members are a prefix
  const int chunk = i / EMB_CH;
  const int lim = min(n, (chunk + 1) * EMB_CH);
  const int j = i + lane;
  const int jpos = j < lim ? spos[j] : 0;
  unsigned long long m = __ballot(j < lim && sid[j] == id);
  const int cnt_all = __popcll(m);
  const bool continues = i + cnt_all == lim && lim < n && sid[lim] == id;
  // rows in position order, RB loads in flight before their (sequential) additions
  constexpr int RB = 8;
  while (m) {
    long rows[RB];
    int cnt = 0;
#pragma unroll
    for (int u = 0; u < RB; ++u) {
      const int l = m ? __ffsll((long long)m) - 1 : 0;
      if (m) ++cnt;
      m &= m - 1;
      rows[u] = __shfl(jpos, l, 64);  // past the piece's end: a valid row, loaded and not added
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int c0 = c * 512 + lane * 8;
      if (c0 >= dim) continue;
      float x[RB][8];
#pragma unroll
      for (int u = 0; u < RB; ++u) {
        if (vec) {
          ld_g<T, 8>(dout + rows[u] * dim + c0, x[u]);
        } else {
#pragma unroll
          for (int k = 0; k < 8; ++k) x[u][k] = c0 + k < dim ? to_f(dout[rows[u] * dim + c0 + k]) : 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < RB; ++u) {
        if (u >= cnt) break;  // wave-uniform
#pragma unroll
        for (int k = 0; k < 8; ++k)
          acc[c][k] += x[u][k] * dropout_scale(seed, stream_id, rows[u] * dim + c0 + k, p);
      }
    }
  }
  // a whole run: into the table; a piece of a longer one: its chunk slot (0 continuation, 1 head)
  float* dst = (head && !continues) ? dtable + (long)id * dim
                                    : ws + ((long)chunk * 2 + (head ? 1 : 0)) * dim;
  const bool add = head && !continues;
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int col = c * 512 + lane * 8 + k;
      if (col < dim) dst[col] = add ? dst[col] + acc[c][k] : acc[c][k];
    }
}

// The runs that cross chunk boundaries: the wave of chunk k takes the run that starts in chunk k
// and continues past its end, and adds its head piece and the continuation pieces of the chunks
// that follow, in chunk order, to the table.
__global__ __launch_bounds__(256) void emb_combine_kernel(int n, int dim, const int* __restrict__ sid,
                                                          const float* __restrict__ ws,
                                                          float* __restrict__ dtable) {
  const int k = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int last = (k + 1) * EMB_CH - 1;
  if (last + 1 >= n) return;
  const int id = sid[last];
  if (sid[last + 1] != id) return;                     // no run crosses this chunk's end
  if (k > 0 && sid[k * EMB_CH - 1] == id) return;      // it started in an earlier chunk
  // the continuation chunks k+1 .. k+cnt, found 64 at a time (lane l tests chunk base + l) instead
  // of one dependent id load per chunk
  int cnt = 0;
  for (int base = k + 1;; base += 64) {
    const int jc = base + lane;
    const unsigned long long m = __ballot(jc * EMB_CH < n && sid[jc * EMB_CH] == id);
    const int run = ~m ? __ffsll((long long)~m) - 1 : 64;
    cnt += run;
    if (run < 64) break;
  }
  constexpr int NC = EMB_MAXDIM / 512;
  constexpr int PB = 8;  // continuation pieces in flight before their (ordered) additions
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int c0 = c * 512 + lane * 8;
    if (c0 >= dim) continue;
    float t[8];
    const float* h = ws + ((long)k * 2 + 1) * dim + c0;
#pragma unroll
    for (int e = 0; e < 8; ++e) t[e] = c0 + e < dim ? h[e] : 0.f;
    for (int j0 = 0; j0 < cnt; j0 += PB) {
      float q[PB][8];
#pragma unroll
      for (int u = 0; u < PB; ++u) {
        const float* qp = ws + (long)(k + 1 + min(j0 + u, cnt - 1)) * 2 * dim + c0;
#pragma unroll
        for (int e = 0; e < 8; ++e) q[u][e] = c0 + e < dim ? qp[e] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < PB; ++u) {
        if (j0 + u >= cnt) break;
#pragma unroll
        for (int e = 0; e < 8; ++e) t[e] += q[u][e];
      }
    }
    float* tp = dtable + (long)id * dim + c0;
#pragma unroll
    for (int e = 0; e < 8; ++e)
      if (c0 + e < dim) tp[e] += t[e];
  }
}

template <typename TI, typename TO>
__global__ void cast_kernel(long n, const TI* __restrict__ x, TO* __restrict__ y) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) y[i] = from_f<TO>(to_f(x[i]));
}

template <typename T>
__global__ void fill_kernel(long n, float v, T* __restrict__ x) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) x[i] = from_f<T>(v);
}

template <typename T>
__global__ void dropout_kernel(long n, const T* __restrict__ x, float p, uint64_t seed0, const uint64_t* seed_ctr,
                               uint32_t sid, T* __restrict__ y) {
  const uint64_t seed = p > 0.f ? eff_seed(seed0, seed_ctr) : seed0;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    y[i] = from_f<T>(to_f(x[i]) * dropout_scale(seed, sid, i, p));
}

__global__ void loss_finalize_kernel(int n, const float* __restrict__ loss_rows, const float* __restrict__ hit5,
                                     const int64_t* __restrict__ tgt, const float* __restrict__ extra,
                                     float* __restrict__ out) {
  __shared__ float red[16];
  float l = 0.f, c = 0.f, h = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    if (tgt[i] >= 0) { l += loss_rows[i]; c += 1.f; h += hit5[i]; }
  }
  l = block_sum(l, red);
  c = block_sum(c, red);
  h = block_sum(h, red);
  if (threadIdx.x == 0) {
    const float cnt = c > 0.f ? c : 1.f;
    out[0] = l / cnt + (extra ? *extra : 0.f);
    out[1] = c;
    out[2] = h;
    out[3] = 1.f / cnt;
  }
}

// out[b, e] = mean_p x[b, p, e]  (decoder.py:64 encoder_out.mean(dim=1))
template <typename TI, typename TO>
__global__ void mean_mid_kernel(int B, int P, int E, const TI* __restrict__ x, TO* __restrict__ out) {
  const long n = (long)B * E;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int b = (int)(i / E), e = (int)(i % E);
    float s = 0.f;
    for (int p = 0; p < P; ++p) s += to_f(x[((long)b * P + p) * E + e]);
    out[i] = from_f<TO>(s / P);
  }
}

// decoder.py:64,79-81 in one launch: sort the batch by caption length (descending, stable --
// the order the engine has always used), gather encoder_out and the captions into that order,
// decode lengths (len - 1, int32) and the pixel mean of each gathered row (decoder.py:64, the
// same p-order fp32 sum as mean_mid_kernel).  Block (r, chunk) = destination row r, 32 16-byte
// column vectors: every block ranks the (<= 256) lengths itself, so no second launch is needed
// for the gather.  The 8 waves' lanes split the pixels (all of a block's loads in flight at
// once, 256 threads busy instead of the 96 of one thread per vector), stage them in LDS, and
// the first 32 threads sum each vector's pixels in p order from there.
template <typename T>
__global__ __launch_bounds__(256) void sort_gather_kernel(int B, int P, int E, int L, const int64_t* __restrict__ lens,
                                                          const T* __restrict__ enc, const int64_t* __restrict__ caps,
                                                          T* __restrict__ enc_out, T* __restrict__ mean_out,
                                                          int64_t* __restrict__ caps_out, int64_t* __restrict__ sort_ind,
                                                          int32_t* __restrict__ dl) {
  extern __shared__ uint4 stage[];  // [P][32] 16-byte vectors
  __shared__ int64_t ls[256];
  __shared__ int src_s;
  const int r = blockIdx.x, tid = threadIdx.x;
  if (tid < B) ls[tid] = lens[tid];
  __syncthreads();
  if (tid < B) {
    const int64_t li = ls[tid];
    int rank = 0;
    for (int j = 0; j < B; ++j) rank += (ls[j] > li) || (ls[j] == li && j < tid);
    if (rank == r) src_s = tid;
  }
  __syncthreads();
  const int src = src_s;
  if (blockIdx.y == 0) {
    if (tid == 0) {
      sort_ind[r] = src;
      dl[r] = (int32_t)(ls[src] - 1);
    }
    for (int i = tid; i < L; i += 256) caps_out[(long)r * L + i] = caps[(long)src * L + i];
  }
  constexpr int VEC = 16 / sizeof(T);
  const int vl = tid & 31, ps = tid >> 5;
  const int v = blockIdx.y * 32 + vl;
  const bool ok = v < E / VEC;
  const T* in = enc + (long)src * P * E;
  T* out = enc_out + (long)r * P * E;
  if (ok) {
    constexpr int PB = 8;  // pixels ps, ps + 8, .. : up to PB loads in flight per thread
    for (int p0 = ps; p0 < P; p0 += 8 * PB) {
      uint4 u[PB];
#pragma unroll
      for (int i = 0; i < PB; ++i)
        if (p0 + 8 * i < P) u[i] = *(const uint4*)(in + (long)(p0 + 8 * i) * E + v * VEC);
#pragma unroll
      for (int i = 0; i < PB; ++i)
        if (p0 + 8 * i < P) {
          *(uint4*)(out + (long)(p0 + 8 * i) * E + v * VEC) = u[i];
          stage[(p0 + 8 * i) * 32 + vl] = u[i];
        }
    }
  }
  __syncthreads();
  if (ps == 0 && ok) {
    float acc[VEC];
#pragma unroll
    for (int k = 0; k < VEC; ++k) acc[k] = 0.f;
    for (int p = 0; p < P; ++p) {
      const uint4 u = stage[p * 32 + vl];
      const T* x = (const T*)&u;
#pragma unroll
      for (int k = 0; k < VEC; ++k) acc[k] += to_f(x[k]);
    }
#pragma unroll
    for (int k = 0; k < VEC; ++k) mean_out[(long)r * E + v * VEC + k] = from_f<T>(acc[k] / P);
  }
}

// The one-block-per-row form (96 threads busy per block at E = 768): kept for B > 32, where it
// measured faster in the C3 step (17.33-17.35k vs 17.23k img/s, tools/gpu/r3_sortg.sh).
template <typename T>
__global__ __launch_bounds__(256) void sort_gather_row_kernel(int B, int P, int E, int L, const int64_t* __restrict__ lens,
                                                          const T* __restrict__ enc, const int64_t* __restrict__ caps,
                                                          T* __restrict__ enc_out, T* __restrict__ mean_out,
                                                          int64_t* __restrict__ caps_out, int64_t* __restrict__ sort_ind,
                                                          int32_t* __restrict__ dl) {
  __shared__ int64_t ls[256];
  __shared__ int src_s;
  const int r = blockIdx.x, tid = threadIdx.x;
  if (tid < B) ls[tid] = lens[tid];
  __syncthreads();
  if (tid < B) {
    const int64_t li = ls[tid];
    int rank = 0;
    for (int j = 0; j < B; ++j) rank += (ls[j] > li) || (ls[j] == li && j < tid);
    if (rank == r) src_s = tid;
  }
  __syncthreads();
  const int src = src_s;
  if (tid == 0) {
    sort_ind[r] = src;
    dl[r] = (int32_t)(ls[src] - 1);
  }
  for (int i = tid; i < L; i += 256) caps_out[(long)r * L + i] = caps[(long)src * L + i];
  constexpr int VEC = 16 / sizeof(T);
  const T* in = enc + (long)src * P * E;
  T* out = enc_out + (long)r * P * E;
  for (int v = tid; v < E / VEC; v += 256) {
    float acc[VEC];
#pragma unroll
    for (int k = 0; k < VEC; ++k) acc[k] = 0.f;
    // pixels in batches of PB independent loads (one memory round trip per batch instead of one
    // per pixel; 34.6 -> 15.5 us at B = 32, P = 49 with batches of 16), summed in p order
    constexpr int PB = 32;
    for (int p0 = 0; p0 < P; p0 += PB) {
      uint4 u[PB];
#pragma unroll
      for (int i = 0; i < PB; ++i)
        if (p0 + i < P) u[i] = *(const uint4*)(in + (long)(p0 + i) * E + v * VEC);
#pragma unroll
      for (int i = 0; i < PB; ++i)
        if (p0 + i < P) {
          *(uint4*)(out + (long)(p0 + i) * E + v * VEC) = u[i];
          const T* x = (const T*)&u[i];
#pragma unroll
          for (int k = 0; k < VEC; ++k) acc[k] += to_f(x[k]);
        }
    }
#pragma unroll
    for (int k = 0; k < VEC; ++k) mean_out[(long)r * E + v * VEC + k] = from_f<T>(acc[k] / P);
  }
}

__global__ __launch_bounds__(256) void zero16_kernel(uint4* p, long n16) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n16; i += (long)gridDim.x * 256) p[i] = make_uint4(0u, 0u, 0u, 0u);
}

static dim3 grid_for(long n) {
  long b = (n + 255) / 256;
  if (b > 4096) b = 4096;
  if (b < 1) b = 1;
  return dim3((unsigned)b);
}

hipError_t zero_async(void* p, size_t bytes, hipStream_t stream) {
  if (bytes == 0) return hipSuccess;
  if ((bytes & 15) || !aligned16(p)) return hipErrorInvalidValue;
  const long n16 = (long)(bytes / 16);
  hipLaunchKernelGGL(zero16_kernel, grid_for(n16), dim3(256), 0, stream, (uint4*)p, n16);
  return hipGetLastError();
}

}  // namespace imgcap

using namespace imgcap;

extern "C" int imgcap_clamp_adam(int64_t n, float* param, const float* grad, float* m, float* v, void* shadow_bf16,
                                 float lr, float beta1, float beta2, float eps, int step, float clip, float grad_div,
                                 const float* skip, void* stream) {
  if (n == 0) return 0;
  IMGCAP_REQUIRE(step >= 1, "imgcap_clamp_adam: step must be >= 1");
  IMGCAP_REQUIRE(aligned16(param) && aligned16(grad) && aligned16(m) && aligned16(v),
                 "imgcap_clamp_adam: buffers must be 16-byte aligned");
  IMGCAP_REQUIRE(shadow_bf16 == nullptr || (((uintptr_t)shadow_bf16) & 7) == 0, "imgcap_clamp_adam: shadow align");
  const double bc1 = 1.0 - std::pow((double)beta1, step);
  const double bc2 = 1.0 - std::pow((double)beta2, step);
  hipLaunchKernelGGL(clamp_adam_kernel, grid_for(n / 4 + 1), dim3(256), 0, (hipStream_t)stream, (long)n, param, grad,
                     m, v, (bf16*)shadow_bf16, lr, beta1, beta2, eps, (float)(lr / bc1), (float)std::sqrt(bc2), clip,
                     1.0f / grad_div, skip);
  IMGCAP_CHECK_LAUNCH("imgcap_clamp_adam");
  return 0;
}

extern "C" int imgcap_embedding_fwd(int dtype, int n, int dim, const int64_t* ids, const float* table, const float* pe,
                                    int L, float drop_p, uint64_t seed, uint32_t drop_stream, void* out, void* stream) {
  if (n == 0) return 0;
  IMGCAP_REQUIRE(pe == nullptr || L > 0, "imgcap_embedding_fwd: L");
  const long total = (long)n * dim;
  const bool v8 = dim % 8 == 0 && total < (1L << 31) && ((uintptr_t)table & 15) == 0 && (!pe || ((uintptr_t)pe & 15) == 0) &&
                  ((uintptr_t)out & 15) == 0;
  if (v8) {
    if (dtype == IMGCAP_BF16)
      hipLaunchKernelGGL(embedding_fwd8_kernel<bf16>, grid_for(total / 8), dim3(256), 0, (hipStream_t)stream, n, dim,
                         ids, table, pe, L, drop_p, seed, g_seed_ctr, drop_stream, (bf16*)out);
    else
      hipLaunchKernelGGL(embedding_fwd8_kernel<float>, grid_for(total / 8), dim3(256), 0, (hipStream_t)stream, n, dim,
                         ids, table, pe, L, drop_p, seed, g_seed_ctr, drop_stream, (float*)out);
    IMGCAP_CHECK_LAUNCH("imgcap_embedding_fwd");
    return 0;
  }
  if (dtype == IMGCAP_BF16)
    hipLaunchKernelGGL(embedding_fwd_kernel<bf16>, grid_for(total), dim3(256), 0, (hipStream_t)stream, n, dim, ids,
                       table, pe, L, drop_p, seed, g_seed_ctr, drop_stream, (bf16*)out);
  else
    hipLaunchKernelGGL(embedding_fwd_kernel<float>, grid_for(total), dim3(256), 0, (hipStream_t)stream, n, dim, ids,
                       table, pe, L, drop_p, seed, g_seed_ctr, drop_stream, (float*)out);
  IMGCAP_CHECK_LAUNCH("imgcap_embedding_fwd");
  return 0;
}

extern "C" int imgcap_embedding_bwd(int dtype, int n, int dim, const int64_t* ids, const void* dout, float drop_p,
                                    uint64_t seed, uint32_t drop_stream, float* dtable, void* stream) {
  if (n == 0) return 0;
  IMGCAP_REQUIRE(n <= EMB_MAXN && dim <= EMB_MAXDIM, "imgcap_embedding_bwd: n <= 2^20 positions, dim <= 2048");
  hipStream_t st = (hipStream_t)stream;
  const size_t rank_bytes = ((size_t)n * sizeof(int) + 15) / 16 * 16;
  const size_t idx_bytes = (2 * (size_t)n * sizeof(int) + 15) / 16 * 16;
  const int nchunks = (n + EMB_CH - 1) / EMB_CH;
  // workspace: ranks + sorted indices (12 B per position) and two dim-wide fp32 slots per chunk for
  // runs crossing a chunk boundary -- ~n * dim / 2 bytes plus 12 n: 0.9 MB at C3 (n = 3,328,
  // dim = 512), 1 GiB at the limits (n = 2^20, dim = 2048); the library workspace keeps its
  // high-water mark for the process (imgcap_workspace_needed / _attach size it)
  int* rank = (int*)workspace(rank_bytes + idx_bytes + (size_t)nchunks * 2 * dim * sizeof(float), st);
  if (!rank) return fail(IMGCAP_EWORKSPACE, std::string("imgcap_embedding_bwd: ") + last_error());
  int* spos = rank + rank_bytes / sizeof(int);
  int* sid = spos + n;
  float* ws = (float*)((char*)rank + rank_bytes + idx_bytes);  // chunk pieces of boundary-crossing runs
  if (zero_async(rank, rank_bytes, st) != hipSuccess) return fail(IMGCAP_EINVAL, "imgcap_embedding_bwd: zeroing failed");
  const int nb = (n + 255) / 256;
  hipLaunchKernelGGL(emb_rank_kernel, dim3(nb, (n + EMB_CHUNK - 1) / EMB_CHUNK), dim3(256), 0, st, n, ids, rank);
  hipLaunchKernelGGL(emb_scatter_kernel, dim3(nb), dim3(256), 0, st, n, ids, rank, spos, sid);
  const dim3 g((n + 3) / 4);
  if (dtype == IMGCAP_BF16)
    hipLaunchKernelGGL(emb_segsum_kernel<bf16>, g, dim3(256), 0, st, n, dim, spos, sid, (const bf16*)dout, drop_p,
                       seed, g_seed_ctr, drop_stream, dtable, ws);
  else
    hipLaunchKernelGGL(emb_segsum_kernel<float>, g, dim3(256), 0, st, n, dim, spos, sid, (const float*)dout,
                       drop_p, seed, g_seed_ctr, drop_stream, dtable, ws);
  if (n > EMB_CH)
    hipLaunchKernelGGL(emb_combine_kernel, dim3((nchunks + 3) / 4), dim3(256), 0, st, n, dim, sid, ws, dtable);
  IMGCAP_CHECK_LAUNCH("imgcap_embedding_bwd");
  return 0;
}

extern "C" int imgcap_dropout(int dtype, int64_t n, const void* x, float p, uint64_t seed, uint32_t drop_stream,
                              void* y, void* stream) {
  if (n == 0) return 0;
  if (dtype == IMGCAP_BF16)
    hipLaunchKernelGGL(dropout_kernel<bf16>, grid_for(n), dim3(256), 0, (hipStream_t)stream, (long)n, (const bf16*)x,
                       p, seed, g_seed_ctr, drop_stream, (bf16*)y);
  else
    hipLaunchKernelGGL(dropout_kernel<float>, grid_for(n), dim3(256), 0, (hipStream_t)stream, (long)n,
                       (const float*)x, p, seed, g_seed_ctr, drop_stream, (float*)y);
  IMGCAP_CHECK_LAUNCH("imgcap_dropout");
  return 0;
}

extern "C" int imgcap_loss_finalize(int n, const float* loss_rows, const float* hit5, const int64_t* targets,
                                    const float* extra, float* out, void* stream) {
  hipLaunchKernelGGL(loss_finalize_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, n, loss_rows, hit5, targets,
                     extra, out);
  IMGCAP_CHECK_LAUNCH("imgcap_loss_finalize");
  return 0;
}

extern "C" int imgcap_mean_mid(int dtype, int B, int P, int E, const void* x, void* out, void* stream) {
  const long n = (long)B * E;
  if (n == 0) return 0;
  if (dtype == IMGCAP_BF16)
    hipLaunchKernelGGL((mean_mid_kernel<bf16, bf16>), grid_for(n), dim3(256), 0, (hipStream_t)stream, B, P, E,
                       (const bf16*)x, (bf16*)out);
  else
    hipLaunchKernelGGL((mean_mid_kernel<float, float>), grid_for(n), dim3(256), 0, (hipStream_t)stream, B, P, E,
                       (const float*)x, (float*)out);
  IMGCAP_CHECK_LAUNCH("imgcap_mean_mid");
  return 0;
}

extern "C" int imgcap_sort_gather_rows(int dtype, int B, int P, int E, int L, const int64_t* lens, const void* enc,
                                       const int64_t* caps, void* enc_out, void* mean_out, int64_t* caps_out,
                                       int64_t* sort_ind, int32_t* dl, void* stream) {
  if (B == 0) return 0;
  IMGCAP_REQUIRE(B >= 1 && B <= 256, "imgcap_sort_gather_rows: 1 <= B <= 256");
  const int vec = dtype == IMGCAP_BF16 ? 8 : 4;
  IMGCAP_REQUIRE(E % vec == 0 && ((uintptr_t)enc & 15) == 0 && ((uintptr_t)enc_out & 15) == 0,
                 "imgcap_sort_gather_rows: 16-byte aligned rows of E elements");
  IMGCAP_REQUIRE(P >= 1 && P <= 256, "imgcap_sort_gather_rows: 1 <= P <= 256 pixels (LDS stage)");
  if (B > 32) {  // measured: the row form is faster in the B = 64 step (see sort_gather_row_kernel)
    if (dtype == IMGCAP_BF16)
      hipLaunchKernelGGL((sort_gather_row_kernel<bf16>), dim3(B), dim3(256), 0, (hipStream_t)stream, B, P, E, L,
                         lens, (const bf16*)enc, caps, (bf16*)enc_out, (bf16*)mean_out, caps_out, sort_ind, dl);
    else
      hipLaunchKernelGGL((sort_gather_row_kernel<float>), dim3(B), dim3(256), 0, (hipStream_t)stream, B, P, E, L,
                         lens, (const float*)enc, caps, (float*)enc_out, (float*)mean_out, caps_out, sort_ind, dl);
    IMGCAP_CHECK_LAUNCH("imgcap_sort_gather_rows");
    return 0;
  }
  // B <= 32: column chunks (C2 step 12.77-12.83k -> 13.04-13.06k img/s, tools/gpu/r3_sortg.sh)
  const dim3 grid((unsigned)B, (unsigned)((E / vec + 31) / 32));
  const size_t smem = (size_t)P * 32 * 16;
  if (dtype == IMGCAP_BF16)
    hipLaunchKernelGGL((sort_gather_kernel<bf16>), grid, dim3(256), smem, (hipStream_t)stream, B, P, E, L, lens,
                       (const bf16*)enc, caps, (bf16*)enc_out, (bf16*)mean_out, caps_out, sort_ind, dl);
  else
    hipLaunchKernelGGL((sort_gather_kernel<float>), grid, dim3(256), smem, (hipStream_t)stream, B, P, E, L, lens,
                       (const float*)enc, caps, (float*)enc_out, (float*)mean_out, caps_out, sort_ind, dl);
  IMGCAP_CHECK_LAUNCH("imgcap_sort_gather_rows");
  return 0;
}

extern "C" int imgcap_cast(int in_dtype, int out_dtype, int64_t n, const void* x, void* y, void* stream) {
  if (n == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (in_dtype == IMGCAP_F32 && out_dtype == IMGCAP_BF16)
    hipLaunchKernelGGL((cast_kernel<float, bf16>), grid_for(n), dim3(256), 0, st, (long)n, (const float*)x, (bf16*)y);
  else if (in_dtype == IMGCAP_BF16 && out_dtype == IMGCAP_F32)
    hipLaunchKernelGGL((cast_kernel<bf16, float>), grid_for(n), dim3(256), 0, st, (long)n, (const bf16*)x, (float*)y);
  else if (in_dtype == IMGCAP_F32 && out_dtype == IMGCAP_F32)
    hipLaunchKernelGGL((cast_kernel<float, float>), grid_for(n), dim3(256), 0, st, (long)n, (const float*)x, (float*)y);
  else
    hipLaunchKernelGGL((cast_kernel<bf16, bf16>), grid_for(n), dim3(256), 0, st, (long)n, (const bf16*)x, (bf16*)y);
  IMGCAP_CHECK_LAUNCH("imgcap_cast");
  return 0;
}

extern "C" int imgcap_fill(int dtype, int64_t n, float value, void* x, void* stream) {
  if (n == 0) return 0;
  if (dtype == IMGCAP_BF16)
    hipLaunchKernelGGL(fill_kernel<bf16>, grid_for(n), dim3(256), 0, (hipStream_t)stream, (long)n, value, (bf16*)x);
  else
    hipLaunchKernelGGL(fill_kernel<float>, grid_for(n), dim3(256), 0, (hipStream_t)stream, (long)n, value, (float*)x);
  IMGCAP_CHECK_LAUNCH("imgcap_fill");
  return 0;
}

// ---- Transformer loss rows (transformerDecoder.py:88-108 + train.py:262-276) -------------------
// One launch for what the decoder's loss needs from the captions: tmask[b, l] = l < len[b] - 1 (the
// decode lengths), targets[b * L + l] = tmask ? caps[b, l + 1] : -1 (position l predicts the next
// token; the last position's target is never valid), and the step's metric words zeroed.
__global__ __launch_bounds__(256) void tf_targets_kernel(int B, int L, const int64_t* __restrict__ caps,
                                                         const int64_t* __restrict__ lens,
                                                         unsigned char* __restrict__ tmask,
                                                         int64_t* __restrict__ targets, float* __restrict__ metrics,
                                                         int n_metrics) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n_metrics) metrics[i] = 0.f;
  if (i >= (long)B * L) return;
  const int b = (int)(i / L), l = (int)(i % L);
  const bool ok = (int64_t)l < lens[b] - 1;
  tmask[i] = ok ? 1 : 0;
  targets[i] = ok ? caps[(long)b * L + (l + 1 < L ? l + 1 : 0)] : (int64_t)-1;
}

extern "C" int imgcap_tf_targets(int B, int L, const int64_t* caps, const int64_t* lens, uint8_t* tmask,
                                 int64_t* targets, float* metrics, int n_metrics, void* stream) {
  IMGCAP_REQUIRE(B >= 0 && L > 0 && n_metrics >= 0 && n_metrics <= 256, "imgcap_tf_targets: bad sizes");
  const long n = std::max((long)B * L, (long)n_metrics);
  if (n == 0) return 0;
  hipLaunchKernelGGL(tf_targets_kernel, grid_for(n), dim3(256), 0, (hipStream_t)stream, B, L, caps, lens, tmask,
                     targets, metrics, n_metrics);
  IMGCAP_CHECK_LAUNCH("imgcap_tf_targets");
  return 0;
}

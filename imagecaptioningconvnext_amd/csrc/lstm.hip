// Teacher-forced "Show, Attend and Tell" LSTM decoder recurrence (models/decoder.py:69-113)
// and its backward-through-time, driven natively: one C-ABI call enqueues all T steps.
//
// Exact algebraic restructuring of the reference loop (results identical up to fp
// reassociation):
//   * att1 = enc W_ea^T + b_ea (decoder.py:26) is computed ONCE outside the loop (the
//     reference recomputes it every step)
//   * the three GEMMs that read h_{t-1} (decoder_att, f_beta, LSTMCell weight_hh) are one
//     GEMM against W_hcat = [W_da; W_fb; W_hh]
//   * the embedding half of weight_ih (and bias_ih) is precomputed for all t (xe); only the
//     attention half (z_t W_ih[:,M:]^T) stays in the loop
//   * fc(dropout(h)) (decoder.py:109) runs once after the loop over all [B*T] rows
//   * rows are never shrunk: rows with t >= decode_length[b] are computed and masked out
//     (alphas = 0 there; the loss never reads their logits; their gradients are zero)
//   * backward keeps only the recurrent chain in the loop: the encoder_att / full_att weight
//     gradients are summed over t in ONE pass afterwards (attn_param_grad_kernel), from the
//     saved softmax-input gradients de[b,t,p]
// Per step, three launches each way:
//   forward : skinny GEMM h_{t-1} -> g1 = [att2 | gate_pre | hh]
//             -> attn_fwd (scores, softmax, context, sigmoid gate)
//             -> gate_cell_fwd (z_t W_ih[:, M:]^T with the four gates of 4 units per 16-column
//                block, LSTMCell pointwise in the epilogue)
//   backward: x_partial (dgates_t . [W_ih[:, M:] | W_hh], K split over the grid into slabs)
//             -> attn_bwd (sums the dz slabs) -> dh_cell (dh_{t-1} = [d att2 | d gate_pre] .
//                [W_da; W_fb] + the W_hh slabs, K split over the grid, last-arriving block per
//                column tile reduces and runs the LSTMCell backward of step t-1 in the epilogue)
// with the weights pre-transposed so every step GEMM is k-major x k-major.
#include <algorithm>

#include "mfma.h"

namespace imgcap {

constexpr int ATT_THREADS = 1024;
constexpr int ATT_WAVES = ATT_THREADS / 64;
constexpr int MAXP = 64;
// default channel chunks per row in attn_fwd.  Swept at C2 (tools/gpu/att_ys.sh, ys = 1..6):
// 8,138-8,226 img/s, all within run-to-run spread -- the step is latency-, not CU-bandwidth-bound.
constexpr int LSTM_ATT_YS = 1;

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

// 8 consecutive elements kept as raw 16-byte words until used (1 word bf16, 2 words fp32)
template <typename T> struct Raw8 { uint4 u[sizeof(T) / 2]; };
template <typename T>
DEV void raw_load(Raw8<T>& r, const T* p) {
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 2); ++i) r.u[i] = *(const uint4*)(p + i * (16 / sizeof(T)));
}
template <typename T>
DEV void raw_to_f(const Raw8<T>& r, float (&x)[8]) { load8<T>((const T*)r.u, x); }

// ---- forward attention step: gridDim.y blocks (16 waves each) per batch row --------------
// Latency-bound (a few hundred KB per step spread over B blocks), so every global load the
// block needs is issued up front, before any reduction.  Block (b, y) recomputes the 49 scores
// and the softmax of row b (att1 is the smaller operand) and owns the context / gate outputs of
// channel chunk y of E (E / gridDim.y channels), so a row's encoder features are read by
// gridDim.y CUs at once instead of one:
//   scores : wave w owns pixels p = w, w+16, ... (<= 4); lane l owns 8 attention units
//            (att1 rows, att2 and w_f slices in registers)
//   context: thread = (8-channel vector v of E, pixel group pg): pixels pg, pg + G, ...
//            (<= MPP enc vectors in registers), partial sums reduced over pg in LDS
template <typename T, int MPP>
__global__ __launch_bounds__(ATT_THREADS) void attn_fwd_kernel(imgcap_lstm_desc d, int t) {
  __shared__ float e_s[MAXP];
  extern __shared__ __attribute__((aligned(16))) float part[];  // [G][E] context partials
  const int b = blockIdx.x;
  const int P = d.P, E = d.E, A = d.A, Tn = d.T;
  const int W3 = A + E + 4 * d.D;
  const int Ec = E / (int)gridDim.y, e0 = blockIdx.y * Ec;  // this block's channel chunk
  const long bt = (long)b * Tn + t;
  const bool active = t < d.dl[b];
  const float* g1 = d.g1 + bt * W3;  // [att2 | gate_pre | hh]
  const T* att1 = (const T*)d.att1 + (long)b * P * A;
  const T* enc = (const T*)d.enc + (long)b * P * E + e0;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int NVE = Ec / 8, G = ATT_THREADS / NVE;
  const int v = threadIdx.x % NVE, pg = threadIdx.x / NVE;
  const bool ctx_thread = pg < G;
  // ---- all loads ----
  const int a0 = lane * 8;
  const bool a_ok = a0 < A;
  float att2[8], wf[8];
  load8<float>(g1 + (a_ok ? a0 : 0), att2);
  load8<float>(d.w_f + (a_ok ? a0 : 0), wf);
  Raw8<T> a1[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int p = w + i * ATT_WAVES;
    raw_load(a1[i], att1 + (long)min(p, P - 1) * A + (a_ok ? a0 : 0));
  }
  Raw8<T> ev[MPP];
#pragma unroll
  for (int i = 0; i < MPP; ++i) {
    const int p = pg + i * G;
    raw_load(ev[i], enc + (long)min(p, P - 1) * E + v * 8);
  }
  // gate pre-activation of the output element(s) this thread writes at the end
  constexpr int EPT = 2;  // E <= EPT * ATT_THREADS (checked on the host)
  float gpre[EPT];
#pragma unroll
  for (int k = 0; k < EPT; ++k) {
    const int e = threadIdx.x + k * ATT_THREADS;
    gpre[k] = e < Ec ? g1[A + e0 + e] : 0.f;
  }
  // ---- scores e_p = w_f . relu(att1_p + att2)   (full_att bias cancels in the softmax) ----
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int p = w + i * ATT_WAVES;
    float x[8];
    raw_to_f(a1[i], x);
    float sc = 0.f;
    if (a_ok) {
#pragma unroll
      for (int j = 0; j < 8; ++j) sc += wf[j] * fmaxf(x[j] + att2[j], 0.f);
    }
    sc = wave_sum(sc);
    if (lane == 0 && p < P) e_s[p] = sc;
  }
  __syncthreads();
  if (w == 0) {
    const float vv = lane < P ? e_s[lane] : -INFINITY;
    const float m = wave_max(vv);
    const float ex = lane < P ? __expf(vv - m) : 0.f;
    const float al = ex / wave_sum(ex);
    if (lane < P) {
      e_s[lane] = al;
      if (blockIdx.y == 0) d.alphas[bt * P + lane] = active ? al : 0.f;
    }
  }
  __syncthreads();
  // ---- context partials over this thread's pixels ----
  if (ctx_thread) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < MPP; ++i) {
      const int p = pg + i * G;
      if (p < P) {
        float x[8];
        raw_to_f(ev[i], x);
        const float al = e_s[p];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += al * x[j];
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) part[pg * Ec + v * 8 + j] = acc[j];
  }
  __syncthreads();
  T* zs = (T*)d.zs + bt * E + e0;
  float* awe = d.awe + bt * E + e0;
#pragma unroll
  for (int k = 0; k < EPT; ++k) {
    const int e = threadIdx.x + k * ATT_THREADS;
    if (e >= Ec) break;
    float s = 0.f;
    for (int q = 0; q < G; ++q) s += part[q * Ec + e];
    const float gate = sigmoidf_(gpre[k]);
    awe[e] = s;
    zs[e] = from_f<T>(gate * s);
  }
}

// ---- forward: input GEMM of the attention half + LSTMCell (torch gate order i, f, g, o) ----
// Block x owns units 4x..4x+3: its 16 columns are gate q = c/4 of unit 4x + c%4 (B row
// q*D + unit of W_ih[:, M:]), so all four gates of a unit meet in one block's tile.
// Rows go in groups of RG = 32 (blockIdx.y).
constexpr int RG = 32;
constexpr int RG_MT = RG / 16;
template <typename T, int SW, int DEPTH>
__global__ __launch_bounds__(64 * SW) void gate_cell_fwd_kernel(imgcap_lstm_desc d, int t) {
  __shared__ __attribute__((aligned(16))) float part[SW][RG][SKINNY_LDT];
  const int D = d.D, E = d.E, Tn = d.T;
  const int W3 = d.A + E + 4 * D;
  const int r0 = blockIdx.y * RG, rows = min(RG, d.B - r0);
  const int c = threadIdx.x & 15;
  const T* brow = (const T*)d.w_ih + (long)((c >> 2) * D + blockIdx.x * 4 + (c & 3)) * (d.M + E) + d.M;
  // the cell's other inputs (x-part + hh-part of the gates, c_{t-1}) are loaded before the GEMM
  // so their latency overlaps it; thread e < rows*4 owns (row e/4, unit 4*blockIdx.x + e%4)
  const int e = threadIdx.x;
  const bool cell_thread = e < rows * 4;
  const int b = r0 + (cell_thread ? (e >> 2) : 0), jj = e & 3, j = blockIdx.x * 4 + jj;
  const long bt = (long)b * Tn + t;
  float pre[4], cp = 0.f;
  if (cell_thread) {
    const float* xe = d.xe + bt * 4 * D;
    const float* hh = d.g1 + bt * W3 + d.A + E;
#pragma unroll
    for (int q = 0; q < 4; ++q) pre[q] = xe[q * D + j] + hh[q * D + j];
    cp = t == 0 ? d.c0[(long)b * D + j] : d.cs[(bt - 1) * D + j];
  }
  skinny_tile<T, RG_MT, SW, DEPTH>((const T*)d.zs + ((long)r0 * Tn + t) * E, (long)Tn * E, rows, brow, true, E,
                                   part);
  if (cell_thread) {
    float g[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) g[q] = part[0][b - r0][q * 4 + jj] + pre[q];
    const float gi = sigmoidf_(g[0]), gf = sigmoidf_(g[1]), gg = tanhf(g[2]), go = sigmoidf_(g[3]);
    const float cn = gf * cp + gi * gg;
    const float h = go * tanhf(cn);
    float* ga = d.gates + bt * 4 * D;
    ga[j] = gi; ga[D + j] = gf; ga[2 * D + j] = gg; ga[3 * D + j] = go;
    d.cs[bt * D + j] = cn;
    ((T*)d.hs)[bt * D + j] = from_f<T>(h);
    if (t + 1 < Tn) ((T*)d.hprev)[(bt + 1) * D + j] = from_f<T>(h);
  }
}

// LSTMCell backward of one (row, unit) at step t given dL/dh_t from the later steps (dh_next,
// without the fc term) and the carried dL/dc_t in d.dc; writes d gates_preact into dcat and
// the carry dL/dc_{t-1}.  Rows past their decode length contribute nothing.  The inputs are
// gathered by cell_bwd_load (so a kernel can issue them early) and consumed by cell_bwd_apply.
struct CellBwdIn {
  float dhs, gi, gf, gg, go, c, cp, dc;
  bool active;
};

template <typename T>
DEV CellBwdIn cell_bwd_load(const imgcap_lstm_desc& d, int t, int b, int j) {
  const int D = d.D, Tn = d.T;
  const long bt = (long)b * Tn + t;
  const long e = (long)b * D + j;
  CellBwdIn in;
  in.active = t < d.dl[b];
  const float* ga = d.gates + bt * 4 * D;
  in.dhs = to_f(((const T*)d.dhs)[bt * D + j]);
  in.gi = ga[j]; in.gf = ga[D + j]; in.gg = ga[2 * D + j]; in.go = ga[3 * D + j];
  in.c = d.cs[bt * D + j];
  in.cp = t == 0 ? d.c0[e] : d.cs[(bt - 1) * D + j];
  in.dc = d.dc[e];
  return in;
}

template <typename T>
DEV void cell_bwd_apply(const imgcap_lstm_desc& d, int t, int b, int j, const CellBwdIn& in, float dh_next,
                        bool has_next) {
  const int D = d.D, Tn = d.T;
  const int W3 = d.A + d.E + 4 * D;
  const long bt = (long)b * Tn + t;
  const long e = (long)b * D + j;
  T* dg = (T*)d.dcat + bt * W3 + d.A + d.E;
  if (!in.active) {
    dg[j] = dg[D + j] = dg[2 * D + j] = dg[3 * D + j] = from_f<T>(0.f);
    d.dc[e] = 0.f;
    return;
  }
  const float dh = in.dhs + (has_next ? dh_next : 0.f);
  const float tc = tanhf(in.c);
  const float dct = (has_next ? in.dc : 0.f) + dh * in.go * (1.f - tc * tc);
  dg[j] = from_f<T>(dct * in.gg * in.gi * (1.f - in.gi));
  dg[D + j] = from_f<T>(dct * in.cp * in.gf * (1.f - in.gf));
  dg[2 * D + j] = from_f<T>(dct * in.gi * (1.f - in.gg * in.gg));
  dg[3 * D + j] = from_f<T>(dh * tc * in.go * (1.f - in.go));
  d.dc[e] = dct * in.gf;
}

// ---- backward: LSTMCell of the last step (no carry from later steps) ------------------
template <typename T>
__global__ __launch_bounds__(256) void cell_bwd_last_kernel(imgcap_lstm_desc d) {
  const long n = (long)d.B * d.D;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < n; e += (long)gridDim.x * 256)
  {
    const int b = (int)(e / d.D), j = (int)(e % d.D);
    cell_bwd_apply<T>(d, d.T - 1, b, j, cell_bwd_load<T>(d, d.T - 1, b, j), 0.f, false);
  }
}

// ---- backward: dgates_t . [W_ih[:, M:] | W_hh]  -> K-slice partial slabs ----------------
// grid (ceil((E+D)/16), x_slices, row groups); slab z = d.dz[z][B][E + D]: columns < E are
// dL/dz_t, the rest the W_hh part of dL/dh_{t-1}.  Consumers add the slabs.
template <typename T, int SW, int DEPTH>
__global__ __launch_bounds__(64 * SW) void x_partial_kernel(imgcap_lstm_desc d, int t, int kslice) {
  __shared__ __attribute__((aligned(16))) float part[SW][RG][SKINNY_LDT];
  const int r0 = blockIdx.z * RG, rows = min(RG, d.B - r0);
  const int D = d.D, E = d.E, NX = E + D, K4 = 4 * D;
  const int W3 = d.A + E + K4;
  const int k0 = blockIdx.y * kslice, klen = min(K4 - k0, kslice);
  const int n0 = blockIdx.x * 16, n = n0 + (threadIdx.x & 15);
  const bool bok = n < NX;
  const T* A = (const T*)d.dcat + ((long)r0 * d.T + t) * W3 + d.A + E + k0;
  const T* brow = (const T*)d.w_zh_t + (long)(bok ? n : 0) * K4 + k0;
  skinny_tile<T, RG_MT, SW, DEPTH>(A, (long)d.T * W3, rows, brow, bok, klen, part);
  float* slab = d.dz + ((long)blockIdx.y * d.B + r0) * NX;
  for (int e = threadIdx.x; e < rows * 16; e += 64 * SW) {
    const int r = e >> 4, c = e & 15;
    if (n0 + c < NX) slab[(long)r * NX + n0 + c] = part[0][r][c];
  }
}

// ---- backward: dh_{t-1} = [d att2 | d gate_pre]_t . [W_da; W_fb] + W_hh slabs, then the
// LSTMCell backward of step t-1 (t >= 1) or dL/dh0 (t == 0).  grid (D/16, y_slices, row
// groups): each block publishes its K-slice tile; the last arriving block of a column tile (agent-scope
// release/acquire around a relaxed ticket, cdna_hip_programming.md §5 "Projection GEMM",
// item 2) sums the slabs in slice order and runs the epilogue.  y_cnt returns to 0.
template <typename T, int SW, int DEPTH>
__global__ __launch_bounds__(64 * SW) void dh_cell_kernel(imgcap_lstm_desc d, int t, int kslice) {
  __shared__ __attribute__((aligned(16))) float part[SW][RG][SKINNY_LDT];
  __shared__ int is_last;
  const int D = d.D, E = d.E, KY = d.A + E, NX = E + D;
  const int W3 = KY + 4 * D;
  const int ntile = gridDim.x, S = gridDim.y;
  const int r0 = blockIdx.z * RG, rows = min(RG, d.B - r0);
  const int tile = blockIdx.z * ntile + blockIdx.x;  // counter / slab index of (row group, columns)
  const int k0 = blockIdx.y * kslice, klen = min(KY - k0, kslice);
  const int n0 = blockIdx.x * 16, n = n0 + (threadIdx.x & 15);
  const T* A = (const T*)d.dcat + ((long)r0 * d.T + t) * W3 + k0;
  const T* brow = (const T*)d.w_att_t + (long)n * KY + k0;
  // epilogue inputs requested before the GEMM (only the last-arriving block uses them, but the
  // critical path is then the slab hand-off alone): W_hh part of dh from the x slabs and the
  // cell-backward operands of step t-1, for this thread's (row, unit) items
  constexpr int PER = RG * 16 / (64 * SW);
  float xh[PER];
  CellBwdIn cin[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int e = threadIdx.x + i * 64 * SW;
    const int b = r0 + min(e >> 4, rows - 1), j = n0 + (e & 15);
    float s = 0.f;
    for (int z = 0; z < d.x_slices; ++z) s += d.dz[((long)z * d.B + b) * NX + E + j];
    xh[i] = s;
    if (t > 0) cin[i] = cell_bwd_load<T>(d, t - 1, b, j);
  }
  skinny_tile<T, RG_MT, SW, DEPTH>(A, (long)d.T * W3, rows, brow, true, klen, part);
  constexpr int TILE = RG * 16;
  const long ntiles = (long)ntile * gridDim.z;
  float* slab = d.ws_y + ((long)blockIdx.y * ntiles + tile) * TILE;
  for (int e = threadIdx.x; e < TILE; e += 64 * SW) slab[e] = part[0][e >> 4][e & 15];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int ticket = __hip_atomic_fetch_add(d.y_cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = ticket == S - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(d.y_cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    is_last = last;
  }
  __syncthreads();
  if (!is_last) return;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int e = threadIdx.x + i * 64 * SW;
    if (e >= rows * 16) continue;
    const int b = r0 + (e >> 4), j = n0 + (e & 15);
    float dh = 0.f;
    for (int z = 0; z < S; ++z) dh += d.ws_y[((long)z * ntiles + tile) * TILE + e];
    dh += xh[i];
    if (t == 0) d.dh[(long)b * D + j] = dh;
    else cell_bwd_apply<T>(d, t - 1, b, j, cin[i], dh, true);
  }
}

// ---- backward attention step: recurrent part only ---------------------------------------
// Same load-everything-first structure as attn_fwd_kernel: the enc vectors (for d alpha =
// enc . d awe), the att1 vectors (for d att2), the dz slabs, gate, context and alphas are all
// requested before the first reduction; the reductions then run through LDS.
template <typename T, int MPP>
__global__ __launch_bounds__(ATT_THREADS) void attn_bwd_kernel(imgcap_lstm_desc d, int t) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int b = blockIdx.x;
  const int P = d.P, E = d.E, A = d.A, Tn = d.T;
  const int W3 = A + E + 4 * d.D;
  const long bt = (long)b * Tn + t;
  T* dcat = (T*)d.dcat + bt * W3;
  float* dawe_o = d.dawe ? d.dawe + ((long)b * (Tn + 1) + t) * E : nullptr;
  if (t >= d.dl[b]) {
    for (int i = threadIdx.x; i < A + E; i += ATT_THREADS) dcat[i] = from_f<T>(0.f);
    if (threadIdx.x < P) d.de[bt * P + threadIdx.x] = 0.f;
    if (dawe_o)
      for (int i = threadIdx.x; i < E; i += ATT_THREADS) dawe_o[i] = 0.f;
    return;
  }
  const int NVE = E / 8, G = ATT_THREADS / NVE;
  const int NVA = A / 8, GA = ATT_THREADS / NVA;
  float* dawe = sm;                  // [E]
  float* al = dawe + E;              // [MAXP]
  float* dal = al + MAXP;            // [MAXP]
  float* red = dal + MAXP;           // [P][NVE] d-alpha partials, then [GA][A] d-att2 partials
  const float* g1 = d.g1 + bt * W3;
  const int NX = E + d.D;
  const T* enc = (const T*)d.enc + (long)b * P * E;
  const T* att1 = (const T*)d.att1 + (long)b * P * A;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int v = tid % NVE, pg = tid / NVE;
  const int va = tid % NVA, pga = tid / NVA;
  // ---- all loads ----
  Raw8<T> ev[MPP];
#pragma unroll
  for (int i = 0; i < MPP; ++i) raw_load(ev[i], enc + (long)min(pg + i * G, P - 1) * E + v * 8);
  Raw8<T> av[MPP];
#pragma unroll
  for (int i = 0; i < MPP; ++i) raw_load(av[i], att1 + (long)min(pga + i * GA, P - 1) * A + va * 8);
  float att2[8];
  load8<float>(g1 + va * 8, att2);
  float gate[8], awe[8], dz[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (pg == 0) {
    load8<float>(g1 + A + v * 8, gate);
    load8<float>(d.awe + bt * E + v * 8, awe);
    for (int z = 0; z < d.x_slices; ++z) {  // dL/dz_t = sum of the x_partial slabs
      float q[8];
      load8<float>(d.dz + ((long)z * d.B + b) * NX + v * 8, q);
#pragma unroll
      for (int j = 0; j < 8; ++j) dz[j] += q[j];
    }
  }
  float alpha_in = 0.f, dalpha_in = 0.f;
  if (tid < P) {
    alpha_in = d.alphas[bt * P + tid];
    if (d.dalpha) dalpha_in = d.dalpha[bt * P + tid];
  }
  constexpr int APT = 1;  // A <= ATT_THREADS (checked on the host)
  const float wf_a = tid < A ? d.w_f[tid] : 0.f;
  // ---- d awe = dz * sigmoid(gate), d gate_pre = dz * awe * s (1 - s) ----
  if (pg == 0) {
    float dg[8];
    float da[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float s = sigmoidf_(gate[j]);
      da[j] = dz[j] * s;
      dawe[v * 8 + j] = da[j];
      dg[j] = dz[j] * awe[j] * s * (1.f - s);
    }
    st_g<T, 8>(dcat + A + v * 8, dg);
    if (dawe_o) st_g<float, 8>(dawe_o + v * 8, da);
  }
  if (tid < P) {
    al[tid] = alpha_in;
    dal[tid] = dalpha_in;  // upstream d alpha, read back by the softmax backward
  }
  __syncthreads();
  // ---- d alpha_p = enc_p . d awe (+ upstream) ----
  if (pg < G) {
    float dv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) dv[j] = dawe[v * 8 + j];
#pragma unroll
    for (int i = 0; i < MPP; ++i) {
      const int p = pg + i * G;
      if (p < P) {
        float x[8];
        raw_to_f(ev[i], x);
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) s += x[j] * dv[j];
        red[p * NVE + v] = s;
      }
    }
  }
  __syncthreads();
  for (int p = w; p < P; p += ATT_WAVES) {
    float s = 0.f;
    for (int q = lane; q < NVE; q += 64) s += red[p * NVE + q];
    s = wave_sum(s);
    if (lane == 0) dal[p] += s;
  }
  __syncthreads();
  if (w == 0) {  // softmax backward -> d score
    const float a = lane < P ? al[lane] : 0.f;
    const float da = lane < P ? dal[lane] : 0.f;
    const float dot = wave_sum(a * da);
    if (lane < P) {
      const float de = a * (da - dot);
      dal[lane] = de;
      d.de[bt * P + lane] = de;
    }
  }
  __syncthreads();
  // ---- d att2[a] = w_f[a] * sum_p de_p [att1[p,a] + att2[a] > 0] ----
  if (pga < GA) {
    float sacc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < MPP; ++i) {
      const int p = pga + i * GA;
      if (p < P) {
        float x[8];
        raw_to_f(av[i], x);
        const float de = dal[p];
#pragma unroll
        for (int j = 0; j < 8; ++j) sacc[j] += (x[j] + att2[j] > 0.f) ? de : 0.f;
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) red[pga * A + va * 8 + j] = sacc[j];
  }
  __syncthreads();
  static_assert(APT == 1, "one attention unit per thread");
  if (tid < A) {
    float s = 0.f;
    for (int q = 0; q < GA; ++q) s += red[q * A + tid];
    dcat[tid] = from_f<T>(s * wf_a);
  }
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

// ---- gradient w.r.t. the encoder output (encoder fine-tuning) ----------------------------
//   denc[sort_ind[b], p, e] = base[b, p, e] + sum_{t<T} alpha[b,t,p] dawe[b,t,e] + dawe[b,T,e] / P
// base = datt1 . W_ea (the attention-projection path, one GEMM), dawe rows t < T = d context
// per step (attn_bwd_kernel), row T = dL/d mean(enc) (init_h / init_c path).  Block = (batch
// row, 256 channels); alpha[b] staged in LDS; each thread keeps its channel's P sums in
// registers while t sweeps.
constexpr int DENC_P = 64;
__global__ __launch_bounds__(256) void lstm_denc_kernel(int T, int P, int E, const float* __restrict__ alphas,
                                                        const float* __restrict__ dawe, const float* __restrict__ base,
                                                        const int64_t* __restrict__ sort_ind,
                                                        float* __restrict__ denc) {
  extern __shared__ float al[];  // [T][P]
  const int b = blockIdx.y;
  for (int i = threadIdx.x; i < T * P; i += 256) al[i] = alphas[(long)b * T * P + i];
  __syncthreads();
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= E) return;
  float acc[DENC_P];
  const float* dw = dawe + (long)b * (T + 1) * E + e;
  const float m = dw[(long)T * E] / (float)P;
#pragma unroll
  for (int p = 0; p < DENC_P; ++p) acc[p] = m;
  for (int t = 0; t < T; ++t) {
    const float g = dw[(long)t * E];
#pragma unroll
    for (int p = 0; p < DENC_P; ++p)
      if (p < P) acc[p] += al[t * P + p] * g;
  }
  const long ob = sort_ind ? sort_ind[b] : b;
  const float* bs = base + (long)b * P * E + e;
  float* o = denc + ob * P * E + e;
#pragma unroll
  for (int p = 0; p < DENC_P; ++p)
    if (p < P) o[(long)p * E] = acc[p] + (base ? bs[(long)p * E] : 0.f);
}

// ---- doubly stochastic attention regularisation (train.py:269) --------------------------
//   reg = alphaC * mean_{b,p} (1 - sum_t alpha[b,t,p])^2
//   dalpha[b,t,p] = d reg / d alpha[b,t,p] for t < dl[b] (the written alphas), else 0
// one block per sample b: thread (p, t-slice) sums alpha over its steps, the per-pixel sums are
// combined in LDS in a fixed order; the block writes dalpha[b] and its share of the loss to
// part[b], summed in a fixed order by attn_reg_sum_kernel (deterministic, no atomics)
constexpr int REG_TS = 16;  // step slices per pixel
__global__ __launch_bounds__(1024) void attn_reg_kernel(int B, int Tn, int P, const float* __restrict__ alphas,
                                                        const int32_t* __restrict__ dl, float alphaC,
                                                        float* __restrict__ dalpha, float* __restrict__ part) {
  __shared__ float ps[REG_TS][MAXP];
  __shared__ float gs[MAXP];
  const int b = blockIdx.x;
  const int p = threadIdx.x % MAXP, ts = threadIdx.x / MAXP;
  const float* a = alphas + (long)b * Tn * P;
  float s = 0.f;
  if (p < P)
    for (int t = ts; t < Tn; t += REG_TS) s += a[(long)t * P + p];
  ps[ts][p] = s;
  __syncthreads();
  if (threadIdx.x < MAXP) {
    float tot = 0.f;
#pragma unroll
    for (int k = 0; k < REG_TS; ++k) tot += ps[k][threadIdx.x];
    const bool on = threadIdx.x < P;
    gs[threadIdx.x] = on ? alphaC * 2.f * (tot - 1.f) / (float)(B * P) : 0.f;
    float sq = on ? (1.f - tot) * (1.f - tot) : 0.f;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sq += __shfl_xor(sq, o);
    if (threadIdx.x == 0) part[b] = sq;
  }
  __syncthreads();
  const int db = dl[b];
  float* da = dalpha + (long)b * Tn * P;
  for (int e = threadIdx.x; e < Tn * P; e += blockDim.x) {
    const int t = e / P, pp = e % P;
    da[e] = t < db ? gs[pp] : 0.f;
  }
}

__global__ void attn_reg_sum_kernel(int B, int P, float alphaC, const float* __restrict__ part,
                                    float* __restrict__ reg_out) {
  if (threadIdx.x == 0) {
    float tot = 0.f;
    for (int b = 0; b < B; ++b) tot += part[b];
    *reg_out = alphaC * tot / (float)(B * P);
  }
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

// pixels per thread of the attention kernels' (vector, pixel-group) mappings
static int attn_mpp(const imgcap_lstm_desc& d) {
  const int G = ATT_THREADS / (d.E / 8), GA = ATT_THREADS / (d.A / 8);
  return std::max((d.P + G - 1) / G, (d.P + GA - 1) / GA);
}
static size_t attn_bwd_shm(const imgcap_lstm_desc& d) {
  const int GA = ATT_THREADS / (d.A / 8);
  const size_t red = std::max((size_t)d.P * (d.E / 8), (size_t)GA * d.A);
  return (d.E + 2 * MAXP + red) * sizeof(float);
}

// SW waves per block and DEPTH k-steps per load round: DEPTH = the wave's k-step count
// rounded up to a power of two (fp32 fragments are twice as wide: at most 2)
static int depth_for(int klen, int sw, bool f32) {
  const int per = ((klen + 31) / 32 + sw - 1) / sw;
  const int dpt = per <= 1 ? 1 : per <= 2 ? 2 : per <= 4 ? 4 : 8;
  return f32 ? std::min(dpt, 2) : dpt;
}

#define LSTM_DEPTH_SWITCH(dpt, KERNEL, SW, ...)                                      \
  do {                                                                               \
    if ((dpt) <= 1) hipLaunchKernelGGL((KERNEL<T, SW, 1>), __VA_ARGS__);             \
    else if ((dpt) <= 2) hipLaunchKernelGGL((KERNEL<T, SW, 2>), __VA_ARGS__);        \
    else if ((dpt) <= 4) hipLaunchKernelGGL((KERNEL<T, SW, (F32 ? 2 : 4)>), __VA_ARGS__); \
    else hipLaunchKernelGGL((KERNEL<T, SW, (F32 ? 2 : 8)>), __VA_ARGS__);            \
  } while (0)

int lstm_fwd_persistent(const imgcap_lstm_desc& d, hipStream_t st, bool* used);  // lstm_persist.hip
int lstm_persist_sync_words(const imgcap_lstm_desc& d);
int lstm_bwd_persistent(const imgcap_lstm_desc& d, hipStream_t st, bool* used);  // lstm_persist.hip

template <typename T>
static int lstm_fwd_impl(const imgcap_lstm_desc& d, hipStream_t st) {
  constexpr bool F32 = sizeof(T) == 4;
  bool used = false;
  if (int rc = lstm_fwd_persistent(d, st, &used)) return rc;
  if (used) return 0;
  const int W3 = d.A + d.E + 4 * d.D;
  const int ct = d.dtype;
  const int nrg = (d.B + RG - 1) / RG;
  const imgcap_epilogue e1 = f32_epi(d.b_hcat);
  const int dpt_g = depth_for(d.E, 8, F32);
  // channel chunks per row of the forward attention kernel (IMGCAP_LSTM_ATT_YS overrides)
  static const int ys_env = [] {
    const char* e = getenv("IMGCAP_LSTM_ATT_YS");
    return e ? atoi(e) : 0;
  }();
  int ys = ys_env > 0 ? ys_env : LSTM_ATT_YS;
  while (ys > 1 && d.E % (8 * ys) != 0) --ys;
  const int Gf = ATT_THREADS / (d.E / ys / 8);
  const int mpp = (d.P + Gf - 1) / Gf;  // <= attn_mpp(d) <= 16 (checked at entry)
  const size_t shm_f = (size_t)Gf * (d.E / ys) * sizeof(float);
  const dim3 gatt(d.B, ys);
  for (int t = 0; t < d.T; ++t) {
    int rc = imgcap_gemm(ct, 1, 1, d.B, W3, d.D, (const T*)d.hprev + (long)t * d.D, (long)d.T * d.D, 0, d.w_hcat,
                         d.D, 0, d.g1 + (long)t * W3, (long)d.T * W3, 0, 1, &e1, st);
    if (rc) return rc;
    if (mpp <= 2)
      hipLaunchKernelGGL((attn_fwd_kernel<T, 2>), gatt, dim3(ATT_THREADS), shm_f, st, d, t);
    else if (mpp <= 4)
      hipLaunchKernelGGL((attn_fwd_kernel<T, 4>), gatt, dim3(ATT_THREADS), shm_f, st, d, t);
    else if (mpp <= 5)
      hipLaunchKernelGGL((attn_fwd_kernel<T, 5>), gatt, dim3(ATT_THREADS), shm_f, st, d, t);
    else if (mpp <= 8)
      hipLaunchKernelGGL((attn_fwd_kernel<T, 8>), gatt, dim3(ATT_THREADS), shm_f, st, d, t);
    else
      hipLaunchKernelGGL((attn_fwd_kernel<T, 16>), gatt, dim3(ATT_THREADS), shm_f, st, d, t);
    IMGCAP_CHECK_LAUNCH("lstm attn_fwd");
    LSTM_DEPTH_SWITCH(dpt_g, gate_cell_fwd_kernel, 8, dim3(d.D / 4, nrg), dim3(512), 0, st, d, t);
    IMGCAP_CHECK_LAUNCH("lstm gate_cell_fwd");
  }
  return 0;
}

template <typename T>
static int lstm_bwd_impl(const imgcap_lstm_desc& d, hipStream_t st) {
  constexpr bool F32 = sizeof(T) == 4;
  const int nrg = (d.B + RG - 1) / RG;
  const int NX = d.E + d.D, K4 = 4 * d.D, KY = d.A + d.E;
  const int kx = ((K4 + d.x_slices - 1) / d.x_slices + 31) / 32 * 32;
  const int ky = ((KY + d.y_slices - 1) / d.y_slices + 31) / 32 * 32;
  const int sx = (K4 + kx - 1) / kx, sy = (KY + ky - 1) / ky;  // non-empty slices
  const int dpt_x = depth_for(kx, 8, F32), dpt_y = depth_for(ky, 4, F32);
  const size_t shm = attn_bwd_shm(d);
  const int mpp = attn_mpp(d);
  imgcap_lstm_desc dd = d;
  dd.x_slices = sx;
  dd.y_slices = sy;
  bool used = false;
  if (int rc = lstm_bwd_persistent(dd, st, &used)) return rc;
  if (!used) {
  hipLaunchKernelGGL(cell_bwd_last_kernel<T>, pw_grid((long)d.B * d.D), dim3(256), 0, st, dd);
  IMGCAP_CHECK_LAUNCH("lstm cell_bwd_last");
  for (int t = d.T - 1; t >= 0; --t) {
    LSTM_DEPTH_SWITCH(dpt_x, x_partial_kernel, 8, dim3((NX + 15) / 16, sx, nrg), dim3(512), 0, st, dd, t, kx);
    IMGCAP_CHECK_LAUNCH("lstm x_partial");
    if (mpp <= 4)
      hipLaunchKernelGGL((attn_bwd_kernel<T, 4>), dim3(d.B), dim3(ATT_THREADS), shm, st, dd, t);
    else if (mpp <= 5)
      hipLaunchKernelGGL((attn_bwd_kernel<T, 5>), dim3(d.B), dim3(ATT_THREADS), shm, st, dd, t);
    else if (mpp <= 8)
      hipLaunchKernelGGL((attn_bwd_kernel<T, 8>), dim3(d.B), dim3(ATT_THREADS), shm, st, dd, t);
    else
      hipLaunchKernelGGL((attn_bwd_kernel<T, 16>), dim3(d.B), dim3(ATT_THREADS), shm, st, dd, t);
    IMGCAP_CHECK_LAUNCH("lstm attn_bwd");
    LSTM_DEPTH_SWITCH(dpt_y, dh_cell_kernel, 4, dim3(d.D / 16, sy, nrg), dim3(256), 0, st, dd, t, ky);
    IMGCAP_CHECK_LAUNCH("lstm dh_cell");
  }
  }
  const size_t shm2 = (size_t)d.T * PCH * sizeof(float);
  const int thr = d.A >= 512 ? 512 : ((d.A + 63) / 64) * 64;
  hipLaunchKernelGGL(attn_param_grad_kernel<T>, dim3((d.P + PCH - 1) / PCH, d.B), dim3(thr), shm2, st, dd);
  IMGCAP_CHECK_LAUNCH("lstm attn_param_grad");
  return 0;
}

static int check_desc(const imgcap_lstm_desc* d) {
  IMGCAP_REQUIRE(d != nullptr, "lstm desc NULL");
  IMGCAP_REQUIRE(d->dtype == IMGCAP_F32 || d->dtype == IMGCAP_BF16, "lstm: dtype");
  IMGCAP_REQUIRE(d->B > 0 && d->T > 0 && d->P > 0 && d->P <= MAXP, "lstm: need 0 < P <= 64");
  IMGCAP_REQUIRE(d->E % 8 == 0 && d->A % 8 == 0 && d->M % 8 == 0 && d->D % 16 == 0, "lstm: E, A, M % 8, D % 16");
  IMGCAP_REQUIRE(d->A <= 512 && d->E <= 2 * ATT_THREADS, "lstm: attention_dim <= 512, encoder_dim <= 2048");
  IMGCAP_REQUIRE(attn_mpp(*d) <= 16, "lstm: too many pixels per attention thread");
  IMGCAP_REQUIRE((size_t)(ATT_THREADS / (d->E / 8)) * d->E * 4 <= 65536 && attn_bwd_shm(*d) <= 65536,
                 "lstm: attention LDS budget");
  return 0;
}

}  // namespace imgcap

using namespace imgcap;

extern "C" int imgcap_lstm_tf_fwd(const imgcap_lstm_desc* d, void* stream) {
  if (int rc = check_desc(d)) return rc;
  if (d->dtype == IMGCAP_BF16) return lstm_fwd_impl<bf16>(*d, (hipStream_t)stream);
  return lstm_fwd_impl<float>(*d, (hipStream_t)stream);
}

extern "C" int imgcap_lstm_sync_words(const imgcap_lstm_desc* d) {
  if (check_desc(d)) return 0;
  return lstm_persist_sync_words(*d);
}

extern "C" int imgcap_lstm_tf_bwd(const imgcap_lstm_desc* d, void* stream) {
  if (int rc = check_desc(d)) return rc;
  IMGCAP_REQUIRE((size_t)d->T * PCH * 4 <= 65536, "lstm bwd: T too large for LDS");
  IMGCAP_REQUIRE(d->w_zh_t && d->w_att_t && d->de && d->dbea && d->ws_y && d->y_cnt,
                 "lstm bwd: transposed weights / de / dbea / ws_y / y_cnt needed");
  IMGCAP_REQUIRE(d->x_slices >= 1 && d->x_slices <= 16 && d->y_slices >= 1 && d->y_slices <= 16,
                 "lstm bwd: x_slices, y_slices in [1, 16]");
  if (d->dtype == IMGCAP_BF16) return lstm_bwd_impl<bf16>(*d, (hipStream_t)stream);
  return lstm_bwd_impl<float>(*d, (hipStream_t)stream);
}

extern "C" int imgcap_attn_reg(int B, int T, int P, const float* alphas, const int32_t* dl, float alphaC,
                               float* dalpha, float* reg_out, float* part, void* stream) {
  IMGCAP_REQUIRE(P <= MAXP, "imgcap_attn_reg: P must be <= 64");
  if (B == 0) return 0;
  if (!part) {
    part = (float*)workspace((size_t)B * sizeof(float), (hipStream_t)stream);
    if (!part) return fail(IMGCAP_EWORKSPACE, std::string("imgcap_attn_reg: ") + last_error());
  }
  hipLaunchKernelGGL(attn_reg_kernel, dim3(B), dim3(REG_TS * MAXP), 0, (hipStream_t)stream, B, T, P, alphas, dl, alphaC,
                     dalpha, part);
  hipLaunchKernelGGL(attn_reg_sum_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, B, P, alphaC, part, reg_out);
  IMGCAP_CHECK_LAUNCH("imgcap_attn_reg");
  return 0;
}

extern "C" int imgcap_lstm_denc(int B, int T, int P, int E, const float* alphas, const float* dawe, const float* base,
                                const int64_t* sort_ind, float* denc, void* stream) {
  IMGCAP_REQUIRE(P <= DENC_P, "imgcap_lstm_denc: P must be <= 64");
  IMGCAP_REQUIRE(denc != base, "imgcap_lstm_denc: denc must not alias base (rows are permuted)");
  if (B == 0 || E == 0) return 0;
  const size_t shm = (size_t)T * P * sizeof(float);
  IMGCAP_REQUIRE(shm <= 64 * 1024, "imgcap_lstm_denc: T*P too large");
  hipLaunchKernelGGL(lstm_denc_kernel, dim3((E + 255) / 256, B), dim3(256), shm, (hipStream_t)stream, T, P, E, alphas,
                     dawe, base, sort_ind, denc);
  IMGCAP_CHECK_LAUNCH("imgcap_lstm_denc");
  return 0;
}

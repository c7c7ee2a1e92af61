// Persistent forward recurrence of the teacher-forced LSTM-attention decoder
// (models/decoder.py:69-113): ONE launch runs every step t < min(T, max decode length).
//
// Why: the per-step kernels of lstm.hip (skinny GEMM -> attention -> gate/cell, three launches
// per step) spend most of each launch refilling registers from L2 and draining; here every
// workgroup keeps its operands resident in LDS for the whole sequence and the steps are chained
// by in-launch hand-offs.
//
// Roles (one 512-thread workgroup per CU; the LDS request keeps it that way):
//   UG blocks [0, NUG):   U role (blk < NU): UPB LSTM units = UC = 4*UPB gate columns (all four
//                         gates of each unit), rows of [W_ih[:, M:] | W_hh] resident in LDS;
//                         gates = xe + [z_t | h_{t-1}] . W^T + b_hh, then the LSTMCell -> h_t.
//                         G role (blk < NG): 32 columns of [W_da; W_fb] resident in LDS;
//                         [att2 | gate_pre]_t = h_{t-1} . W^T + b  (decoder.py:27,104).
//   R blocks [NUG, +B*RS): batch row b, channel chunk s of E: att1[b] and enc[b][:, chunk]
//                         resident in LDS; scores, softmax, context, sigmoid gate -> z_t[b]
//                         (decoder.py:25-31, 102-105).
// Per step three hand-offs: h_{t-1} (all U blocks) -> G and U;  [att2 | gate_pre] (all G
// blocks) -> R;  z_t (all R blocks) -> U.
//   g and z: tagged granules -- every value travels in a naturally aligned 8-byte {value bits,
//   epoch} granule written by one write-through (sc1) store (a 16-byte store carries two), and
//   the consumer's sc1 loads of the granules are the poll: no drain, no separate flag, no second
//   round trip (MI355X_MICROARCH.md handoff-1to1 vs handoff-flag; granules observed untorn on
//   gfx950 / ROCm 7.2, also as 16-byte halves).  A U block polls one sentinel granule pair per
//   lane before sweeping its 48 KB of z granules.  z granules live in two slots by step parity
//   (a slot is rewritten two steps later, by which time every consumer has read it: the chain
//   z_t -> h_t -> g_{t+1} -> z_{t+1} passes through every block), tag = step + 1.
//   h: write-through hs rows + one flag per U block (drained sc1 stores, then a relaxed agent-
//   scope flag store; the consumer's wave 0 polls the flags, a barrier, sc1 payload loads).  As
//   granules (IMGCAP_LSTM_HGRAN=1, the HG instantiation) the h hop measured 3.3-3.4 us against 2.0
//   (32 KB of granules per consumer instead of a 16 KB payload), the step 15.1 vs 14.6 us.
// The flag / granule area is zeroed by a kernel before the launch.
// Every spin is bounded: on timeout (or when another block already gave up) the block writes
// the error word and returns, so the grid always drains.
//
// Outputs are those of the per-step path (imgcap_lstm_tf_fwd), except g1's hh columns, which
// only the per-step gate kernel reads.  Steps t >= max decode length are not computed; their
// outputs are written as zeros (every row is past its decode length there, so the loss and
// the backward never use them).
#include <algorithm>

#include "mfma.h"

namespace imgcap {

static int device_cus();

namespace {

constexpr int PT = 512;            // threads per workgroup (8 waves: two per SIMD hide each other's latency)
constexpr int PWV = PT / 64;       // waves
constexpr int GCOLS = 32;          // G columns per workgroup
constexpr int SPIN_LIMIT = 1 << 21;
template <typename T> struct MaxKs { static constexpr int N = sizeof(T) == 2 ? 16 : 8; };  // U-phase k-steps per wave
// forward: k-steps per wave by row tiles (the granule polls hold every step's loads in flight;
// MT = 1 has 8 K parts, so 8 steps cover K = E + D <= 2048)
template <typename T, int MT> struct MaxKsF { static constexpr int N = sizeof(T) == 2 && MT == 2 ? 16 : 8; };
constexpr int SYNC_HDR = 16;       // words before the flags (word 0: error)

typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
typedef __amdgpu_buffer_rsrc_t rsrc_t;

DEV rsrc_t make_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
// 16-byte write-through (sc1) load / store
DEV uint4 ld_wt(rsrc_t r, uint32_t off) {
  const u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16);
  return make_uint4(v[0], v[1], v[2], v[3]);
}
DEV void st_wt(rsrc_t r, uint32_t off, uint4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{v.x, v.y, v.z, v.w}, r, off, 0, 16);
}

struct Geo {
  int NU, NG, NUG, RS, Ec, NR, UPB, KU, ldu, ldg, rc;
  int ug_red, ug_hst, r_enc, r_red, r_red2, r_es;  // byte offsets into dynamic LDS
  long long* stamps;  // diagnostics (IMGCAP_LSTM_STAMPS=1): per step, s_memrealtime at phase edges
  int gran_off;       // sync word offset of the [B][A + E] {epoch, value} granules (G -> R hand-off)
  int r_gv;           // R: LDS offset of the row's [att2 | gate_pre chunk] values
  int ldE;            // R: LDS pitch (elements) of the enc rows: Ec + 32, see lstm_fwd_body
  int* err;           // the launch's error word (shared by the row groups)
  int fault_step;     // test knob (IMGCAP_LSTM_FAULT_FWD): U block 0 never publishes h of this step
  int hg_off, zg_off; // sync word offsets of the h / z granule slots: [2][B][D or E / VPG] {value(s), epoch}
  int hgran;          // h_t hand-off: 1 = tagged granules, 0 = write-through hs rows + per-block flags
  int poll_sleep;     // s_sleep rounds after an incomplete granule poll pass (0 = spin)
};

// thread 0 of block 0 (U+G) and of the first R block records [role][t][k]
DEV void stamp(const Geo& g, int role, int t, int k, bool drain = false) {
  if (g.stamps && threadIdx.x == 0 && (blockIdx.x == 0 || (int)blockIdx.x == g.NUG)) {
    if (drain) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    g.stamps[(role * 64 + t) * 16 + k] = (long long)__builtin_amdgcn_s_memrealtime();
    if (k == 0) g.stamps[(role * 64 + t) * 16 + 15] = (long long)__builtin_amdgcn_s_memtime();
  }
}

// Wave 0 polls n per-producer flags (plus the error word) until all reach `epoch`; the result
// is shared through LDS and a workgroup barrier follows (the other waves load after it).
DEV bool poll_once(const int* flags, int n, int epoch, int* err, int lane, bool& bad) {
  bool all = true;
  bad = false;
  for (int i = lane; i <= n; i += 64) {
    const int v = __hip_atomic_load(i < n ? flags + i : err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (i < n) all = all && v >= epoch;
    else bad = v != 0;
  }
  return all;
}

// Wave 0 polls n per-producer flags (plus the error word) until all reach `epoch`; the result
// is shared through LDS and a workgroup barrier follows (the other waves load after it).
DEV bool block_wait(const int* flags, int n, int epoch, int* err, int* s_ok) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    bool ok = false;
    for (int spins = 0;; ++spins) {
      bool bad;
      const bool all = poll_once(flags, n, epoch, err, lane, bad);
      if (__any(bad)) break;
      if (__all(all)) { ok = true; break; }
      if (spins >= SPIN_LIMIT) {
        if (lane == 0) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
    if (lane == 0) *s_ok = ok;
  }
  __syncthreads();
  return *s_ok != 0;
}

// every storing wave drains its write-through stores, then one lane publishes the flag
DEV void block_publish(int* flag, int epoch) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(flag, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <typename T> struct VecOf { static constexpr int N = 16 / sizeof(T); };

// wave64 reductions on DPP (quad_perm, row mirrors, row_bcast15/31): the total lands in lane 63
// and is broadcast with readlane -- no LDS round trip (ds_bpermute) per step
#define IMGCAP_DPP(v, ctrl, rmask) \
  __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), ctrl, rmask, 0xF, false))
DEV float wave_sum_dpp(float v) {
  v += IMGCAP_DPP(v, 0xB1, 0xF);   // quad_perm [1,0,3,2]
  v += IMGCAP_DPP(v, 0x4E, 0xF);   // quad_perm [2,3,0,1]
  v += IMGCAP_DPP(v, 0x141, 0xF);  // row_half_mirror
  v += IMGCAP_DPP(v, 0x140, 0xF);  // row_mirror
  v += IMGCAP_DPP(v, 0x142, 0xA);  // row_bcast15
  v += IMGCAP_DPP(v, 0x143, 0xC);  // row_bcast31
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}
#define IMGCAP_DPP_MAX(v, ctrl, rmask)                                                              \
  __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, -INFINITY),         \
                                                        __builtin_bit_cast(int, v), ctrl, rmask, 0xF, false))
DEV float wave_max_dpp(float v) {
  v = fmaxf(v, IMGCAP_DPP_MAX(v, 0xB1, 0xF));
  v = fmaxf(v, IMGCAP_DPP_MAX(v, 0x4E, 0xF));
  v = fmaxf(v, IMGCAP_DPP_MAX(v, 0x141, 0xF));
  v = fmaxf(v, IMGCAP_DPP_MAX(v, 0x140, 0xF));
  v = fmaxf(v, IMGCAP_DPP_MAX(v, 0x142, 0xA));
  v = fmaxf(v, IMGCAP_DPP_MAX(v, 0x143, 0xC));
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}
// sum over the 4 lanes of a quad, every lane of the quad gets it
DEV float quad_sum_dpp(float v) {
  v += IMGCAP_DPP(v, 0xB1, 0xF);
  v += IMGCAP_DPP(v, 0x4E, 0xF);
  return v;
}
// Eight wave sums at once: lane l returns the sum over all 64 lanes of v[(l >> 3) & 7].  Each
// exchange halves the values a lane carries (32 -> 4, 16 -> 2, 8 -> 1 values), then three more
// for the last one: 10 shuffles instead of 8 x (6 DPP steps + readlane).
DEV float wave_sum8_t(const float (&v)[8], int lane) {
  const bool h5 = lane & 32, h4 = lane & 16, h3 = lane & 8;
  float a[4], b[2];
#pragma unroll
  for (int k = 0; k < 4; ++k) a[k] = (h5 ? v[4 + k] : v[k]) + __shfl_xor(h5 ? v[k] : v[4 + k], 32, 64);
#pragma unroll
  for (int k = 0; k < 2; ++k) b[k] = (h4 ? a[2 + k] : a[k]) + __shfl_xor(h4 ? a[k] : a[2 + k], 16, 64);
  float c = (h3 ? b[1] : b[0]) + __shfl_xor(h3 ? b[0] : b[1], 8, 64);
  c += __shfl_xor(c, 4, 64);
  c += __shfl_xor(c, 2, 64);
  c += __shfl_xor(c, 1, 64);
  return c;
}

DEV void unpack8(const uint4& a, const uint4& b, float (&v)[8]) {
  v[0] = __uint_as_float(a.x); v[1] = __uint_as_float(a.y); v[2] = __uint_as_float(a.z); v[3] = __uint_as_float(a.w);
  v[4] = __uint_as_float(b.x); v[5] = __uint_as_float(b.y); v[6] = __uint_as_float(b.z); v[7] = __uint_as_float(b.w);
}

// B fragment from LDS, zero for k0 >= K (a register select: the MFMA stays wave-uniform)
template <typename T>
DEV Frag<T> lds_frag_k(const T* row, int k0, int K) {
  const bool ok = k0 < K;
  Frag<T> f = lds_frag<T>(row + (ok ? k0 : 0));
  if (!ok) f = frag_from<T>(make_uint4(0u, 0u, 0u, 0u), make_uint4(0u, 0u, 0u, 0u));
  return f;
}

// A fragment (8 k of one row) from a write-through buffer; zero outside [0, rows) x [0, K)
template <typename T>
DEV Frag<T> frag_wt(rsrc_t r, uint32_t off, bool ok) {
  // branch-free: a masked fragment reads past the buffer's range, which the buffer load returns
  // as zeros (a conditional load leaves the compiler's vmcnt waits conservative)
  const uint32_t o = ok ? off : 0x80000000u;
  const uint4 lo = ld_wt(r, o);
  const uint4 hi = sizeof(T) == 4 ? ld_wt(r, o + 16) : lo;
  return frag_from<T>(lo, hi);
}

// Tagged granules: one naturally aligned 8-byte {value bits, epoch} pair written by ONE store (a
// 16-byte write-through store carries two); the data is its own flag (no drain, no separate flag,
// no second round trip; MI355X_MICROARCH.md handoff-1to1 vs handoff-flag).  Values per granule:
// two bf16 or one fp32.  A fragment (8 consecutive values of one row) is 4 (bf16) / 8 (fp32)
// granules = 2 / 4 sixteen-byte loads.
template <typename T> struct GranOf {
  static constexpr int VPG = sizeof(T) == 2 ? 2 : 1;  // values per granule
  static constexpr int NL = 4 / VPG;                  // 16-byte loads per fragment
};
// One pass over a fragment's granules: the fragment and whether every tag is `ep` (an offset
// past the buffer's range returns zeros without a memory access: the caller passes one for a
// fragment it already holds or does not need)
template <typename T>
DEV bool frag_gran(rsrc_t r, uint32_t off, unsigned ep, Frag<T>& f) {
  constexpr int NL = GranOf<T>::NL;
  uint4 q[NL];
#pragma unroll
  for (int i = 0; i < NL; ++i) q[i] = ld_wt(r, off + 16 * i);
  bool ok = true;
#pragma unroll
  for (int i = 0; i < NL; ++i) ok = ok && q[i].y == ep && q[i].w == ep;
  const uint4 lo = make_uint4(q[0].x, q[0].z, q[1].x, q[1].z);
  const uint4 hi = NL == 4 ? make_uint4(q[NL / 2].x, q[NL / 2].z, q[NL - 1].x, q[NL - 1].z) : lo;
  f = frag_from<T>(lo, hi);
  return ok;
}
// 8 values (one fragment's worth, packed as T in lo/hi) stored as tagged granules at byte `off`
template <typename T>
DEV void store_gran8(rsrc_t r, uint32_t off, const uint4& lo, const uint4& hi, unsigned ep) {
  if constexpr (sizeof(T) == 2) {
    st_wt(r, off, make_uint4(lo.x, ep, lo.y, ep));
    st_wt(r, off + 16, make_uint4(lo.z, ep, lo.w, ep));
  } else {
    st_wt(r, off, make_uint4(lo.x, ep, lo.y, ep));
    st_wt(r, off + 16, make_uint4(lo.z, ep, lo.w, ep));
    st_wt(r, off + 32, make_uint4(hi.x, ep, hi.y, ep));
    st_wt(r, off + 48, make_uint4(hi.z, ep, hi.w, ep));
  }
}
// Wave-level poll of up to N fragments: fragment i is wanted where (want >> i) & 1, at byte
// offset base + i * stride, tag ep.  Spins until every wanted fragment of every lane carries the
// tag; a bounded spin (or an error word already set by another block) returns false.
template <typename T, int N>
DEV bool poll_frags(rsrc_t r, int base, int stride, unsigned want, unsigned ep, Frag<T> (&fa)[N], int* err,
                    int sleep) {
  // sentinel: until the first granule pair of each lane's first wanted fragment carries the tag,
  // poll only that (16 bytes per lane per pass instead of every fragment); a producer writes all
  // of a row's granules within one phase, so the full pass that follows usually completes at once
  {
    const uint32_t so = want ? (uint32_t)(base + __builtin_ctz(want) * stride) : 0x80000000u;
    for (int spins = 0;; ++spins) {
      const uint4 q = ld_wt(r, so);
      if (__all(!want || q.y == ep)) break;
      if ((spins & 255) == 255 &&
          (spins >= SPIN_LIMIT || __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return false;
      }
    }
  }
  unsigned pending = want;
  for (int spins = 0;; ++spins) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      Frag<T> f;
      const bool need = (pending >> i) & 1u;
      const bool ok = frag_gran<T>(r, need ? (uint32_t)(base + i * stride) : 0x80000000u, ep, f);
      if (need && ok) {
        fa[i] = f;
        pending &= ~(1u << i);
      }
    }
    if (__all(pending == 0u)) return true;
    for (int q = 0; q < sleep; ++q) __builtin_amdgcn_s_sleep(2);
    if ((spins & 63) == 63 &&
        (spins >= SPIN_LIMIT / 8 || __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
      __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
  }
}

template <typename T, int MT, bool HG>
DEV void lstm_fwd_body(const imgcap_lstm_desc& d, const Geo& g, const int blk) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int* s_ok = (int*)smem;
  const int B = d.B, P = d.P, E = d.E, A = d.A, D = d.D, M = d.M, Tn = d.T;
  const int W3 = A + E + 4 * D;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int* err = g.err;
  // steps actually run: every row is past its decode length from max(dl) on
  if (tid < 64) {
    int m = 0;
    for (int i = lane; i < B; i += 64) m = max(m, d.dl[i]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = max(m, __shfl_xor(m, o, 64));
    if (lane == 0) s_ok[1] = m;
  }
  __syncthreads();
  const int Tmax = max(0, min(Tn, s_ok[1]));
  constexpr int VEC = VecOf<T>::N;
  const rsrc_t r_h0 = make_rsrc(d.hprev, (uint32_t)((long)B * Tn * D * sizeof(T)));
  const rsrc_t r_hs = make_rsrc(d.hs, (uint32_t)((long)B * Tn * D * sizeof(T)));
  int* fh = d.sync + SYNC_HDR;  // per-U-block h flags (hgran == 0)
  const rsrc_t r_gr = make_rsrc(d.sync + g.gran_off, (uint32_t)((long)B * (A + E) * 8));

  if (blk < g.NUG) {
    // ======================= U / G workgroup =======================================
    constexpr int KP = PWV / MT;         // K parts: wave w -> row tile w % MT, K part w / MT
    constexpr int NTU = 2;  // UPB = 8 units = 32 gate columns
    constexpr int UC = 16 * NTU;
    constexpr int MAXKS = MaxKsF<T, MT>::N;
    const int UPB = g.UPB;
    const bool isU = blk < g.NU, isG = blk < g.NG;
    const int u0 = blk * UPB;
    const int KU = g.KU, ldu = g.ldu, ldg = g.ldg, RC = g.rc;
    T* wu = (T*)(smem + 16);
    T* wg = wu + UC * ldu;
    float* red = (float*)(smem + g.ug_red);  // [KP][16*MT][RC]
    T* hst = (T*)(smem + g.ug_hst);          // [16*MT][UPB]
    // ---- resident weights ----
    if (isU) {
      const int cpr = KU / VEC;
      for (int i = tid; i < UC * cpr; i += PT) {
        const int c = i / cpr, k = (i % cpr) * VEC;
        const int row = (c / UPB) * D + u0 + c % UPB;
        const T* src = k < E ? (const T*)d.w_ih + (long)row * (M + E) + M + k
                             : (const T*)d.w_hcat + (long)(A + E + row) * D + (k - E);
        *(uint4*)(wu + c * ldu + k) = *(const uint4*)src;
      }
    }
    if (isG) {
      const int cpr = D / VEC;
      for (int i = tid; i < GCOLS * cpr; i += PT) {
        const int c = i / cpr, k = (i % cpr) * VEC;
        const int col = blk * GCOLS + c;
        *(uint4*)(wg + c * ldg + k) =
            col < A + E ? *(const uint4*)((const T*)d.w_hcat + (long)col * D + k) : make_uint4(0u, 0u, 0u, 0u);
      }
    }
    // ---- cell state of this thread's (row, unit) items ----
    constexpr int CPT = (16 * MT * 8 + PT - 1) / PT;  // (row, unit) items per thread
    float creg[CPT], bh[CPT][4];
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      const int i = tid + k * PT, b = i / UPB, j = u0 + i % UPB;
      const bool ok = isU && b < B;
      creg[k] = ok ? d.c0[(long)b * D + j] : 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) bh[k][q] = ok ? d.b_hcat[A + E + q * D + j] : 0.f;
    }
    // G output bias: a thread always stores the same 4 columns (PT is a multiple of GCOLS / 4)
    float gb[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = blk * GCOLS + (tid % (GCOLS / 4)) * 4 + j;
      gb[j] = isG && col < A + E ? d.b_hcat[col] : 0.f;
    }
    if (tid == 0) s_ok[2] = 1;  // cleared (for good) by a wave whose granule poll gave up
    __syncthreads();
    const int mi = w % MT, kp = w / MT;
    const int fr = lane & 15, fk = 8 * (lane >> 4);
    const int m = mi * 16 + fr;
    const bool mok = m < B;
    constexpr int VPG = GranOf<T>::VPG;
    const rsrc_t r_hg = make_rsrc(d.sync + g.hg_off, (uint32_t)(2L * B * (D / VPG) * 8));
    const rsrc_t r_zg = make_rsrc(d.sync + g.zg_off, (uint32_t)(2L * B * (E / VPG) * 8));
    for (int t = 0; t < Tmax; ++t) {
      stamp(g, 0, t, 0);
      // h_{t-1} rows: h0 (hprev slot 0) at t = 0, else the U blocks' h granules of step t-1
      const long hrow = (long)m * Tn;
      // U prefetch (issued before the G phase so its round trip overlaps it): xe, h part of A
      float xe[CPT][4];
#pragma unroll
      for (int k = 0; k < CPT; ++k) {
        const int i = tid + k * PT, b = i / UPB, j = u0 + i % UPB;
#pragma unroll
        for (int q = 0; q < 4; ++q) xe[k][q] = isU && b < B ? d.xe[((long)b * Tn + t) * 4 * D + q * D + j] : 0.f;
      }
      // A = [z_t | h_{t-1}]: the h part is available now, the z part after the R blocks'
      // hand-off; every fragment of this wave's K range is requested in one round trip each.
      // The G product (h_{t-1} [W_da; W_fb]^T) multiplies the SAME h fragments, so G blocks
      // (U blocks or not) request them too and G runs on them: one round trip of h per block.
      const int nks = (KU + 31) / 32, per = (nks + KP - 1) / KP;
      const int ks0 = kp * per, ks1 = min(nks, ks0 + per);
      const long zrow = (long)m * Tn + t;
      Frag<T> fa[MAXKS];
      unsigned hwant = 0u, zwant = 0u;
#pragma unroll
      for (int i = 0; i < MAXKS; ++i) {
        const int k0 = (ks0 + i) * 32 + fk;
        const bool in = mok && ks0 + i < ks1;
        const bool hk = (isU || isG) && in && k0 >= E && k0 < KU;
        fa[i] = frag_from<T>(make_uint4(0u, 0u, 0u, 0u), make_uint4(0u, 0u, 0u, 0u));
        if (t == 0) {
          fa[i] = frag_wt<T>(r_h0, (uint32_t)((hrow * D + (k0 - E)) * sizeof(T)), hk);
        } else if (hk) {
          hwant |= 1u << i;
        }
        if (isU && in && k0 < E) zwant |= 1u << i;
      }
      // granule byte offsets of this wave's first k-step (affine in the step: 32 / VPG granules)
      constexpr int GSTRIDE = 32 / VPG * 8;
      const int k00 = ks0 * 32 + fk;
      const int hbase = ((((t - 1) & 1) * B + m) * (D / VPG) + (k00 - E) / VPG) * 8;
      const int zbase = (((t & 1) * B + m) * (E / VPG) + k00 / VPG) * 8;
      if (t > 0 && HG) {
        if (!poll_frags<T, MAXKS>(r_hg, hbase, GSTRIDE, hwant, (unsigned)t, fa, err, g.poll_sleep) && lane == 0)
          s_ok[2] = 0;
      } else if (t > 0) {  // every U block's flag, then the write-through hs rows of step t-1
        if (!block_wait(fh, g.NU, t, err, s_ok + 3)) return;
        const long hprow = (long)m * Tn + t - 1;
#pragma unroll
        for (int i = 0; i < MAXKS; ++i) {
          const int k0 = (ks0 + i) * 32 + fk;
          if ((hwant >> i) & 1u) fa[i] = frag_wt<T>(r_hs, (uint32_t)((hprow * D + (k0 - E)) * sizeof(T)), true);
        }
      }
      stamp(g, 0, t, 1);
      // ---------------- G: [att2 | gate_pre]_t ----------------
      if (isG) {
        f32x4 acc[2];
        acc[0] = acc[1] = f32x4{0.f, 0.f, 0.f, 0.f};
        stamp(g, 0, t, 9, true);
#pragma unroll
        for (int i = 0; i < MAXKS; ++i) {
          const int kb = (ks0 + i) * 32;
          if (ks0 + i < ks1 && kb + 32 > E) {  // uniform: the k-step holds h columns
            // lanes left of E carry zero A fragments; their B read is clamped to a valid column
            const int kg = max(kb + fk - E, 0);
#pragma unroll
            for (int ni = 0; ni < 2; ++ni) mma(acc[ni], fa[i], lds_frag_k<T>(wg + (ni * 16 + fr) * ldg, kg, D));
          }
        }
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
#pragma unroll
          for (int r = 0; r < 4; ++r) red[(kp * 16 * MT + mi * 16 + 4 * (lane >> 4) + r) * RC + ni * 16 + fr] = acc[ni][r];
        __syncthreads();
        if (s_ok[2] == 0) return;
        // 16-byte write-through stores: row b, 4 consecutive columns per thread
        const int col0 = blk * GCOLS;
        for (int i = tid; i < 16 * MT * (GCOLS / 4); i += PT) {
          const int b = i / (GCOLS / 4), c = (i % (GCOLS / 4)) * 4;
          if (b >= B || col0 + c >= A + E) continue;
          float v[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float s = gb[j];
#pragma unroll
            for (int q = 0; q < KP; ++q) s += red[(q * 16 * MT + b) * RC + c + j];
            v[j] = s;
          }
          // hand-off to the R blocks as 8-byte {epoch, value} granules: the data is its own flag
          // (no drain, no separate flag; R2 of cdna_hip_programming.md Guideline 16); two
          // granules per 16-byte write-through store, each 8-byte half written whole
          const unsigned ep = (unsigned)(t + 1);
          const uint32_t go = (uint32_t)(((long)b * (A + E) + col0 + c) * 8);
          st_wt(r_gr, go, make_uint4(__float_as_uint(v[0]), ep, __float_as_uint(v[1]), ep));
          st_wt(r_gr, go + 16, make_uint4(__float_as_uint(v[2]), ep, __float_as_uint(v[3]), ep));
          *(f32x4*)(d.g1 + ((long)b * Tn + t) * W3 + col0 + c) = f32x4{v[0], v[1], v[2], v[3]};  // saved for bwd
        }
        stamp(g, 0, t, 2);
        stamp(g, 0, t, 3);
      }
      // ---------------- U: gates, LSTMCell -> h_t ----------------
      if (isU) {
        // the z part of A: the R blocks' z_t granules (slot t & 1, tag t + 1)
        if (!poll_frags<T, MAXKS>(r_zg, zbase, GSTRIDE, zwant, (unsigned)(t + 1), fa, err, g.poll_sleep) && lane == 0)
          s_ok[2] = 0;
        stamp(g, 0, t, 4);
        stamp(g, 0, t, 8, true);
        f32x4 acc[NTU][2];  // two K-interleaved chains per column tile
#pragma unroll
        for (int ni = 0; ni < NTU; ++ni) acc[ni][0] = acc[ni][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i0 = 0; i0 < MAXKS; i0 += 4) {
          if (ks0 + i0 < ks1) {  // uniform; steps past ks1 inside a group have zero A fragments
#pragma unroll
            for (int i = i0; i < i0 + 4; ++i) {
              const int k0 = (ks0 + i) * 32 + fk;
#pragma unroll
              for (int ni = 0; ni < NTU; ++ni)
                mma(acc[ni][i & 1], fa[i], lds_frag_k<T>(wu + (ni * 16 + fr) * ldu, k0, KU));
            }
          }
        }
#pragma unroll
        for (int ni = 0; ni < NTU; ++ni)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            red[(kp * 16 * MT + mi * 16 + 4 * (lane >> 4) + r) * RC + ni * 16 + fr] = acc[ni][0][r] + acc[ni][1][r];
        __syncthreads();
        if (s_ok[2] == 0) return;
        stamp(g, 0, t, 5);
        float cell[CPT][5];  // activated i, f, g, o and c_t, stored after the hand-off
#pragma unroll
        for (int k = 0; k < CPT; ++k) {
          const int i = tid + k * PT, b = i / UPB, jj = i % UPB;
          if (b >= B) continue;
          float gq[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            float s = xe[k][q] + bh[k][q];
#pragma unroll
            for (int p = 0; p < KP; ++p) s += red[(p * 16 * MT + b) * RC + q * UPB + jj];
            gq[q] = s;
          }
          const float gi = sigmoidf_(gq[0]), gf = sigmoidf_(gq[1]), gg = tanhf(gq[2]), go = sigmoidf_(gq[3]);
          const float cn = gf * creg[k] + gi * gg;
          const float h = go * tanhf(cn);
          creg[k] = cn;
          cell[k][0] = gi; cell[k][1] = gf; cell[k][2] = gg; cell[k][3] = go; cell[k][4] = cn;
          hst[b * UPB + jj] = from_f<T>(h);
        }
        __syncthreads();
        // h_t of this block's units as granules (slot t & 1, tag t + 1): one row per thread; the
        // saved hs / hprev copies with plain stores
        const int pieces = UPB * (int)sizeof(T) / 16;  // UPB * sizeof(T) is 16 or 32
        const bool publish = t != g.fault_step || blk != 0;
        if constexpr (HG) {
          if (publish)
            for (int b = tid; b < B; b += PT) {
              const uint4 lo = *(const uint4*)(hst + b * UPB);
              const uint4 hi = pieces == 2 ? *(const uint4*)(hst + b * UPB + VecOf<T>::N) : lo;
              store_gran8<T>(r_hg, (uint32_t)((((long)(t & 1) * B + b) * (D / VPG) + u0 / VPG) * 8), lo, hi,
                             (unsigned)(t + 1));
            }
          stamp(g, 0, t, 6);
          for (int i = tid; i < B * pieces; i += PT) {
            const int b = i / pieces, pc = i % pieces;
            const uint4 v = *(const uint4*)(hst + b * UPB + pc * VEC);
            *(uint4*)((T*)d.hs + ((long)b * Tn + t) * D + u0 + pc * VEC) = v;
          }
        } else {
          for (int i = tid; i < B * pieces; i += PT) {
            const int b = i / pieces, pc = i % pieces;
            const uint4 v = *(const uint4*)(hst + b * UPB + pc * VEC);
            st_wt(r_hs, (uint32_t)((((long)b * Tn + t) * D + u0 + pc * VEC) * sizeof(T)), v);
          }
          stamp(g, 0, t, 6);
          if (publish) block_publish(fh + blk, t + 1);
        }
        stamp(g, 0, t, 7);
        // outputs nobody in this launch reads: after the hand-off
#pragma unroll
        for (int k = 0; k < CPT; ++k) {
          const int i = tid + k * PT, b = i / UPB, jj = i % UPB, j = u0 + jj;
          if (b >= B) continue;
          const long bt = (long)b * Tn + t;
          float* ga = d.gates + bt * 4 * D;
          ga[j] = cell[k][0]; ga[D + j] = cell[k][1]; ga[2 * D + j] = cell[k][2]; ga[3 * D + j] = cell[k][3];
          d.cs[bt * D + j] = cell[k][4];
        }
        if (t + 1 < Tn)
          for (int i = tid; i < B * pieces; i += PT) {
            const int b = i / pieces, pc = i % pieces;
            const long off = ((long)b * Tn + t) * D + u0 + pc * VEC;
            *(uint4*)((T*)d.hprev + off + D) = *(const uint4*)(hst + b * UPB + pc * VEC);
          }
      }
    }
    // ---- steps past every decode length: zero outputs ----
    if (Tmax < Tn) {
      if (isU) {
        for (int i = tid; i < B * (Tn - Tmax) * UPB; i += PT) {
          const int jj = i % UPB, rest = i / UPB, b = rest % B, t = Tmax + rest / B, j = u0 + jj;
          const long bt = (long)b * Tn + t;
#pragma unroll
          for (int q = 0; q < 4; ++q) d.gates[bt * 4 * D + q * D + j] = 0.f;
          d.cs[bt * D + j] = 0.f;
          ((T*)d.hs)[bt * D + j] = from_f<T>(0.f);
          if (t + 1 < Tn) ((T*)d.hprev)[(bt + 1) * D + j] = from_f<T>(0.f);
        }
      }
      if (isG) {
        for (int i = tid; i < B * (Tn - Tmax) * GCOLS; i += PT) {
          const int c = i % GCOLS, rest = i / GCOLS, b = rest % B, t = Tmax + rest / B;
          const int col = blk * GCOLS + c;
          if (col < A + E) d.g1[((long)b * Tn + t) * W3 + col] = 0.f;
        }
      }
    }
    return;
  }
  // ======================= R workgroup: attention of row b, channel chunk s ================
  const int rr = blk - g.NUG, b = rr / g.RS, s = rr % g.RS;
  const int Ec = g.Ec, e0 = s * Ec;
  constexpr int VPG = GranOf<T>::VPG;
  const rsrc_t r_zg = make_rsrc(d.sync + g.zg_off, (uint32_t)(2L * B * (E / VPG) * 8));
  T* att1s = (T*)(smem + 16);                   // [P][A]
  // [P][ldE]: a lane quad reads 4 consecutive pixels of one 8-channel vector in the context
  // loop; with rows of Ec (a multiple of 128 elements) the quad hit one bank group (4-way,
  // SQ_LDS_BANK_CONFLICT 3.3 per LDS instruction), rows padded by 64 B spread them over the 64 banks
  const int ldE = g.ldE;
  T* encs = (T*)(smem + g.r_enc);
  float* red2 = (float*)(smem + g.r_red2);      // [64] scores
  float* es = (float*)(smem + g.r_es);          // [64] alpha
  float* gv = (float*)(smem + g.r_gv);          // [A + Ec] att2 | gate_pre chunk of this step
  if (tid == 0) s_ok[2] = 1;
  {
    const T* a1 = (const T*)d.att1 + (long)b * P * A;
    for (int i = tid; i < P * A / VEC; i += PT) *(uint4*)(att1s + i * VEC) = *(const uint4*)(a1 + i * VEC);
    const T* en = (const T*)d.enc + (long)b * P * E + e0;
    const int cpr = Ec / VEC;
    for (int i = tid; i < P * cpr; i += PT) {
      const int p = i / cpr, k = (i % cpr) * VEC;
      *(uint4*)(encs + p * ldE + k) = *(const uint4*)(en + (long)p * E + k);
    }
  }
  const int dlb = d.dl[b];
  const int NVA = A / 8;                          // <= 64 (A <= 512)
  const bool aok = lane < NVA;
  float wf[8];
  {
    const float* wp = d.w_f + (aok ? lane * 8 : 0);
    unpack8(*(const uint4*)wp, *(const uint4*)(wp + 4), wf);
  }
  // context mapping: thread = (8-channel vector v, pixel group pg = lane & 3); the four pixel
  // groups of a vector are one lane quad, summed with two DPP steps (no LDS round trip)
  const int NVE = Ec / 8;
  const int pg = lane & 3;
  __syncthreads();
  for (int t = 0; t < Tmax; ++t) {
    stamp(g, 1, t, 0);
    // [att2 | gate_pre of this chunk] of row b: poll the G blocks' granules until every tag is
    // this step's epoch, values into LDS (pairs of granules per 16-byte write-through load)
    {
      const unsigned ep = (unsigned)(t + 1);
      const int npair = (A + Ec) / 2;
      bool bad = false;
      for (int j = tid; j < npair; j += PT) {
        const int col = 2 * j < A ? 2 * j : A + e0 + (2 * j - A);
        const uint32_t off = (uint32_t)(((long)b * (A + E) + col) * 8);
        for (int spins = 0;; ++spins) {
          const uint4 q = ld_wt(r_gr, off);
          if (q.y == ep && q.w == ep) {
            gv[2 * j] = __uint_as_float(q.x);
            gv[2 * j + 1] = __uint_as_float(q.z);
            break;
          }
          if ((spins & 255) == 255 &&
              (spins >= SPIN_LIMIT || __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
            bad = true;
            break;
          }
        }
        if (bad) break;
      }
      if (bad) {
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_ok[2] = 0;
      }
      __syncthreads();
      if (s_ok[2] == 0) return;
    }
    stamp(g, 1, t, 1);
    const long bt = (long)b * Tn + t;
    // att2 slice of this lane (the gate pre-activations are read by the context threads below)
    float a2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) a2[j] = aok ? gv[lane * 8 + j] : 0.f;
    stamp(g, 1, t, 5, true);
    // scores e_p = w_f . relu(att1_p + att2): wave w takes pixels w, w+PWV, ..; lane = 8 units;
    // each pixel's 64 lane partials summed by DPP, the total written by one lane
    {
      constexpr int H = sizeof(T) / 2;  // 16-byte words per 8 elements
      constexpr int NPW = 64 / PWV;
      uint4 xr[NPW][H];
#pragma unroll
      for (int i = 0; i < NPW; ++i) {
        const int p = min(w + PWV * i, P - 1);
#pragma unroll
        for (int h = 0; h < H; ++h) xr[i][h] = *(const uint4*)(att1s + p * A + (aok ? lane * 8 : 0) + h * VEC);
      }
      if constexpr (NPW == 8) {  // every pixel's partial first, then one transposed reduction
        float part[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const T* x8 = (const T*)&xr[i][0];
          float sc = 0.f;
#pragma unroll
          for (int j = 0; j < 8; ++j) sc += wf[j] * fmaxf(to_f(x8[j]) + a2[j], 0.f);
          part[i] = aok ? sc : 0.f;
        }
        const float sum = wave_sum8_t(part, lane);
        const int p = w + PWV * ((lane >> 3) & 7);
        if ((lane & 7) == 0 && p < P) red2[p] = sum;
      } else {
#pragma unroll
        for (int i = 0; i < NPW; ++i) {
          const int p = w + PWV * i;
          if (p < P) {
            const T* x8 = (const T*)&xr[i][0];
            float sc = 0.f;
#pragma unroll
            for (int j = 0; j < 8; ++j) sc += wf[j] * fmaxf(to_f(x8[j]) + a2[j], 0.f);
            sc = wave_sum_dpp(aok ? sc : 0.f);
            if (lane == 0) red2[p] = sc;
          }
        }
      }
    }
    __syncthreads();
    stamp(g, 1, t, 6);
    if (tid < 64) {  // softmax over the P scores (full_att's bias cancels)
      const float e = tid < P ? red2[tid] : -INFINITY;
      const float mx = wave_max_dpp(e);
      const float ex = tid < P ? __expf(e - mx) : 0.f;
      const float al = ex / wave_sum_dpp(ex);
      if (tid < P) es[tid] = al;
    }
    __syncthreads();
    stamp(g, 1, t, 7);
    for (int v = tid >> 2; v < NVE; v += PT / 4) {
      // gate pre-activation of this vector (only the quad leader uses it)
      float gp[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) gp[j] = gv[A + v * 8 + j];
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      constexpr int H = sizeof(T) / 2;
      for (int p0 = pg; p0 < P; p0 += 32) {
        uint4 xr[8][H];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int p = min(p0 + 4 * i, P - 1);
#pragma unroll
          for (int h = 0; h < H; ++h) xr[i][h] = *(const uint4*)(encs + p * ldE + v * 8 + h * VEC);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int p = p0 + 4 * i;
          const float al = p < P ? es[min(p, P - 1)] : 0.f;
          const T* x8 = (const T*)&xr[i][0];
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] += al * to_f(x8[j]);
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = quad_sum_dpp(acc[j]);
      if (pg == 0) {
        uint4 zz[2];
        T* zt = (T*)zz;
#pragma unroll
        for (int j = 0; j < 8; ++j) zt[j] = from_f<T>(sigmoidf_(gp[j]) * acc[j]);
        // z_t to the U blocks as tagged granules (slot t & 1, tag t + 1); the saved zs copy plain
        store_gran8<T>(r_zg, (uint32_t)((((long)(t & 1) * B + b) * (E / VPG) + (e0 + v * 8) / VPG) * 8), zz[0],
                       zz[1], (unsigned)(t + 1));
        T* zsp = (T*)d.zs + bt * E + e0 + v * 8;
        *(uint4*)zsp = zz[0];
        if (sizeof(T) == 4) *(uint4*)(zsp + 4) = zz[1];
        float* aw = d.awe + bt * E + e0 + v * 8;  // saved context (nobody in this launch reads it)
        *(f32x4*)aw = f32x4{acc[0], acc[1], acc[2], acc[3]};
        *(f32x4*)(aw + 4) = f32x4{acc[4], acc[5], acc[6], acc[7]};
      }
    }
    stamp(g, 1, t, 3);
    stamp(g, 1, t, 4);
    if (s == 0 && tid < P) d.alphas[bt * P + tid] = t < dlb ? es[tid] : 0.f;
  }
  if (Tmax < Tn) {
    for (int i = tid; i < (Tn - Tmax) * Ec; i += PT) {
      const long bt = (long)b * Tn + Tmax + i / Ec;
      const int e = e0 + i % Ec;
      d.awe[bt * E + e] = 0.f;
      ((T*)d.zs)[bt * E + e] = from_f<T>(0.f);
    }
    if (s == 0)
      for (int i = tid; i < (Tn - Tmax) * P; i += PT) d.alphas[((long)b * Tn + Tmax) * P + i] = 0.f;
  }
}

// Row groups: rows [0, B0) and [B0, B) are independent recurrences (no term couples two batch
// rows), run side by side in ONE launch -- each group with its own blocks, descriptor view
// (row-offset pointers) and flag / granule area; blocks [0, nb0) are group 0.  Halving the
// rows per chain shortens each step's payload loads and MFMA work (measured per step at
// B = 16 vs 32: forward 15.7 vs 17.4 us, backward 17.8 vs 21.2 us).
template <typename T, int MT, bool HG>
__global__ __launch_bounds__(PT) void lstm_fwd_persist_kernel(imgcap_lstm_desc d0, Geo g0, imgcap_lstm_desc d1,
                                                              Geo g1, int nb0) {
  // one inlined body over the selected group's (kernel-argument) descriptor: two inlined copies
  // doubled the code and ran out of SGPRs (1,000+ SGPR spills to VGPR lanes)
  const bool second = (int)blockIdx.x >= nb0;
  lstm_fwd_body<T, MT, HG>(second ? d1 : d0, second ? g1 : g0, second ? (int)blockIdx.x - nb0 : (int)blockIdx.x);
}

size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

DEV void ldf8(const float* p, float (&v)[8]) {
  unpack8(*(const uint4*)p, *(const uint4*)(p + 4), v);
}
// 8 floats as T in 16-byte words (hi unused for bf16), in registers
template <typename T> DEV void pack8(const float (&v)[8], uint4& lo, uint4& hi);
template <> DEV void pack8<bf16>(const float (&v)[8], uint4& lo, uint4& hi) {
  bf16x8 x;
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = (bf16)v[j];
  lo = __builtin_bit_cast(uint4, x);
  hi = lo;
}
template <> DEV void pack8<float>(const float (&v)[8], uint4& lo, uint4& hi) {
  lo = make_uint4(__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3]));
  hi = make_uint4(__float_as_uint(v[4]), __float_as_uint(v[5]), __float_as_uint(v[6]), __float_as_uint(v[7]));
}

// =========================================================================================
// Persistent BACKWARD recurrence (backpropagation through time of decoder.py:69-113): ONE
// launch runs every step t = max(decode length) - 1 .. 0 of what imgcap_lstm_tf_bwd's per-step
// path does with three launches per step (x_partial -> attn_bwd -> dh_cell).
//
// Roles (one 512-thread workgroup per CU):
//   U blocks [0, NU):       UPB LSTM units; rows of [W_hh | W_da; W_fb] for those units resident
//                           in LDS.  Per step: the LSTMCell backward of (row, unit) items ->
//                           dgates_t (published), then dh_{t-1}[:, units] = dgates_t . W_hh[:,
//                           units] + [d att2 | d gate_pre]_t . [W_da; W_fb][:, units] -- the
//                           recurrent dh the next (earlier) step's cell backward adds to dhs.
//   X blocks [NU, +NX):     16 columns of W_ih[:, M:] resident; dz_t[:, cols] = dgates_t . W_ih
//                           [:, M + cols], handed to the R blocks as {value, epoch} granules.
//   R blocks [NU+NX, +B):   batch row b; att1[b] (and enc[b] when it fits) resident; the
//                           attention backward (decoder.py:25-31,102-105 reversed): d awe, d
//                           gate_pre, d alpha, softmax backward -> de, d att2 (published).
// Per step three hand-offs: dgates_t (U -> X, U), dz_t (X -> R, granules), [d att2 | d
// gate_pre]_t (R -> U).  dgates and d att are stored write-through into dcat itself (the
// weight-gradient GEMMs after the launch read the same rows), published with per-producer flags
// (block_publish / block_wait, epoch = steps done + 1), and loaded with sc1 loads.  The U blocks
// request the dgates part of their product right after its flags, so only the d att part sits
// on the R -> U edge.  Outputs equal the per-step path's up to summation order (dcat, de, dawe,
// dh = dL/dh0, dc = dL/dc0); steps t >= max decode length are zeros, as there.
struct BGeo {
  int NU, UPB, NX, NR;
  int ldu, ldx;                 // LDS row pitches (elements) of the resident weights
  int u_red, u_dg, x_red;       // byte offsets (U / X)
  int r_enc, r_dz, r_dawe, r_red, r_al, r_dal, r_dtt;  // byte offsets (R); r_enc < 0: enc from global
  int gran_off;                 // sync word offset of the [B][E] dz granules
  long long* stamps;            // diagnostics (IMGCAP_LSTM_STAMPS=1): [role U/X/R][step][16]
  int* err;                     // the launch's error word (shared by the row groups)
  int fault_step;               // test knob (IMGCAP_LSTM_FAULT_BWD): U block 0 never publishes dgates of this step
};

// thread 0 of the first U, X and R block records s_memrealtime at phase edges of step t
DEV void bstamp(const BGeo& g, int role, int t, int k) {
  const int b0 = role == 0 ? 0 : role == 1 ? g.NU : g.NU + g.NX;
  if (g.stamps && threadIdx.x == 0 && (int)blockIdx.x == b0 && t < 64)
    g.stamps[(role * 64 + t) * 16 + k] = (long long)__builtin_amdgcn_s_memrealtime();
}

struct CellIn {
  float gi, gf, gg, go, c, cp, dhs;
};

template <typename T>
DEV CellIn cell_in_load(const imgcap_lstm_desc& d, int t, int b, int j) {
  const int D = d.D, Tn = d.T;
  const long bt = (long)b * Tn + t;
  const float* ga = d.gates + bt * 4 * D;
  CellIn in;
  in.gi = ga[j]; in.gf = ga[D + j]; in.gg = ga[2 * D + j]; in.go = ga[3 * D + j];
  in.c = d.cs[bt * D + j];
  in.cp = t == 0 ? d.c0[(long)b * D + j] : d.cs[(bt - 1) * D + j];
  in.dhs = to_f(((const T*)d.dhs)[bt * D + j]);
  return in;
}

template <typename T, int MT>
DEV void lstm_bwd_body(const imgcap_lstm_desc& d, const BGeo& g, const int blk) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int* s_ok = (int*)smem;
  const int B = d.B, P = d.P, E = d.E, A = d.A, D = d.D, Tn = d.T;
  const int KY = A + E, K4 = 4 * D, W3 = KY + K4;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int* err = g.err;
  int* fdg = d.sync + SYNC_HDR;  // U blocks: dgates_t published
  int* fdt = fdg + g.NU;         // R blocks: [d att2 | d gate_pre]_t published
  if (tid < 64) {
    int m = 0;
    for (int i = lane; i < B; i += 64) m = max(m, d.dl[i]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = max(m, __shfl_xor(m, o, 64));
    if (lane == 0) s_ok[1] = m;
  }
  __syncthreads();
  const int Tmax = max(0, min(Tn, s_ok[1]));
  constexpr int VEC = VecOf<T>::N;
  constexpr int KP = PWV / MT;                      // K parts: wave w -> row tile w % MT, K part w / MT
  constexpr int KCH = sizeof(T) == 2 ? 16 : 8;      // A fragments requested per round trip
  const rsrc_t r_dcat = make_rsrc(d.dcat, (uint32_t)((long)B * Tn * W3 * sizeof(T)));
  const rsrc_t r_gr = make_rsrc(d.sync + g.gran_off, (uint32_t)((long)B * E * 8));
  const int mi = w % MT, kp = w / MT;
  const int fr = lane & 15, fk = 8 * (lane >> 4);
  const int m = mi * 16 + fr;
  const bool mok = m < B;
  const int nk1 = K4 / 32, nk2 = (KY + 31) / 32;   // k-steps of the dgates / d att parts
  const int per1 = (nk1 + KP - 1) / KP, per2 = (nk2 + KP - 1) / KP;
  const uint4 zero4 = make_uint4(0u, 0u, 0u, 0u);

  if (blk < g.NU + g.NX) {
    // ======================= U and X workgroups ==========================================
    const bool isU = blk < g.NU;
    const int UPB = g.UPB, u0 = blk * UPB;
    const int x0 = (blk - g.NU) * 16;
    const int ld = isU ? g.ldu : g.ldx;
    const int KW = isU ? K4 + KY : K4;  // resident k per weight row
    const int nrows = isU ? UPB : 16;
    T* wr = (T*)(smem + 16);
    float* red = (float*)(smem + (isU ? g.u_red : g.x_red));  // [KP][16 * MT][20]
    T* dgs = (T*)(smem + g.u_dg);                              // U: [B][4][UPB] staged dgates
    {
      const int cpr = KW / VEC;
      for (int i = tid; i < nrows * cpr; i += PT) {
        const int c = i / cpr, k = (i % cpr) * VEC;
        uint4 v = zero4;
        if (isU) {
          const int j = u0 + c;
          v = k < K4 ? *(const uint4*)((const T*)d.w_zh_t + (long)(E + j) * K4 + k)
                     : *(const uint4*)((const T*)d.w_att_t + (long)j * KY + (k - K4));
        } else if (x0 + c < E) {
          v = *(const uint4*)((const T*)d.w_zh_t + (long)(x0 + c) * K4 + k);
        }
        *(uint4*)(wr + c * ld + k) = v;
      }
    }
    // this thread's (row, unit) item of the cell backward (U)
    const int ib = tid / UPB, ijj = tid % UPB, ij = u0 + ijj;
    const bool iok = isU && tid < B * UPB;
    const int dlb = iok ? d.dl[ib] : 0;
    float dc = 0.f, dh_rec = 0.f;
    CellIn cin{};
    if (iok && Tmax > 0 && Tmax - 1 < dlb) cin = cell_in_load<T>(d, Tmax - 1, ib, ij);
    const bool bok = fr < nrows;  // B fragment rows past UPB are zero
    __syncthreads();
    const int role = isU ? 0 : 1;
    for (int t = Tmax - 1; t >= 0; --t) {
      const int ep = Tmax - t;
      const long mbt = (long)m * Tn + t;
      bstamp(g, role, t, 0);
      if (isU) {
        // ---- LSTMCell backward of step t (cell_bwd_apply of lstm.hip) ----
        if (iok) {
          float dg[4] = {0.f, 0.f, 0.f, 0.f};
          if (t < dlb) {
            const float dh = cin.dhs + dh_rec;
            const float tc = tanhf(cin.c);
            const float dct = dc + dh * cin.go * (1.f - tc * tc);
            dg[0] = dct * cin.gg * cin.gi * (1.f - cin.gi);
            dg[1] = dct * cin.cp * cin.gf * (1.f - cin.gf);
            dg[2] = dct * cin.gi * (1.f - cin.gg * cin.gg);
            dg[3] = dh * tc * cin.go * (1.f - cin.go);
            dc = dct * cin.gf;
          } else {
            dc = 0.f;
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) dgs[(ib * 4 + q) * UPB + ijj] = from_f<T>(dg[q]);
        }
        __syncthreads();
        // dgates_t rows of this block's units -> dcat (write-through): row b, gate q, UPB elements
        const int pieces = UPB * (int)sizeof(T) / 16;
        for (int i = tid; i < B * 4 * pieces; i += PT) {
          const int pc = i % pieces, bq = i / pieces, b = bq / 4, q = bq % 4;
          const uint4 v = *(const uint4*)(dgs + bq * UPB + pc * VEC);
          const long off = ((long)b * Tn + t) * W3 + KY + (long)q * D + u0 + pc * VEC;
          st_wt(r_dcat, (uint32_t)(off * sizeof(T)), v);
        }
        if (t != g.fault_step || blk != 0) block_publish(fdg + blk, ep);
        bstamp(g, 0, t, 1);
        // cell inputs of the next (earlier) step: independent of every hand-off
        if (iok && t > 0 && t - 1 < dlb) cin = cell_in_load<T>(d, t - 1, ib, ij);
      }
      // ---- dgates_t . W[:, cols]  (U: W_hh part of dh_{t-1}; X: dz_t) ----
      if (!block_wait(fdg, g.NU, ep, err, s_ok + 2)) return;
      bstamp(g, role, t, 2);
      f32x4 acc[2];
      acc[0] = acc[1] = f32x4{0.f, 0.f, 0.f, 0.f};
      {
        const int ks0 = kp * per1, ks1 = min(nk1, ks0 + per1);
        for (int ks = ks0; ks < ks1; ks += KCH) {
          Frag<T> fa[KCH];
#pragma unroll
          for (int i = 0; i < KCH; ++i) {
            const int k0 = (ks + i) * 32 + fk;
            fa[i] = frag_wt<T>(r_dcat, (uint32_t)((mbt * W3 + KY + k0) * sizeof(T)), mok && ks + i < ks1);
          }
#pragma unroll
          for (int i = 0; i < KCH; ++i) {  // steps past ks1 have zero A fragments
            const int k0 = (ks + i) * 32 + fk;
            Frag<T> fb = lds_frag_k<T>(wr + (bok ? fr : 0) * ld, k0, K4);
            if (!bok) fb = frag_from<T>(zero4, zero4);
            mma(acc[i & 1], fa[i], fb);
          }
        }
      }
      bstamp(g, role, t, 3);
      if (isU) {
        // ---- + [d att2 | d gate_pre]_t . [W_da; W_fb][:, units]: after the R blocks ----
        if (!block_wait(fdt, g.NR, ep, err, s_ok + 3)) return;
        bstamp(g, 0, t, 4);
        const int ks0 = kp * per2, ks1 = min(nk2, ks0 + per2);
        for (int ks = ks0; ks < ks1; ks += KCH) {
          Frag<T> fa[KCH];
#pragma unroll
          for (int i = 0; i < KCH; ++i) {
            const int k0 = (ks + i) * 32 + fk;
            fa[i] = frag_wt<T>(r_dcat, (uint32_t)((mbt * W3 + k0) * sizeof(T)), mok && ks + i < ks1 && k0 < KY);
          }
#pragma unroll
          for (int i = 0; i < KCH; ++i) {
            const int k0 = (ks + i) * 32 + fk;
            Frag<T> fb = lds_frag_k<T>(wr + (bok ? fr : 0) * ld + K4, k0, KY);
            if (!bok) fb = frag_from<T>(zero4, zero4);
            mma(acc[i & 1], fa[i], fb);
          }
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r)
        red[(kp * 16 * MT + mi * 16 + 4 * (lane >> 4) + r) * 20 + fr] = acc[0][r] + acc[1][r];
      __syncthreads();
      if (isU) {
        if (iok) {
          float s = 0.f;
#pragma unroll
          for (int q = 0; q < KP; ++q) s += red[(q * 16 * MT + ib) * 20 + ijj];
          dh_rec = s;
          if (t == 0) d.dh[(long)ib * D + ij] = s;  // dL/dh0
        }
      } else {
        // dz_t granules {value, epoch} of this block's 16 columns, two per 16-byte store
        for (int i = tid; i < B * 8; i += PT) {
          const int b = i / 8, c = (i % 8) * 2;
          float v0 = 0.f, v1 = 0.f;
#pragma unroll
          for (int q = 0; q < KP; ++q) {
            v0 += red[(q * 16 * MT + b) * 20 + c];
            v1 += red[(q * 16 * MT + b) * 20 + c + 1];
          }
          if (x0 + c < E)
            st_wt(r_gr, (uint32_t)(((long)b * E + x0 + c) * 8),
                  make_uint4(__float_as_uint(v0), (unsigned)ep, __float_as_uint(v1), (unsigned)ep));
        }
      }
      __syncthreads();  // red is rewritten next step
      bstamp(g, role, t, 5);
    }
    if (isU) {
      if (iok) d.dc[(long)ib * D + ij] = dc;  // dL/dc0
      // steps past every decode length: zero dgates rows (as the per-step path leaves them)
      for (int i = tid; i < B * (Tn - Tmax) * 4 * UPB; i += PT) {
        const int jj = i % UPB, rest = i / UPB, q = rest % 4, rest2 = rest / 4, b = rest2 % B, t = Tmax + rest2 / B;
        ((T*)d.dcat)[((long)b * Tn + t) * W3 + KY + (long)q * D + u0 + jj] = from_f<T>(0.f);
      }
      if (Tmax == 0 && iok) {
        d.dh[(long)ib * D + ij] = 0.f;
        d.dc[(long)ib * D + ij] = 0.f;
      }
    }
    return;
  }

  // ======================= R workgroup: attention backward of row b ======================
  const int b = blk - g.NU - g.NX;
  T* att1s = (T*)(smem + 16);                       // [P][A]
  const bool enc_lds = g.r_enc >= 0;
  const T* encs = enc_lds ? (const T*)(smem + g.r_enc) : (const T*)d.enc + (long)b * P * E;  // [P][E]
  float* dzs = (float*)(smem + g.r_dz);             // [E]
  float* dawes = (float*)(smem + g.r_dawe);         // [E]
  float* red = (float*)(smem + g.r_red);            // [GA][A]
  float* als = (float*)(smem + g.r_al);             // [64]
  float* dal = (float*)(smem + g.r_dal);            // [64]
  T* dtt = (T*)(smem + g.r_dtt);                    // [A] d att2 staged for 16-byte stores
  {
    const T* a1 = (const T*)d.att1 + (long)b * P * A;
    for (int i = tid; i < P * A / VEC; i += PT) *(uint4*)(att1s + i * VEC) = *(const uint4*)(a1 + i * VEC);
    if (enc_lds) {
      const T* en = (const T*)d.enc + (long)b * P * E;
      for (int i = tid; i < P * E / VEC; i += PT) *(uint4*)((T*)encs + i * VEC) = *(const uint4*)(en + i * VEC);
    }
  }
  if (tid == 0) s_ok[2] = 1;
  const int dlb = d.dl[b];
  const int NVE = E / 8, NVA = A / 8, GA = PT / NVA;
  const int va = tid % NVA, pga = tid / NVA;
  const float wf_a = tid < A ? d.w_f[tid] : 0.f;
  __syncthreads();
  for (int t = Tmax - 1; t >= 0; --t) {
    const int ep = Tmax - t;
    const long bt = (long)b * Tn + t;
    float* dawe_o = d.dawe ? d.dawe + ((long)b * (Tn + 1) + t) * E : nullptr;
    if (t >= dlb) {  // past this row's decode length: zero outputs, publish at once
      for (int i = tid; i < KY / VEC; i += PT) st_wt(r_dcat, (uint32_t)((bt * W3 + i * VEC) * sizeof(T)), zero4);
      if (tid < P) d.de[bt * P + tid] = 0.f;
      if (dawe_o)
        for (int i = tid; i < E; i += PT) dawe_o[i] = 0.f;
      block_publish(fdt + b, ep);
      continue;
    }
    bstamp(g, 2, t, 0);
    // ---- operands independent of the hand-off, requested first ----
    const float* g1 = d.g1 + bt * W3;
    float gp[8], aw[8], a2[8];
    const bool vth = tid < NVE;
    if (vth) {
      ldf8(g1 + A + tid * 8, gp);
      ldf8(d.awe + bt * E + tid * 8, aw);
    }
    ldf8(g1 + va * 8, a2);  // att2 slice of this thread's 8 units
    float alpha_in = 0.f, dalpha_in = 0.f;
    if (tid < P) {
      alpha_in = d.alphas[bt * P + tid];
      if (d.dalpha) dalpha_in = d.dalpha[bt * P + tid];
    }
    // ---- dz_t[b] from the X blocks' granules ----
    {
      bool bad = false;
      for (int j = tid; j < E / 2; j += PT) {
        const uint32_t off = (uint32_t)(((long)b * E + 2 * j) * 8);
        for (int spins = 0;; ++spins) {
          const uint4 q = ld_wt(r_gr, off);
          if (q.y == (unsigned)ep && q.w == (unsigned)ep) {
            dzs[2 * j] = __uint_as_float(q.x);
            dzs[2 * j + 1] = __uint_as_float(q.z);
            break;
          }
          if ((spins & 255) == 255 &&
              (spins >= SPIN_LIMIT || __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
            bad = true;
            break;
          }
        }
        if (bad) break;
      }
      if (bad) {
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_ok[2] = 0;
      }
      __syncthreads();
      if (s_ok[2] == 0) return;
    }
    bstamp(g, 2, t, 1);
    // ---- d awe = dz * sigmoid(gate), d gate_pre = dz * awe * s (1 - s) ----
    if (vth) {
      float da[8], dg[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float dz = dzs[tid * 8 + j];
        const float s = sigmoidf_(gp[j]);
        da[j] = dz * s;
        dg[j] = dz * aw[j] * s * (1.f - s);
        dawes[tid * 8 + j] = da[j];
      }
      uint4 lo, hi;
      pack8<T>(dg, lo, hi);
      const uint32_t off = (uint32_t)((bt * W3 + A + tid * 8) * sizeof(T));
      st_wt(r_dcat, off, lo);
      if (sizeof(T) == 4) st_wt(r_dcat, off + 16, hi);
      if (dawe_o) {
        *(f32x4*)(dawe_o + tid * 8) = f32x4{da[0], da[1], da[2], da[3]};
        *(f32x4*)(dawe_o + tid * 8 + 4) = f32x4{da[4], da[5], da[6], da[7]};
      }
    }
    if (tid < P) {
      als[tid] = alpha_in;
      dal[tid] = dalpha_in;  // upstream d alpha
    }
    __syncthreads();
    bstamp(g, 2, t, 2);
    // ---- d alpha_p += enc_p . d awe: wave w takes pixels w, w + 8, ..; lane = 8-channel vectors ----
    if (enc_lds && sizeof(T) == 2) {
      // enc rows resident in LDS (bf16): per 64-channel-vector slot, every pixel's 16-byte piece
      // is requested before the first product, the dot partials of the wave's <= 8 pixels are
      // kept in registers and reduced by DPP at the end (one round trip, no serial chain)
      const T* el = (const T*)(smem + g.r_enc);
      constexpr int PPW = 64 / PWV;  // pixels per wave (P <= 64)
      float part[PPW];
#pragma unroll
      for (int i = 0; i < PPW; ++i) part[i] = 0.f;
      for (int v0 = 0; v0 < NVE; v0 += 64) {  // wave-uniform
        const int v = v0 + lane;
        const bool vok = v < NVE;
        float dv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) dv[j] = vok ? dawes[v * 8 + j] : 0.f;
        uint4 ev[PPW];
#pragma unroll
        for (int i = 0; i < PPW; ++i) {
          const int p = min(w + PWV * i, P - 1);
          ev[i] = vok ? *(const uint4*)(el + p * E + v * 8) : make_uint4(0u, 0u, 0u, 0u);
        }
#pragma unroll
        for (int i = 0; i < PPW; ++i) {
          const bf16x8 x = __builtin_bit_cast(bf16x8, ev[i]);
#pragma unroll
          for (int j = 0; j < 8; ++j) part[i] += (float)x[j] * dv[j];
        }
      }
      bstamp(g, 2, t, 6);
      if constexpr (PPW == 8) {  // all eight pixel sums in one transposed reduction
        const float sum = wave_sum8_t(part, lane);
        const int p = w + PWV * ((lane >> 3) & 7);
        if ((lane & 7) == 0 && p < P) dal[p] += sum;
      } else {
#pragma unroll
        for (int i = 0; i < PPW; ++i) {
          const int p = w + PWV * i;
          if (p < P) {  // wave-uniform
            const float s = wave_sum_dpp(part[i]);
            if (lane == 0) dal[p] += s;
          }
        }
      }
      bstamp(g, 2, t, 7);
    } else {
      for (int p = w; p < P; p += PWV) {
        float s = 0.f;
        for (int v = lane; v < NVE; v += 64) {
          float x[8];
          ld_g<T, 8>(encs + (long)p * E + v * 8, x);
#pragma unroll
          for (int j = 0; j < 8; ++j) s += x[j] * dawes[v * 8 + j];
        }
        s = wave_sum_dpp(s);
        if (lane == 0) dal[p] += s;
      }
    }
    __syncthreads();
    bstamp(g, 2, t, 3);
    if (w == 0) {  // softmax backward -> d score (stamps 8-10: the d att2 sub-phases)
      const float a = lane < P ? als[lane] : 0.f;
      const float da = lane < P ? dal[lane] : 0.f;
      const float dot = wave_sum_dpp(a * da);
      if (lane < P) {
        const float de = a * (da - dot);
        dal[lane] = de;
        d.de[bt * P + lane] = de;
      }
    }
    __syncthreads();
    bstamp(g, 2, t, 8);
    // ---- d att2[a] = w_f[a] * sum_p de_p [att1[p, a] + att2[a] > 0] ----
    if (pga < GA) {
      float sacc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (sizeof(T) == 2 && GA == PWV) {  // A = 512: <= 8 pixels per thread, loads issued first
        constexpr int PPT = 64 / PWV;
        uint4 xv[PPT];
        float dep[PPT];
#pragma unroll
        for (int i = 0; i < PPT; ++i) {
          const int p = pga + GA * i;
          xv[i] = *(const uint4*)(att1s + min(p, P - 1) * A + va * 8);
          dep[i] = p < P ? dal[min(p, P - 1)] : 0.f;
        }
#pragma unroll
        for (int i = 0; i < PPT; ++i) {
          const bf16x8 x = __builtin_bit_cast(bf16x8, xv[i]);
#pragma unroll
          for (int j = 0; j < 8; ++j) sacc[j] += ((float)x[j] + a2[j] > 0.f) ? dep[i] : 0.f;
        }
      } else {
        for (int p = pga; p < P; p += GA) {
          float x[8];
          ld_g<T, 8>(att1s + p * A + va * 8, x);
          const float de = dal[p];
#pragma unroll
          for (int j = 0; j < 8; ++j) sacc[j] += (x[j] + a2[j] > 0.f) ? de : 0.f;
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) red[pga * A + va * 8 + j] = sacc[j];
    }
    bstamp(g, 2, t, 9);
    __syncthreads();
    bstamp(g, 2, t, 10);
    if (tid < A) {
      float s = 0.f;
      for (int q = 0; q < GA; ++q) s += red[q * A + tid];
      dtt[tid] = from_f<T>(s * wf_a);
    }
    __syncthreads();
    bstamp(g, 2, t, 4);
    for (int i = tid; i < A / VEC; i += PT)
      st_wt(r_dcat, (uint32_t)((bt * W3 + i * VEC) * sizeof(T)), *(const uint4*)(dtt + i * VEC));
    block_publish(fdt + b, ep);
    bstamp(g, 2, t, 5);
  }
  // steps past every decode length: zero outputs
  for (int t = Tmax; t < Tn; ++t) {
    const long bt = (long)b * Tn + t;
    for (int i = tid; i < KY; i += PT) ((T*)d.dcat)[bt * W3 + i] = from_f<T>(0.f);
    if (tid < P) d.de[bt * P + tid] = 0.f;
    if (d.dawe)
      for (int i = tid; i < E; i += PT) d.dawe[((long)b * (Tn + 1) + t) * E + i] = 0.f;
  }
}

template <typename T, int MT>
__global__ __launch_bounds__(PT) void lstm_bwd_persist_kernel(imgcap_lstm_desc d0, BGeo g0, imgcap_lstm_desc d1,
                                                              BGeo g1, int nb0) {
  // two inlined bodies here: the single selected-descriptor body (lstm_fwd_persist_kernel) cut the
  // backward's SGPR spills 600 -> 77 but measured 20.3 -> 23.5 us per step
  if ((int)blockIdx.x < nb0) lstm_bwd_body<T, MT>(d0, g0, blockIdx.x);
  else lstm_bwd_body<T, MT>(d1, g1, blockIdx.x - nb0);
}

}  // namespace

// Geometry + LDS plan; false when the shape is outside what the persistent kernel covers.
static bool persist_plan(const imgcap_lstm_desc& d, int esz, Geo& g, size_t& lds, int& mt, int& words,
                         int force_mt = 0) {
  const size_t LDS_MAX = 160 * 1024;
  if (d.B < 1 || d.B > 32 || d.P > 64 || d.A > 512 || d.A % 8 || d.E % 8 || d.D % 8 || d.M % 8) return false;
  mt = force_mt ? force_mt : d.B <= 16 ? 1 : 2;
  g.UPB = 8;
  const int UC = 4 * g.UPB;
  g.NU = d.D / g.UPB;
  g.NG = (d.A + d.E + GCOLS - 1) / GCOLS;
  g.NUG = std::max(g.NU, g.NG);
  g.KU = d.E + d.D;
  const int pad = 16 / esz;
  g.ldu = g.KU + pad;
  g.ldg = d.D + pad;
  g.rc = std::max(UC, GCOLS) + 4;
  const int KP = PWV / mt;
  const int maxks = esz == 2 ? (mt == 2 ? MaxKsF<bf16, 2>::N : MaxKsF<bf16, 1>::N) : MaxKsF<float, 1>::N;
  if (((g.KU + 31) / 32 + KP - 1) / KP > maxks) return false;
  size_t o = 16 + (size_t)UC * g.ldu * esz + (size_t)GCOLS * g.ldg * esz;
  g.ug_red = (int)align16(o);
  o = g.ug_red + (size_t)KP * 16 * mt * g.rc * 4;
  g.ug_hst = (int)align16(o);
  const size_t ug = align16(g.ug_hst + (size_t)16 * mt * g.UPB * esz);
  // R blocks: smallest channel split that fits
  size_t r = 0;
  g.RS = 0;
  for (int rs = 1; rs <= 8; ++rs) {
    if (d.E % (8 * rs)) continue;
    const int Ec = d.E / rs;
    if (Ec > 2048) continue;
    size_t q = align16(16 + (size_t)d.P * d.A * esz);
    const size_t enc = q;
    q = align16(q + (size_t)d.P * (Ec + 32) * esz);
    const size_t rd = q;
    q = align16(q + 16);
    const size_t rd2 = q;
    q = align16(q + PWV * 64 * 4);
    const size_t ees = q;
    q = align16(q + 64 * 4);
    const size_t gvo = q;
    q = align16(q + (size_t)(d.A + Ec) * 4);
    if (q <= LDS_MAX) {
      g.r_gv = (int)gvo;
      g.RS = rs;
      g.Ec = Ec;
      g.ldE = Ec + 32;
      g.r_enc = (int)enc;
      g.r_red = (int)rd;
      g.r_red2 = (int)rd2;
      g.r_es = (int)ees;
      r = q;
      break;
    }
  }
  if (!g.RS) return false;
  g.NR = d.B * g.RS;
  if (g.NUG + g.NR > device_cus()) return false;
  // at least 81 KB: one workgroup per CU (the visibility form used here is the one measured so)
  lds = std::max(std::max(ug, r), (size_t)81 * 1024);
  if (lds > LDS_MAX) return false;
  g.gran_off = (SYNC_HDR + g.NU + g.NG + g.NR + 63) / 64 * 64;  // 256-byte aligned granule block
  const int vpg = esz == 2 ? 2 : 1;
  g.hg_off = (g.gran_off + d.B * (d.A + d.E) * 2 + 63) / 64 * 64;  // [2][B][D / vpg] h granules
  g.zg_off = g.hg_off + 2 * d.B * (d.D / vpg) * 2;                 // [2][B][E / vpg] z granules
  words = g.zg_off + 2 * d.B * (d.E / vpg) * 2;
  return true;
}

// The descriptor restricted to rows [r0, r0 + nb) (every per-row array is batch-major) with its
// own flag area at sync word `soff`.
static imgcap_lstm_desc rows_view(const imgcap_lstm_desc& d, int r0, int nb, int esz, int soff) {
  imgcap_lstm_desc v = d;
  const long T = d.T, P = d.P, E = d.E, A = d.A, D = d.D, W3 = A + E + 4 * D, r = r0;
  const auto cb = [&](const void* p, long elems) { return p ? (const char*)p + r * elems * esz : nullptr; };
  const auto mb = [&](void* p, long elems) { return p ? (char*)p + r * elems * esz : nullptr; };
  const auto cf = [&](const float* p, long elems) { return p ? p + r * elems : nullptr; };
  const auto mf = [&](float* p, long elems) { return p ? p + r * elems : nullptr; };
  v.B = nb;
  v.enc = cb(d.enc, P * E);
  v.att1 = cb(d.att1, P * A);
  v.xe = cf(d.xe, T * 4 * D);
  v.c0 = cf(d.c0, D);
  v.dl = d.dl + r0;
  v.g1 = mf(d.g1, T * W3);
  v.alphas = mf(d.alphas, T * P);
  v.awe = mf(d.awe, T * E);
  v.zs = mb(d.zs, T * E);
  v.gates = mf(d.gates, T * 4 * D);
  v.cs = mf(d.cs, T * D);
  v.hs = mb(d.hs, T * D);
  v.hprev = mb(d.hprev, T * D);
  v.dhs = cb(d.dhs, T * D);
  v.dalpha = cf(d.dalpha, T * P);
  v.dcat = mb(d.dcat, T * W3);
  v.dh = mf(d.dh, D);
  v.dc = mf(d.dc, D);
  v.de = mf(d.de, T * P);
  v.dawe = mf(d.dawe, (T + 1) * E);
  v.sync = d.sync + soff;
  v.sync_words = d.sync_words - soff;
  return v;
}

// Row-group split: two groups when every row group still has a persistent plan and the two
// fit on the chip.  Mask (d.row_groups when bit 2 is set, else IMGCAP_LSTM_GROUPS, else 0):
// bit 0 splits the forward, bit 1 the backward.  Measured (C2 bench, 1x MI355X): the
// encoder / decoder pipeline, whose encoder branch runs on the CUs the recurrence leaves,
// 11.8k img/s unsplit, 12.1k forward-only, 12.1k backward-only, 11.5k both; the sequential
// schedule 7.9k unsplit, 8.3k both.  Returns the first group's row count (B when not split).
static int split_rows(const imgcap_lstm_desc& d, bool fwd) {
  static const int env = [] {
    const char* e = getenv("IMGCAP_LSTM_GROUPS");
    return e ? atoi(e) : 0;
  }();
  const int mask = (d.row_groups & 4) ? d.row_groups : env;
  if (!(mask & (fwd ? 1 : 2)) || d.B <= 16 || d.B > 64) return d.B;
  return (d.B + 1) / 2;
}

// Compute units of the current device (every persistent workgroup must be resident at once: one
// per CU, the LDS request keeps it that way).  Cached per device.
static int device_cus() {
  static int cache[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  if (!cache[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    cache[dev] = n;
  }
  return cache[dev];
}

// Integer knob from the environment (read once), `dflt` when unset.
static int env_or(const char* name, int dflt) {
  const char* e = getenv(name);
  return e && *e ? atoi(e) : dflt;
}

// Test knob: a step index from the environment (read at every launch), -1 when unset.
static int env_step(const char* name) {
  const char* e = getenv(name);
  return e && *e ? atoi(e) : -1;
}

// Whether `kernel` with `lds` bytes of dynamic LDS gets at least one resident workgroup per CU
// (raises the dynamic LDS limit first; the answer is cached per kernel and LDS size).
static bool resident_one_per_cu(const void* kernel, size_t lds) {
  struct Entry { const void* k; size_t lds; int ok; };
  static Entry seen[64];
  static int n_seen = 0;
  for (int i = 0; i < n_seen; ++i)
    if (seen[i].k == kernel && seen[i].lds == lds) return seen[i].ok;
  int blocks = 0;
  const bool ok = hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess &&
                  hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, kernel, PT, lds) == hipSuccess && blocks >= 1;
  if (n_seen < 64) seen[n_seen++] = Entry{kernel, lds, ok ? 1 : 0};
  return ok;
}

struct FwdLaunch {
  imgcap_lstm_desc d[2];
  Geo g[2];
  int groups = 0, nb0 = 0, nblk = 0, mt = 0, words = 0;
  size_t lds = 0;
};

// Plans the forward launch (two row groups, else one); false = the per-step path.
static bool fwd_launch_plan(const imgcap_lstm_desc& d, int esz, FwdLaunch& L) {
  const int b0 = split_rows(d, true);
  for (int groups = b0 < d.B ? 2 : 1; groups >= 1; --groups) {
    L = FwdLaunch();
    L.groups = groups;
    const int rows[2] = {groups == 2 ? b0 : d.B, d.B - b0};
    L.mt = rows[0] <= 16 ? 1 : 2;
    int soff = 0;
    bool ok = true;
    for (int i = 0; i < groups && ok; ++i) {
      L.d[i] = groups == 2 ? rows_view(d, i ? b0 : 0, rows[i], esz, soff) : d;
      size_t lds;
      int m, words;
      ok = persist_plan(L.d[i], esz, L.g[i], lds, m, words, L.mt);
      L.lds = std::max(L.lds, lds);
      if (i == 0) L.nb0 = L.g[0].NUG + L.g[0].NR;
      L.nblk += L.g[i].NUG + L.g[i].NR;
      soff += (words + 63) / 64 * 64;
      L.words = groups == 2 ? soff : words;
    }
    if (!ok || L.nblk > device_cus()) continue;
    for (int i = 0; i < groups; ++i) L.g[i].err = d.sync;
    if (groups == 1) {
      L.d[1] = L.d[0];
      L.g[1] = L.g[0];
    }
    return true;
  }
  return false;
}

// (the h hand-off as tagged granules, the HG = true form, measured slower -- 15.1 vs 14.6 us per
// step -- and is no longer instantiated, round 4)
static const void* fwd_kernel_of(int esz, int mt) {
  if (esz == 2)
    return mt == 1 ? (const void*)lstm_fwd_persist_kernel<bf16, 1, false> : (const void*)lstm_fwd_persist_kernel<bf16, 2, false>;
  return mt == 1 ? (const void*)lstm_fwd_persist_kernel<float, 1, false> : (const void*)lstm_fwd_persist_kernel<float, 2, false>;
}

template <typename T, int MT, bool HG>
static int launch_persist(const FwdLaunch& L, hipStream_t st) {
  hipLaunchKernelGGL((lstm_fwd_persist_kernel<T, MT, HG>), dim3(L.nblk), dim3(PT), L.lds, st, L.d[0], L.g[0], L.d[1],
                     L.g[1], L.nb0);
  IMGCAP_CHECK_LAUNCH("lstm persistent forward");
  return 0;
}

int lstm_persist_sync_words(const imgcap_lstm_desc& d);

// Runs the whole forward recurrence in one launch when the shape fits; *used = false leaves
// the call to the per-step path.
int lstm_fwd_persistent(const imgcap_lstm_desc& d, hipStream_t st, bool* used) {
  *used = false;
  static const int env = [] {
    const char* e = getenv("IMGCAP_LSTM_PERSIST");
    return e ? atoi(e) : 1;
  }();
  if (!env || d.T < 2 || !d.sync) return 0;
  const int esz = d.dtype == IMGCAP_BF16 ? 2 : 4;
  FwdLaunch L;
  if (!fwd_launch_plan(d, esz, L)) return 0;
  // every workgroup resident at once (the hand-offs spin on each other): else the per-step path
  if (!resident_one_per_cu(fwd_kernel_of(esz, L.mt), L.lds)) return 0;
  L.g[0].fault_step = L.g[1].fault_step = env_step("IMGCAP_LSTM_FAULT_FWD");
  L.g[0].hgran = L.g[1].hgran = 0;
  L.g[0].poll_sleep = L.g[1].poll_sleep = 0;
  static const bool stamps = getenv("IMGCAP_LSTM_STAMPS") && atoi(getenv("IMGCAP_LSTM_STAMPS"));
  L.g[0].stamps = L.g[1].stamps = nullptr;
  if (stamps && d.T <= 64) {  // group 0 only, after every group's sync words (fwd and bwd)
    const int base = (lstm_persist_sync_words(d) + 63) / 64 * 64 + 64;
    if (d.sync_words >= base + 2 * 64 * 16 * 2) L.g[0].stamps = (long long*)(d.sync + base);
  }
  IMGCAP_REQUIRE(d.sync_words >= L.words, "lstm persistent: sync workspace too small");
  IMGCAP_REQUIRE(aligned16(d.sync), "lstm persistent: sync workspace must be 16-byte aligned");
  // zero the error word and every flag (a kernel node when captured)
  if (zero_async(d.sync, align16((size_t)L.words * 4), st) != hipSuccess)
    return fail(IMGCAP_EINVAL, "lstm persistent: zeroing of the sync words failed");
  *used = true;
#define LP_CASE(TT, M_) \
  if (L.mt == M_) return launch_persist<TT, M_, false>(L, st);
  if (esz == 2) {
    LP_CASE(bf16, 1) LP_CASE(bf16, 2)
  } else {
    LP_CASE(float, 1) LP_CASE(float, 2)
  }
#undef LP_CASE
  return fail(IMGCAP_EINVAL, "lstm persistent: no instantiation");
}

// ---- backward ------------------------------------------------------------------------------
static bool bwd_plan(const imgcap_lstm_desc& d, int esz, BGeo& g, size_t& lds, int& mt, int& words,
                     int force_mt = 0) {
  const size_t LDS_MAX = 160 * 1024;
  if (d.B < 1 || d.B > 32 || d.P > 64 || d.A > 512 || d.A % 8 || d.E % 16 || d.D % 16) return false;
  mt = force_mt ? force_mt : d.B <= 16 ? 1 : 2;
  const int KY = d.A + d.E, K4 = 4 * d.D;
  if (KY % 8) return false;
  const int pad = 16 / esz;
  // U: 16 units per block in bf16, 8 in fp32 (rows of 4D + A + E elements in LDS)
  g.UPB = esz == 2 ? 16 : 8;
  if (d.D % g.UPB || d.B * g.UPB > PT) return false;
  g.NU = d.D / g.UPB;
  g.NX = d.E / 16;
  g.NR = d.B;
  if (g.NU + g.NX + g.NR > device_cus()) return false;
  g.ldu = K4 + KY + pad;
  g.ldx = K4 + pad;
  const size_t red = (size_t)(PWV / mt) * 16 * mt * 20 * 4;
  size_t o = align16(16 + (size_t)g.UPB * g.ldu * esz);
  g.u_red = (int)o;
  o = align16(o + red);
  g.u_dg = (int)o;
  o = align16(o + (size_t)d.B * 4 * g.UPB * esz);
  const size_t u = o;
  o = align16(16 + (size_t)16 * g.ldx * esz);
  g.x_red = (int)o;
  const size_t x = align16(o + red);
  // R: att1[b] always, enc[b] when it fits
  const int GA = PT / (d.A / 8);
  size_t r = 0;
  for (int enc_in = 1; enc_in >= 0; --enc_in) {
    o = align16(16 + (size_t)d.P * d.A * esz);
    g.r_enc = enc_in ? (int)o : -1;
    if (enc_in) o = align16(o + (size_t)d.P * d.E * esz);
    g.r_dz = (int)o;
    o = align16(o + (size_t)d.E * 4);
    g.r_dawe = (int)o;
    o = align16(o + (size_t)d.E * 4);
    g.r_red = (int)o;
    o = align16(o + (size_t)GA * d.A * 4);
    g.r_al = (int)o;
    o = align16(o + 64 * 4);
    g.r_dal = (int)o;
    o = align16(o + 64 * 4);
    g.r_dtt = (int)o;
    o = align16(o + (size_t)d.A * esz);
    r = o;
    if (r <= LDS_MAX) break;
  }
  lds = std::max(std::max(std::max(u, x), r), (size_t)81 * 1024);  // one workgroup per CU
  if (lds > LDS_MAX) return false;
  g.gran_off = (SYNC_HDR + g.NU + g.NR + 63) / 64 * 64;
  words = g.gran_off + d.B * d.E * 2;
  return true;
}

struct BwdLaunch {
  imgcap_lstm_desc d[2];
  BGeo g[2];
  int groups = 0, nb0 = 0, nblk = 0, mt = 0, words = 0;
  size_t lds = 0;
};

static bool bwd_launch_plan(const imgcap_lstm_desc& d, int esz, BwdLaunch& L) {
  const int b0 = split_rows(d, false);
  for (int groups = b0 < d.B ? 2 : 1; groups >= 1; --groups) {
    L = BwdLaunch();
    L.groups = groups;
    const int rows[2] = {groups == 2 ? b0 : d.B, d.B - b0};
    L.mt = rows[0] <= 16 ? 1 : 2;
    int soff = 0;
    bool ok = true;
    for (int i = 0; i < groups && ok; ++i) {
      L.d[i] = groups == 2 ? rows_view(d, i ? b0 : 0, rows[i], esz, soff) : d;
      size_t lds;
      int m, words;
      ok = bwd_plan(L.d[i], esz, L.g[i], lds, m, words, L.mt) && aligned16(L.d[i].dcat);
      L.lds = std::max(L.lds, lds);
      if (i == 0) L.nb0 = L.g[0].NU + L.g[0].NX + L.g[0].NR;
      L.nblk += L.g[i].NU + L.g[i].NX + L.g[i].NR;
      soff += (words + 63) / 64 * 64;
      L.words = groups == 2 ? soff : words;
    }
    if (!ok || L.nblk > device_cus()) continue;
    for (int i = 0; i < groups; ++i) L.g[i].err = d.sync;
    if (groups == 1) {
      L.d[1] = L.d[0];
      L.g[1] = L.g[0];
    }
    return true;
  }
  return false;
}

static const void* bwd_kernel_of(int esz, int mt) {
  if (esz == 2) return mt == 1 ? (const void*)lstm_bwd_persist_kernel<bf16, 1> : (const void*)lstm_bwd_persist_kernel<bf16, 2>;
  return mt == 1 ? (const void*)lstm_bwd_persist_kernel<float, 1> : (const void*)lstm_bwd_persist_kernel<float, 2>;
}

template <typename T, int MT>
static int launch_bwd_persist(const BwdLaunch& L, hipStream_t st) {
  hipLaunchKernelGGL((lstm_bwd_persist_kernel<T, MT>), dim3(L.nblk), dim3(PT), L.lds, st, L.d[0], L.g[0], L.d[1],
                     L.g[1], L.nb0);
  IMGCAP_CHECK_LAUNCH("lstm persistent backward");
  return 0;
}

// Runs the whole backward recurrence in one launch when the shape fits (outputs: dcat, de,
// dawe, dh, dc); *used = false leaves the call to the per-step path.
int lstm_bwd_persistent(const imgcap_lstm_desc& d, hipStream_t st, bool* used) {
  *used = false;
  static const int env = [] {
    const char* e = getenv("IMGCAP_LSTM_BWD_PERSIST");
    return e ? atoi(e) : 1;
  }();
  if (!env || d.T < 2 || !d.sync) return 0;
  const int esz = d.dtype == IMGCAP_BF16 ? 2 : 4;
  BwdLaunch L;
  if (!bwd_launch_plan(d, esz, L)) return 0;
  if (!resident_one_per_cu(bwd_kernel_of(esz, L.mt), L.lds)) return 0;
  L.g[0].fault_step = L.g[1].fault_step = env_step("IMGCAP_LSTM_FAULT_BWD");
  IMGCAP_REQUIRE(d.w_zh_t && d.w_att_t, "lstm persistent backward: transposed weights needed");
  IMGCAP_REQUIRE(d.sync_words >= L.words, "lstm persistent backward: sync workspace smaller than imgcap_lstm_sync_words");
  static const bool stamps = getenv("IMGCAP_LSTM_STAMPS") && atoi(getenv("IMGCAP_LSTM_STAMPS"));
  L.g[0].stamps = L.g[1].stamps = nullptr;
  if (stamps && d.T <= 64) {  // same diagnostics area as the forward's: after max(fwd, bwd) words
    const int base = (lstm_persist_sync_words(d) + 63) / 64 * 64 + 64;
    if (d.sync_words >= base + 3 * 64 * 16 * 2) L.g[0].stamps = (long long*)(d.sync + base);
  }
  IMGCAP_REQUIRE(aligned16(d.sync) && aligned16(d.dcat), "lstm persistent backward: 16-byte aligned sync / dcat");
  if (zero_async(d.sync, align16((size_t)L.words * 4), st) != hipSuccess)
    return fail(IMGCAP_EINVAL, "lstm persistent backward: zeroing of the sync words failed");
  *used = true;
  if (esz == 2) return L.mt == 1 ? launch_bwd_persist<bf16, 1>(L, st) : launch_bwd_persist<bf16, 2>(L, st);
  return L.mt == 1 ? launch_bwd_persist<float, 1>(L, st) : launch_bwd_persist<float, 2>(L, st);
}

int lstm_persist_sync_words(const imgcap_lstm_desc& d) {
  const int esz = d.dtype == IMGCAP_BF16 ? 2 : 4;
  FwdLaunch f;
  BwdLaunch b;
  const int fw = fwd_launch_plan(d, esz, f) ? f.words : 0;
  const int bw = bwd_launch_plan(d, esz, b) ? b.words : 0;
  return std::max(fw, bw);
}

}  // namespace imgcap

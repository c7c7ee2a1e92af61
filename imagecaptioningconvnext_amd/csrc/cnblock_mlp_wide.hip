// Fused ConvNeXt block MLP for the wide stages (C = 384, 512: stage 3 of Tiny / Base; torchvision
// CNBlock reached via encoder.py:18-24):
//   x[m, :] += gamma * sd[m / rows_per_sample] * (GELU(LN(y)[m, :] W1^T + b1) W2^T + b2)
// with the 4C hidden on chip.  MEASURED SLOWER than the LayerNorm + two-GEMM path these stages run
// (DESIGN.md §3e): kept as a tested opt-in (the encoder does not call it); the numbers and the
// diagnosis are there.
//
// Block = 8 waves (two per SIMD), 64 rows: the waves of a pair (w, w ^ 4) own the same 16 rows.
// GEMM1 runs swapped (H^T = W1 Z^T, Z fragments resident in registers after the LayerNorm) with
// the pair splitting each 32-unit hidden chunk (wave w computes hidden 16t .. 16t + 15, t = w >> 2);
// after bias + GELU each lane's 4 values go to LDS and the partner lane's 4 come back, which makes
// the lane's B fragment of GEMM2 (swapped too: O^T = W2 H^T; the pair splits the C output
// channels, the accumulators hold 4 consecutive channels of one row per fragment).
//
// Weights: packed once (imgcap_cnblock_mlp_wide_pack) into chunk-major LDS images -- per 32 hidden
// units one W1 image [32][C] and one W2 image [C][32] (k order permuted as GEMM1's output leaves
// the hidden in a lane), 16-byte granules pre-swizzled so every ds_read_b128 lane group covers
// the 64 banks once (SQ_LDS_BANK_CONFLICT measured 0) -- so a chunk half is a contiguous 64C-byte
// copy: LDS-DMA (global_load_lds_dwordx4), no staging registers, into a ring of NSLOT half-slots
// consumed W1(0), W2(0), W1(1), ...  One raw barrier per half (wait for the half's DMA with a
// counted vmcnt, barrier); the refill of the slot the previous half used is issued behind the
// first MFMA group; NSLOT - 1 halves stay in flight.
//
// Rows: the stages' row counts are small (B*196), so when 64-row tiles alone would leave the chip
// idle the hidden is split in two (S = 2): blocks 2t and 2t+1 walk hidden halves of tile t and the
// second to finish adds the first one's fp32 partial (write-through slab + flag: the first
// finisher's stores drain, one lane stores the flag; MI355X_MICROARCH.md hand-off table row 1) --
// in the fixed order p0 + p1 whichever block finishes last, so results are bitwise repeatable.
// The ticket / flag words are left zero for the next launch.
#include <algorithm>
#include <cstdlib>

#include "mfma.h"

namespace imgcap {
namespace {

typedef unsigned wu32x4_t __attribute__((ext_vector_type(4)));
typedef __amdgpu_buffer_rsrc_t wrsrc_t;

DEV wrsrc_t w_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
DEV f32x4 w_ld_wt(wrsrc_t r, uint32_t off) {  // 16-byte write-through (sc1) load
  const wu32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16);
  return __builtin_bit_cast(f32x4, v);
}
DEV void w_st_wt(wrsrc_t r, uint32_t off, f32x4 v) {  // 16-byte write-through (sc1) store
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(wu32x4_t, v), r, off, 0, 16);
}

template <int C>
struct WideCfg {
  static constexpr int HID = 4 * C;
  static constexpr int NJ = HID / 32;            // 32-unit hidden chunks
  static constexpr int HALF = 64 * C;            // bytes of one W1 (or W2) chunk image
  static constexpr int THREADS = 512;            // 8 waves: two per SIMD
  static constexpr int RING = 144 * 1024;        // LDS for the ring
  static constexpr int NSLOT = RING / HALF > 6 ? 6 : RING / HALF;
  static constexpr int NPH = HALF / (THREADS * 16);  // LDS-DMA instructions per thread per half
  static constexpr int KS1 = C / 32;             // GEMM1 k-steps
  static constexpr int TNW = C / 32;             // GEMM2 output fragments per wave (half the channels)
  static constexpr int GRP = C == 384 ? 6 : 4;   // fragments per software-pipelined read group
  static constexpr int B1_OFF = NSLOT * HALF;
  static constexpr int HX_OFF = B1_OFF + HID * 4;  // b1 of the block's hidden range (<= HID)
  static constexpr int SMEM = HX_OFF + 8 * 64 * 8;  // + the hidden exchange [wave][lane] (8 B); the ticket reuses it
  static_assert(NSLOT >= 3 && NPH * THREADS * 16 == HALF && SMEM <= 160 * 1024, "LDS plan");
  static_assert(NJ % 2 == 0 && KS1 % GRP == 0 && TNW % GRP == 0, "chunking");
};

constexpr int WIDE_SPIN_LIMIT = 1 << 22;

#ifdef WIDE_STAMPS  // diagnostic build only (tools/kbench/wide_bench.hip): s_memtime at phase edges
__device__ long long* g_wide_stamps;
#define WSTAMP(k)                                                                                      \
  do {                                                                                               \
    if (g_wide_stamps && blockIdx.x < 32 && (threadIdx.x & 63) == 0 && (k) < 64)                   \
      g_wide_stamps[(blockIdx.x * 8 + (threadIdx.x >> 6)) * 64 + (k)] = (long long)__builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define WSTAMP(k) \
  do {            \
  } while (0)
#endif

// granule swizzles of the packed images (the reads below and the pack kernel agree):
//   W1 [32][C]: granule g of row i at g ^ (i & 15)  (rows are a multiple of 256 B: the 16 lanes of
//               a ds_read_b128 group -- rows fr, granule 4ks + fq -- land on 16 distinct slots)
//   W2 [C][32]: granule q of row n at q ^ (n & 8 ? 3 : 0)  (64-byte rows: 4 rows share a bank row)
DEV int w2_swz(int n) { return (n & 8) ? 3 : 0; }

template <int C>
DEV void wide_ln(bf16x8 (&zf)[C / 32], const float* __restrict__ lnw, const float* __restrict__ lnb, int fq) {
  constexpr int KS = C / 32;
  float s = 0.f;
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
#pragma unroll
    for (int j = 0; j < 8; ++j) s += (float)zf[ks][j];
  s += __shfl_xor(s, 16, 64);
  s += __shfl_xor(s, 32, 64);
  const float mean = s * (1.f / C);
  float q = 0.f;
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float d = (float)zf[ks][j] - mean;
      q += d * d;
    }
  q += __shfl_xor(q, 16, 64);
  q += __shfl_xor(q, 32, 64);
  const float rstd = rsqrtf(q * (1.f / C) + 1e-6f);
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int k = ks * 32 + 8 * fq;
    const f32x4 g0 = *(const f32x4*)(lnw + k), g1 = *(const f32x4*)(lnw + k + 4);
    const f32x4 c0 = *(const f32x4*)(lnb + k), c1 = *(const f32x4*)(lnb + k + 4);
    const float gg[8] = {g0[0], g0[1], g0[2], g0[3], g1[0], g1[1], g1[2], g1[3]};
    const float cc[8] = {c0[0], c0[1], c0[2], c0[3], c1[0], c1[1], c1[2], c1[3]};
#pragma unroll
    for (int j = 0; j < 8; ++j) zf[ks][j] = (bf16)(((float)zf[ks][j] - mean) * rstd * gg[j] + cc[j]);
  }
}

template <int C>
DEV void issue_half(const char* __restrict__ wimg, int j0, int q, char* slot, int w, int lane) {
  using G = WideCfg<C>;
  const char* src = wimg + ((long)j0 * 2 + q) * G::HALF;  // halves in image order: W1(j), W2(j), ...
#pragma unroll
  for (int i = 0; i < G::NPH; ++i) {
    const int p0 = (i * 8 + w) * 64;  // first 16-byte piece of this wave-instruction
    __builtin_amdgcn_global_load_lds((const void*)(src + (long)(p0 + lane) * 16),
                                     (__attribute__((address_space(3))) void*)(slot + p0 * 16), 16, 0, 0);
  }
}

// this thread's DMAs of the half being waited for have landed when at most n*NPH newer ones are out
template <int NPH>
DEV void wait_halves(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NPH) : "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NPH) : "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * NPH) : "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * NPH) : "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(5 * NPH) : "memory"); break;
  }
}

template <int C>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void cnblock_mlp_wide_kernel(
    int M, int S, const bf16* __restrict__ y, const float* __restrict__ lnw, const float* __restrict__ lnb,
    const char* __restrict__ wimg, const float* __restrict__ b1, const float* __restrict__ b2,
    const float* __restrict__ gamma, const float* __restrict__ sd, int rows_per_sample, bf16* __restrict__ x,
    float* __restrict__ part, int* __restrict__ sync, int dbg) {
  using G = WideCfg<C>;
  // ONE static LDS object (with the dynamic-LDS base the compiler put vmcnt(0) -- a drain of every
  // DMA in flight -- before the first LDS read of each half)
  __shared__ __attribute__((aligned(16))) char smem[G::SMEM];
  float* b1s = (float*)(smem + G::B1_OFF);
  uint2* hx = (uint2*)(smem + G::HX_OFF);
  int* ticket = (int*)(smem + G::HX_OFF);
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int wr = w & 3, t = w >> 2;  // row slab; hidden half of GEMM1 and channel half of GEMM2
  const int tile = blockIdx.x / S, s = blockIdx.x - tile * S;
  const int nj = G::NJ / S, j0 = s * nj, nq = 2 * nj;
  const int row = tile * 64 + wr * 16 + fr;
  const bool rok = row < M;
  WSTAMP(40);

  // this wave's Z rows first (the oldest loads: waiting for them never drains the ring's DMA),
  // b1 of the block's hidden range -> LDS, then ring halves 0 .. NSLOT-1
  bf16x8 zf[G::KS1];
  {
    const bf16* zp = y + (long)(rok ? row : 0) * C + 8 * fq;
#pragma unroll
    for (int ks = 0; ks < G::KS1; ++ks) {
      const uint4 v = *(const uint4*)(zp + ks * 32);
      zf[ks] = __builtin_bit_cast(bf16x8, rok ? v : make_uint4(0u, 0u, 0u, 0u));
    }
  }
  for (int i = threadIdx.x; i < nj * 32; i += G::THREADS) b1s[i] = b1[j0 * 32 + i];
#pragma unroll
  for (int q = 0; q < G::NSLOT; ++q)
    if (q < nq && dbg != 2) issue_half<C>(wimg, j0, q, smem + q * G::HALF, w, lane);
  if (lnw) wide_ln<C>(zf, lnw, lnb, fq);
  // the fragments' loads retire here, outside the loop (a first use inside it made the compiler
  // wait vmcnt(0) -- every DMA in flight -- before MFMAs in every half)
#pragma unroll
  for (int ks = 0; ks < G::KS1; ++ks) asm volatile("" : "+v"(zf[ks]));

  f32x4 acc2[G::TNW];
#pragma unroll
  for (int tn = 0; tn < G::TNW; ++tn) acc2[tn] = f32x4{0.f, 0.f, 0.f, 0.f};

  // start of half q: its DMA landed for every thread, the slot of half q-1 is free for half
  // q-1+NSLOT (every wave has passed this barrier, so it is done reading that slot)
  int pend = -1;
  auto begin_half = [&](int q) -> const char* {
    if (q >= 8 && q < 24) WSTAMP(2 * (q - 8));
    const int issued = min(nq, G::NSLOT + max(q - 1, 0));
    if (dbg != 2) wait_halves<G::NPH>(issued - q - 1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (q >= 8 && q < 24) WSTAMP(2 * (q - 8) + 1);
    pend = q >= 1 && q - 1 + G::NSLOT < nq && dbg != 2 ? q - 1 + G::NSLOT : -1;
    return smem + (q % G::NSLOT) * G::HALF;
  };
  // the refill of the previous half's slot, issued behind the first MFMA group of this half (its
  // DMA instructions' issue cost then overlaps MFMAs in flight instead of delaying them)
  auto refill = [&]() {
    if (pend >= 0) issue_half<C>(wimg, j0, pend, smem + ((pend - G::NSLOT) % G::NSLOT) * G::HALF, w, lane);
  };
  // Fragment reads are software-pipelined by groups: group g+1 is requested before group g's
  // MFMAs, and a scheduling barrier keeps the compiler from pairing each read with its MFMA (its
  // default: one read in flight, the MFMA waiting out the LDS latency -- 5x the MFMA time).
  // GEMM1 (swapped) of local chunk jl, this wave's hidden half t: a1 = b1 + W1[16t + .., :] Z^T
  // -> hidden 16t + 4fq + r of row fr; GELU'd into the exchange slot of this lane
  auto gemm1 = [&](const char* img, int jl) {
    f32x4 a1 = *(const f32x4*)(b1s + 32 * jl + 16 * t + 4 * fq);
    if (dbg != 1) {
      constexpr int NG = G::KS1 / G::GRP;
      bf16x8 a[2][G::GRP];
      const char* rowp = img + (16 * t + fr) * (2 * C);
      auto load = [&](int gi, bf16x8 (&dst)[G::GRP]) {
#pragma unroll
        for (int i = 0; i < G::GRP; ++i) dst[i] = *(const bf16x8*)(rowp + (((4 * (G::GRP * gi + i) + fq) ^ fr) << 4));
      };
      load(0, a[0]);
#pragma unroll
      for (int gi = 0; gi < NG; ++gi) {
        if (gi + 1 < NG) load(gi + 1, a[(gi + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < G::GRP; ++i)
          a1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[gi & 1][i], zf[G::GRP * gi + i], a1, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        if (gi == 0) refill();
      }
    } else {
      refill();
    }
    bf16x4 h;
#pragma unroll
    for (int r = 0; r < 4; ++r) h[r] = (bf16)gelu_sig(a1[r]);
    hx[w * 64 + lane] = __builtin_bit_cast(uint2, h);
  };
  // GEMM2 (swapped): acc2[tn] += W2[16(tn + t C/32) + .., chunk] H^T -> channels 16(tn + t C/32) + 4fq + r
  // of row fr; H = this lane's GELU'd hidden half and the partner wave's (same lane): element e
  // <-> hidden 16(e / 4) + 4fq + e % 4, the W2 image's k order
  auto gemm2 = [&](const char* img) {
    const uint2 mine = hx[w * 64 + lane], other = hx[(w ^ 4) * 64 + lane];
    const uint4 hv = t == 0 ? make_uint4(mine.x, mine.y, other.x, other.y) : make_uint4(other.x, other.y, mine.x, mine.y);
    const bf16x8 h = __builtin_bit_cast(bf16x8, hv);
    if (dbg == 1) {
      refill();
      return;
    }
    const int sw = (fq ^ w2_swz(fr)) << 4;
    const char* base = img + (16 * t * G::TNW + fr) * 64 + sw;
    constexpr int NG = G::TNW / G::GRP;
    bf16x8 a[2][G::GRP];
    auto load = [&](int gi, bf16x8 (&dst)[G::GRP]) {
#pragma unroll
      for (int i = 0; i < G::GRP; ++i) dst[i] = *(const bf16x8*)(base + 16 * (G::GRP * gi + i) * 64);
    };
    load(0, a[0]);
#pragma unroll
    for (int gi = 0; gi < NG; ++gi) {
      if (gi + 1 < NG) load(gi + 1, a[(gi + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < G::GRP; ++i)
        acc2[G::GRP * gi + i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[gi & 1][i], h, acc2[G::GRP * gi + i], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      if (gi == 0) refill();
    }
  };

  // halves W1(0), W2(0), W1(1), ...: the hidden exchange of chunk j is written in half W1(j) and
  // read in half W2(j), the barrier of begin_half in between (and the next write comes after the
  // following barrier)
  for (int jl = 0; jl < nj; ++jl) {
    gemm1(begin_half(2 * jl), jl);
    gemm2(begin_half(2 * jl + 1));
  }

  WSTAMP(41);
  // ---- epilogue: x += gamma * sd * (sum of the slices' partials + b2) ----
  if (S > 1) {
    // ticket: the first finisher publishes its partial, the second adds it
    __syncthreads();
    if (threadIdx.x == 0) *ticket = __hip_atomic_fetch_add(sync + 2 * tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const int first = *ticket == 0;
    const uint32_t pbytes = (uint32_t)(64 * C * 4);
    const wrsrc_t rp = w_rsrc(part + (long)tile * 64 * C, pbytes);
    const uint32_t lbase = (uint32_t)((w * G::TNW) * 64 + lane) * 16;
    if (first) {
#pragma unroll
      for (int tn = 0; tn < G::TNW; ++tn) w_st_wt(rp, lbase + tn * 64 * 16, acc2[tn]);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) __hip_atomic_store(sync + 2 * tile + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    // second finisher: the first one took its ticket earlier, so it is resident and publishing
    if (threadIdx.x == 0) {
      int ok = 0;
      for (int spins = 0; spins < WIDE_SPIN_LIMIT; ++spins)
        if (__hip_atomic_load(sync + 2 * tile + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 1) {
          ok = 1;
          break;
        }
      __hip_atomic_store(sync + 2 * tile + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(sync + 2 * tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *ticket = ok ? 1 : -1;
    }
    __syncthreads();
    const bool ok = *ticket == 1;  // a lost partner leaves NaN outputs (loud in the loss)
#pragma unroll
    for (int tn = 0; tn < G::TNW; ++tn) {
      const f32x4 o = w_ld_wt(rp, lbase + tn * 64 * 16);
      // fixed order p0 + p1 (fp32 addition is commutative: the same bits whichever block adds)
      acc2[tn] = ok ? acc2[tn] + o : f32x4{__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""), __builtin_nanf("")};
    }
  }
  if (rok) {
    const float sc = sd ? sd[row / rows_per_sample] : 1.f;
    uint2 xr[G::TNW];
    const int c0 = 16 * t * G::TNW + 4 * fq;
#pragma unroll
    for (int tn = 0; tn < G::TNW; ++tn) xr[tn] = *(const uint2*)(x + (long)row * C + c0 + tn * 16);
#pragma unroll
    for (int tn = 0; tn < G::TNW; ++tn) {
      const int c = c0 + tn * 16;
      asm volatile("" ::: "memory");  // gamma / b2 per fragment (hoisting all of them spilled)
      const f32x4 g = *(const f32x4*)(gamma + c), bb = *(const f32x4*)(b2 + c);
      const bf16x4 xv = __builtin_bit_cast(bf16x4, xr[tn]);
      bf16x4 o;
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = (bf16)((float)xv[r] + (acc2[tn][r] + bb[r]) * g[r] * sc);
      *(bf16x4*)(x + (long)row * C + c) = o;
    }
  }
}

// chunk images: [NJ][2][64C bytes]; one thread per 16-byte granule of the image
template <int C>
__global__ void cnblock_mlp_wide_pack_kernel(const bf16* __restrict__ w1, const bf16* __restrict__ w2,
                                             bf16* __restrict__ img) {
  using G = WideCfg<C>;
  const long gi = (long)blockIdx.x * blockDim.x + threadIdx.x;  // granule index
  const long per_chunk = 2L * G::HALF / 16;
  if (gi >= (long)G::NJ * per_chunk) return;
  const int j = (int)(gi / per_chunk), rem = (int)(gi % per_chunk);
  bf16x8 v;
  if (rem < G::HALF / 16) {  // W1 [32][C]: stored granule gs of row i holds granule gs ^ (i & 15)
    const int i = rem / (C / 8), gs = rem % (C / 8);
    const int g = gs ^ (i & 15);
    v = *(const bf16x8*)(w1 + (long)(32 * j + i) * C + 8 * g);
  } else {  // W2 [C][32]: stored granule qs of row n holds hidden {16e/4 + 4q + e%4}, q = qs ^ swz(n)
    const int r2 = rem - G::HALF / 16;
    const int n = r2 / 4, qs = r2 % 4, q = qs ^ w2_swz(n);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = w2[(long)n * G::HID + 32 * j + 16 * (e >> 2) + 4 * q + (e & 3)];
  }
  *(bf16x8*)(img + gi * 8) = v;
}

int wide_dbg() {  // kernel-timing experiments only (IMGCAP_WIDE_DBG: 1 = DMA only, 2 = compute only)
  static const int v = [] {
    const char* e = getenv("IMGCAP_WIDE_DBG");
    return e ? atoi(e) : 0;
  }();
  return v;
}

int wide_slices(int M) {
  const int tiles = (M + 63) / 64;
  return tiles < 128 ? 2 : 1;
}

}  // namespace
}  // namespace imgcap

using namespace imgcap;

extern "C" int imgcap_cnblock_mlp_wide_pack(int C, const void* w1, const void* w2, void* img, void* stream) {
  IMGCAP_REQUIRE(C == 384 || C == 512, "imgcap_cnblock_mlp_wide_pack: C must be 384 or 512");
  IMGCAP_REQUIRE(aligned16(w1) && aligned16(w2) && aligned16(img), "imgcap_cnblock_mlp_wide_pack: alignment");
  hipStream_t st = (hipStream_t)stream;
  const long granules = (long)(C / 8) * 2 * 64 * C / 16;
  const int blocks = (int)((granules + 255) / 256);
#define PK_(CC) \
  hipLaunchKernelGGL(cnblock_mlp_wide_pack_kernel<CC>, dim3(blocks), dim3(256), 0, st, (const bf16*)w1, (const bf16*)w2, (bf16*)img)
  if (C == 384) PK_(384);
  else PK_(512);
#undef PK_
  IMGCAP_CHECK_LAUNCH("imgcap_cnblock_mlp_wide_pack");
  return 0;
}

extern "C" int imgcap_cnblock_mlp_wide_scratch(int M, int C, uint64_t* part_bytes, uint64_t* sync_bytes) {
  IMGCAP_REQUIRE(part_bytes && sync_bytes, "imgcap_cnblock_mlp_wide_scratch: null output");
  const int tiles = (M + 63) / 64;
  const bool split = wide_slices(M) > 1;
  *part_bytes = split ? (uint64_t)tiles * 64 * C * 4 : 0;
  *sync_bytes = split ? (uint64_t)tiles * 2 * sizeof(int) : 0;
  return 0;
}

extern "C" int imgcap_cnblock_mlp_wide(int M, int C, const void* y, const float* ln_w, const float* ln_b,
                                       const void* wimg, const float* b1, const float* b2, const float* gamma,
                                       const float* sd, int rows_per_sample, void* x, void* part, int* sync,
                                       void* stream) {
  if (M == 0) return 0;
  IMGCAP_REQUIRE(C == 384 || C == 512, "imgcap_cnblock_mlp_wide: C must be 384 or 512");
  IMGCAP_REQUIRE(aligned16(y) && aligned16(wimg) && aligned16(x) && aligned16(b1) && aligned16(b2) &&
                     aligned16(gamma),
                 "imgcap_cnblock_mlp_wide: operands must be 16-byte aligned");
  IMGCAP_REQUIRE(sd == nullptr || rows_per_sample > 0, "imgcap_cnblock_mlp_wide: rows_per_sample");
  IMGCAP_REQUIRE((ln_w == nullptr) == (ln_b == nullptr) && (ln_w == nullptr || (aligned16(ln_w) && aligned16(ln_b))),
                 "imgcap_cnblock_mlp_wide: ln_w / ln_b");
  const int S = wide_slices(M);
  IMGCAP_REQUIRE(S == 1 || (part && sync && aligned16(part)),
                 "imgcap_cnblock_mlp_wide: split launch needs part / sync scratch (imgcap_cnblock_mlp_wide_scratch)");
  hipStream_t st = (hipStream_t)stream;
  const int grid = ((M + 63) / 64) * S;
  auto launch = [&](auto kern, int) {
    hipLaunchKernelGGL(kern, dim3(grid), dim3(512), 0, st, M, S, (const bf16*)y, ln_w, ln_b, (const char*)wimg,
                       b1, b2, gamma, sd, rows_per_sample, (bf16*)x, (float*)part, sync, wide_dbg());
  };
  if (C == 384) launch(cnblock_mlp_wide_kernel<384>, WideCfg<384>::SMEM);
  else launch(cnblock_mlp_wide_kernel<512>, WideCfg<512>::SMEM);
  IMGCAP_CHECK_LAUNCH("imgcap_cnblock_mlp_wide");
  return 0;
}

// Weight-stationary short-K bf16 GEMM -- included by gemm.hip.
//
// C[M, N] = epilogue(A[M, K] . B[N, K]^T) for K = 384 / 512 with both operands k-major (activations
// x nn.Linear weights): the forward pointwise Linears of the ConvNeXt stage-3 blocks
// (12544 x 1536 x 384 at C3, torchvision CNBlock via encoder.py:24), the 1->2 downsample and the
// Transformer decoder's d = 512 projections (transformerDecoder.py:82-83,104).  At such K a
// tile's whole k-loop is a few steps, so tiled kernels are paid for by what surrounds the loop
// (prologue, epilogue, per-tile operand re-reads: the 64x64 LDS-DMA tile moves ~460 MB through
// L2 for the stage-3 product's 11 MB of operands).  Here the weight slice never moves:
//
//   * a block owns a slice of 32*NW output columns; each wave keeps its 32 columns x K of B in
//     registers for the whole launch (KS = K/16 fragments of 4 VGPRs, loaded once);
//   * the block walks a contiguous range of rows in chunks of 32, each chunk (32 x K of A) brought
//     into LDS by buffer_load ... lds (S-stage ring, one barrier per chunk, counted vmcnt waits),
//     every wave reading the chunk for its own 32 columns: per 16-deep k-step one ds_read_b128 and
//     one v_mfma_f32_32x32x16_bf16;
//   * MFMA as D^T = B_slice . A_chunk^T, so a lane holds one output row and 4 x 4 consecutive
//     columns: the epilogue (alpha, bias, GELU / ReLU, dropout, column scale) runs on the
//     accumulators and leaves as four 8-byte buffer stores per lane (out-of-range rows / columns
//     dropped by the descriptor's range check, so every wave issues the same store count);
//   * block -> (row group, column slice) through an XCD-contiguous bijection: the blocks of one XCD
//     share row groups (A chunks hit that XCD's L2) and column slices (B slices likewise).
// Per CU the operand bytes are (its rows + its columns) x K x 2 once each, against
// 2 x rows x columns x K of MFMA work; for the stage-3 product ~0.42 MB and 59 MFLOP.
//
// LDS chunk image: [32 rows][K] bf16, 16-byte granule g of row r stored at slot g ^ (r & 15)
// (K % 128 == 0): the 16 lanes of each ds_read_b128 lane group read 16 distinct slots of the
// 256-byte bank row -- conflict-free.  The DMA writes the image linearly (lane = slot) and reads
// the source granule slot ^ (r & 15) instead.

typedef __amdgpu_buffer_rsrc_t ws_rsrc_t;
typedef unsigned ws_u32x4 __attribute__((ext_vector_type(4)));
typedef float ws_f32x16 __attribute__((ext_vector_type(16)));

struct WsArgs {
  const bf16* A;
  const bf16* B;
  void* C;
  long lda, ldb, ldc;
  int M, N;
  int slices;        // column slices of 32 * NW
  int row_groups;    // blocks per column slice
  int chunks_per;    // 32-row chunks per row group
  imgcap_epilogue ep;
  const uint64_t* seed_ctr;
  int64_t b_bytes, c_bytes;
};

DEV ws_rsrc_t ws_rsrc(const void* base, int64_t bytes) {
  const int n = bytes <= 0 ? 0 : bytes > 0x7fffffffLL ? 0x7fffffff : (int)bytes;
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, n, 0x00020000);
}

// s_waitcnt vmcnt(n), n uniform at run time (cases up to 63)
#define WS_VMW(N) \
  case N:         \
    asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); \
    break;
DEV void ws_vmwait(int n) {
  switch (n) {
    WS_VMW(0) WS_VMW(1) WS_VMW(2) WS_VMW(3) WS_VMW(4) WS_VMW(5) WS_VMW(6) WS_VMW(7) WS_VMW(8) WS_VMW(9)
    WS_VMW(10) WS_VMW(11) WS_VMW(12) WS_VMW(13) WS_VMW(14) WS_VMW(15) WS_VMW(16) WS_VMW(17) WS_VMW(18)
    WS_VMW(19) WS_VMW(20) WS_VMW(21) WS_VMW(22) WS_VMW(23) WS_VMW(24) WS_VMW(25) WS_VMW(26) WS_VMW(27)
    WS_VMW(28) WS_VMW(29) WS_VMW(30) WS_VMW(31) WS_VMW(32) WS_VMW(33) WS_VMW(34) WS_VMW(35) WS_VMW(36)
    default:
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      break;
  }
}
#undef WS_VMW

// the PW pieces of one 32-row chunk (rows row0 ..) into the stage image st (this wave's pieces)
template <int PW, int NW>
DEV void ws_issue(const bf16* A, long lda, int M, long row0, char* st, int w, const uint32_t (&voff)[PW]) {
  const ws_rsrc_t rs = ws_rsrc(A + row0 * lda, ((long)M - row0) * lda * 2);
#pragma unroll
  for (int j = 0; j < PW; ++j)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(st + (j * NW + w) * 1024), 16,
                                             voff[j], 0, 0, 0);
}

// ACT: the epilogue's activation (IMGCAP_ACT_NONE / GELU / RELU); bias, alpha, dropout and the
// column scale as the epilogue asks (no operand reads in the loop)
// STG: the chunk's output tile staged through LDS ([32 rows][32*NW columns] bf16, 16-byte padded
// rows) and stored as whole row segments (16 B per lane, 32*NW*2 contiguous bytes per row) instead
// of 8-byte pieces of 32 rows per wave-instruction; needs N % 8 == 0.
template <int KS, int NW, int S, int ACT, bool STG = false>
__global__ __launch_bounds__(NW * 64, 2) void gemm_ws_kernel(WsArgs a) {
  constexpr int K = KS * 16;
  constexpr int G = K / 8;                  // 16-byte granules per row
  constexpr int CHUNK = 32 * K * 2;         // bytes of one 32-row chunk image
  constexpr int PIECES = CHUNK / 1024;      // 1 KB wave-instructions per chunk
  constexpr int PW = PIECES / NW;           // ... per wave
  static_assert(PW * NW == PIECES && G % 16 == 0, "chunk vs block");
  constexpr int OROW = 32 * NW * 2 + 16;    // staged output row pitch (bytes)
  constexpr int OSEG = 32 * NW * 2 / 16;    // 16-byte segments of one staged row
  constexpr int NST = STG ? 32 * OSEG / (64 * NW) : 4;  // stores per lane per chunk
  static_assert(!STG || NST * 64 * NW == 32 * OSEG, "staged output vs block");
  __shared__ __attribute__((aligned(16))) char sm[S * CHUNK + (STG ? 32 * OROW : 0)];

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 31, h = lane >> 5;

  // block -> (row group, column slice): XCD x = b % 8 holds G/8 + (x < G%8) consecutive slots
  const int GB = gridDim.x, b = blockIdx.x;
  const int xq = GB / 8, xr = GB % 8, xb = b % 8;
  const int slot = xb * xq + min(xb, xr) + b / 8;
  const int grp = slot / a.slices, sl = slot - grp * a.slices;
  const int M = a.M, N = a.N;
  const int nchunks_all = (M + 31) / 32;
  const int c0 = grp * a.chunks_per;
  const int nch = max(0, min(a.chunks_per, nchunks_all - c0));
  if (nch == 0) return;  // uniform per block: every wave leaves together
  const int n0 = sl * 32 * NW + 32 * w;     // this wave's first column
  const bool active = n0 < N;               // wave-uniform

  imgcap_epilogue ep = a.ep;
  const bool drop = ep.drop_p > 0.f;
  if (drop) ep.seed = eff_seed(ep.seed, a.seed_ctr);
  const long lda = a.lda;

  // ---- DMA sources of this lane for the PW pieces of a chunk (offsets from the chunk's row 0)
  uint32_t voff[PW];
#pragma unroll
  for (int j = 0; j < PW; ++j) {
    const int p = (j * NW + w) * 64 + lane;  // slot of the chunk image this lane writes
    const int rr = p / G, gs = p - rr * G;
    voff[j] = (uint32_t)(((long)rr * lda + 8 * (gs ^ (rr & 15))) * 2);
  }
  // chunk c (0-based within the group) into stage c % S
#define WS_ISSUE(c_) ws_issue<PW, NW>(a.A, lda, M, (long)(c0 + (c_)) * 32, sm + ((c_) % S) * CHUNK, w, voff)

  // ---- prologue: the first S-1 chunks in flight, then this wave's weight slice into registers
#pragma unroll
  for (int c = 0; c < S - 1; ++c)
    if (c < nch) WS_ISSUE(c);
  bf16x8 wf[KS];
  {
    const ws_rsrc_t rb = ws_rsrc(a.B, a.b_bytes);
    const int n = n0 + r;
    const uint32_t base = n < N ? (uint32_t)(((long)n * a.ldb + 8 * h) * 2) : 0x80000000u;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      wf[ks] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rb, base + 32 * ks, 0, 0));
  }
  // epilogue column operands of this lane's 16 columns n0 + 8g + 4h + e (fixed for the launch)
  float bias[16], csc[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int n = n0 + 8 * (i >> 2) + 4 * h + (i & 3);
    bias[i] = (ep.bias && n < N) ? ep.bias[n] : 0.f;
    csc[i] = (ep.colscale && n < N) ? ep.colscale[n] : 1.f;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  const ws_rsrc_t rc = ws_rsrc(a.C, (int64_t)a.c_bytes);
  const int lds_row = r * (K * 2);
  for (int c = 0; c < nch; ++c) {
    // chunk c landed (issued S-1 iterations ago; the younger ops of this wave since then: the
    // stores of the S-1 epilogues before this one and the pieces of the chunks issued after it)
    if (c >= S - 1) ws_vmwait((active || STG ? NST : 0) * (S - 1) + PW * min(S - 2, nch - 1 - c));
    __builtin_amdgcn_s_barrier();  // chunk c visible to every wave; stage (c-1) % S free
    if (c + S - 1 < nch) WS_ISSUE(c + S - 1);
    if (!active && !STG) continue;
    const char* st = sm + (c % S) * CHUNK + lds_row;
    ws_f32x16 acc = {};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int g = 2 * ks + h;
      const bf16x8 xf = *(const bf16x8*)(st + ((g ^ (r & 15)) << 4));
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[ks], xf, acc, 0, 0, 0);
    }
    // epilogue: row m = chunk row r, columns n0 + 8g + 4h + e (e = 0..3) in acc[4g + e]
    const int m = (c0 + c) * 32 + r;
    const bool row_ok = m < M;
    float v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = acc[i] * ep.alpha + bias[i];
    if constexpr (ACT == IMGCAP_ACT_GELU) {
      // the sigmoid form (common.h gelu_sig: |error| <= 5.5e-5, below the bf16 rounding of the
      // stored hidden value): 12544 x 1536 x 384 33.4 -> 31.3 us against the polynomial erf
      // (gelu_fast2), C3 +0.5 % on one box (tools/gpu/r6_wsgelu.sh)
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = gelu_sig(v[i]);
    } else if constexpr (ACT == IMGCAP_ACT_RELU) {
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = fmaxf(v[i], 0.f);
    }
    if (drop) {
      const uint64_t rowi = (uint64_t)m * ep.drop_ld + n0 + 4 * h;
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] *= dropout_scale(ep.seed, ep.drop_stream, rowi + 8 * (i >> 2) + (i & 3), ep.drop_p);
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] *= csc[i];
    if constexpr (STG) {
      // this wave's 32 x 32 tile into the staged block row image, then every wave stores whole
      // row segments: lane e of store j = segment (j*64*NW + w*64 + e) of the [32][OSEG] image
      char* ost = sm + S * CHUNK;
      typedef unsigned ws_u32x2s __attribute__((ext_vector_type(2)));
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const bf16x2 lo = {(bf16)v[4 * g], (bf16)v[4 * g + 1]}, hi = {(bf16)v[4 * g + 2], (bf16)v[4 * g + 3]};
        *(ws_u32x2s*)(ost + r * OROW + (32 * w + 8 * g + 4 * h) * 2) =
            ws_u32x2s{__builtin_bit_cast(uint32_t, lo), __builtin_bit_cast(uint32_t, hi)};
      }
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's staging writes done
      __builtin_amdgcn_s_barrier();
      const int cb = sl * 32 * NW;  // the block's first column
#pragma unroll
      for (int j = 0; j < NST; ++j) {
        const int q = (j * NW + w) * 64 + lane, rr = q / OSEG, sg = q - rr * OSEG;
        const uint4 val = *(const uint4*)(ost + rr * OROW + sg * 16);
        const int mm = (c0 + c) * 32 + rr, n = cb + 8 * sg;
        const uint32_t off = (mm < M && n < N) ? (uint32_t)(((long)mm * a.ldc + n) * 2) : 0x80000000u;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(ws_u32x4, val), rc, off, 0, 0);
      }
      continue;
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int n = n0 + 8 * g + 4 * h;
      const uint32_t off = (row_ok && n < N) ? (uint32_t)(((long)m * a.ldc + n) * 2) : 0x80000000u;
      const bf16x2 lo = {(bf16)v[4 * g], (bf16)v[4 * g + 1]}, hi = {(bf16)v[4 * g + 2], (bf16)v[4 * g + 3]};
      typedef unsigned ws_u32x2 __attribute__((ext_vector_type(2)));
      const ws_u32x2 pk = {__builtin_bit_cast(uint32_t, lo), __builtin_bit_cast(uint32_t, hi)};
      __builtin_amdgcn_raw_buffer_store_b64(pk, rc, off, 0, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#undef WS_ISSUE
}

#ifdef IMGCAP_STAMPS  // measured slower (35.1-38.2 us vs 32.2): diagnostic build only
// ---- software-pipelined form -------------------------------------------------------------------
// The loop above runs each chunk as [barrier, MFMAs, epilogue VALU, stores] in lockstep over the
// block's waves, so the matrix pipe idles through every epilogue (measured: ~2.6 us per chunk
// against ~0.64 us of MFMA work at 12544 x 1536 x 384).  Here iteration c multiplies chunk c into
// one accumulator while the epilogue of chunk c-1 runs from the other, in the same basic block, so
// the scheduler can put the epilogue's VALU and stores into the MFMAs' issue gaps; the loop is
// unrolled by two so both accumulators keep static registers.  The LDS fragment addresses are 8
// per-lane offsets (the granule swizzle repeats every 8 k-steps) plus immediates.  No column scale.

// epilogue of one chunk: row m, this lane's columns n0 + 8g + 4h + e from acc[4g + e]
template <int ACT>
DEV void ws_epi(const ws_f32x16& acc, const float (&bias)[16], const imgcap_epilogue& ep, bool drop, int m, int M,
                int N, int n0, int h, long ldc, ws_rsrc_t rc) {
  float v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = acc[i] * ep.alpha + bias[i];
  if constexpr (ACT == IMGCAP_ACT_GELU) {
#pragma unroll
    for (int i = 0; i < 16; i += 2) {
      const f32x2 gv = gelu_fast2(f32x2{v[i], v[i + 1]});
      v[i] = gv[0];
      v[i + 1] = gv[1];
    }
  } else if constexpr (ACT == IMGCAP_ACT_RELU) {
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = fmaxf(v[i], 0.f);
  }
  if (drop) {
    const uint64_t rowi = (uint64_t)m * ep.drop_ld + n0 + 4 * h;
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] *= dropout_scale(ep.seed, ep.drop_stream, rowi + 8 * (i >> 2) + (i & 3), ep.drop_p);
  }
  typedef unsigned ws_u32x2p __attribute__((ext_vector_type(2)));
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int n = n0 + 8 * g + 4 * h;
    const uint32_t off = (m < M && n < N) ? (uint32_t)(((long)m * ldc + n) * 2) : 0x80000000u;
    const bf16x2 lo = {(bf16)v[4 * g], (bf16)v[4 * g + 1]}, hi = {(bf16)v[4 * g + 2], (bf16)v[4 * g + 3]};
    __builtin_amdgcn_raw_buffer_store_b64(ws_u32x2p{__builtin_bit_cast(uint32_t, lo), __builtin_bit_cast(uint32_t, hi)},
                                          rc, off, 0, 0);
  }
}

template <int KS, int NW, int S, int ACT>
__global__ __launch_bounds__(NW * 64, 2) void gemm_wsp_kernel(WsArgs a) {
  constexpr int K = KS * 16;
  constexpr int G = K / 8;
  constexpr int CHUNK = 32 * K * 2;
  constexpr int PIECES = CHUNK / 1024;
  constexpr int PW = PIECES / NW;
  static_assert(PW * NW == PIECES && G % 16 == 0 && KS % 8 == 0, "chunk vs block");
  constexpr int NST = 4;
  __shared__ __attribute__((aligned(16))) char sm[S * CHUNK];

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 31, h = lane >> 5;
  const int GB = gridDim.x, b = blockIdx.x;
  const int xq = GB / 8, xr = GB % 8, xb = b % 8;
  const int slot = xb * xq + min(xb, xr) + b / 8;
  const int grp = slot / a.slices, sl = slot - grp * a.slices;
  const int M = a.M, N = a.N;
  const int nchunks_all = (M + 31) / 32;
  const int c0 = grp * a.chunks_per;
  const int nch = max(0, min(a.chunks_per, nchunks_all - c0));
  if (nch == 0) return;
  const int n0 = sl * 32 * NW + 32 * w;
  const bool active = n0 < N;
  imgcap_epilogue ep = a.ep;
  const bool drop = ep.drop_p > 0.f;
  if (drop) ep.seed = eff_seed(ep.seed, a.seed_ctr);
  const long lda = a.lda;
  uint32_t voff[PW];
#pragma unroll
  for (int j = 0; j < PW; ++j) {
    const int p = (j * NW + w) * 64 + lane;
    const int rr = p / G, gs = p - rr * G;
    voff[j] = (uint32_t)(((long)rr * lda + 8 * (gs ^ (rr & 15))) * 2);
  }
#define WSP_ISSUE(c_) ws_issue<PW, NW>(a.A, lda, M, (long)(c0 + (c_)) * 32, sm + ((c_) % S) * CHUNK, w, voff)
#pragma unroll
  for (int c = 0; c < S - 1; ++c)
    if (c < nch) WSP_ISSUE(c);
  bf16x8 wf[KS];
  {
    const ws_rsrc_t rb = ws_rsrc(a.B, a.b_bytes);
    const int n = n0 + r;
    const uint32_t base = n < N ? (uint32_t)(((long)n * a.ldb + 8 * h) * 2) : 0x80000000u;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      wf[ks] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rb, base + 32 * ks, 0, 0));
  }
  float bias[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int n = n0 + 8 * (i >> 2) + 4 * h + (i & 3);
    bias[i] = (ep.bias && n < N) ? ep.bias[n] : 0.f;
  }
  // per-lane byte offsets of the fragment of k-step ks (mod 8) inside a chunk image; k-step ks
  // reads offset[ks % 8] + 256 * (ks / 8)
  uint32_t foff[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) foff[q] = r * (K * 2) + (((2 * q + h) ^ (r & 15)) << 4);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  const ws_rsrc_t rc = ws_rsrc(a.C, (int64_t)a.c_bytes);

  // one iteration: chunk c into `cur`, the epilogue of chunk c-1 from `prev` (a macro, not a
  // lambda: device builtins inside a lambda of the kernel body lose the host stub, see above).
  // The two halves of the block run the two parts in opposite orders (the first half MFMAs then
  // epilogue, the second half epilogue then MFMAs): a SIMD's two waves (w and w + NW/2 under the
  // cyclic wave placement) then pair one wave's MFMAs with the other's epilogue VALU instead of
  // both doing the same thing between two barriers.
  const bool late = w >= NW / 2;
#define WSP_BODY(c_, cur, prev)                                                                        \
  do {                                                                                                 \
    const int cc = (c_);                                                                               \
    if (cc >= S - 1) {                                                                                 \
      /* younger than chunk cc's pieces: the stores of iterations cc-S+1 .. cc-1 (iteration 0 has   \
         none) and the pieces of the chunks issued after it */                                         \
      const int st_it = (S - 1) - (cc - S + 1 == 0 ? 1 : 0);                                           \
      ws_vmwait((active ? NST : 0) * st_it + PW * min(S - 2, nch - 1 - cc));                           \
    }                                                                                                  \
    __builtin_amdgcn_s_barrier();                                                                      \
    if (cc + S - 1 < nch) WSP_ISSUE(cc + S - 1);                                                       \
    if (active) {                                                                                      \
      const char* st = sm + (cc % S) * CHUNK;                                                          \
      if (late && cc > 0) ws_epi<ACT>(prev, bias, ep, drop, (c0 + cc - 1) * 32 + r, M, N, n0, h, a.ldc, rc); \
      cur = ws_f32x16{};                                                                               \
      _Pragma("unroll") for (int ks = 0; ks < KS; ++ks) {                                              \
        const bf16x8 xf = *(const bf16x8*)(st + foff[ks & 7] + 256 * (ks >> 3));                      \
        cur = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[ks], xf, cur, 0, 0, 0);                       \
      }                                                                                                \
      if (!late && cc > 0) ws_epi<ACT>(prev, bias, ep, drop, (c0 + cc - 1) * 32 + r, M, N, n0, h, a.ldc, rc); \
    }                                                                                                  \
  } while (0)
  ws_f32x16 acc0 = {}, acc1 = {};
  int c = 0;
  for (; c + 1 < nch; c += 2) {
    WSP_BODY(c, acc0, acc1);
    WSP_BODY(c + 1, acc1, acc0);
  }
  if (c < nch) {
    WSP_BODY(c, acc0, acc1);
    if (active) ws_epi<ACT>(acc0, bias, ep, drop, (c0 + c) * 32 + r, M, N, n0, h, a.ldc, rc);
  } else if (active) {
    ws_epi<ACT>(acc1, bias, ep, drop, (c0 + c - 1) * 32 + r, M, N, n0, h, a.ldc, rc);
  }
#undef WSP_BODY
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#undef WSP_ISSUE
}

#endif  // IMGCAP_STAMPS

// explicit instantiations of the launched forms (ACT 0 / 1 / 2 = IMGCAP_ACT_NONE / GELU / RELU).
// (A device builtin called inside a lambda of the kernel body is an error in the host-side pass,
// which clang reports only as a "substitution failure" of the kernel template -- or, without these
// instantiations, not at all: no host stub, an undefined symbol at load time; hence ws_issue and
// the WSP_BODY macro.)
#define WS_I3(KS_, NW_, S_, STG_)                                      \
  template __global__ void gemm_ws_kernel<KS_, NW_, S_, 0, STG_>(WsArgs); \
  template __global__ void gemm_ws_kernel<KS_, NW_, S_, 1, STG_>(WsArgs); \
  template __global__ void gemm_ws_kernel<KS_, NW_, S_, 2, STG_>(WsArgs);
WS_I3(24, 8, 3, false)
WS_I3(24, 4, 3, false)
WS_I3(32, 8, 3, false)
WS_I3(32, 4, 2, false)
#ifdef IMGCAP_STAMPS  // deeper rings (IMGCAP_WS_DEEP): within 2 %, diagnostic build only
WS_I3(24, 8, 6, false)
WS_I3(32, 8, 4, false)
#endif
WS_I3(24, 8, 5, true)
WS_I3(24, 4, 2, true)
WS_I3(32, 8, 4, true)
WS_I3(32, 4, 2, true)
#undef WS_I3
#ifdef IMGCAP_STAMPS
#define WSP_I3(KS_, NW_, S_)                                        \
  template __global__ void gemm_wsp_kernel<KS_, NW_, S_, 0>(WsArgs); \
  template __global__ void gemm_wsp_kernel<KS_, NW_, S_, 1>(WsArgs); \
  template __global__ void gemm_wsp_kernel<KS_, NW_, S_, 2>(WsArgs);
WSP_I3(24, 8, 4)
WSP_I3(24, 4, 3)
WSP_I3(32, 8, 3)
WSP_I3(32, 4, 2)
#undef WSP_I3
#endif

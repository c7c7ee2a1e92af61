// Tiled MFMA GEMM (M > 64) — included by gemm.hip.
//
// 256 threads = 4 wave64s (2 x 2), BM x BN output tile, BK-deep k-tiles (32 or 64).
// LDS images per operand:
//   k-major operand ([rows][K] in memory): image [row][k] (row stride BK + 8), 16-byte stores,
//     fragments by one ds_read_b128 per 32-k step
//   m/n-major operand ([K][rows] in memory): image [k][row] (row stride ROWS + 8) filled with
//     the SAME 16-byte vector stores (no per-element transpose), fragments by two
//     ds_read_b64_tr_b16 hardware-transposed reads (bf16; f32 falls back to scalar writes)
// Staging is register-based and branch-free (clamped addresses + zero select); the next
// k-tile's global loads are in flight under the current tile's MFMAs.  The block index is
// remapped so that the 8 blocks dealt round-robin to one XCD work on neighbouring M tiles
// (shared B panel, L2 reuse).

template <typename T, int BM, int BN, int BK, bool AK, bool BKM>
struct GemmCfg {
  static constexpr int VEC = 16 / sizeof(T);
  static constexpr bool TR = sizeof(T) == 2;  // hardware transposed reads available (16-bit)
  static constexpr int LDK = BK + VEC;        // k-major image row stride
  static constexpr int LDA_T = BM + VEC;      // [k][m] image row stride
  static constexpr int LDB_T = BN + VEC;
  static constexpr int A_ELEMS = AK ? BM * LDK : (TR ? BK * LDA_T : BM * LDK);
  static constexpr int B_ELEMS = BKM ? BN * LDK : (TR ? BK * LDB_T : BN * LDK);
  static constexpr int TM = BM / 2 / 16;
  static constexpr int TN = BN / 2 / 16;
  static constexpr int A_VECS = BM * BK / VEC / 256;
  static constexpr int B_VECS = BN * BK / VEC / 256;
  static constexpr int STAGE_BYTES = (A_ELEMS + B_ELEMS) * (int)sizeof(T);
  static constexpr int EPI_ROWS = BM / 2;
  static constexpr int LDT = BN + 4;
  static constexpr int EPI_BYTES = EPI_ROWS * LDT * 4;
  static constexpr int SMEM = STAGE_BYTES > EPI_BYTES ? STAGE_BYTES : EPI_BYTES;
  static_assert(A_VECS >= 1 && B_VECS >= 1, "tile too small for 256 threads");
};

// Load one operand tile (ROWS x BK) into registers.  KMAJ: element (r,k) at P[r*ld + k].
template <typename T, int ROWS, int BK, int NV, bool KMAJ>
DEV void tile_load(uint4 (&reg)[NV], const T* __restrict__ P, long ld, int r0, int k0, int R, int K) {
  constexpr int VEC = 16 / sizeof(T);
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int v = tid + i * 256;
    int r, k;
    if (KMAJ) { r = v / (BK / VEC); k = (v % (BK / VEC)) * VEC; }
    else      { k = v / (ROWS / VEC); r = (v % (ROWS / VEC)) * VEC; }
    const int gr = r0 + r, gk = k0 + k;
    const int cr = gr < R ? gr : R - 1;  // clamped (always-valid) address
    const int ck = gk < K ? gk : K - 1;
    const uint4 x = KMAJ ? *(const uint4*)(P + (long)cr * ld + (ck / VEC) * VEC)
                         : *(const uint4*)(P + (long)ck * ld + (cr / VEC) * VEC);
    const bool ok = gr < R && gk < K;
    reg[i] = ok ? x : make_uint4(0u, 0u, 0u, 0u);
    if (KMAJ && gk + VEC > K) reg[i] = mask_tail<T>(reg[i], K - gk);
  }
}

// Store the registers into the LDS image (see header for the two image kinds).
template <typename T, int ROWS, int BK, int NV, bool KMAJ, int LDK, int LDT_>
DEV void tile_store(T* S, const uint4 (&reg)[NV]) {
  constexpr int VEC = 16 / sizeof(T);
  constexpr bool TR = sizeof(T) == 2;
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int v = tid + i * 256;
    if (KMAJ) {
      const int r = v / (BK / VEC), k = (v % (BK / VEC)) * VEC;
      *(uint4*)(S + r * LDK + k) = reg[i];
    } else if (TR) {
      const int k = v / (ROWS / VEC), r = (v % (ROWS / VEC)) * VEC;
      *(uint4*)(S + k * LDT_ + r) = reg[i];
    } else {  // f32, m/n-major: transpose element-wise into a [row][k] image
      const int k = v / (ROWS / VEC), r = (v % (ROWS / VEC)) * VEC;
      const uint32_t w[4] = {reg[i].x, reg[i].y, reg[i].z, reg[i].w};
      uint32_t* s32 = (uint32_t*)S;
#pragma unroll
      for (int j = 0; j < 4; ++j) s32[(r + j) * LDK + k] = w[j];
    }
  }
}

typedef short v4s16 __attribute__((ext_vector_type(4)));

// 8-k fragment of row `row` (k = kk + 8*(lane>>4) + 0..7) from an image
template <typename T, bool KMAJ, int LDK, int LDT_>
DEV Frag<T> img_frag(const T* S, int row0, int kk, int lane) {
  if constexpr (KMAJ || sizeof(T) == 4) {
    return lds_frag<T>(S + (row0 + (lane & 15)) * LDK + kk + 8 * (lane >> 4));
  } else {
    // ds_read_b64_tr_b16: lane 4q+p of a 16-lane group addresses row (k) q, columns 4p..4p+3;
    // lane i receives column i of the 4 rows.  Two reads give k = 8g..8g+3 and 8g+4..8g+7.
    const int i16 = lane & 15, q = i16 >> 2, p = i16 & 3, g = lane >> 4;
    const T* base = S + (kk + 8 * g + q) * LDT_ + row0 + 4 * p;
    typedef __attribute__((address_space(3))) v4s16 lds_v4s16;
    const v4s16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s16*)(base));
    const v4s16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s16*)(base + 4 * LDT_));
    Frag<T> f;
    typedef short v8s16 __attribute__((ext_vector_type(8)));
    const v8s16 all = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    f = __builtin_bit_cast(Frag<T>, all);
    return f;
  }
}

// XCD-aware remap of a 2-D grid (x = N tiles fastest): consecutive linear block ids are dealt
// round-robin over the 8 XCDs, so give each XCD a contiguous run of tiles (bijective form of
// cdna_hip_programming.md §5 T1).  Only changes speed, never results.
DEV void xcd_remap(int& bx, int& by) {
  const int nx = gridDim.x, nwg = gridDim.x * gridDim.y;
  const int orig = blockIdx.y * nx + blockIdx.x;
  int id = orig;
  if (nwg >= 64) {
    const int xcd = orig % 8, q = nwg / 8, r = nwg % 8;
    id = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
  }
  bx = id % nx;
  by = id / nx;
}

template <typename T, int BM, int BN, int BK, bool AK, bool BKM>
__global__ __launch_bounds__(256) void gemm_kernel(const T* __restrict__ A, long lda, long sA,
                                                   const T* __restrict__ B, long ldb, long sB,
                                                   void* __restrict__ C, long ldc, long sC,
                                                   int M, int N, int K, imgcap_epilogue ep, int vec_ok,
                                                   const uint64_t* seed_ctr, int kslice) {
  using G = GemmCfg<T, BM, BN, BK, AK, BKM>;
  if (ep.drop_p > 0.f) ep.seed = eff_seed(ep.seed, seed_ctr);
  __shared__ __attribute__((aligned(16))) char smem[G::SMEM];
  T* As = (T*)smem;
  T* Bs = As + G::A_ELEMS;

  // grid.z = batch entries, or K slices (kslice > 0: slice z covers k in [z*kslice, +kslice)
  // and stores its partial tile into plane z of the fp32 workspace C = P[z][M][N])
  const int bz = kslice ? 0 : blockIdx.z;
  const int kt0 = kslice ? blockIdx.z * (kslice / BK) : 0;
  A += bz * sA;
  B += bz * sB;
  const long cbase = (long)bz * sC;
  int bx, by;
  xcd_remap(bx, by);
  const int m0 = by * BM, n0 = bx * BN;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int rb = wm * (BM / 2), cb = wn * (BN / 2);

  f32x4 acc[G::TM][G::TN];
#pragma unroll
  for (int i = 0; i < G::TM; ++i)
#pragma unroll
    for (int j = 0; j < G::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  uint4 ra[G::A_VECS], rbv[G::B_VECS];
  tile_load<T, BM, BK, G::A_VECS, AK>(ra, A, lda, m0, kt0 * BK, M, K);
  tile_load<T, BN, BK, G::B_VECS, BKM>(rbv, B, ldb, n0, kt0 * BK, N, K);
  tile_store<T, BM, BK, G::A_VECS, AK, G::LDK, G::LDA_T>(As, ra);
  tile_store<T, BN, BK, G::B_VECS, BKM, G::LDK, G::LDB_T>(Bs, rbv);
  __syncthreads();

  const int nk = kslice ? min((K + BK - 1) / BK, kt0 + kslice / BK) : (K + BK - 1) / BK;
  for (int kt = kt0; kt < nk; ++kt) {
    const bool more = kt + 1 < nk;
    if (more) {
      tile_load<T, BM, BK, G::A_VECS, AK>(ra, A, lda, m0, (kt + 1) * BK, M, K);
      tile_load<T, BN, BK, G::B_VECS, BKM>(rbv, B, ldb, n0, (kt + 1) * BK, N, K);
    }
#pragma unroll
    for (int kk = 0; kk < BK; kk += 32) {
      Frag<T> af[G::TM], bfr[G::TN];
#pragma unroll
      for (int i = 0; i < G::TM; ++i) af[i] = img_frag<T, AK, G::LDK, G::LDA_T>(As, rb + i * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < G::TN; ++j) bfr[j] = img_frag<T, BKM, G::LDK, G::LDB_T>(Bs, cb + j * 16, kk, lane);
#pragma unroll
      for (int i = 0; i < G::TM; ++i)
#pragma unroll
        for (int j = 0; j < G::TN; ++j) mma(acc[i][j], af[i], bfr[j]);
    }
    __syncthreads();
    if (more) {
      tile_store<T, BM, BK, G::A_VECS, AK, G::LDK, G::LDA_T>(As, ra);
      tile_store<T, BN, BK, G::B_VECS, BKM, G::LDK, G::LDB_T>(Bs, rbv);
      __syncthreads();
    }
  }

  // epilogue: two passes of BM/2 rows (one wave-row each) through LDS
  float* tile = (float*)smem;
  const int fr = lane & 15;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    if (wm == pass) {
#pragma unroll
      for (int i = 0; i < G::TM; ++i)
#pragma unroll
        for (int j = 0; j < G::TN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            tile[(i * 16 + 4 * (lane >> 4) + r) * G::LDT + cb + j * 16 + fr] = acc[i][j][r];
    }
    __syncthreads();
    if (kslice)
      partial_from_lds<BN>(tile, G::LDT, G::EPI_ROWS, m0 + pass * G::EPI_ROWS, n0, M, N,
                           (float*)C + (long)blockIdx.z * M * N);
    else
      epilogue_from_lds<BN>(ep, tile, G::LDT, G::EPI_ROWS, m0 + pass * G::EPI_ROWS, n0, M, N, C, ldc, cbase,
                            vec_ok != 0);
    __syncthreads();
  }
}

template <typename T, int BM, int BN, int BK>
static int launch_tiled(int ak, int bk, int M, int N, int K, const void* A, long lda, long sA, const void* B,
                        long ldb, long sB, void* C, long ldc, long sC, int batch, const imgcap_epilogue& ep,
                        int vec_ok, hipStream_t st, int split = 1) {
  // split > 1 (batch == 1): K cut into `split` BK-aligned slices, one grid.z layer each, whose
  // partial products go to workspace planes; splitk_reduce_kernel then finishes C
  const int kslice = split > 1 ? ((K + split - 1) / split + BK - 1) / BK * BK : 0;
  const int zdim = split > 1 ? (K + kslice - 1) / kslice : batch;
  void* Cout = C;
  if (split > 1) {
    C = workspace((size_t)zdim * M * N * sizeof(float), st);
    if (!C) return fail(IMGCAP_EWORKSPACE, std::string("imgcap_gemm: split-K ") + last_error());
  }
  dim3 grid((N + BN - 1) / BN, (M + BM - 1) / BM, zdim);
  const T* a = (const T*)A;
  const T* b = (const T*)B;
#define L_(AKV, BKV)                                                                                             \
  hipLaunchKernelGGL((gemm_kernel<T, BM, BN, BK, AKV, BKV>), grid, dim3(256), 0, st, a, lda, sA, b, ldb, sB, C, ldc, \
                     sC, M, N, K, ep, vec_ok, g_seed_ctr, kslice)
  if (ak && bk) L_(true, true);
  else if (ak && !bk) L_(true, false);
  else if (!ak && bk) L_(false, true);
  else L_(false, false);
#undef L_
  if (split > 1) {
    const long total = (long)M * N;
    const int blocks = (int)std::min<long>((total + 255) / 256, 2048);
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3(blocks), dim3(256), 0, st, M, N, zdim, (const float*)C, Cout, ldc,
                       ep, g_seed_ctr);
  }
  IMGCAP_CHECK_LAUNCH("imgcap_gemm");
  return 0;
}

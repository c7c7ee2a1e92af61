// Row-complete GEMM + post-norm residual LayerNorm, forward and backward -- included by gemm.hip
// after gemm_pt.h (PtSrc LDS-DMA sources, glds_frag_op fragment reads).
//
// nn.TransformerDecoderLayer's post-norm blocks (transformerDecoder.py:82,104, norm_first=False)
// end every sub-layer with x' = LN(x + dropout(y)), y the sub-layer's last Linear.  A 512-wide
// (d_model) output row fits one block: 32 rows x 512 columns, 4 waves of 32 x 128, the weight
// streamed through LDS 64 k at a time.  The LayerNorm then runs on the accumulators -- row
// statistics by lane shuffles + one LDS exchange between the 4 waves -- instead of a separate
// add_ln launch that re-reads y from HBM (forward), and the LayerNorm backward runs on the
// accumulators of the product that produces its incoming gradient (dx = dZ W (+ the residual
// gradient already accumulated)), writing dS, the sub-layer's dropout-masked dY and per-block
// dgamma / dbeta partials for the deferred column sums.
//
// Arithmetic matches the unfused path element for element: y rounded to bf16, s = bf16(x +
// y * mask), the statistics over the stored bf16 s (what the backward recomputes from), mask
// index row * 512 + column on the same dropout stream.

constexpr int RL_BM = 32, RL_BN = 512, RL_S = 2;

struct RowLnArgs {
  const bf16* A;
  const bf16* B;
  long lda, ldb;
  int M, K;
  int64_t a_bytes, b_bytes;
  // forward: y = A B^T + bias; s = x + dropout(y); out = LN(s) * gamma + beta
  const float* bias;
  const bf16* x;
  long ldx;
  const float* gamma;
  const float* beta;
  float eps;
  // backward: dx = A B (+ res); dS = LN_bwd(dx; s, mean, rstd, gamma); dr = dS * mask
  const bf16* res;
  long ldr;
  const bf16* s;
  long lds;
  const float* mean_in;
  const float* rstd_in;
  float* part;  // [gridDim.x][2][512]: sum over the block's rows of dx * xhat, dx
  // dropout of the residual branch
  float drop_p;
  uint64_t seed;
  const uint64_t* seed_ctr;
  uint32_t drop_stream;
  // outputs: forward out0 = s, out1 = LN(s); backward out0 = dS, out1 = dr (may be null)
  bf16* out0;
  bf16* out1;
  long ldo;
  float* mean_out;
  float* rstd_out;
};

DEV void rl_ld4(const bf16* p, float (&v)[4]) {
  const uint2 u = *(const uint2*)p;
  v[0] = pt_bf_lo(u.x);
  v[1] = pt_bf_hi(u.x);
  v[2] = pt_bf_lo(u.y);
  v[3] = pt_bf_hi(u.y);
}
DEV void rl_st4(bf16* p, const float (&v)[4]) {
  *(uint2*)p = make_uint2(pt_pack(v[0], v[1]), pt_pack(v[2], v[3]));
}
DEV float rl_bfr(float x) { return (float)(bf16)x; }

// MODE 0: forward (B = the Linear weight [512, K], k-major); MODE 1: backward (B [K, 512] row-major)
template <int MODE>
__global__ __launch_bounds__(256, 1) void gemm_rowln_kernel(RowLnArgs a) {
  constexpr bool BKM = MODE == 0;
  constexpr int NW = 4, TA = RL_BM * 128, TB = RL_BN * 128, STAGE = TA + TB;
  constexpr int FM = RL_BM / 16, FN = RL_BN / NW / 16;
  using SrcA = PtSrc<RL_BM, true, NW>;
  using SrcB = PtSrc<RL_BN, BKM, NW>;
  constexpr int LPT = SrcA::PER + SrcB::PER;  // DMA pieces per thread per k-step
  __shared__ __attribute__((aligned(16))) char smem[RL_S * STAGE];
  __shared__ float red[2][NW][RL_BM];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int m0 = blockIdx.x * RL_BM, cb = w * (RL_BN / NW);
  const int nk = a.K / 64;
  SrcA srcA;
  SrcB srcB;
  srcA.set(a.lda, m0, a.M, w, lane);
  srcB.set(a.ldb, 0, RL_BN, w, lane);
  auto issue = [&](int g, char* st) {
    const long offA = (long)g * 128;
    const long offB = BKM ? (long)g * 128 : (long)g * 64 * a.ldb * 2;
    const pt_rsrc_t ra = pt_rsrc((const char*)a.A + offA, a.a_bytes - offA);
    const pt_rsrc_t rb = pt_rsrc((const char*)a.B + offB, a.b_bytes - offB);
#pragma unroll
    for (int q = 0; q < SrcA::PER; ++q) srcA.issue(q, ra, st, w);
#pragma unroll
    for (int q = 0; q < SrcB::PER; ++q) srcB.issue(q, rb, st + TA, w);
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  issue(0, smem);
  if (nk > 1) issue(1, smem + STAGE);
  for (int g = 0; g < nk; ++g) {
    char* cur = smem + (g & 1) * STAGE;
    if (g + 1 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LPT) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    pt_lgkm0();
    __builtin_amdgcn_s_barrier();  // step g in LDS for every wave
    asm volatile("" ::: "memory");
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 fa[FM], fb[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) fa[i] = glds_frag_op<RL_BM, true>(cur, 16 * i, kk, lane);
#pragma unroll
      for (int j = 0; j < FN; ++j) fb[j] = glds_frag_op<RL_BN, BKM>(cur + TA, cb + 16 * j, kk, lane);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)  // D^T: a lane ends with 4 consecutive columns of one row
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
    }
    pt_lgkm0();
    __builtin_amdgcn_s_barrier();  // every wave is done reading the stage: refill it
    asm volatile("" ::: "memory");
    if (g + 2 < nk) issue(g + 2, cur);
  }

  // ---- epilogue: lane rows m0 + 16 i + fr, columns cb + 16 j + 4 fq + (0..3) ----
  const uint64_t seed = (a.drop_p > 0.f) ? eff_seed(a.seed, a.seed_ctr) : a.seed;
  const float inv_n = 1.f / RL_BN;
  int mrow[FM];
  bool valid[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int m = m0 + 16 * i + fr;
    valid[i] = m < a.M;
    mrow[i] = valid[i] ? m : a.M - 1;
  }
  // row sums of q[i] over the block's 512 columns: 4-lane shuffles, then the 4 waves via LDS
  auto row_sum2 = [&](float (&q0)[FM], float (&q1)[FM]) {
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      q0[i] += __shfl_xor(q0[i], 16, 64);
      q0[i] += __shfl_xor(q0[i], 32, 64);
      q1[i] += __shfl_xor(q1[i], 16, 64);
      q1[i] += __shfl_xor(q1[i], 32, 64);
      if (fq == 0) {
        red[0][w][16 * i + fr] = q0[i];
        red[1][w][16 * i + fr] = q1[i];
      }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int r = 16 * i + fr;
      q0[i] = ((red[0][0][r] + red[0][1][r]) + red[0][2][r]) + red[0][3][r];
      q1[i] = ((red[1][0][r] + red[1][1][r]) + red[1][2][r]) + red[1][3][r];
    }
    __syncthreads();
  };

  if constexpr (MODE == 0) {
    float sum[FM], dummy[FM];
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      sum[i] = 0.f;
      dummy[i] = 0.f;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = cb + 16 * j + 4 * fq;
        const f32x4 bias = *(const f32x4*)(a.bias + n);
        float xv[4];
        rl_ld4(a.x + (long)mrow[i] * a.ldx + n, xv);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float y = rl_bfr(acc[i][j][r] + bias[r]);
          const float sv = rl_bfr(xv[r] + y * dropout_scale(seed, a.drop_stream, (uint64_t)mrow[i] * RL_BN + n + r,
                                                             a.drop_p));
          acc[i][j][r] = sv;
          sum[i] += sv;
        }
      }
    }
    row_sum2(sum, dummy);
    float mean[FM], sq[FM];
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      mean[i] = sum[i] * inv_n;
      sq[i] = 0.f;
      dummy[i] = 0.f;
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float dv = acc[i][j][r] - mean[i];
          sq[i] += dv * dv;
        }
    }
    row_sum2(sq, dummy);
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const float rstd = rsqrtf(sq[i] * inv_n + a.eps);
      if (valid[i]) {
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int n = cb + 16 * j + 4 * fq;
          const f32x4 gm = *(const f32x4*)(a.gamma + n), bt = *(const f32x4*)(a.beta + n);
          float sv[4], o[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            sv[r] = acc[i][j][r];
            o[r] = (sv[r] - mean[i]) * rstd * gm[r] + bt[r];
          }
          const long off = (long)mrow[i] * a.ldo + n;
          rl_st4(a.out0 + off, sv);
          rl_st4(a.out1 + off, o);
        }
        if (w == 0 && fq == 0) {
          a.mean_out[mrow[i]] = mean[i];
          a.rstd_out[mrow[i]] = rstd;
        }
      }
    }
  } else {
    float s1[FM], s2[FM], mean[FM], rstd[FM];
    float xh[FM][FN][4];
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      mean[i] = a.mean_in[mrow[i]];
      rstd[i] = a.rstd_in[mrow[i]];
      s1[i] = 0.f;
      s2[i] = 0.f;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = cb + 16 * j + 4 * fq;
        const f32x4 gm = *(const f32x4*)(a.gamma + n);
        float sv[4], rv[4] = {0.f, 0.f, 0.f, 0.f};
        rl_ld4(a.s + (long)mrow[i] * a.lds + n, sv);
        if (a.res) rl_ld4(a.res + (long)mrow[i] * a.ldr + n, rv);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float dxv = acc[i][j][r] + rv[r];  // the incoming gradient dy of the LayerNorm
          acc[i][j][r] = dxv;
          xh[i][j][r] = (sv[r] - mean[i]) * rstd[i];
          const float gdy = dxv * gm[r];
          s1[i] += gdy;
          s2[i] += gdy * xh[i][j][r];
        }
      }
    }
    row_sum2(s1, s2);
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      s1[i] *= inv_n;
      s2[i] *= inv_n;
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = cb + 16 * j + 4 * fq;
      const f32x4 gm = *(const f32x4*)(a.gamma + n);
      float pg[4] = {0.f, 0.f, 0.f, 0.f}, pb[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        float d[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float dxv = acc[i][j][r];
          d[r] = rstd[i] * (dxv * gm[r] - s1[i] - xh[i][j][r] * s2[i]);
          if (valid[i]) {
            pg[r] += dxv * xh[i][j][r];
            pb[r] += dxv;
          }
        }
        if (valid[i]) {
          const long off = (long)mrow[i] * a.ldo + n;
          rl_st4(a.out0 + off, d);
          if (a.out1) {
#pragma unroll
            for (int r = 0; r < 4; ++r)
              d[r] *= dropout_scale(seed, a.drop_stream, (uint64_t)mrow[i] * RL_BN + n + r, a.drop_p);
            rl_st4(a.out1 + off, d);
          }
        }
      }
      // column partials over the block's rows: the 16 lanes of one fq hold the 16 row offsets
#pragma unroll
      for (int r = 0; r < 4; ++r) {
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          pg[r] += __shfl_xor(pg[r], o, 64);
          pb[r] += __shfl_xor(pb[r], o, 64);
        }
      }
      if (fr == 0) {
        float* p = a.part + (long)blockIdx.x * 2 * RL_BN + n;
        *(f32x4*)p = f32x4{pg[0], pg[1], pg[2], pg[3]};
        *(f32x4*)(p + RL_BN) = f32x4{pb[0], pb[1], pb[2], pb[3]};
      }
    }
  }
}

// explicit instantiations (host stubs of kernel templates first named inside a host function
// were left undefined in this library otherwise)
template __global__ void gemm_rowln_kernel<0>(RowLnArgs);
template __global__ void gemm_rowln_kernel<1>(RowLnArgs);

static int64_t rl_kmajor_bytes(int rows, int K, long ld) { return ((int64_t)(rows - 1) * ld + (K + 7) / 8 * 8) * 2; }

extern "C" int imgcap_gemm_add_ln_fwd(int M, int K, const void* A, int64_t lda, const void* W, int64_t ldw,
                                      const float* bias, const void* x, int64_t ldx, float drop_p, uint64_t seed,
                                      uint32_t drop_stream, const float* gamma, const float* beta, float eps,
                                      void* s_out, void* y, int64_t ldo, float* mean, float* rstd, void* stream) {
  IMGCAP_REQUIRE(M >= 0 && K > 0 && K % 64 == 0, "imgcap_gemm_add_ln_fwd: K must be a positive multiple of 64");
  IMGCAP_REQUIRE(A && W && bias && x && gamma && beta && s_out && y && mean && rstd, "imgcap_gemm_add_ln_fwd: null");
  IMGCAP_REQUIRE(lda % 8 == 0 && ldw % 8 == 0 && ldx % 8 == 0 && ldo % 8 == 0 && aligned16(A) && aligned16(W) &&
                     aligned16(bias) && aligned16(gamma) && aligned16(beta) && aligned16(x) && aligned16(s_out) &&
                     aligned16(y),
                 "imgcap_gemm_add_ln_fwd: operand alignment");
  if (M == 0) return 0;
  RowLnArgs a{};
  a.A = (const bf16*)A;
  a.B = (const bf16*)W;
  a.lda = lda;
  a.ldb = ldw;
  a.M = M;
  a.K = K;
  a.a_bytes = rl_kmajor_bytes(M, K, lda);
  a.b_bytes = rl_kmajor_bytes(RL_BN, K, ldw);
  IMGCAP_REQUIRE(a.a_bytes < 0x7fffffffLL && a.b_bytes < 0x7fffffffLL, "imgcap_gemm_add_ln_fwd: operand over 2 GiB");
  a.bias = bias;
  a.x = (const bf16*)x;
  a.ldx = ldx;
  a.gamma = gamma;
  a.beta = beta;
  a.eps = eps;
  a.drop_p = drop_p;
  a.seed = seed;
  a.seed_ctr = g_seed_ctr;
  a.drop_stream = drop_stream;
  a.out0 = (bf16*)s_out;
  a.out1 = (bf16*)y;
  a.ldo = ldo;
  a.mean_out = mean;
  a.rstd_out = rstd;
  hipLaunchKernelGGL(gemm_rowln_kernel<0>, dim3((M + RL_BM - 1) / RL_BM), dim3(256), 0, (hipStream_t)stream, a);
  IMGCAP_CHECK_LAUNCH("imgcap_gemm_add_ln_fwd");
  return 0;
}

extern "C" int imgcap_gemm_ln_bwd(int M, int K, const void* A, int64_t lda, const void* B, int64_t ldb,
                                  const void* res, int64_t ldr, const void* s, int64_t lds, const float* mean,
                                  const float* rstd, const float* gamma, float drop_p, uint64_t seed,
                                  uint32_t drop_stream, void* ds, void* dr, int64_t ldo, float* part, void* stream) {
  IMGCAP_REQUIRE(M >= 0 && K > 0 && K % 64 == 0, "imgcap_gemm_ln_bwd: K must be a positive multiple of 64");
  IMGCAP_REQUIRE(A && B && s && mean && rstd && gamma && ds && part, "imgcap_gemm_ln_bwd: null");
  IMGCAP_REQUIRE(lda % 8 == 0 && ldb % 8 == 0 && lds % 8 == 0 && ldr % 8 == 0 && ldo % 8 == 0 && aligned16(A) &&
                     aligned16(B) && aligned16(gamma) && aligned16(part) && aligned16(s) && aligned16(ds) &&
                     (!res || aligned16(res)) && (!dr || aligned16(dr)),
                 "imgcap_gemm_ln_bwd: operand alignment");
  if (M == 0) return 0;
  RowLnArgs a{};
  a.A = (const bf16*)A;
  a.B = (const bf16*)B;
  a.lda = lda;
  a.ldb = ldb;
  a.M = M;
  a.K = K;
  a.a_bytes = rl_kmajor_bytes(M, K, lda);
  a.b_bytes = ((int64_t)(K - 1) * ldb + RL_BN) * 2;
  IMGCAP_REQUIRE(a.a_bytes < 0x7fffffffLL && a.b_bytes < 0x7fffffffLL, "imgcap_gemm_ln_bwd: operand over 2 GiB");
  a.res = (const bf16*)res;
  a.ldr = ldr;
  a.s = (const bf16*)s;
  a.lds = lds;
  a.mean_in = mean;
  a.rstd_in = rstd;
  a.gamma = gamma;
  a.part = part;
  a.drop_p = drop_p;
  a.seed = seed;
  a.seed_ctr = g_seed_ctr;
  a.drop_stream = drop_stream;
  a.out0 = (bf16*)ds;
  a.out1 = (bf16*)dr;
  a.ldo = ldo;
  hipLaunchKernelGGL(gemm_rowln_kernel<1>, dim3((M + RL_BM - 1) / RL_BM), dim3(256), 0, (hipStream_t)stream, a);
  IMGCAP_CHECK_LAUNCH("imgcap_gemm_ln_bwd");
  return 0;
}

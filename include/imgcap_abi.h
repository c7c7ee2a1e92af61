/*
 * imgcap_abi.h — C ABI of libimgcap_hip.so, the MI355X (gfx950) kernels behind the
 * teacher-forced image-captioning train step of sa06840/ImageCaptioningConvNeXt.
 *
 * The reference has no native code and no FFI: its boundary is the PyTorch
 * nn.Module surface of models/encoder.py, models/decoder.py, models/transformerDecoder.py and
 * the train-step functions of train.py / trainMultiGPU.py.  Each entry point below replaces
 * the torch/cuDNN/cuBLAS/NCCL work reached from one reference line (cited per function).
 *
 * Conventions
 *   - Plain pointers to device memory + sizes; no torch types.  `stream` is a hipStream_t
 *     (passed as void*); every call only enqueues work on it (no allocation, no sync), so a
 *     caller may capture calls into a hipGraph.
 *   - `dtype`: IMGCAP_F32 or IMGCAP_BF16 = element type of the activation/weight operands.
 *     Accumulation is always fp32.  Optimizer state and master weights are fp32.
 *   - Return 0 on success, a hipError_t (>0) or IMGCAP_E* (<0) otherwise;
 *     imgcap_last_error_string() describes the last failure (thread-local).
 *   - The caller owns every buffer.  Ops with split reductions draw scratch from a per-device,
 *     per-slot workspace the caller attaches (imgcap_workspace_attach); a call whose scratch
 *     would not fit returns IMGCAP_EWORKSPACE before enqueuing anything, and
 *     imgcap_workspace_needed gives the size to attach before retrying it.  Only a (device,
 *     slot) the caller never attached makes the library allocate (grow-only, never freed: a
 *     captured graph may reference it).  Op-specific workspaces (the LSTM hand-off words) are
 *     passed in the op's arguments.
 */
#ifndef IMGCAP_ABI_H
#define IMGCAP_ABI_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

enum { IMGCAP_F32 = 0, IMGCAP_BF16 = 1 };
/* Block-scaled fp8 (OCP MX-FP8): e4m3fn bytes, one E8M0 scale byte (2^(s-127)) per 32
 * consecutive elements of a row.  Only as an imgcap_epilogue.c_dtype (imgcap_gemm_mx output)
 * and as the operands of imgcap_gemm_mx. */
enum { IMGCAP_FP8MX = 2 };
enum { IMGCAP_OK = 0, IMGCAP_EINVAL = -1, IMGCAP_EUNSUPPORTED = -2, IMGCAP_EWORKSPACE = -3 };
/* ACT_GELU with an aux operand also writes the pre-activation to aux (the saved input of the
 * backward pass); ACT_DGELU multiplies by GELU'(aux[m, n]) (aux = that saved pre-activation). */
enum { IMGCAP_ACT_NONE = 0, IMGCAP_ACT_GELU = 1, IMGCAP_ACT_RELU = 2, IMGCAP_ACT_DGELU = 3 };

const char* imgcap_last_error_string(void);
/* Split-reduction scratch slot (0 default, 1, 2) of the calling thread: calls whose kernels may
 * run concurrently with slot-0 work on another stream use another slot (the trainer's encoder
 * pipeline 1, the decoder engines' side streams 2).  Inside one captured graph the library
 * refuses a slot's scratch to a second stream (the call fails, nothing is enqueued). */
int imgcap_workspace_slot(int slot);
/* Attach the caller's device buffer (256-byte aligned; NULL detaches) as the split-reduction
 * scratch of `slot` on the current device. */
int imgcap_workspace_attach(int slot, void* ptr, uint64_t bytes);
/* Largest scratch request seen so far in `slot` on the current device (what to attach). */
int imgcap_workspace_needed(int slot, uint64_t* bytes);
/* ABI revision of this header; imgcap_version() returns the library's.  Bumped whenever an
 * entry point changes meaning or arity (6: imgcap_add_layernorm_bwd's per-block partials
 * argument, imgcap_gemm_get_pt; bindings refuse a library of another revision). */
#define IMGCAP_ABI_VERSION 6
int imgcap_version(void);

/* Device-resident step counter mixed into every dropout / stochastic-depth seed at kernel
 * run time: mask = f(seed ^ g(*counter), stream, index).  Lets a captured HIP graph draw new
 * masks on each replay (the counter is bumped by a node inside the graph) while the seeds in
 * its kernel arguments stay fixed.  NULL (the default) = seeds used as given.  Process-wide;
 * read at launch-enqueue time, so set it before capturing. */
int imgcap_set_seed_counter(const uint64_t* counter);

/* ---------------------------------------------------------------------------------------
 * GEMM with fused epilogue (MFMA: bf16 16x16x32 / f32 16x16x4).
 *   acc[m,n] = sum_k A(m,k) * B(k,n)
 *   A(m,k) = A[m*lda + k] if a_kmajor else A[k*lda + m]
 *   B(k,n) = B[n*ldb + k] if b_kmajor else B[k*ldb + n]      (b_kmajor = nn.Linear weight [N][K])
 *   v = alpha*acc (+bias[n]) -> act -> dropout(p; seed,stream, index m*drop_ld+n)
 *       -> (*= aux[m,n] > 0 ? aux_scale : 0; or *= GELU'(aux[m,n]) for ACT_DGELU)
 *       -> (*= colscale[n]) -> (*= rowscale[m/rows_per_scale])
 *       -> (+= res[m,n]) -> (+= beta*C[m,n]) -> C[m,n] (c_dtype)
 * Replaces every nn.Linear / 1x1-conv / patchify-conv / projection matmul on the path:
 * decoder.py:26-27,65-66,104-109; transformerDecoder.py:95,104,106; torchvision CNBlock
 * Linear pair + layer_scale + residual (reached via encoder.py:24); and their backward.
 * -------------------------------------------------------------------------------------- */
typedef struct imgcap_epilogue {
  const float* bias;       /* [N] or NULL */
  const float* colscale;   /* [N] or NULL (ConvNeXt layer_scale) */
  const float* rowscale;   /* [M/rows_per_scale] or NULL (stochastic depth, per sample) */
  const void* res;         /* residual [M, ldr] of c_dtype, or NULL */
  const void* aux;         /* relu/dropout mask source [M, ldaux] of c_dtype, or NULL */
  int64_t ldr;
  int64_t ldaux;
  int64_t drop_ld;
  uint64_t seed;
  float alpha;
  float beta;
  float drop_p;
  float aux_scale;
  int32_t act;
  int32_t c_dtype;
  int32_t rows_per_scale;
  uint32_t drop_stream;
  int32_t split_k;         /* 0/1: off.  n > 1: K split n ways, -1: library picks n.  Only for
                              fp32 C = alpha*A.B + beta*C (no other epilogue, batch 1): slices
                              write fp32 partials to library scratch, a second kernel adds them
                              in fixed order (deterministic) */
  uint8_t* c_scale;        /* c_dtype IMGCAP_FP8MX: the E8M0 block scales of C, [M][ldc / 32] */
} imgcap_epilogue;

int imgcap_gemm(int dtype, int a_kmajor, int b_kmajor, int M, int N, int K,
                const void* A, int64_t lda, int64_t strideA,
                const void* B, int64_t ldb, int64_t strideB,
                void* C, int64_t ldc, int64_t strideC, int batch,
                const imgcap_epilogue* epi, void* stream);

/* Grouped product launch: C_i = alpha_i * op(A_i) op(B_i) + beta_i * C_i, fp32 C, bf16 operands,
 * one operand layout for all problems (a_kmajor / b_kmajor as imgcap_gemm), <= 48 problems.  The
 * weight gradients of a backward pass (dW = dY^T X, K = rows) in one grid of 128x128 tiles. */
typedef struct imgcap_gemm_problem {
  const void* A;
  const void* B;
  float* C;
  int64_t lda, ldb, ldc;
  int32_t M, N, K;
  float alpha, beta;
} imgcap_gemm_problem;
int imgcap_gemm_grouped(int a_kmajor, int b_kmajor, int n, const imgcap_gemm_problem* probs, void* stream);

/* Block-scaled fp8 GEMM (v_mfma_scale_f32_16x16x128_f8f6f4): C = epilogue(A . B^T) with
 * A [M][K] e4m3fn bytes (row pitch lda bytes) and its E8M0 scales As [M][K/32], B [N][K]
 * (nn.Linear weight layout, pitch ldb) and Bs [N][K/32]; K % 128 == 0, pitches % 16 == 0.
 * The epilogue is imgcap_gemm's (bias, act, colscale, rowscale, res; no dropout, aux, beta or
 * split-K) with c_dtype IMGCAP_BF16 / IMGCAP_F32, or IMGCAP_FP8MX (N % 32 == 0): C then gets
 * e4m3fn bytes and ep->c_scale the block scales -- the next product's A operand.  The frozen
 * ConvNeXt pointwise Linears of config C5 ("frozen stages in fp8"). */
int imgcap_gemm_mx(int M, int N, int K, const void* A, int64_t lda, const uint8_t* As, const void* B,
                   int64_t ldb, const uint8_t* Bs, void* C, int64_t ldc, const imgcap_epilogue* epi,
                   void* stream);
/* Rows of x [R][K] (dtype, pitch ldx elements), optionally LayerNorm'd first (ln_w/ln_b not
 * NULL: y = LN(x)*ln_w + ln_b, eps), to MX-FP8: q [R][K] bytes, s [R][K/32]; K % 32 == 0.
 * Per block of 32: e = floor(log2(amax)) - 8, s = e + 127, q = e4m3(clamp(v * 2^-e, +-448)). */
int imgcap_mx_quant_rows(int dtype, int R, int K, const void* x, int64_t ldx, const float* ln_w,
                         const float* ln_b, float eps, uint8_t* q, uint8_t* s, void* stream);

/* out[c, r] = in[r, c]  (weight transposes for the k-major skinny GEMMs) */
/* Which kernel imgcap_gemm launches for these operands (diagnostics and the bench's roofline):
 * returns one of IMGCAP_GEMM_*; *splits (if not NULL) = K slices (1 = none). */
enum { IMGCAP_GEMM_SKINNY = 1, IMGCAP_GEMM_TILED64 = 2, IMGCAP_GEMM_TILED128 = 3, IMGCAP_GEMM_GLDS = 4,
       IMGCAP_GEMM_GLDS256 = 5, IMGCAP_GEMM_GLDS64 = 6, IMGCAP_GEMM_GLDS128X64 = 7,
       /* stream-tile kernel (persistent, epilogue from registers, bf16 C): 256x128, 128x256, 128x128,
        * 128x192 tiles of 8 waves; 128x128 of 4 waves, two blocks a CU; 128x128 of 8 waves with
        * 128-deep k-steps */
       IMGCAP_GEMM_PT = 8, IMGCAP_GEMM_PT128X256 = 9, IMGCAP_GEMM_PT128 = 10, IMGCAP_GEMM_PT128X192 = 11,
       IMGCAP_GEMM_PT128X2 = 12, IMGCAP_GEMM_PT128K = 13, IMGCAP_GEMM_WS = 14, IMGCAP_GEMM_WS4 = 15 };
int imgcap_gemm_plan(int dtype, int a_kmajor, int b_kmajor, int M, int N, int K, int64_t lda, int64_t ldb,
                     int batch, int split_k, int* splits);
/* The same, knowing the call's epilogue (the persistent-tile kernel serves bf16 outputs only). */
int imgcap_gemm_plan_ep(int dtype, int a_kmajor, int b_kmajor, int M, int N, int K, int64_t lda, int64_t ldb,
                        int batch, const imgcap_epilogue* epi, int* splits);
/* Stream-tile GEMM policy: -1 by shape (the library default: the encoder's large forward pointwise
 * products, where a step census measured it ahead of the LDS-staged tiles), 0 never, 1 wherever
 * eligible (tile by the cost model), 2..7 wherever eligible with config 1..6 (IMGCAP_GEMM_PT ..
 * IMGCAP_GEMM_PT128K; a config not built for the call's epilogue form or K falls back to the cost
 * model).  Configs 1 / 2 (modes 2 / 3: 256x128, 128x256) exist in the diagnostic build only; the
 * product library returns IMGCAP_EUNSUPPORTED for those modes. */
int imgcap_gemm_set_pt(int mode);
/* The current stream-tile policy (what imgcap_gemm_set_pt last set; -1 unless changed). */
int imgcap_gemm_get_pt(void);
/* Weight-stationary short-K kernel (K = 384 / 512, A and B k-major, bf16 C; epilogue: alpha,
 * bias, GELU / ReLU, dropout, column scale): -1 by shape (default), 0 never, 1 wherever eligible
 * with 8-wave blocks (IMGCAP_GEMM_WS), 2 with 4-wave blocks (IMGCAP_GEMM_WS4); checked before
 * the stream-tile policy. */
int imgcap_gemm_set_ws(int mode);
int imgcap_gemm_get_ws(void);
/* Kernel-selection policy for A/B tests and benchmarks: glds256 >= 1 serves every eligible
 * GEMM (bf16, unsplit, 16-byte operand pitches) with the 256x256 tile (1: 64-deep k-steps x 2
 * stages, 2: 32-deep x 4 stages, 3: 32-deep x 3 stages), 0 never, 4 = the 128x128 LDS-DMA tile
 * wherever eligible, 5 = register-staged tiles only, -1 by shape (default); 6 = the 64x64
 * LDS-DMA tile wherever eligible and unsplit; 7 / 8 = by shape, but grids under 128 128x128
 * tiles on the 128x64 LDS-DMA tile (diagnostic build only: IMGCAP_EUNSUPPORTED in the product
 * library) / the register-staged 64x64 tile.
 * Process-wide; set before capturing graphs. */
int imgcap_gemm_set_policy(int glds256);
int imgcap_transpose(int dtype, int rows, int cols, const void* in, int64_t ldi, void* out, int64_t ldo,
                     void* stream);

/* Many column sums in one launch: out_i = beta_i*out_i + colsum(x_i)  (the bias gradients of a
 * whole backward pass, deferred to its end; <= 48 items per call; vec_ok is set by the library;
 * deterministic fixed-order sums; no library scratch) */
typedef struct imgcap_colsum_item {
  const void* x;      /* [rows, ld] of dtype */
  float* out;         /* [cols] fp32 */
  int64_t ld;
  int32_t rows, cols, dtype, vec_ok;
  float beta;
} imgcap_colsum_item;
int imgcap_colsum_multi(int n, const imgcap_colsum_item* items, void* stream);
/* The same in two launches with caller-owned fp32 scratch part[sum_i ceil(rows_i / 256) * cols_i]:
 * per-(256-row chunk, 64 columns) partial sums, then each column's chunk partials added in order
 * -- deterministic, the same sums in a different association than imgcap_colsum_multi. */
int imgcap_colsum_multi_part(int n, const imgcap_colsum_item* items, float* part, int64_t part_floats,
                             void* stream);

/* column sums of a [rows, cols] matrix into fp32 out[cols] (bias gradients); beta=1 accumulates */
int imgcap_colsum(int dtype, int rows, int cols, const void* x, int64_t ldx, float* out, float beta,
                  void* stream);

/* ---------------------------------------------------------------------------------------
 * LayerNorm over the last dim, optionally of a sum:  s = x + dropout(r);  y = LN(s)*g + b.
 * Replaces nn.TransformerDecoderLayer's post-norm residual blocks (norm_first=False,
 * transformerDecoder.py:82,104) incl. the sublayer dropout.  Saves s, mean, rstd for bwd.
 * -------------------------------------------------------------------------------------- */
int imgcap_add_layernorm_fwd(int dtype, int rows, int cols, const void* x, const void* r,
                             float drop_p, uint64_t seed, uint32_t drop_stream,
                             const float* gamma, const float* beta, float eps,
                             void* s_out, void* y, float* mean, float* rstd, void* stream);
/* dS = LN backward of dy;  dx = dS;  dr = dS * dropmask  (dr may be NULL);
 * dgamma/dbeta accumulated (+=) in fp32 -- or, with part != NULL (and dgamma = dbeta = NULL),
 * the per-block partial sums are written to part[nblk][2][cols] (nblk =
 * imgcap_add_layernorm_bwd_blocks(rows); [b][0] of dy * xhat, [b][1] of dy) for the caller's
 * deferred column sums (dgamma = colsum(part[:, 0]), dbeta = colsum(part[:, 1]):
 * imgcap_colsum_multi). */
int imgcap_add_layernorm_bwd(int dtype, int rows, int cols, const void* dy, const void* s,
                             const float* mean, const float* rstd, const float* gamma,
                             float drop_p, uint64_t seed, uint32_t drop_stream,
                             void* dx, void* dr, float* dgamma, float* dbeta, float* part, void* stream);
int imgcap_add_layernorm_bwd_blocks(int rows);

/* ---------------------------------------------------------------------------------------
 * ConvNeXt trunk (torchvision features reached via encoder.py:24), NHWC activations.
 * -------------------------------------------------------------------------------------- */
/* features[0]: Conv2d(3,C0,4,s4)+LayerNorm2d(eps 1e-6).  images: f32 NCHW [B,3,H,W];
 * w: f32 [C0][48] (ci,kh,kw order as torch); out: dtype NHWC [B,H/4,W/4,C0]. */
int imgcap_convnext_stem(int dtype, int B, int H, int W, int C0, const float* images,
                         const float* w, const float* bias, const float* ln_w, const float* ln_b,
                         void* out, void* stream);
/* Same, from the reference's raw images: uint8 [B,3,H,W] (the HDF5 'images' dataset,
 * dataLoader.py:43-46), normalised in the patch load exactly as the reference does on the host:
 * x = float(u / 255.), (x - mean3[c]) / std3[c] (train.py:152, ImageNet mean/std). */
int imgcap_convnext_stem_u8(int dtype, int B, int H, int W, int C0, const uint8_t* images, const float* mean3,
                            const float* std3, const float* w, const float* bias, const float* ln_w,
                            const float* ln_b, void* out, void* stream);
/* CNBlock head: depthwise 7x7 (pad 3, bias) + LayerNorm(C, eps 1e-6).  w: f32 [49][C]. */
/* Depthwise 7x7 conv + bias only, y [B,H,W,C] (the LayerNorm is applied by the consumer:
 * imgcap_cnblock_mlp's prologue or imgcap_add_layernorm_fwd).  C % 32 == 0, W <= 64.
 * w [49][C] (tap-major), fp32. */
int imgcap_dwconv7(int dtype, int B, int H, int W, int C, const void* x, const float* w, const float* bias,
                   void* y, void* stream);
int imgcap_dwconv7_ln(int dtype, int B, int H, int W, int C, const void* x, const float* w,
                      const float* bias, const float* ln_w, const float* ln_b, void* out,
                      void* stream);
/* features[2,4,6] head: LayerNorm2d(C) then gather 2x2/s2 patches into rows
 * out[B*(H/2)*(W/2)][4C] ordered (kh, kw, c) (weights repacked to match; cmajor = 0) or
 * (c, kh, kw) (cmajor = 1: the torch Conv2d weight [2C][C][2][2] is the GEMM operand as is). */
int imgcap_ln_patchify2(int dtype, int B, int H, int W, int C, const void* x, const float* ln_w,
                        const float* ln_b, int cmajor, void* out, void* stream);
/* AdaptiveAvgPool2d((OH,OW)) on NHWC (encoder.py:20,25) */
int imgcap_adaptive_pool_nhwc(int dtype, int B, int H, int W, int C, int OH, int OW,
                              const void* x, void* out, void* stream);
/* Fused ConvNeXt CNBlock MLP, bf16 (torchvision CNBlock via encoder.py:18):
 *   x[m, :] += gamma * sd[m / rows_per_sample] * (GELU(z[m, :] W1^T + b1) W2^T + b2)
 * z = LayerNorm(y; ln_w, ln_b, eps 1e-6) of the dwconv7 output y [M, C] (or z = y when ln_w is
 * NULL); w1 [4C, C], w2 [C, 4C] (nn.Linear weights); gamma = layer_scale; sd = per-sample
 * stochastic-depth scales or NULL.  The 4C hidden stays on chip.
 * C in {96, 128, 192} (IMGCAP_EUNSUPPORTED otherwise: the wide, short stages run faster as two
 * GEMMs with full-chip parallelism). */
int imgcap_cnblock_mlp(int M, int C, const void* y, const float* ln_w, const float* ln_b, const void* w1,
                       const float* b1, const void* w2, const float* b2, const float* gamma, const float* sd,
                       int rows_per_sample, void* x, void* stream);
/* ---------------------------------------------------------------------------------------
 * Backward of the trainable ConvNeXt children (Encoder.fine_tune, encoder.py:29-34; the
 * encoder half of loss.backward() / encoderOptimizer.step() at train.py:278-290).
 * -------------------------------------------------------------------------------------- */
/* dx = res + dwconv7^T(dz): the depthwise 7x7 data gradient (the forward kernel with flipped
 * taps, no bias).  w: the forward weights [49][C] (tap-major).  res may alias dx (or be NULL);
 * dz may not. */
int imgcap_dwconv7_bwd_data(int dtype, int B, int H, int W, int C, const void* dz, const float* w,
                            const void* res, void* dx, void* stream);
/* Depthwise weight / bias gradients: dw[c][kh*7+kw] = sum_{b,h,w} dz[b,h,w,c] *
 * x[b,h+kh-3,w+kw-3,c] (zero padded), db[c] = sum dz[..., c]  (torch layout [C,1,7,7]; written,
 * not accumulated; fixed-order reduction). */
int imgcap_dwconv7_wgrad(int dtype, int B, int H, int W, int C, const void* dz, const void* x, float* dw,
                         float* db, void* stream);
/* Layer-scale backward of one CNBlock from G = (sd*dout)^T GELU(h)  [C][C4] fp32 and
 * cs = colsum(sd*dout): dw2 = gamma*G, wg = gamma*w2 (dtype; operand of the d-hidden GEMM),
 * dgamma = rowsum(w2*G) + b2*cs, db2 = gamma*cs. */
int imgcap_layer_scale_grad(int dtype, int C, int C4, const float* G, const float* w2, const float* b2,
                            const float* gamma, const float* cs, float* dw2, void* wg, float* dgamma,
                            float* db2, void* stream);
/* y[r, :] = x[r, :] * s[r / rows_per_scale]  (per-sample stochastic-depth scale; y may be x) */
int imgcap_rowscale(int dtype, int64_t rows, int cols, const void* x, const float* s, int rows_per_scale,
                    void* y, void* stream);
/* Backward of imgcap_ln_patchify2 (features[2,4,6] LayerNorm2d + 2x2 patch gather): dpatches
 * [B*(H/2)*(W/2)][4C] -> dx [B,H,W,C]; dln_w / dln_b written (statistics recomputed from x). */
int imgcap_ln_patchify2_bwd(int dtype, int B, int H, int W, int C, const void* x, const void* dpatches,
                            const float* ln_w, int cmajor, void* dx, float* dln_w, float* dln_b, void* stream);
/* Backward of imgcap_adaptive_pool_nhwc (AdaptiveAvgPool2d, encoder.py:20,25). */
int imgcap_adaptive_pool_bwd_nhwc(int dtype, int B, int H, int W, int C, int OH, int OW, const void* dy,
                                  void* dx, void* stream);
/* Fixed-order sum of `slices` partial rows ws[s*ld + i], i < n:
 *   split == 0: out0[i] = beta*out0[i] + t_i;  split > 0: i >= split goes to out1[i - split];
 *   split < 0:  depthwise layout i = c*50 + k -> out0[c*49 + k] (k < 49) / out1[c] (k = 49). */
int imgcap_slice_reduce(int64_t n, int slices, const float* ws, int64_t ld, float beta, int64_t split,
                        float* out0, float* out1, void* stream);

/* StochasticDepth(p_i, "row") per-sample scales of every CNBlock (torchvision convnext,
 * train mode; encoder.py:18 builds it): out[i*B + b] = keep ? 1/(1-p_i) : 0, keep drawn from
 * the counter RNG (seed, drop_stream, index i*B+b).  probs: device fp32 [nblocks]. */
int imgcap_stochastic_depth_scales(int nblocks, int B, const float* probs, uint64_t seed,
                                   uint32_t drop_stream, float* out, void* stream);

/* ---------------------------------------------------------------------------------------
 * Token embedding (+ dropout, + positional encoding) — decoder.py:84,
 * transformerDecoder.py:97-98.  out[n, :] = drop(table[ids[n], :]) + (pe ? pe[n % L, :] : 0)
 * -------------------------------------------------------------------------------------- */
int imgcap_embedding_fwd(int dtype, int n, int dim, const int64_t* ids, const float* table,
                         const float* pe, int L, float drop_p, uint64_t seed, uint32_t drop_stream,
                         void* out, void* stream);
/* dtable[ids[n], :] += dout[n, :] * dropmask   (fp32 atomics) */
/* Deterministic: positions are ranked in (id, position) order and every table row is the sum
 * of its occurrences in position order -- bitwise the same on every run (no float atomics).
 * Scratch: the split-reduction workspace.  dtable rows are accumulated into (+=). */
int imgcap_embedding_bwd(int dtype, int n, int dim, const int64_t* ids, const void* dout,
                         float drop_p, uint64_t seed, uint32_t drop_stream, float* dtable,
                         void* stream);

/* ---------------------------------------------------------------------------------------
 * Cross-entropy over rows of logits (train.py:266-268,274-276 CrossEntropyLoss on packed
 * scores) with fused top-5 hit (utils.py:248-250).  target < 0 = ignored row.
 * fwd: lse[n], loss[n] = lse - logit[target] (0 if ignored), hit5[n] in {0,1}.
 * bwd: dlogits = (softmax - onehot) * scale  (0 rows for ignored / padded columns)
 * -------------------------------------------------------------------------------------- */
int imgcap_ce_fwd(int dtype, int n, int V, const void* logits, int64_t ld, const int64_t* targets,
                  float* lse, float* loss, float* hit5, void* stream);
int imgcap_ce_bwd(int dtype, int n, int V, const void* logits, int64_t ld, const int64_t* targets,
                  const float* lse, const float* scale, void* dlogits, int64_t ldd, void* stream);
/* fwd + bwd in one pass over the logits (the training step): scale[0] = 1 / (rows with a
 * target) is computed first and written, then lse / loss / hit5 as imgcap_ce_fwd and
 * dlogits = (softmax - onehot) * scale[0] as imgcap_ce_bwd; one read + one write of [n, V]
 * (train.py:266-276 -- the loss, its gradient and utils.py:248-250's top-5 of one step).
 * Rows: 16-byte aligned, pitches multiples of 8 (bf16) / 4 (fp32) elements, V <= 24576 / 12288;
 * dlogits' padding columns up to the next multiple of 8 / 4 are written as 0. */
int imgcap_ce_fused(int dtype, int n, int V, const void* logits, int64_t ld, const int64_t* targets,
                    float* scale, float* lse, float* loss, float* hit5, void* dlogits, int64_t ldd,
                    void* stream);

/* ---------------------------------------------------------------------------------------
 * clip_gradient (utils.py:183-192, clamp to +-clip) + torch.optim.Adam step
 * (train.py:110,289-291) over a flat fp32 parameter buffer; optionally refreshes a bf16
 * shadow copy of the weights used by the bf16 kernels.  grad is divided by grad_div first
 * (DDP mean over ranks, trainMultiGPU.py:233,384).  skip (device, may be NULL): when *skip != 0
 * at run time the update is not applied (the step's error word: a timed-out persistent LSTM
 * hand-off made its gradients invalid; the step is reported failed by the metrics).
 * -------------------------------------------------------------------------------------- */
int imgcap_clamp_adam(int64_t n, float* param, const float* grad, float* m, float* v,
                      void* shadow_bf16, float lr, float beta1, float beta2, float eps,
                      int step, float clip, float grad_div, const float* skip, void* stream);

/* ---------------------------------------------------------------------------------------
 * LSTM + soft-attention decoder, teacher forced (decoder.py:69-113, Attention 25-31,
 * LSTMCell at :141).  One call enqueues all T steps (3 kernels per step each way).
 * Batch-major buffers [B, T, .]; rows sorted by decode length (decoder.py:79);
 * W3 = A + E + 4D.
 * fwd requires: hprev[:,0,:] = h0, c0, xe = emb_t W_ih[:, :M]^T + b_ih, att1
 *   (b_hh rides in b_hcat).
 * bwd requires: the saved forward buffers, dhs (dL/dh_t from fc), dalpha, the transposed
 * weights; produces dcat (= per-step [d att2 | d gate_pre | d gates_preact]) for the
 * weight-gradient GEMMs, dh/dc (= dL/dh0, dL/dc0), datt1 (sum over t of dL/datt1) and the
 * dwf / dbea partials.  Step GEMMs with long K are split over the grid: x_slices K-slices of
 * dgates . [W_ih[:, M:] | W_hh] into the dz slabs, y_slices of [d att2 | d gate_pre] .
 * [W_da; W_fb] into ws_y, reduced in-kernel by the last arriving block (y_cnt counters).
 * -------------------------------------------------------------------------------------- */
typedef struct imgcap_lstm_desc {
  int32_t dtype, B, P, E, A, D, M, T;
  const void* w_hcat;   /* [W3, D] = [W_da; W_fb; W_hh]             */
  const float* b_hcat;  /* [W3]   = [b_da; b_fb; b_hh]              */
  const void* w_ih;     /* [4D, M+E] LSTMCell weight_ih             */
  const float* w_f;     /* [A] full_att weight                      */
  const void* enc;      /* [B, P, E] encoder_out (sorted)           */
  const void* att1;     /* [B, P, A]                                */
  const float* xe;      /* [B, T, 4D] emb W_ih[:, :M]^T + b_ih      */
  const float* c0;      /* [B, D]                                   */
  const int32_t* dl;    /* [B] decode lengths (sorted, device)      */
  float* g1;            /* [B, T, W3] saved [att2 | gate_pre | hh]  */
  float* alphas;        /* [B, T, P]  output (0 where t >= dl[b])   */
  float* awe;           /* [B, T, E]  saved attention context       */
  void* zs;             /* [B, T, E]  gate * context (LSTM input)   */
  float* gates;         /* [B, T, 4D] activated i, f, g, o          */
  float* cs;            /* [B, T, D]                                */
  void* hs;             /* [B, T, D]  h_t                           */
  void* hprev;          /* [B, T, D]  h_{t-1}; slot 0 = h0          */
  const void* w_zh_t;   /* [E + D, 4D] = [W_ih[:, M:] | W_hh]^T (bwd) */
  const void* w_att_t;  /* [D, A + E]  = [W_da; W_fb]^T        (bwd) */
  const void* dhs;      /* [B, T, D]  bwd input                     */
  const float* dalpha;  /* [B, T, P]  bwd input dL/dalpha or NULL   */
  void* dcat;           /* [B, T, W3] bwd output                    */
  float* dz;            /* [x_slices, B, E + D] workspace (slabs)   */
  float* ws_y;          /* [y_slices, ceil(B/32) * D/16, 512] workspace */
  int32_t* y_cnt;       /* [ceil(B/32) * D/16] zero-initialised counters (left at 0) */
  float* dh;            /* [B, D] out: dL/dh0                       */
  float* dc;            /* [B, D] out: dL/dc0                       */
  float* de;            /* [B, T, P] workspace: dL/d(attention score) */
  void* datt1;          /* [B, P, A] out: sum_t dL/datt1 (dtype)    */
  float* dwf;           /* [B*ceil(P/7), A] out: partials of dL/dw_f  */
  float* dbea;          /* [B*ceil(P/7), A] out: partials of dL/db_ea */
  int32_t x_slices;     /* 1..16 */
  int32_t y_slices;     /* 1..16 */
  float* dawe;          /* [B, T+1, E] out or NULL: dL/d(attention context) per step (rows t < T;
                           row T is left to the caller) -- the encoder-gradient path */
  int32_t* sync;        /* caller-owned, 16-byte aligned, at least imgcap_lstm_sync_words() int32
                           words (NULL: per-step launches only).  fwd: the persistent recurrence's
                           hand-off flags, zeroed by the library (a memset on the stream) before
                           each launch; word 0 is left non-zero if a hand-off timed out. */
  int32_t sync_words;
  int32_t row_groups;   /* persistent recurrences: 0 = library default (IMGCAP_LSTM_GROUPS, else
                           one chain); 4 | mask = explicit, mask bit 0 runs the forward, bit 1 the
                           backward as two row groups [0, ceil(B/2)), [ceil(B/2), B) side by side in
                           the one launch (B > 16; more CUs, shorter steps) */
} imgcap_lstm_desc;

/* fwd: with d->sync set and T >= 2, the whole recurrence is ONE persistent launch when the
 * shape fits (B <= 64, P <= 64, A <= 512, E, D, M % 8 == 0; steps t >= max(dl) are skipped and
 * their outputs zeroed); otherwise three launches per step.  Same outputs either way, except
 * that g1's hh columns are written by the per-step path only. */
int imgcap_lstm_tf_fwd(const imgcap_lstm_desc* d, void* stream);
/* int32 words of imgcap_lstm_desc.sync the persistent forward needs for this shape (0: the
 * shape runs on the per-step path) */
int imgcap_lstm_sync_words(const imgcap_lstm_desc* d);
int imgcap_lstm_tf_bwd(const imgcap_lstm_desc* d, void* stream);
/* dL/d encoder_out for encoder fine-tuning (the decoder.py:75-113 paths back into encoder_out):
 *   denc[sort_ind[b], p, :] = base[b, p, :] + sum_{t<T} alphas[b,t,p] dawe[b,t,:] + dawe[b,T,:] / P
 * base [B, P, E] fp32 = datt1 . W_ea (sorted order, may be NULL); dawe [B, T+1, E] fp32 as
 * imgcap_lstm_desc.dawe with row T = dL/d mean(encoder_out); sort_ind NULL = identity; P <= 64. */
int imgcap_lstm_denc(int B, int T, int P, int E, const float* alphas, const float* dawe, const float* base,
                     const int64_t* sort_ind, float* denc, void* stream);
/* train.py:269: reg = alphaC*mean_{b,p}(1-sum_t alpha)^2 -> *reg_out;
 * dalpha[b,t,p] = d reg / d alpha[b,t,p] (0 where t >= dl[b]).  part: B floats of per-row partial
 * sums, caller-owned (NULL: library scratch -- not from a stream that runs beside other scratch
 * users; the LSTM engine calls this on its side stream and passes its own). */
int imgcap_attn_reg(int B, int T, int P, const float* alphas, const int32_t* dl, float alphaC, float* dalpha,
                    float* reg_out, float* part, void* stream);

/* ---------------------------------------------------------------------------------------
 * Multi-head attention of nn.TransformerDecoderLayer (transformerDecoder.py:82,104): one
 * workgroup per (batch, head), head dim 64, Lq, Lk <= 64.  q/k/v/o are row-major [B*L, ld]
 * activations with head h at column offset h*64 (the packed in_proj output can be passed
 * directly).  Masks: causal (key j > query i), key padding (key_ids[b, j] == pad_id).
 * Dropout p on the attention probabilities (nn.MultiheadAttention dropout).
 * fwd saves lse[B, H, Lq]; bwd recomputes P from it and writes dq, dk, dv.
 * -------------------------------------------------------------------------------------- */
typedef struct imgcap_mha_desc {
  int32_t dtype, B, H, Lq, Lk, dh, causal;
  int64_t pad_id;
  int64_t ldq, ldk, ldv, ldo;
  const void* q;
  const void* k;
  const void* v;
  void* o;
  float* lse;
  const int64_t* key_ids;
  float scale;
  float drop_p;
  uint64_t seed;
  uint32_t drop_stream;
  const void* dout;
  int64_t lddo;
  void* dq;
  void* dk;
  void* dv;
  int64_t lddq, lddk, lddv;
  int64_t kv_rows;     /* fwd only: rows between consecutive batch entries of k / v (0 = Lk): a
                          [B][Lmax] key/value cache read at its first Lk rows (incremental decode) */
  float* probs;        /* fwd only, optional: the attention probabilities [B, H, Lq, Lk] fp32 as
                          nn.MultiheadAttention returns them with need_weights=True,
                          average_attn_weights=False (after dropout) -- transformerDecoderAttVis.py:72,83 */
} imgcap_mha_desc;

int imgcap_mha_fwd(const imgcap_mha_desc* d, void* stream);
/* One greedy decoding step (decoder.py:150-161, transformerDecoder.py:137-155) for rows not yet
 * finished: predictions[b, t, :V] = logits[b, :V] (fp32), sequences[b, t] = argmax (first index
 * of the maximum, as torch), alphas[b, t, :P] = alpha[b, :P] (if alpha), next_ids[b] = argmax,
 * finished[b] |= (argmax == end_id).  Finished rows are left untouched (the outputs start zeroed,
 * as the reference's torch.zeros).  logits: [B, ldl] of dtype. */
int imgcap_greedy_select(int dtype, int B, int V, const void* logits, int64_t ldl, int t, int maxlen,
                         int64_t end_id, uint8_t* finished, int64_t* next_ids, int64_t* sequences,
                         float* predictions, const float* alpha, float* alphas, int P, void* stream);
int imgcap_mha_bwd(const imgcap_mha_desc* d, void* stream);

/* y = x * dropmask(seed, stream, i) (nn.Dropout, decoder.py:109 / transformer dropouts) */
int imgcap_dropout(int dtype, int64_t n, const void* x, float p, uint64_t seed, uint32_t drop_stream, void* y,
                   void* stream);
/* Token-mean loss finalisation without host sync (train.py:268 + reduceLossAndTokens inputs):
 * out[0] = sum(loss_rows)/count + (extra ? *extra : 0), out[1] = count (valid targets),
 * out[2] = sum(hit5), out[3] = 1/count (the CE backward scale) */
int imgcap_loss_finalize(int n, const float* loss_rows, const float* hit5, const int64_t* targets,
                         const float* extra, float* out, void* stream);

/* Transformer loss rows from the captions, one launch (transformerDecoder.py:88-108, train.py:262-276):
 * tmask[b*L+l] = l < lens[b] - 1 (uint8), targets[b*L+l] = tmask ? caps[b, l+1] : -1, metrics[0..n) = 0
 * (caps [B, L] int64, lens [B] int64 caption lengths incl. <start>/<end>) */
int imgcap_tf_targets(int B, int L, const int64_t* caps, const int64_t* lens, uint8_t* tmask, int64_t* targets,
                      float* metrics, int n_metrics, void* stream);

/* out[b, e] = mean_p x[b, p, e] (decoder.py:64, input of init_h/init_c) */
int imgcap_mean_mid(int dtype, int B, int P, int E, const void* x, void* out, void* stream);
/* decoder.py:64,79-81 fused: rows sorted by caption length (descending, stable), enc_out[r] =
 * enc[sort_ind[r]] ([B,P,E]), caps_out[r] = caps[sort_ind[r]] ([B,L] int64), dl[r] = len - 1
 * (int32), mean_out[r] = mean over P of enc_out[r]; B <= 256, E rows 16-byte aligned */
int imgcap_sort_gather_rows(int dtype, int B, int P, int E, int L, const int64_t* lens, const void* enc,
                            const int64_t* caps, void* enc_out, void* mean_out, int64_t* caps_out, int64_t* sort_ind,
                            int32_t* dl, void* stream);

/* elementwise helpers */
int imgcap_cast(int in_dtype, int out_dtype, int64_t n, const void* x, void* y, void* stream);
int imgcap_fill(int dtype, int64_t n, float value, void* x, void* stream);

#ifdef __cplusplus
}
#endif
#endif

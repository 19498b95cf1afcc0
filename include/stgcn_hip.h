/*
 * stgcn_hip.h — C-ABI of libstgcn_hip.so, the MI355X (gfx950) ST-GCN block.
 *
 * This is the drop-in boundary for ONE hot path of nagyrajmund/st-gcn: the
 * ST-GCN block in training (and eval) mode,
 *
 *   y = ReLU(BN2(Conv9x1(SpatialConv(BN1(x)))))                 (default)
 *   y = ReLU(Conv9x1(ReLU(BN2(SpatialConv(ReLU(BN1(x)))))) + R(x))
 *                                          (flags & STGCN_F_RESIDUAL)
 *
 * with R = identity (C_in == C_out, stride 1) or a 1x1 Conv2d with temporal
 * stride (st_graphconv.py:24-28), i.e. SpatialTemporalConv.forward
 * (src/network/st_graphconv.py:85-109, residual_block :60-82) with
 * SpatialConv.forward (st_graphconv.py:139-152) and its autograd backward.
 * Dropout (p > 0, training) is fused into the block's output pass
 * (stgcn_fwd_args_t.dropout_p / seed, ABI 2); training and eval mode are
 * both differentiable (eval: BatchNorm with the running statistics as
 * constants, ABI 4).
 * The reference has no FFI of its own (pure Python over PyTorch); the entry
 * points below are what its module boundary binds to (the ctypes binding in
 * st-gcn_amd/hip_lib.py, shown in INTEGRATION.md):
 *
 *   stgcn_block_fwd  replaces SpatialTemporalConv.forward, st_graphconv.py:85-109
 *                    (BatchNorm2d :34/:98, SpatialConv :139-152, temporalConv
 *                    :41-43/:99, BatchNorm2d :46/:100, ReLU :49/:105;
 *                    residual_block :60-82 with apply_residual :24-28)
 *   stgcn_block_bwd  replaces the autograd backward of the same ops
 *                    (driven by lightning_model.py:199-205 -> loss.backward())
 *   stgcn_spatial_fwd / stgcn_spatial_bwd  replace SpatialConv.forward used on
 *                    its own (st_graphconv.py:139-152) and its backward (ABI 4)
 *
 * Conventions
 *   - All tensors are caller-owned, contiguous, fp32, device memory, layout
 *     NCTV (N clips, C channels, T frames, V joints) as in the reference.
 *   - A is (K,V,V), W is (K*C_out, C_in) (the reference's 1x1 Conv2d weight),
 *     Wt is (C_out, C_out, 9) (the (9,1) Conv2d weight).
 *   - The workspace is caller-allocated (query *_workspace_bytes first); the
 *     library allocates nothing on the hot path and keeps no mutable global
 *     state besides the thread-local error string.
 *   - Every launch goes on the caller's stream (a hipStream_t passed as void*).
 *   - Return 0 on success, a negative STGCN_E* code otherwise; the message is
 *     in stgcn_last_error() (thread-local).
 */
#ifndef STGCN_HIP_H
#define STGCN_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define STGCN_ABI_VERSION 11

/* ABI 7: words of max |y| after the 5 * C sums of a y_stats block */
#define STGCN_STATS_AMAX_WORDS 2048
#define STGCN_Y_STATS_BYTES(C) (8 * 5 * (size_t)(C) + 4 * (size_t)STGCN_STATS_AMAX_WORDS)

/* stgcn_desc_t.flags */
#define STGCN_F_RESIDUAL 1 /* full pre-activation residual block (st_graphconv.py:60-82) */
#define STGCN_F_BF16 2     /* channel GEMMs (W, temporal conv fwd/dgrad/wgrad, projection)
                            * on bf16 MFMA: operands rounded to bf16, fp32 accumulate;
                            * A / BatchNorm stay fp32 (BASELINE cfg3/5). x, y, U, stats and
                            * every gradient the caller receives are fp32. Z (the saved
                            * spatial output) is OPAQUE under this flag: on stride-1
                            * non-residual blocks with C_in >= 16 it holds bf16 values in
                            * the first half of its fp32-sized buffer (every reader rounds
                            * it to bf16 anyway), so only stgcn_block_bwd may read it.
                            * Applies for V in {18, 25, 50} and reductions over >= 16
                            * channels; other GEMMs run the fp32 kernels. */
#define STGCN_F_F32X3 4    /* fp32 channel GEMMs on the bf16 matrix cores by exact 3-way
                            * operand splits (x = h + m + l, six partial products, fp32
                            * accumulate): fp32-GEMM accuracy at up to 2.67x the fp32
                            * MFMA rate. Applies for V in {18, 25} over >= 16 channels to
                            * the temporal conv forward (stride 1 and 2), data-grad and
                            * weight-grad, and to the spatial weight-grad dW'; other GEMMs
                            * run the fp32 kernels. Every tensor stays fp32. On non-residual
                            * blocks with K = 1, V = 18 and C_in >= 16 the SpatialConv
                            * channel GEMM is folded into the temporal conv's weights
                            * (Wc_q = Wt_q W'): Z is never formed, and its buffer is
                            * OPAQUE (it carries Wc from stgcn_block_fwd to
                            * stgcn_block_bwd). Exclusive with STGCN_F_BF16. */
#define STGCN_F_F16X2 8    /* ABI 6, with STGCN_F_F32X3 only: the folded block's temporal
                            * conv forward, data-grad and weight-grad GEMMs as 2-way fp16 splits
                            * (x s = h + l, 22 significant bits, three partial products,
                            * fp32 accumulate) of operands scaled by powers of two s from
                            * their max |x| (so h <= 2^14 and no element underflows
                            * relative to the tensor's maximum); the result is scaled back
                            * exactly. Same fp32 gate as STGCN_F_F32X3, half its MFMAs.
                            * At V = 18 the data gradient runs on the fp16 splits too
                            * (with the SpatialConv backward fused into it); BN1's
                            * nearly cancelling sum of dxhat (its bias gradient) is
                            * formed from the fp64 per-tap dU sums instead of from the
                            * 22-bit data gradient. (The 3-way bf16 data gradient is an
                            * A/B measurement build only: STGCN_AB_F16X2_DGRAD=0.) At
                            * V = 25 (folded, K = 1) the data gradient stays on the
                            * 3-way bf16 splits. ABI 8: an unfolded non-residual V = 18,
                            * K = 1 block with C_out >= 16 (the first block, C_in = 3)
                            * runs its temporal forward and weight gradient on the fp16
                            * splits (bounds by max-|x| passes over Z and Wt), its data
                            * gradient on the 3-way bf16 splits. stgcn_block_plan reports
                            * STGCN_PLAN_F16X2 wherever any GEMM of the block uses them. */

#define STGCN_F_NO_G 16    /* ABI 7, with STGCN_F_F16X2 only (memory-lean folded block):
                            * G = BN1(x) A^T is never formed or kept -- the forward GEMM
                            * reads x (BN1 in its loader, the joint contraction in its
                            * epilogue), the weight gradient reads x against dU A formed
                            * by the ReLU + BN2 backward pass -- so the N*C_in*T*V*4-byte
                            * G buffer is not kept between forward and backward
                            * (stgcn_keep_g_bytes then returns only the bound words).
                            * Same fp32 gate; measured slower than the G path on cfg2
                            * (DESIGN.md), hence opt-in. */

enum {
  STGCN_OK = 0,
  STGCN_E_INVALID = -1,     /* bad pointer / shape / parameter            */
  STGCN_E_UNSUPPORTED = -2, /* V > 256, gamma != 9, unknown flags ...      */
  STGCN_E_HIP = -3          /* a HIP launch / runtime error               */
};

/* Block descriptor (one SpatialTemporalConv, st_graphconv.py:9). */
typedef struct stgcn_desc {
  int32_t N, C_in, C_out, T, T_out, V, K;
  int32_t gamma;       /* temporal kernel size: 9 (lightning_model.py:263)   */
  int32_t stride;      /* temporal stride 1 or 2                             */
  int32_t pad;         /* temporal padding (gamma-1)/2 = 4                   */
  float eps;           /* BatchNorm eps 1e-5                                 */
  float momentum;      /* BatchNorm momentum 0.1                             */
  int32_t training;    /* 1: batch statistics + running-stat update          */
  int32_t need_dx;     /* backward: write dx (0 for the network's first block)*/
  int32_t flags;       /* STGCN_F_RESIDUAL | (STGCN_F_BF16 or STGCN_F_F32X3
                        * [| STGCN_F_F16X2 [| STGCN_F_NO_G]])                  */
} stgcn_desc_t;

/* Forward arguments. Saved tensors (Z, U, stats; residual: Z, Za, y, stats)
 * are kept by the caller for stgcn_block_bwd. stats holds mean1[C_in],
 * invstd1[C_in], mean2[C_out], invstd2[C_out] (fp32) as used by the forward.
 * Residual block: BN2 normalizes Z (the spatial output, st_graphconv.py:76),
 * U is not used, Za = ReLU(BN2(Z)) is the temporal conv input, Wr/br is the
 * projection (C_out, C_in) + (C_out) when C_in != C_out or stride != 1
 * (apply_residual, st_graphconv.py:27), else null. */
typedef struct stgcn_fwd_args {
  const float *x;                       /* N,C_in,T,V                         */
  const float *A, *W, *bW, *Wt, *bWt;   /* SpatialConv.A / W ; temporalConv   */
  const float *g1, *b1, *g2, *b2;       /* batch_n / batch_n_2 affine         */
  float *rm1, *rv1, *rm2, *rv2;         /* running stats (updated if training)*/
  float *y;                             /* out: N,C_out,T_out,V (ABI 8: may be
                                         * null, see prev_U below; ABI 9: null
                                         * with y_stats null, see
                                         * stgcn_head_fwd_u)                  */
  float *Z;                             /* saved: spatial output N,C_out,T,V
                                         * (fp32-sized; opaque under STGCN_F_BF16) */
  float *U;                             /* saved: temporal output N,C_out,T_out,V */
  float *stats;                         /* saved: 2*C_in + 2*C_out floats     */
  /* ABI 2 (residual block; null otherwise) */
  const float *Wr, *br;                 /* apply_residual Conv2d (projection) */
  float *Za;                            /* saved: ReLU(BN2(Z)) N,C_out,T,V    */
  /* ABI 2, optional: keep the joint contraction G = f(BN1(x)) A^T for the
   * backward instead of recomputing it: stgcn_keep_g_bytes(d) bytes; fp32
   * (N, K*C_in, T, V), or, where the bf16 path's fused spatial kernel runs
   * (STGCN_F_BF16, C_in >= 16), bf16 in frame tiles (ABI 4: opaque to the caller).
   * Under STGCN_F_F16X2 the words after G carry its operand bound max |G| to
   * the backward's weight gradient: a kept G is valid only for a backward with
   * the SAME descriptor (flags included) as the forward that wrote it. */
  float *G;
  /* ABI 2, optional stack chaining (training): x_stats = [sum(C_in), sumsq(C_in)]
   * of x over (n,t,v) in fp64 (produced by the previous block's y_stats: the
   * BN1 statistics pass is skipped); y_stats (out) = the same for y (C_out).
   * ABI 5: y_stats holds 5 * C_out doubles; a non-residual block without
   * dropout also writes, with its ReLU mask m = y > 0 and uhat = (U - mean2) *
   * invstd2, [cnt = sum m | su = sum m uhat | xu = sum y uhat] after the two
   * (the next block's deferred-dx chain, stgcn_bwd_args_t.x_stats). */
  const double *x_stats;
  double *y_stats;
  /* ABI 7: x_stats / y_stats blocks are STGCN_Y_STATS_BYTES(C) bytes: the 5 * C
   * doubles above, then STGCN_STATS_AMAX_WORDS uint32 words that receive max |y|
   * (as float bits, the largest word wins): the operand bound of the next block's
   * fp16-split GEMMs, which read y itself (STGCN_PLAN_FOLD_NO_G). */
  /* ABI 2, optional fused dropout on y (training only; st_graphconv.py:53-58,
   * :107-109): element e of y is kept iff splitmix64(seed + e * 0x9E3779B97F4A7C15)
   * >> 32 >= dropout_p * 2^32, then scaled by 1/(1 - dropout_p). 0: no dropout. */
  float dropout_p;
  uint64_t seed;
  /* ABI 7, optional (folded blocks): the block's stgcn_fold_prep buffer of this
   * training step -- its weight-only operands are then not formed again */
  const void *prep;
  /* ABI 8, optional stack chaining without the block output in HBM
   * (STGCN_PLAN_X_FROM_U; training, with x_stats; non-residual previous block
   * without dropout): the block input is x = ReLU(BN2_prev(prev_U)), formed
   * where the block reads it, from the previous block's U, [mean2 | invstd2]
   * (its stats + 2 * C_in_prev) and BN2 affine; x may then be null. The
   * previous block's forward ran with y = null (a non-residual block without
   * dropout, with y_stats: only the statistics of y are formed), and this
   * block's backward is called with x = null, its kept G and the deferred-dx
   * chain arguments (stgcn_bwd_args_t prev_*, x_stats, dx_coef, dx_deferred). */
  const float *prev_U, *prev_stats, *prev_g2, *prev_b2;
} stgcn_fwd_args_t;

/* Backward arguments: the gradients of every input of the forward. */
typedef struct stgcn_bwd_args {
  const float *dy;                      /* N,C_out,T_out,V                    */
  const float *x, *Z, *U, *stats;       /* saved by the forward               */
  const float *A, *W, *bW, *Wt, *g1, *b1, *g2, *b2;
  float *dx;                            /* N,C_in,T,V (ignored if !need_dx)   */
  float *dA, *dW, *dbW, *dWt, *dbWt;
  float *dg1, *db1, *dg2, *db2;
  /* ABI 2 (residual block; null otherwise) */
  const float *Wr;                      /* projection weight or null          */
  const float *Za, *y;                  /* saved by the forward               */
  float *dWr, *dbr;                     /* projection gradients or null       */
  const float *G;                       /* optional: G kept by the forward    */
  /* optional stack chaining (non-residual blocks):
   * dy_sums = [sum dy*m, sum dy*m*uhat] (2*C_out, fp64) of this block's
   * ReLU+BN2 backward, produced by the next block (its reduction pass is
   * skipped); prev_g2/prev_b2 = BN2 affine of the (non-residual) block that
   * produced x, prev_sums (out, 2*C_in) = that block's dy_sums, computed while
   * writing dx (needs need_dx). */
  const double *dy_sums;
  const float *prev_g2, *prev_b2;
  double *prev_sums;
  float dropout_p;                      /* the forward's dropout (same seed)  */
  uint64_t seed;
  /* ABI 4, optional with prev_sums: the previous block's saved pre-BN2 tensor
   * U (N, C_in, T, V) and its stats (mean2[C_in], invstd2[C_in]). Channels
   * where reconstructing uhat = (x - prev_b2) / prev_g2 from x is
   * ill-conditioned (|prev_b2| > 4 |prev_g2|, including prev_g2 == 0) read
   * uhat from U instead. Null: reconstruct everywhere. */
  const float *prev_U;
  const float *prev_stats;
  /* ABI 5, optional deferred dx (training, non-residual block, with the
   * prev_* chain arguments above and prev_U / prev_stats): this block's BN1
   * backward apply is folded into the PREVIOUS block's ReLU+BN2 backward
   * apply. When the library takes it (*dx_deferred = 1; it does where its
   * spatial-backward kernel reads the previous block's U in place of x), dx
   * receives dxhat (the gradient at BN1's output) instead of the gradient of
   * x, dx_coef (5 * C_in floats [a | md | mu | is | mdn]) the BN1 backward
   * coefficients (dx = a * (dxhat - md - (x - mu) * is * mdn)) and prev_sums
   * the previous block's dy_sums; the previous block's stgcn_block_bwd then
   * takes dy = that dxhat with dy_coef = dx_coef and dy_sums = prev_sums.
   * x_stats: the 5 * C_in y_stats the previous block's forward wrote. */
  const double *x_stats;
  float *dx_coef;
  int32_t *dx_deferred;                 /* host int: 1 deferred, 0 dx written */
  /* ABI 5, in: dy holds the next block's dxhat, to be combined as above with
   * these 5 * C_out coefficients (needs dy_sums; non-residual, no dropout) */
  const float *dy_coef;
  /* ABI 7, optional: the same stgcn_fold_prep buffer as the forward's */
  const void *prep;
  /* ABI 10, optional: the gradient of y is constant over (T_out, V) --
   * dy[n, c, t, v] = dy_nc[n * C_out + c] (N * C_out floats), as the average-pool
   * head gives it (stgcn_head_bwd_nc) -- and dy may be null: the ReLU + BN2
   * backward reads one value per (clip, channel) instead of the dy tensor.
   * Non-residual blocks; STGCN_E_UNSUPPORTED where the block's backward needs
   * the full dy (the caller then passes it). */
  const float *dy_nc;
  /* ABI 8: x may be null when the forward took its input from prev_U
   * (STGCN_PLAN_X_FROM_U); the call then needs the kept G and the deferred-dx
   * arguments (prev_U, prev_stats, prev_g2, prev_b2, prev_sums, x_stats, dx_coef,
   * dx_deferred) and fails with STGCN_E_INVALID where it could not defer. */
} stgcn_bwd_args_t;

int stgcn_abi_version(void);
const char *stgcn_last_error(void);

/* Validate a descriptor without touching the GPU (0 = supported). */
int stgcn_check_desc(const stgcn_desc_t *d);

size_t stgcn_fwd_workspace_bytes(const stgcn_desc_t *d);
/* ABI 4: bytes of the optional kept-G buffer (stgcn_fwd_args_t.G / bwd G) */
size_t stgcn_keep_g_bytes(const stgcn_desc_t *d);
size_t stgcn_bwd_workspace_bytes(const stgcn_desc_t *d);

int stgcn_block_fwd(const stgcn_desc_t *d, const stgcn_fwd_args_t *a,
                    void *workspace, size_t workspace_bytes, void *stream);
int stgcn_block_bwd(const stgcn_desc_t *d, const stgcn_bwd_args_t *a,
                    void *workspace, size_t workspace_bytes, void *stream);

/* ---------------------------------------------------------------------------
 * ABI 4: SpatialConv on its own (st_graphconv.py:139-152):
 *   out[n,c,t,v] = sum_k sum_w A[k,v,w] * (W_k x[n,:,t,w] + bW_k)[c]
 * computed as out = sum_k W_k (x A_k^T) + sum_k bW_k rowsum(A_k) (the block's
 * form (1), no BatchNorm). x (N, C_in, T, V), A (K, V, V), W (K*C_out, C_in),
 * bW (K*C_out), out (N, C_out, T, V); flags: STGCN_F_BF16 runs the channel
 * GEMMs on bf16 MFMA (fp32 otherwise). Backward: dout -> dx (may be null),
 * dA, dW, dbW.
 */
typedef struct stgcn_spatial_desc {
  int32_t N, C_in, C_out, T, V, K;
  int32_t flags;       /* 0 or STGCN_F_BF16                                 */
} stgcn_spatial_desc_t;

size_t stgcn_spatial_workspace_bytes(const stgcn_spatial_desc_t *d, int backward);
int stgcn_spatial_fwd(const stgcn_spatial_desc_t *d, const float *x, const float *A,
                      const float *W, const float *bW, float *out, void *workspace,
                      size_t workspace_bytes, void *stream);
int stgcn_spatial_bwd(const stgcn_spatial_desc_t *d, const float *dout, const float *x,
                      const float *A, const float *W, const float *bW, float *dx, float *dA,
                      float *dW, float *dbW, void *workspace, size_t workspace_bytes,
                      void *stream);

/* ABI 6: the kernel plan the library selects for a descriptor (a bitmask of
 * STGCN_PLAN_*), so a caller or a test can pin which path its calls take. */
#define STGCN_PLAN_FOLD 1          /* K = 1 fp32 split path: the SpatialConv channel GEMM W'
                                    * folded into the temporal conv's weights (Wc_q = Wt_q W');
                                    * Z and dZ are never formed (capi.hip fold_w)         */
#define STGCN_PLAN_SP_FWD_FUSED 2  /* SpatialConv forward in one kernel (k_sp_fwd_*)     */
#define STGCN_PLAN_SP_BWD_FUSED 4  /* SpatialConv backward in one kernel (H never in HBM) */
#define STGCN_PLAN_ACT_BF16 8      /* Z / dU stored in bf16 (bf16 path)                  */
#define STGCN_PLAN_WSP_SPLIT 16    /* spatial dW' on exact split products (k_wgrad_sp X3) */
#define STGCN_PLAN_TCONV_SPLIT 32  /* temporal conv forward on the split pipeline         */
#define STGCN_PLAN_TWGRAD_SPLIT 64 /* temporal weight gradient on the split kernel        */
#define STGCN_PLAN_F16X2 128       /* the folded GEMMs on 2-way fp16 splits (STGCN_F_F16X2) */
#define STGCN_PLAN_FOLD_NO_G 256   /* ABI 7, with F16X2: G = BN1(x) A^T is never formed: the
                                    * forward GEMM reads x (BN1 in its loader, the joint
                                    * contraction in its epilogue), the weight gradient reads
                                    * x against dU A; the kept-G buffer (stgcn_keep_g_bytes)
                                    * then carries only max |x| to the backward          */
#define STGCN_PLAN_X_FROM_U 512    /* ABI 8: the training forward can take its input as
                                    * ReLU(BN2(U)) of the previous block
                                    * (stgcn_fwd_args_t.prev_U): that block's y is never
                                    * written                                             */
int stgcn_block_plan(const stgcn_desc_t *d, uint32_t *plan);

/* ABI 7: the weight-only operands of a stack's folded blocks (STGCN_PLAN_FOLD),
 * formed together once per training step (the weights change every optimizer
 * step): bZ = bW rowsum(A), the composite weights Wc_q = Wt_q W', the per-frame
 * bias table, max |Wc|, the packed split planes of the forward and data-gradient
 * GEMMs and the backward's operand re-layouts -- a dozen launches for the whole
 * stack instead of ~11 small launches per block. stgcn_fold_prep_bytes(d) is the
 * block's buffer size (0: the block does not fold); the buffer is then passed as
 * stgcn_fwd_args_t.prep / stgcn_bwd_args_t.prep of that block in the same step
 * (same weights). Blocks whose size is 0 are skipped. The block's backward also
 * uses the buffer's fp64 scratch for its activation-dependent per-tap dU sums
 * (the Tq re-layout): one prep buffer must not serve two backward passes that
 * run concurrently (e.g. micro-batches on separate streams). */
typedef struct stgcn_fold_weights {
  const float *A, *W, *bW, *Wt, *bWt;   /* as in stgcn_fwd_args_t            */
} stgcn_fold_weights_t;
size_t stgcn_fold_prep_bytes(const stgcn_desc_t *d);
int stgcn_fold_prep(int nblocks, const stgcn_desc_t *descs, const stgcn_fold_weights_t *weights,
                    void *const *prep, void *stream);

/* Measurement (bench.py roofline): time one of the block's GEMM kernels,
 * launched `iters` times with the exact parameters the block uses for this
 * descriptor, between two hipEvents on `stream`. which: 0 temporal conv fwd,
 * 1 temporal conv data-grad, 2 temporal conv weight-grad, 3 spatial channel
 * GEMM (the fused SpatialConv forward where it runs), 4 spatial backward
 * (dZ -> dx, dA, BN1 sums), 5 / 6 the H GEMM / the joint kernel of a spatial
 * backward that runs unfused (STGCN_E_UNSUPPORTED where it is one kernel).
 * scratch (>= stgcn_time_kernel_bytes) supplies operand memory.
 * *flops receives the algorithmic FLOPs of one launch. */
size_t stgcn_time_kernel_bytes(const stgcn_desc_t *d, int which);
int stgcn_time_kernel(const stgcn_desc_t *d, int which, void *scratch, size_t scratch_bytes,
                      int iters, void *stream, float *avg_ms, double *flops);

/* ---------------------------------------------------------------------------
 * ABI 3: training-step ops around the stack.
 *
 * Classification head: global average pool over (T, V) + Linear + cross
 * entropy (lightning_model.py:105-107 avg_pool2d + fc_layer, :202
 * F.cross_entropy with mean reduction). y is the last block's output
 * (N, C, L = T*V); W (classes, C), bias (classes), labels int64 (N).
 * stgcn_head_fwd writes pooled (N, C), logits (N, classes), lossv (N, per-clip
 * loss) and loss (1, the mean). stgcn_head_bwd takes dloss (1) and writes
 * dlogits (N, classes, scratch), dpooled (N, C, scratch), dy (N, C, L: the
 * gradient of y), dW, dbias. Deterministic (no atomics).
 */
typedef struct stgcn_head_desc {
  int32_t N, C, L, classes;
} stgcn_head_desc_t;

int stgcn_head_fwd(const stgcn_head_desc_t *d, const float *y, const float *W, const float *bias,
                   const int64_t *labels, float *pooled, float *logits, float *lossv, float *loss,
                   void *stream);
int stgcn_head_bwd(const stgcn_head_desc_t *d, const float *pooled, const float *logits,
                   const float *W, const int64_t *labels, const float *dloss, float *dlogits,
                   float *dpooled, float *dy, float *dW, float *dbias, void *stream);
/* ABI 10: stgcn_head_bwd with the gradient of y as its per-(n, c) value only:
 * dy_nc (N, C) = dpooled / L, the value stgcn_head_bwd writes to every one of
 * the L positions of row (n, c) -- for stgcn_bwd_args_t.dy_nc (no (N, C, L)
 * tensor written or read). */
int stgcn_head_bwd_nc(const stgcn_head_desc_t *d, const float *pooled, const float *logits,
                      const float *W, const int64_t *labels, const float *dloss, float *dlogits,
                      float *dpooled, float *dy_nc, float *dW, float *dbias, void *stream);
/* ABI 9: stgcn_head_fwd with the last block's output never written: the pool
 * reads that block's pre-BN2 tensor U (N, C, L) and forms y = ReLU(BN2(U)) on
 * load with the block's stats2 = [mean2 (C) | invstd2 (C)] (its stats buffer
 * from C_in * 2 on) and BN2 affine g2 / b2, as the block's output pass would
 * (bit-identical pooled). The block runs with stgcn_fwd_args_t.y and .y_stats
 * both null (training, non-residual, no dropout: no output pass at all).
 * stgcn_head_bwd is unchanged (its dy is the gradient of that unwritten y). */
int stgcn_head_fwd_u(const stgcn_head_desc_t *d, const float *U, const float *stats2,
                     const float *g2, const float *b2, const float *W, const float *bias,
                     const int64_t *labels, float *pooled, float *logits, float *lossv,
                     float *loss, void *stream);

/* Multi-tensor Adam (torch.optim.Adam, amsgrad=False, maximize=False;
 * lightning_model.py:196-197): ONE launch updates every tensor of a table.
 * stgcn_adam_build_table fills a HOST buffer (stgcn_adam_table_bytes; pinned
 * memory, so the caller can copy it to the device asynchronously) with the
 * tensor list and its chunk prefix sums and returns the chunk count;
 * stgcn_adam_step reads the DEVICE copy, with the 1-based step count; the
 * hyper-parameters are doubles (Python floats): 1 - beta and the bias
 * corrections are formed in double and rounded to float, as torch does. */
typedef struct stgcn_adam_tensor {
  float *param;
  const float *grad;
  float *exp_avg;
  float *exp_avg_sq;
  int64_t numel;
} stgcn_adam_tensor_t;

size_t stgcn_adam_table_bytes(int ntensors);
int stgcn_adam_build_table(const stgcn_adam_tensor_t *tensors, int ntensors, void *host_table,
                           size_t table_bytes, int64_t *total_chunks);
int stgcn_adam_step(const void *dev_table, int ntensors, int64_t total_chunks, double lr,
                    double beta1, double beta2, double eps, double weight_decay, int64_t step,
                    void *stream);
/* ABI 11: the same update with the step count in DEVICE memory (a float, as
 * torch.optim.Adam(capturable=True) keeps it): *step += 1 on the stream, then
 * the update with the bias corrections formed on the device from the new count
 * (in double, rounded to float: the values stgcn_adam_step forms on the host).
 * No host value changes between steps, so the launch can be captured once in a
 * HIP graph and replayed every training step (train_ops.FusedAdam
 * (capturable=True), train_ops.GraphedStep). Replaces the host-step launch of
 * stgcn_adam_step (torch optim/adam.py _multi_tensor_adam, capturable branch). */
int stgcn_adam_step_dev(const void *dev_table, int ntensors, int64_t total_chunks, double lr,
                        double beta1, double beta2, double eps, double weight_decay, float *step,
                        void *stream);

#ifdef __cplusplus
}
#endif
#endif /* STGCN_HIP_H */

// Internal kernel-launch interface of libstgcn_hip.so (not part of the C-ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ab_switches.h"

namespace stgcn {

// Fused dropout (st_graphconv.py:53-58, :107-109): element e of the block
// output is kept iff hash(seed, e) >= thresh (thresh = p * 2^32) and then
// scaled by 1/(1-p). thresh == 0: no dropout. The hash (splitmix64 of
// seed + e * golden ratio) is counter-based: the backward regenerates the
// mask instead of storing it.
struct Dropout {
  uint64_t seed = 0;
  uint32_t thresh = 0;
  float scale = 1.f;
};

__host__ __device__ inline bool dropout_keep(const Dropout &d, uint64_t e) {
  uint64_t z = d.seed + e * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (uint32_t)(z >> 32) >= d.thresh;
}

// Deferred-dx chain (ABI 5; capi.hip "deferred dx"): the spatial backward of
// block i reads the PREVIOUS block's pre-BN2 tensor U in place of its input x
// and rebuilds x = ReLU((U - mean) * invstd * g + b) exactly as that block's
// output pass did; with the mask m = x > 0 and uhat = (U - mean) * invstd it
// adds s1[c] += sum m * dxhat, s2[c] += sum m * dxhat * uhat (fp64). mean ==
// nullptr: off (x read as is).
struct PrevBn {
  const float *mean = nullptr, *invstd = nullptr, *g = nullptr, *b = nullptr;
  double *s1 = nullptr, *s2 = nullptr;
};

// f16x2 operand bounds: kAmaxSlots words kAmaxStride apart per bound
// (device_common.h block_amax / amax_read)
constexpr int kAmaxSlots = 64, kAmaxStride = 32, kAmaxWords = kAmaxSlots * kAmaxStride;

constexpr int kTileRows = 64;   // output rows per workgroup (2 MFMA 32-row tiles)
constexpr int kTileCols = 256;  // max (frames x V) columns per workgroup (8 MFMA 32-col tiles)

// Generic temporal-conv-shaped GEMM on MFMA (v_mfma_f32_32x32x2_f32):
//   out[n, r, s_out*m + p_out, v] = bias_r[r] + bias_rv[r, v]
//        + sum_{c<C} sum_{q<NQ} w[r*w_sr + c*w_sc + q*w_sq] * in[n, c, s_in*m + q + off, v]
// with in[] zero outside [0, T_src). Covers: the spatial W GEMM (NQ=1), the
// (9,1) temporal conv forward (NQ=9), its data-gradient (flipped taps; stride-2
// split into two phases, NQ=5/4) and the spatial H = W^T dZ GEMM (NQ=1).
struct ConvGemmParams {
  const float *in, *w;
  float *wpk;            // workspace for the packed weights (conv_gemm_wpk_floats)
  float *out;
  const float *bias_r;   // [R] or null
  const float *bias_rv;  // [R][V] or null
  double *stat_sum, *stat_sq;  // [R] per-row sum / sum of squares, or null
  // (k_conv_x3's row-major epilogue: per-tile partials [2][R][n * n_mtiles + mt]
  // written with plain stores instead of the stat_sum / stat_sq atomics --
  // launch_bn_finalize_parts reduces them; deterministic, and no fp64 atomics
  // whose latency ends every tile)
  double *stat_part;
  int64_t in_bstride, out_bstride;  // elements per clip
  int64_t w_sr, w_sc, w_sq;
  int C, R, NQ;
  int s_in, off, s_out, p_out;
  int M;      // logical output frames
  int T_src;  // input frames
  int T_dst;  // output physical frames
  int V, FT;  // joints; frames per tile (FT*V <= kTileCols)
  int n_mtiles, n_rtiles, N;
  int Cpad;  // set by launch_conv_gemm
  // epilogue extras (residual block): out = f(acc + bias + res), f = ReLU if relu_out
  const float *res;  // same layout and clip stride as out, or null
  int res_shared;    // 1: res has no clip axis (one [R][T_dst][V] table for every clip:
                     // the folded block's per-frame bias table, capi.hip fold_w)
  int relu_out;
  Dropout drop;      // applied after relu_out (element index = flat index in out)
  int bf16;          // 1: operands rounded to bf16 on v_mfma_f32_32x32x16_bf16 (fp32
                     // accumulate, fp32 in/out), where k_conv_bf16 covers the shape;
                     // 3: fp32 GEMM as exact 3-way bf16 splits (k_conv_x3) where covered
  int in_bf16;       // in[] holds bf16 (same element strides; k_conv_x3 one-plane only)
  int out_bf16;      // out[] is written as bf16 (same element strides; the shared
                     // epilogues; no residual input)
  // f16x2 (with bf16 == 3): the fp32 GEMM as 2-way fp16 splits (k_conv_x3
  // NPL = 2, three products) of power-of-two-scaled operands; amax_in / amax_w:
  // device words holding max |in| / max |w| as float bits (f16x2_scale)
  int f16x2;
  const unsigned *amax_in, *amax_w;
  unsigned *amax_keep;  // (or null) block 0 copies *amax_in there (the kept G's bound)
  // spb (the folded block's data gradient, V = 18, K = 1; kernels_x3.hip
  // spb_epilogue): the tile holds H = W'^T dZ (rows = input channels). Instead of
  // storing H the epilogue forms dxhat = H A (stored to out, null: not stored),
  // the BN1 backward sums sd / sdn (and, prev.mean set, the deferred-dx chain's
  // s1 / s2 over the previous block's U read from sx) and dA += H^T BN1(x):
  // the SpatialConv backward never round-trips H through HBM.
  int spb;
  int sd_given;  // sd already holds sum dxhat (launch_fold_small_sd): the epilogue adds only sdn
  const float *sx, *sA, *mean1, *invstd1, *g1, *b1;
  PrevBn prev;
  double *sd, *sdn;
  float *dA;
  // dA_part (non-null): the workgroup's dA partial (V*V floats, summed in a fixed
  // order) is stored at dA_part[blockIdx.x * V * V] instead of added to dA with
  // fp32 atomics; launch_dA_reduce then adds the partials to dA in launch order
  // (run-to-run deterministic dA)
  float *dA_part;
  // wpk already holds the packed split planes of w (stgcn_fold_prep): no pack launch
  int wpk_ready;
  // bna (with f16x2, V = 18, the folded block's forward; kernels_x3.hip): in[] is
  // the block input x, BN1 (mean1, invstd1, g1, b1) is applied in the window
  // loader and the joint contraction with sA in the epilogue -- G is never formed;
  // amax_in holds max |x| (the fp16 operand bound is formed in the kernel)
  int bna;
  // w4 (the fp16-split stride-1 forward; kernels_x3.hip x3_w4): 4-wave 64-row
  // tiles, two workgroups per CU. Set by the caller where it packs AND where it
  // launches (capi.hip fwd_w4), so the weight layout and the kernel agree
  int w4;
};

// Weight-gradient GEMM with split-K partial slabs:
//   slab[split, r, c*NQ + q] = sum_{(n, m-tile) in split} sum_{m, v}
//        P[n, r, m, v] * Q[n, c, s_in*m + q + off, v]
struct WgradParams {
  const float *P, *Q;
  float *slab;
  int64_t p_bstride, q_bstride;
  int R, C, NQ, s_in, off;
  int M;      // frames of P
  int T_src;  // frames of Q
  int V, FT;
  int n_mtiles, n_rtiles, n_jtiles, S, N;
  int CT;  // k_wgrad_sp (NQ = 1): output columns per workgroup (64 or 128)
  int bf16;  // set by plan_wgrad_bf16: run k_wgrad_bf16 (bf16 operands, fp32 accumulate);
             // 3: set by plan_wgrad_x3 (fp32 via exact bf16 splits, k_wgrad_x3)
  int p_bf16, q_bf16;  // P / Q hold bf16 (same element strides; k_wgrad_bf16 only)
  // f16x2 (with bf16 == 3): k_wgrad_x3 on 2-way fp16 splits (NPL = 2) of the
  // power-of-two-scaled P / Q; amax_p / amax_q: device max |P| / max |Q| bits
  int f16x2;
  const unsigned *amax_p, *amax_q;
  // (f16x2 only) Q is the block input x of the folded block: BN1 (q_mean,
  // q_invstd, q_g, q_b) is applied while staging Q (0 in padded frames), amax_q
  // holds max |x|; P is dU contracted with A (dU A), so the product is dWc
  const float *q_mean, *q_invstd, *q_g, *q_b;
  int x3_mr;  // k_wgrad_x3 row tiles of 64 x_mr rows (2: with f16x2 only; set by plan_wgrad_x3)
};

hipError_t launch_conv_gemm(const ConvGemmParams &p, hipStream_t s);
// amax[0] = max(amax[0], max |x[i]|) as float bits (x of n floats; amax zeroed
// by the caller): the operand bound of the fp16-split GEMMs (f16x2)
hipError_t launch_absmax(const float *x, int64_t n, unsigned *amax, hipStream_t s);
// The folded block (kernels_fold.hip; capi.hip fold_w): composite weights
// Wc[o][i][q] = sum_c Wt[o][c][q] W'[c][i], the per-frame bias table, the dU
// sums (total, boundary frames, per tap Tq) and the weight gradients from dWc.
// (scratch: fold_fwd_scratch_floats / fold_bwd_scratch_floats of padded
// operand re-layouts; dwc: fold_dwc_floats)
size_t fold_fwd_scratch_floats(int R, int C, int V);
size_t fold_bwd_scratch_floats(int R, int C);
size_t fold_sdz_scratch_doubles(int R, int C, int V);
size_t fold_dwc_floats(int R, int C);
hipError_t launch_fold_w(const float *Wt, const float *W, int R, int C, float *Wc, float *scratch,
                         hipStream_t s);
hipError_t launch_fold_fwd(const float *Wt, const float *W, const float *bt, const float *bZ, int R,
                           int C, int V, int T, int To, int st, float *Wc, double *bq, float *BT,
                           float *scratch, hipStream_t s);
hipError_t launch_fold_prep_bwd(const float *Wt, const float *W, int R, int C, float *scratch,
                                hipStream_t s);
// Tq (and, tqT non-null, its fp64 re-layout in launch_fold_sdz's scratch:
// fold_sdz_tq_slot) from the clip-chunk sums
hipError_t launch_fold_tq(const double *cs, int nz, int R, int T, int To, int V, int st,
                          double *Tq, double *tqT, hipStream_t s);
double *fold_sdz_tq_slot(double *scratch, int R, int C);
// SdZ = sum_{n,t} dZ and (Wc, SdH non-null) SdH = sum_{n,t} H from Tq, fp64
// (pre: the scratch already holds the Wt / Wc re-layouts, launch_fold_prep;
// tqT: where launch_fold_tq wrote Tq's re-layout, default the scratch's slot --
// with pre the caller's own workspace, so the shared weight-only prep buffer
// never holds step data)
hipError_t launch_fold_sdz(double *scratch, const float *Wt, const float *Wc, const double *Tq,
                           int R, int C, int V, double *SdZ, double *SdH, hipStream_t s,
                           bool pre = false, const double *tqT = nullptr);
// BN1's sd (db1) of the folded block from SdH: sd[c] = sum_v SdH[c][v] rowsum(A)[v]
// launch_spatial_small (K = 1) and BN1's sd of the folded block (from SdH) in one launch
hipError_t launch_fold_small_sd(const double *SdZ, const float *A, const float *bW, int R, int V,
                                float *dbW, float *dA, const double *SdH, int C, double *sd,
                                hipStream_t s);
// The weight-only operands of several folded blocks, formed together once per
// training step (capi.hip stgcn_fold_prep): bZ = bW rowsum(A), Wc = Wt W', the
// bias table BT, max |Wc|, and the re-layouts the backward's small GEMMs read
// (fscr_b: launch_fold_prep_bwd's; f64: launch_fold_sdz's Wt / Wc parts)
struct FoldPrepSpec {
  const float *A, *W, *bW, *Wt, *bWt;
  int R, C, V, T, To, stride;
  float *bZ, *Wc, *BT, *fscr_f, *fscr_b;
  double *bq, *f64;
  unsigned *amax;
};
hipError_t launch_fold_prep(const FoldPrepSpec *specs, int n, hipStream_t s);
hipError_t launch_fold_grads(const float *slab, int S, const float *scratch, const float *bZ,
                             const double *Tq, int R, int C, int V, float *dwc, float *dWt,
                             float *dW, hipStream_t s);
// k_bn_relu_bwd_apply that also writes the clip-chunk sums of dU,
// cs[z][C][L] for z < apply_cols_chunks(N) (kernels.hip)
int apply_cols_chunks(int N);
hipError_t launch_bn_relu_bwd_apply_cols(const float *dy, const float *U, const float *mean,
                                         const float *invstd, const float *g, const float *b,
                                         const double *sg, const double *sgu, float *dU,
                                         double *sdu, int N, int C, int L, int training,
                                         Dropout drop, hipStream_t s, int du_bf16,
                                         const float *dy_coef, double *cs,
                                         unsigned *amax = nullptr, const float *dync = nullptr);
// ... frame-wise (V = 18), also writing dUA = dU A (the folded block without G,
// capi.hip fold_bna) and the fp16 operand bounds max |dU| (amax), max |dUA| (amaxa)
hipError_t launch_bn_relu_bwd_apply_fr(const float *dy, const float *U, const float *mean,
                                       const float *invstd, const float *g, const float *b,
                                       const double *sg, const double *sgu, float *dU, float *dUA,
                                       double *sdu, int N, int C, int To, int V, int training,
                                       Dropout drop, const float *dy_coef, double *cs,
                                       unsigned *amax, unsigned *amaxa, const float *A,
                                       hipStream_t s);
// bf16 path (kernels_bf16.hip): the reference's graphs (V = 18, 25, 50) with
// the fp32 path's tile plan (FT = kTileCols / V); launch_conv_gemm dispatches here
// when p.bf16 and conv_bf16_supported(p).
bool conv_bf16_supported(const ConvGemmParams &p);
size_t conv_bf16_lds_bytes(const ConvGemmParams &p);
hipError_t launch_conv_bf16(const ConvGemmParams &p, hipStream_t s);
// fp32 via exact bf16 splits (kernels_x3.hip): stride-1 temporal conv forward /
// data-grad (NQ = 9, 5, 4) for V = 18, 25 over >= 16 channels; launch_conv_gemm
// dispatches here when p.bf16 == 3 and conv_x3_supported(p).
bool conv_x3_supported(const ConvGemmParams &p);
// The weight pack of k_conv_x3 (split planes [row tile][chunk][tap group][plane]
// [tap][octet][rows][8]) as a job, so several tensors pack in one launch
// (stgcn_fold_prep); conv_x3_pack_bytes: its size (npl: 3 bf16 / 2 fp16 planes)
constexpr int kPackJobs = 16;
struct PackJob {
  const float *w;
  void *wpk;
  int R, C, NQ, TG, nch, rows, npl;
  int64_t w_sr, w_sc, w_sq, total;
  const unsigned *amax_w;
};
PackJob conv_x3_pack_job(const ConvGemmParams &p, int npl);
size_t conv_x3_pack_bytes(const ConvGemmParams &p, int npl);
hipError_t launch_pack_jobs(const PackJob *jobs, int n, hipStream_t s);
// the bna forward's extra LDS (BN1 table of C channels + A rows) fits
bool conv_x3_bna_supported(const ConvGemmParams &p);
size_t conv_x3_wpk_bytes(const ConvGemmParams &p);
hipError_t launch_conv_x3(const ConvGemmParams &p, hipStream_t s);
// bf16 temporal-conv GEMMs on the one-plane k_conv_x3 pipeline (kernels_x3.hip)
bool conv_b1_supported(const ConvGemmParams &p);
hipError_t launch_conv_b1(const ConvGemmParams &p, hipStream_t s);
// Re-plans the temporal weight gradient (NQ = 9, stride 1, V = 18) for
// k_wgrad_x3 (sets FT, tiles, S, bf16 = 3); false (w unchanged) otherwise.
// launch_wgrad_taps dispatches to launch_wgrad_x3 when w.bf16 == 3.
bool plan_wgrad_x3(WgradParams &w, bool f16x2);
hipError_t launch_wgrad_x3(const WgradParams &p, hipStream_t s);
// Re-plans a weight gradient (NQ = 9 temporal taps or NQ = 1) for k_wgrad_bf16
// (sets FT, n_mtiles, n_rtiles, n_jtiles, S, bf16 = 1) when the shape is
// covered; returns false (w unchanged) otherwise. launch_wgrad / launch_wgrad_taps
// dispatch to launch_wgrad_bf16 when w.bf16.
bool plan_wgrad_bf16(WgradParams &w);
hipError_t launch_wgrad_bf16(const WgradParams &p, hipStream_t s);
hipError_t launch_wgrad(const WgradParams &p, hipStream_t s);
// Plan of the NQ = 1 weight gradient (plain split-K GEMM over (n, t*V) chunks of
// wgrad_sp_kc(CT) columns): sets CT, n_rtiles, n_jtiles, n_mtiles (chunks per
// clip), S. Requires s_in = 1, off = 0, M = T_src.
void plan_wgrad_sp(WgradParams &p);
bool wgrad_sp_applies(const WgradParams &p);
inline int wgrad_sp_kc(int CT) { return CT == 64 ? 64 : 32; }
// Temporal-conv weight gradient (NQ = 9) with taps-inner tiles; n_jtiles
// counts channel blocks of wgrad_taps_cb(p) channels. Slab = (R, C, 9).
hipError_t launch_wgrad_taps(const WgradParams &p, hipStream_t s);
int wgrad_taps_cb(const WgradParams &p);
size_t wgrad_taps_lds_bytes(const WgradParams &p);
bool wgrad_taps_supported(const WgradParams &p);
size_t conv_gemm_lds_bytes(const ConvGemmParams &p);
size_t conv_gemm_wpk_floats(const ConvGemmParams &p);
bool conv_gemm_supported(const ConvGemmParams &p);
size_t wgrad_lds_bytes(const WgradParams &p);
bool wgrad_supported(const WgradParams &p);
int wgrad_ntiles_j(int C, int NQ);

// Reduction of split-K slabs: dst = sum_s slab[s]. mode 0: identity layout;
// mode 1: slab is [R][K*C] (packed W'), dst is the (K*R, C) Conv2d weight.
hipError_t launch_slab_reduce(const float *slab, int S, int64_t n, float *dst, int mode,
                              int R, int K, int C, hipStream_t s);

// BatchNorm helpers (fp64 accumulation of per-channel sums).
// (amax, or null: max |x| as float bits, device_common.h block_amax)
hipError_t launch_bn_stats(const float *x, int N, int C, int L, double *sum, double *sq,
                           hipStream_t s, unsigned *amax = nullptr);
hipError_t launch_bn_finalize(const double *sum, const double *sq, int C, int64_t M,
                              float eps, float momentum, int training, float *rm, float *rv,
                              float *mean_out, float *invstd_out, hipStream_t s, unsigned *zw = nullptr,
                              int nzw = 0);
// y = ReLU(BN(U)); ysum/ysq (or null): per-channel sum / sum of squares of y;
// yext (or null, 3*C: [cnt | su | xu]): with the ReLU mask m = y > 0 and
// uhat = (U - mean) * invstd, cnt += sum m, su += sum m * uhat, xu += sum y * uhat
// (the deferred-dx chain's forward sums)
// ymax (or null): max y as float bits (block_amax): the next block's operand bound
hipError_t launch_bn_relu_fwd(const float *U, const float *mean, const float *invstd,
                              const float *g, const float *b, float *y, int N, int C, int L,
                              double *ysum, double *ysq, Dropout drop, hipStream_t s,
                              double *yext = nullptr, unsigned *ymax = nullptr);
hipError_t launch_bn_relu_bwd_reduce(const float *dy, const float *U, const float *mean,
                                     const float *invstd, const float *g, const float *b,
                                     int N, int C, int L, double *sg, double *sgu, Dropout drop,
                                     hipStream_t s, const float *dync = nullptr);
hipError_t launch_bn_relu_bwd_apply(const float *dy, const float *U, const float *mean,
                                    const float *invstd, const float *g, const float *b,
                                    const double *sg, const double *sgu, float *dU,
                                    double *sdu, int N, int C, int L, int training,
                                    Dropout drop, hipStream_t s, int du_bf16 = 0,
                                    const float *dy_coef = nullptr, const float *dync = nullptr);
// (dync non-null, ABI 10 stgcn_bwd_args_t.dy_nc: dy[n, c, :] == dync[n * C + c];
// the three ReLU + BN2 backward passes then read no dy tensor)
// Deferred-dx chain: block i's BN1 backward folded into block i-1's ReLU+BN2
// backward. dy_coef (5*C: [a | md | mu | is | mdn], launch_chain_coef) makes
// launch_bn_relu_bwd_apply read dy as the next block's dxhat and form
//   dy = a * (dxhat - md - (y - mu) * is * mdn),  y = ReLU((U - mean) * invstd * g + b)
// (k_bn1_bwd_apply's arithmetic) instead of reading a materialised dy.
// launch_chain_coef (block i, C = its C_in): from its BN1 sums sd / sdn, its BN1
// statistics (mean1, invstd1, g1), the prev-mode sums s1 / s2 of its spatial
// backward and xst (5*C: the previous block's output sums [sum | sumsq | cnt |
// su | xu]) -> dg1 = sdn, db1 = sd, coef (5*C) and psum (2*C: the previous
// block's [sum m dy | sum m dy uhat]). M = N*T*V.
hipError_t launch_chain_coef(const double *sd, const double *sdn, const float *mean1,
                             const float *invstd1, const float *g1, const double *s1,
                             const double *s2, const double *xst, int C, int64_t M,
                             float *dg1, float *db1, float *coef, double *psum, hipStream_t s);
hipError_t launch_bn_grads_out(const double *sg, const double *sgu, const double *sdu, int C,
                               float *dgamma, float *dbeta, float *dbias, hipStream_t s);
// add (same layout as dx, or null) is added after the BN1 backward (residual path)
// training = 0: eval-mode BatchNorm backward (running statistics are constants)
// pg2/pb2/psum (or null): also the previous block's ReLU+BN2 backward sums;
// pU/pmean/pinvstd (or null): that block's pre-BN2 tensor and statistics, read
// for channels where uhat = (x - b2) / g2 is ill-conditioned
hipError_t launch_bn1_bwd_apply(float *dx, const float *x, const float *mean,
                                const float *invstd, const float *g, const double *sd,
                                const double *sdn, const float *add, int N, int C, int L,
                                int64_t M, int training, const float *pg2, const float *pb2,
                                double *psum, const float *pU, const float *pmean,
                                const float *pinvstd, hipStream_t s);
// dout = dy * (y > 0) (the final ReLU of the residual block), sum[c] += sum dout
// (with dropout: y is the dropped output; dout = dy * scale where y > 0)
hipError_t launch_relu_bwd(const float *dy, const float *y, float *dout, double *sum, int N,
                           int C, int L, float scale, hipStream_t s);

// Spatial (graph) helpers.
hipError_t launch_pack_w(const float *W, float *Wpk, int K, int R, int C, hipStream_t s);
hipError_t launch_bias_rv(const float *A, const float *bW, float *bias_rv, int K, int R, int V,
                          hipStream_t s);
// G = f(BN1(x)) A^T with f = identity, or ReLU when relu != 0 (residual block)
// amax (or null): max |G| as float bits (atomicMax; zeroed by the caller), the
// f16x2 operand bound of the folded temporal GEMMs
// BN statistics from per-tile partials [2][C][ntiles] (ConvGemmParams.stat_part):
// one workgroup per channel, fixed summation order
hipError_t launch_bn_finalize_parts(const double *part, int ntiles, int C, int64_t M, float eps,
                                    float momentum, int training, float *rm, float *rv,
                                    float *mean_out, float *invstd_out, hipStream_t s,
                                    double *ys_zero = nullptr, int nw = 0);
hipError_t launch_gather_fwd(const float *x, const float *mean, const float *invstd,
                             const float *g, const float *b, const float *A, float *G, int N,
                             int C, int T, int V, int K, int relu, hipStream_t s,
                             unsigned *amax = nullptr, const PrevBn *pv = nullptr);
// pv (x = ReLU(BN2_prev(U)) from the previous block's U, ABI 8) runs on
// k_gather4 only: K = 1, 16-byte aligned x / G and these shapes
bool gather_prev_supported(int C, int T, int V);
hipError_t launch_sum_nt(const float *X, int N, int C, int T, int V, double *out,
                         hipStream_t s, int x_bf16 = 0);
hipError_t launch_spatial_small(const double *SdZ, const float *A, const float *bW, int K,
                                int R, int V, float *dbW, float *dA, hipStream_t s);
hipError_t launch_spatial_dx(const float *H, const float *x, const float *mean,
                             const float *invstd, const float *g, const float *b,
                             const float *A, float *dx, float *dA, double *sd, double *sdn,
                             int N, int C, int T, int V, int K, int write_dx, int relu,
                             int bf16ops, hipStream_t s, const PrevBn *prev = nullptr,
                             float *dA_part = nullptr, int64_t part_cap = 0,
                             int64_t *nparts = nullptr);
int conv_x3_tile_rows(const ConvGemmParams &p, int npl);
// Deterministic dA: adds nparts partials part[i][n] (i in order) to dA[n], in two
// fixed-order passes (lvl: kDaLvl * n doubles of scratch)
constexpr int kDaLvl = 64;
hipError_t launch_dA_reduce(const float *part, int64_t nparts, int n, double *lvl, float *dA,
                            hipStream_t s);
// launch_spatial_dx takes a PrevBn for this shape (its k_spatial_bwd5 / _bwd6
// paths; 16-byte aligned tensors assumed, as torch allocates them)
bool spatial_dx_prev_supported(int N, int C, int T, int V, int K);

// Fused spatial graph convolution of the bf16 path (kernels_fused.hip):
// Z = W' (f(BN1(x)) A^T) + biasZ in one kernel (BN1 + joint contraction on MFMA
// with A in LDS + W' GEMM; G never materialised in fp32). Optionally keeps G in
// bf16 (Gk, layout [n][k*C + ci][frame tile][256]) for the weight gradient.
bool sp_fwd_bf16_supported(int C, int V, int K, int R, bool residual);
size_t sp_fwd_bf16_wpk_bytes(int C, int R, int K, int V);  // packed W' + A image
size_t sp_keep_g_bytes(int N, int C, int T, int V, int K);
hipError_t launch_sp_fwd_bf16(const float *x, const float *mean, const float *invstd,
                              const float *g, const float *b, const float *A, const float *W,
                              const float *biasZ, void *wpk, float *Z, int z_bf16, __bf16 *Gk,
                              double *ssum,
                              double *ssq, int N, int C, int R, int T, int V, int K, int relu,
                              hipStream_t s, const PrevBn *prev = nullptr);
// dW' = dZ Gk^T from the kept bf16 G (P = dZ fp32, Q = Gk, C = K*C_in).
void plan_wgrad_gk(WgradParams &w, int T);
hipError_t launch_wgrad_gk(const WgradParams &p, hipStream_t s);

// Fused SpatialConv backward of the bf16 path (kernels_spbwd.hip): from dZ to
// dx (BN1 input side, before the BN1 backward apply), dA += sum H_k^T f(BN1(x))
// and the BN1 backward sums, H = W'^T dZ never in HBM. wpk: scratch of
// sp_bwd_fused_wpk_bytes (packed W' + the A image).
// x3: the fp32 path of STGCN_F_F32X3 (exact bf16 splits) instead of the bf16 path
bool sp_bwd_fused_supported(int C, int V, int K, int R, int T, bool x3);
size_t sp_bwd_fused_wpk_bytes(int C, int R, int K, int V);
hipError_t launch_sp_bwd_fused(const float *dZ, const float *x, const float *mean,
                               const float *invstd, const float *g, const float *b,
                               const float *A, const float *W, void *wpk, float *dx, float *dA,
                               double *sd, double *sdn, int N, int C, int R, int T, int V, int K,
                               int write_dx, int relu, bool x3, hipStream_t s,
                               const PrevBn *prev = nullptr, int dz_bf16 = 0, int only = 0);
// V = 50 runs the fused backward as two kernels (k_sp50_dx, k_sp50_dA); only = 1 / 2
// launches just the first / second of them (timing entry point), 0 both.

}  // namespace stgcn

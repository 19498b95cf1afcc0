// C-ABI entry points of libstgcn_hip.so (declared in include/stgcn_hip.h).
//
// stgcn_block_fwd / stgcn_block_bwd enqueue the kernel sequence of one
// ST-GCN block on the caller's stream. The reference op order of the default
// (non-residual) block
// (st_graphconv.py:97-109, :148-150) is
//     BN1 -> Y = W x + b -> Z = sum_k Y_k A_k^T -> Conv9x1 -> BN2 -> ReLU;
// here the joint contraction is applied on the narrower (input-channel) side,
//     Z = sum_k W_k (BN1(x) A_k^T) + (sum_k b_k rowsum(A_k))          (1)
// which is the same linear map (exact in real arithmetic) and never
// materialises the K*C_out-channel Y. The residual block (st_graphconv.py:60-82)
// reuses the same kernels: ReLU folded into the joint contraction's BN1
// input, BN2 statistics from the spatial GEMM epilogue, and the residual add +
// final ReLU in the temporal conv's epilogue.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/stgcn_hip.h"
#include "internal.h"

using namespace stgcn;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg) {
  g_err = msg;
  return code;
}

}  // namespace

namespace stgcn {
void set_last_error(const std::string &msg) { g_err = msg; }
}  // namespace stgcn

namespace {

#define HIP_TRY(expr)                                                                      \
  do {                                                                                     \
    hipError_t e_ = (expr);                                                                \
    if (e_ != hipSuccess)                                                                  \
      return fail(STGCN_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));        \
  } while (0)

size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }
// bytes of a y_stats / x_stats block (ABI 7): 5 * C doubles of sums, then the
// max |y| words (block_amax slots)
size_t y_stats_bytes(int C) {
  return sizeof(double) * 5 * C + sizeof(unsigned) * STGCN_STATS_AMAX_WORDS;
}
static_assert(STGCN_STATS_AMAX_WORDS == kAmaxWords, "ABI 7: the amax block of y_stats");

// Frames per conv tile: as many whole frames as fit 256 columns.
int conv_ft(int V) { return std::max(1, kTileCols / V); }
// Frames per wgrad work item: as many whole frames as fit 80 columns.
int wgrad_ft(int V) { return std::max(1, 80 / V); }

// Upper bound of the packed-weight scratch any conv_gemm launch of this block needs.
size_t wpk_floats(const stgcn_desc_t *d) {
  const int rows = std::max(d->C_out, d->K * d->C_in);  // (stacked H GEMM: K*C_in rows)
  const int red = std::max(d->C_out, d->K * d->C_in);
  // reduction padded to a whole number of chunks for any chunk size <= 32
  size_t n = (size_t)((rows + 63) / 64 * 64) * ((red + 31) / 32 * 32 + 32) * 9;
  // STGCN_F_F32X3: three bf16 planes of the weights (1.5x the fp32 floats)
  if (d->flags & STGCN_F_F32X3) n *= 2;
  // the fused bf16 spatial forward: packed W' + the A image
  if (d->flags & STGCN_F_BF16)
    n = std::max(n, (sp_fwd_bf16_wpk_bytes(d->C_in, d->C_out, d->K, d->V) + 3) / 4);
  // the fused spatial backward: packed W' planes + its A image
  if (d->flags & (STGCN_F_BF16 | STGCN_F_F32X3))
    n = std::max(n, (sp_bwd_fused_wpk_bytes(d->C_in, d->C_out, d->K, d->V) + 3) / 4);
  return n;
}

int64_t nT(const stgcn_desc_t *d) { return (int64_t)d->T * d->V; }
int64_t nTo(const stgcn_desc_t *d) { return (int64_t)d->T_out * d->V; }
bool residual(const stgcn_desc_t *d) { return (d->flags & STGCN_F_RESIDUAL) != 0; }
bool bf16(const stgcn_desc_t *d) { return (d->flags & STGCN_F_BF16) != 0; }
bool f32x3(const stgcn_desc_t *d) { return (d->flags & STGCN_F_F32X3) != 0; }
bool f16x2_flag(const stgcn_desc_t *d) { return (d->flags & STGCN_F_F16X2) != 0; }
// the fused dropout of a call (training and 0 < p < 1; p >= 1: everything dropped)
Dropout make_dropout(const stgcn_desc_t *d, float p, uint64_t seed) {
  Dropout dr;
  if (!d->training || !(p > 0.f)) return dr;
  dr.seed = seed;
  const double t = (double)p * 4294967296.0;
  dr.thresh = t >= 4294967295.0 ? 0xffffffffu : (uint32_t)t;
  dr.scale = p < 1.f ? (float)(1.0 / (1.0 - (double)p)) : 0.f;
  return dr;
}
// the fused spatial forward (kernels_fused.hip) of the bf16 path applies
// (STGCN_AB_UNFUSED_SP build: the unfused gather + GEMM kernels, A/B measurement only)
bool fused_sp(const stgcn_desc_t *d) {
  constexpr bool off = STGCN_AB_UNFUSED_SP != 0;
  return !off && bf16(d) && sp_fwd_bf16_supported(d->C_in, d->V, d->K, d->C_out, residual(d));
}
// the fused spatial backward (kernels_spbwd.hip) applies: bf16 path, or the fp32
// split path (STGCN_AB_UNFUSED_SPB build: the H GEMM + k_spatial_bwd5/6 pair, A/B only)
bool fused_spb(const stgcn_desc_t *d) {
  constexpr bool off = STGCN_AB_UNFUSED_SPB != 0;
  return !off && (bf16(d) || f32x3(d)) &&
         sp_bwd_fused_supported(d->C_in, d->V, d->K, d->C_out, d->T, f32x3(d));
}
// the fused backward of the two-person graph: two kernels (k_sp50_dx, k_sp50_dA),
// timed apart as which 5 / 6
bool fused_spb50(const stgcn_desc_t *d) { return fused_spb(d) && d->V == 50; }
// The folded block (kernels_fold.hip): with one adjacency partition the
// SpatialConv channel GEMM W' folds into the temporal conv's weights
// (Wc_q = Wt_q W'), so the temporal conv reads G = BN1(x) A^T (C_in channels)
// and Z / dZ are never formed; the backward's data gradient yields H directly.
// fp32 split path, K = 1: V = 18 (cfg2) and V = 25 (the reference's default
// L_STGCN graph: NTU joints, unilabeling partition, lightning_model.py:271),
// non-residual blocks over >= 16 input and output channels (the data gradient
// reduces over C_out: k_conv_x3 needs >= 16 there) (STGCN_AB_NO_FOLD build: the
// unfolded kernels, A/B only).
bool fold_w(const stgcn_desc_t *d) {
  constexpr bool off = STGCN_AB_NO_FOLD != 0;
  return !off && f32x3(d) && !residual(d) && d->K == 1 && d->C_in >= 16 && d->C_out >= 16 &&
         (d->V == 18 || d->V == 25) && !fused_spb(d);
}
// The folded block's SpatialConv backward inside its data gradient (kernels_x3.hip
// spb_epilogue, V = 18): dxhat = H A, dA, the BN1 / chain sums from the tile
// while H is on chip. V = 25 (and the STGCN_AB_SPB_PAIR build): the data gradient
// stores H and the unfused spatial backward (k_spatial_bwd5) reads it.
bool fold_spb(const stgcn_desc_t *d) {
  return fold_w(d) && d->V == 18 && STGCN_AB_SPB_PAIR == 0;
}

// The folded block's temporal GEMMs on 2-way fp16 splits (STGCN_F_F16X2; k_conv_x3 /
// k_wgrad_x3 with NPL = 2), operand scales from max |x| words (launch_absmax)
bool f16x2(const stgcn_desc_t *d) { return fold_w(d) && f16x2_flag(d); }
// ... and the unfolded K = 1 split block (the first block: C_in < 16) with its
// temporal conv forward and weight gradient on fp16 splits: max |Z| by a pass
// over Z, kept after G for the backward;
// its data gradient stays on the 3-way splits (it feeds BN1's nearly cancelling sums)
bool f16x2_unfold(const stgcn_desc_t *d) {
  return f16x2_flag(d) && f32x3(d) && !fold_w(d) && !residual(d) && d->K == 1 && d->V == 18 &&
         d->C_out >= 16;
}
// the temporal forward / weight gradient on fp16 splits (folded or not)
bool f16x2_tw(const stgcn_desc_t *d) { return f16x2(d) || f16x2_unfold(d); }
// ... the data gradient included: its output feeds BN1's sum of dxhat over N T V
// elements of a zero-mean dU (heavy cancellation; the 2^-22 operand
// representation measured 2.5x the fp32 reference's own error on the BN1 bias
// gradient at N = 32, T = 300), which the folded block takes from the fp64 dU
// sums instead (kernels_fold.hip k_fold_sd). STGCN_AB_F16X2_DGRAD=0 build: the
// 3-way bf16 splits there (A/B only).
// (only where BN1's sum comes from the fp64 dU sums: the fused backward, fold_spb)
bool f16x2_dgrad(const stgcn_desc_t *d) {
  return f16x2(d) && fold_spb(d) && STGCN_AB_F16X2_DGRAD != 0;
}
// ... and G never formed (north star N1; kernels_x3.hip bna_contract): the
// forward GEMM reads x, applies BN1 in its window loader and the joint
// contraction with A in its epilogue (U = A U' + BT), the weight gradient reads
// x (BN1 at staging) against dU A (written by the ReLU + BN2 backward apply
// pass), so the gather kernel and G's HBM round trips are gone
// Opt-in (STGCN_F_NO_G, the memory-lean mode: G is not kept between forward and
// backward): measured 4% slower per cfg2 step than forming G once with k_gather4
//  -- the joint contraction then runs on the VALU inside
// latency-bound GEMM kernels instead of inside an HBM-bound pass.
bool fold_bna(const stgcn_desc_t *d);
// The fp16-split stride-1 temporal forward (folded, or the unfolded first
// block) on 4-wave 64-row tiles, two workgroups per CU (kernels_x3.hip x3_w4):
// marks the GEMM's parameters wherever its weights are packed or it is launched
bool fwd_w4(const stgcn_desc_t *d) {
  return d->stride == 1 && ((f16x2(d) && !fold_bna(d)) || f16x2_unfold(d));
}
bool fold_bna(const stgcn_desc_t *d) {
  if (!f16x2(d) || !(d->flags & STGCN_F_NO_G)) return false;
  ConvGemmParams p{};
  p.V = d->V;
  p.FT = conv_ft(d->V);
  p.NQ = 9;
  p.C = d->C_in;
  p.R = d->C_out;
  p.s_in = d->stride;
  p.s_out = 1;
  return conv_x3_bna_supported(p);
}
// ABI 8 (STGCN_PLAN_X_FROM_U): the training forward of a folded block that forms
// G (k_gather4) can read its input as ReLU(BN2_prev(U_prev)) of the previous
// block -- that block then writes only y's statistics, not y -- and its fused
// backward (spb_epilogue, deferred dx) already reads U_prev in place of x
// The bf16 blocks (cfg3 / cfg5) too (verdict r5 item 4): their fused spatial
// forward (k_sp_fwd_bf16 / k_sp_fwd_wide) forms ReLU(BN2_prev(U_prev)) on
// staging, and their spatial backward (k_sp_bwd_fused, k_sp50_*, or the H GEMM
// + joint kernel) reads U_prev in prev mode wherever dx defers; the weight
// gradient of W' reads the kept bf16 G -- so x is read by nothing.
bool x_from_u(const stgcn_desc_t *d) {
  if (!d->training || residual(d)) return false;
  if (fused_sp(d))
    return fused_spb(d) || spatial_dx_prev_supported(d->N, d->C_in, d->T, d->V, d->K);
  return fold_spb(d) && !fold_bna(d) && d->K == 1 && gather_prev_supported(d->C_in, d->T, d->V);
}

// sum_{n,t} dZ of the non-residual block from per-tap sums of dU (clip-chunk
// sums written by the ReLU + BN2 backward apply, k_fold_tq, one small GEMM with
// Wt) instead of a pass over dZ (the folded block has no dZ at all): cfg3 5632
// vs 5604, cfg5 2658 vs 2631 clips/s in one A/B call (STGCN_AB_SUM_NT build:
// the pass over dZ on unfolded blocks, A/B only).
bool cols_sums(const stgcn_desc_t *d) {
  return !residual(d) && (fold_w(d) || STGCN_AB_SUM_NT == 0);
}
// The folded forward leaves Wc in the (otherwise unused) Z buffer for the
// backward when it fits (Z is opaque to the caller under STGCN_F_F32X3 then)
bool fold_wc_in_z(const stgcn_desc_t *d) {
  return fold_w(d) && (int64_t)d->N * d->C_out * d->T * d->V >= (int64_t)d->C_out * d->C_in * 9;
}
// Clips per slice of the unfused spatial backward (H GEMM + joint kernel). The
// shipped build runs the whole batch as one slice. STGCN_AB_SLICE build (A/B
// only): the slice's H, dZ, x and dx (fp32) within ~160 MiB, so the Infinity
// Cache (256 MiB; MI355X_MICROARCH.md) could serve H's read-back -- measured
// SLOWER in one A/B call (round 3: cfg5 2126 vs 2324, cfg2 4182 vs 4432 clips/s):
// the persistent joint kernels (k_spatial_bwd5/6) flush their dA accumulators
// and BN1 sums once per launch, so 16 launches per layer (8-clip slices at cfg5)
// multiply that tail and underfill the grid.
int spatial_bwd_slice(const stgcn_desc_t *d) {
  constexpr bool on = STGCN_AB_SLICE != 0;
  if (!on) return d->N;
  const int64_t per_clip =
      (int64_t)4 * d->T * d->V * ((int64_t)d->K * d->C_in + d->C_out + 2 * d->C_in);
  const int64_t budget = (int64_t)160 << 20;
  const int ns = (int)std::max<int64_t>(8, budget / std::max<int64_t>(per_clip, 1));
  return std::min(ns, d->N);
}
// residual block with a 1x1 projection (apply_residual Conv2d, st_graphconv.py:27)
bool projection(const stgcn_desc_t *d) {
  return residual(d) && (d->C_in != d->C_out || d->stride != 1);
}

struct Carve {
  char *base;
  size_t off = 0;
  explicit Carve(void *b) : base((char *)b) {}
  template <class T>
  T *take(size_t count) {
    T *p = base ? (T *)(base + off) : nullptr;
    off += align_up(count * sizeof(T));
    return p;
  }
};

int wgrad_splits(int tiles, int items) {
  int S = (512 + tiles - 1) / tiles;
  return std::max(1, std::min(S, items));
}

WgradParams make_wgrad(const stgcn_desc_t *d, const float *P, int64_t pb, int R, int Mframes,
                       const float *Q, int64_t qb, int C, int T_src, int NQ, int s_in, int off,
                       float *slab) {
  WgradParams w{};
  w.P = P;
  w.Q = Q;
  w.slab = slab;
  w.p_bstride = pb;
  w.q_bstride = qb;
  w.R = R;
  w.C = C;
  w.NQ = NQ;
  w.s_in = s_in;
  w.off = off;
  w.M = Mframes;
  w.T_src = T_src;
  w.V = d->V;
  w.FT = wgrad_ft(d->V);
  while (w.FT > 1 && wgrad_lds_bytes(w) > 80 * 1024) --w.FT;  // 2 workgroups per CU
  w.n_mtiles = (Mframes + w.FT - 1) / w.FT;
  w.n_rtiles = (R + 63) / 64;
  w.n_jtiles = wgrad_ntiles_j(C, NQ);
  w.N = d->N;
  w.S = wgrad_splits(w.n_rtiles * w.n_jtiles, d->N * w.n_mtiles);
  if (wgrad_sp_applies(w)) plan_wgrad_sp(w);
  if (bf16(d)) plan_wgrad_bf16(w);  // k_wgrad_bf16 where it covers the shape
  // fp32 path of STGCN_F_F32X3: the spatial dW' on exact bf16 splits (k_wgrad_sp<.., X3>)
  if (f32x3(d) && wgrad_sp_applies(w) && !STGCN_AB_WSP_F32) w.bf16 = 3;
  return w;
}

// Temporal-conv weight gradient plan (k_wgrad_taps): dWt = sum dU (x) Z(shifted).
// (Cq: channels of the Q operand, C_out; C_in for the folded block's dWc = sum dU G^T)
WgradParams make_wgrad_taps(const stgcn_desc_t *d, const float *dU, const float *Z,
                            float *slab, int Cq = 0) {
  const int R = d->C_out;
  if (Cq <= 0) Cq = R;
  WgradParams w{};
  w.P = dU;
  w.Q = Z;
  w.slab = slab;
  w.p_bstride = (int64_t)R * d->T_out * d->V;
  w.q_bstride = (int64_t)Cq * d->T * d->V;
  w.R = R;
  w.C = Cq;
  w.NQ = 9;
  w.s_in = d->stride;
  w.off = -d->pad;
  w.M = d->T_out;
  w.T_src = d->T;
  w.V = d->V;
  w.N = d->N;
  w.FT = std::max(1, 80 / d->V);
  while (w.FT > 1 && !wgrad_taps_supported(w)) --w.FT;
  w.n_mtiles = (w.M + w.FT - 1) / w.FT;
  w.n_rtiles = (R + 63) / 64;
  w.n_jtiles = (Cq + wgrad_taps_cb(w) - 1) / wgrad_taps_cb(w);
  const int tiles = w.n_rtiles * w.n_jtiles;
  w.S = std::max(1, std::min((256 + tiles - 1) / tiles, d->N * w.n_mtiles));
  if (bf16(d)) plan_wgrad_bf16(w);
  // k_wgrad_x3 where it covers the shape (its S x R x C x 9 slab fits the fp32
  // plan's: twice the tiles, half the splits)
  if (f32x3(d)) plan_wgrad_x3(w, f16x2_tw(d));
  return w;
}

struct BwdLayout {
  double *sg, *sgu, *sdu, *sd, *sdn, *SdZ;
  double *s1, *s2;  // deferred-dx chain: the prev-mode sums of the spatial backward
  unsigned *amax;
  float *dU, *dZ, *G, *H, *slab, *wpk;
  float *Wpk;  // W' = [W_0 | ... | W_{K-1}] (C_out, K*C_in) for the stacked H GEMM
  float *Rg;  // residual projection data-grad (N, C_in, T, V)
  // the folded block: dU summed over clips, per-tap sums Tq, dWc, partials, Wc, bZ
  double *fcs, *ftq, *f64scr, *SdH;
  float *dWc, *fscr;  // the fold GEMMs' operand re-layouts (kernels_fold.hip)
  float *Wc, *bZ;
  // deterministic dA: the spatial backward's per-workgroup partials (dA_cap
  // slots of K V V floats) and the reduction's fp64 scratch
  float *dApart;
  double *dAlvl;
  int64_t dA_cap;
  size_t dbl_bytes, total;
};

// Partial slots the block's dA-producing launches need (0: fp32 atomics stay):
// the folded data gradient's workgroups (spb_epilogue; both stride-2 phases,
// counted at 64-row tiles: an upper bound), or the unfused spatial backward's
// joint kernel -- persistent k_spatial_bwd5 (<= 2048 workgroups) / _bwd6 (two
// slots per workgroup, <= 512), or the flat-row k_spatial_bwd3 (>= 64 rows per
// workgroup). (The fused bf16 spatial backward kernels keep their atomics.)
static int64_t dA_part_cap(const stgcn_desc_t *d) {
  const int64_t N = d->N, C = d->C_in, T = d->T;
  if (fold_spb(d)) {
    const int FT = conv_ft(d->V);
    const int64_t mt = d->stride == 1 ? (T + FT - 1) / FT
                                      : ((T + 1) / 2 + FT - 1) / FT + (T / 2 + FT - 1) / FT;
    return N * mt * ((C + 63) / 64);
  }
  if (fused_spb(d)) return 0;
  const int64_t bwd3 = C < 16 ? (N * C * T + 63) / 64 : 0;
  return std::max<int64_t>(d->V == 50 ? 512 : 2048, bwd3);
}

BwdLayout bwd_layout(const stgcn_desc_t *d, void *ws) {
  Carve c(ws);
  BwdLayout L{};
  const int R = d->C_out, C = d->C_in, K = d->K;
  L.sg = c.take<double>(R);
  L.sgu = c.take<double>(R);
  L.sdu = c.take<double>(R);
  L.sd = c.take<double>(C);
  L.sdn = c.take<double>(C);
  L.SdZ = c.take<double>((size_t)R * d->V);
  L.s1 = c.take<double>(C);
  L.s2 = c.take<double>(C);
  // f16x2: max |dU|, |Wc|, |G| (bna: |dU A|), |x| (bna without a kept bound); zeroed with the sums
  L.amax = c.take<unsigned>(4 * kAmaxWords);
  L.dbl_bytes = c.off;
  if (!residual(d)) {  // clip-chunk sums of dU -> Tq -> sum_{n,t} dZ (kernels_fold.hip)
    L.fcs = c.take<double>((size_t)apply_cols_chunks(d->N) * R * nTo(d));
    L.ftq = c.take<double>((size_t)9 * R * d->V);
    L.f64scr = c.take<double>(fold_sdz_scratch_doubles(R, C, d->V));
  }
  if (fold_w(d)) {
    L.dWc = c.take<float>(fold_dwc_floats(R, C));
    L.fscr = c.take<float>(std::max(fold_bwd_scratch_floats(R, C),
                                    fold_fwd_scratch_floats(R, C, d->V)));
    L.SdH = c.take<double>((size_t)C * d->V);
    L.Wc = c.take<float>((size_t)R * C * 9);
    L.bZ = c.take<float>((size_t)R * d->V);
  }
  L.dU = c.take<float>((size_t)d->N * R * nTo(d));
  L.dZ = c.take<float>((size_t)d->N * R * nT(d));
  L.G = c.take<float>((size_t)d->N * K * C * nT(d));
  L.H = c.take<float>((size_t)d->N * K * C * nT(d));
  WgradParams w1 = make_wgrad_taps(d, nullptr, nullptr, nullptr);
  WgradParams w2 =
      make_wgrad(d, nullptr, 0, R, d->T, nullptr, 0, K * C, d->T, 1, 1, 0, nullptr);
  size_t slab = std::max((size_t)w1.S * R * R * 9, (size_t)w2.S * R * K * C);
  if (fold_w(d)) {
    WgradParams wf = make_wgrad_taps(d, nullptr, nullptr, nullptr, C);
    slab = std::max(slab, (size_t)wf.S * R * C * 9);
  }
  if (fused_sp(d)) {  // dW' from the kept bf16 G (k_wgrad_gemm_gk)
    WgradParams wg{};
    wg.R = R;
    wg.C = K * C;
    wg.V = d->V;
    wg.N = d->N;
    plan_wgrad_gk(wg, d->T);
    slab = std::max(slab, (size_t)wg.S * R * K * C);
  }
  if (projection(d)) {
    WgradParams w3 = make_wgrad(d, nullptr, 0, R, d->T_out, nullptr, 0, C, d->T, 1, d->stride, 0,
                                nullptr);
    slab = std::max(slab, (size_t)w3.S * R * C);
    if (d->need_dx) L.Rg = c.take<float>((size_t)d->N * C * nT(d));
  }
  L.slab = c.take<float>(slab);
  L.wpk = c.take<float>(wpk_floats(d));
  L.Wpk = c.take<float>((size_t)R * K * C);
  L.dA_cap = dA_part_cap(d);
  if (L.dA_cap) {
    const size_t kvv = (size_t)K * d->V * d->V;
    L.dApart = c.take<float>((size_t)L.dA_cap * kvv);
    L.dAlvl = c.take<double>((size_t)kDaLvl * kvv);
  }
  L.total = c.off;
  return L;
}

struct FwdLayout {
  double *s1, *q1, *s2, *q2;
  unsigned *amax;  // f16x2: max |G|, |Wc|
  float *G, *Wpk, *biasZ, *wpk;
  float *Rp;  // residual projection output (N, C_out, T_out, V)
  float *Wc, *BT;  // the folded block: composite weights, per-frame bias table
  double *bq;      // ... and its per-tap bias products
  float *fscr;     // ... and its GEMM operand re-layouts
  double *s2part;  // ... and its BN2 statistics per GEMM tile [2][C_out][N * n_mtiles]
  size_t dbl_bytes, total;
};

ConvGemmParams fold_fwd_wparams(const stgcn_desc_t *d, const float *Wc);
// The folded training forward's BN2 statistics as per-tile partials
// (k_conv_x3's row-major epilogue; ConvGemmParams.stat_part)
bool fold_stat_parts(const stgcn_desc_t *d) {
  return fold_w(d) && d->training && conv_x3_supported(fold_fwd_wparams(d, nullptr));
}

int fold_stat_tiles(const stgcn_desc_t *d) {
  return d->N * ((d->T_out + conv_ft(d->V) - 1) / conv_ft(d->V));
}

FwdLayout fwd_layout(const stgcn_desc_t *d, void *ws) {
  Carve c(ws);
  FwdLayout L{};
  const int R = d->C_out, C = d->C_in, K = d->K;
  L.s1 = c.take<double>(C);
  L.q1 = c.take<double>(C);
  L.s2 = c.take<double>(R);
  L.q2 = c.take<double>(R);
  L.amax = c.take<unsigned>(2 * kAmaxWords);  // f16x2: max |G|, |Wc|
  L.dbl_bytes = c.off;
  L.G = c.take<float>((size_t)d->N * K * C * nT(d));
  L.Wpk = c.take<float>((size_t)R * K * C);
  L.biasZ = c.take<float>((size_t)R * d->V);
  L.wpk = c.take<float>(wpk_floats(d));
  if (projection(d)) L.Rp = c.take<float>((size_t)d->N * R * nTo(d));
  if (fold_w(d)) {
    L.Wc = c.take<float>((size_t)R * C * 9);
    L.BT = c.take<float>((size_t)R * nTo(d));
    L.bq = c.take<double>((size_t)9 * R * d->V);
    L.fscr = c.take<float>(fold_fwd_scratch_floats(R, C, d->V));
    if (d->training) L.s2part = c.take<double>((size_t)fold_stat_tiles(d) * 2 * R);
  }
  L.total = c.off;
  return L;
}

ConvGemmParams conv_base(const stgcn_desc_t *d, float *wpk) {
  ConvGemmParams p{};
  p.wpk = wpk;
  p.V = d->V;
  p.FT = conv_ft(d->V);
  p.N = d->N;
  p.bf16 = bf16(d) ? 1 : (f32x3(d) ? 3 : 0);
  return p;
}

void conv_tiles(ConvGemmParams &p) {
  p.n_mtiles = (p.M + p.FT - 1) / p.FT;
  p.n_rtiles = (p.R + kTileRows - 1) / kTileRows;
}

// The weight operand fields of the folded block's temporal GEMMs (Wc [R][C][9])
// -- everything the split-plane pack reads (conv_x3_pack_job): the forward
// (R = C_out rows over C_in), and the data gradient's launch `ph` (flipped taps;
// stride 2: phase 0 taps 8, 6, .., 0 and phase 1 taps 7, .., 1)
ConvGemmParams fold_fwd_wparams(const stgcn_desc_t *d, const float *Wc) {
  ConvGemmParams p = conv_base(d, nullptr);
  p.w = Wc;
  p.w_sr = (int64_t)d->C_in * 9;
  p.w_sc = 9;
  p.w_sq = 1;
  p.C = d->C_in;
  p.R = d->C_out;
  p.NQ = 9;
  p.s_in = d->stride;
  p.s_out = 1;
  p.w4 = fwd_w4(d) ? 1 : 0;
  return p;
}
ConvGemmParams fold_dgrad_wparams(const stgcn_desc_t *d, const float *Wc, int ph) {
  ConvGemmParams p = conv_base(d, nullptr);
  p.w_sr = 9;
  p.w_sc = (int64_t)d->C_in * 9;
  p.C = d->C_out;
  p.R = d->C_in;
  p.s_in = 1;
  if (d->stride == 1) {
    p.w = Wc + 8;
    p.w_sq = -1;
    p.NQ = 9;
    p.s_out = 1;
  } else {
    p.w = Wc + (ph == 0 ? 8 : 7);
    p.w_sq = -2;
    p.NQ = ph == 0 ? 5 : 4;
    p.s_out = 2;
  }
  return p;
}
int fold_fwd_npl(const stgcn_desc_t *d) { return f16x2(d) ? 2 : 3; }
int fold_dgrad_npl(const stgcn_desc_t *d) { return f16x2_dgrad(d) ? 2 : 3; }

// A folded block's stgcn_fold_prep buffer (ABI 7)
struct PrepLayout {
  float *bZ, *Wc, *BT, *fscr_f, *fscr_b;
  double *bq, *f64;
  unsigned *amax;  // max |Wc| (kAmaxWords, every slot written)
  char *wpk_f, *wpk_d[2];
  size_t total;
};

PrepLayout prep_layout(const stgcn_desc_t *d, const void *base) {
  Carve c(const_cast<void *>(base));
  PrepLayout P{};
  const int R = d->C_out, C = d->C_in, V = d->V;
  P.amax = c.take<unsigned>(kAmaxWords);
  P.bq = c.take<double>((size_t)9 * R * V);
  P.f64 = c.take<double>(fold_sdz_scratch_doubles(R, C, V));
  P.bZ = c.take<float>((size_t)R * V);
  P.Wc = c.take<float>((size_t)R * C * 9);
  P.BT = c.take<float>((size_t)R * nTo(d));
  P.fscr_f = c.take<float>(fold_fwd_scratch_floats(R, C, V));
  P.fscr_b = c.take<float>(fold_bwd_scratch_floats(R, C));
  P.wpk_f = c.take<char>(conv_x3_pack_bytes(fold_fwd_wparams(d, nullptr), fold_fwd_npl(d)));
  for (int ph = 0; ph < (d->stride == 1 ? 1 : 2); ++ph)
    P.wpk_d[ph] =
        c.take<char>(conv_x3_pack_bytes(fold_dgrad_wparams(d, nullptr, ph), fold_dgrad_npl(d)));
  P.total = c.off;
  return P;
}
// (the block takes a prep buffer: folded, with split-plane forward and data gradient)
bool prep_applies(const stgcn_desc_t *d) {
  if (!fold_w(d)) return false;
  if (!conv_x3_supported(fold_fwd_wparams(d, nullptr))) return false;
  for (int ph = 0; ph < (d->stride == 1 ? 1 : 2); ++ph)
    if (!conv_x3_supported(fold_dgrad_wparams(d, nullptr, ph))) return false;
  return true;
}

// Activations stored in bf16 on the bf16 path's non-residual blocks: Z (the
// SpatialConv output) and dU (the gradient at the temporal conv output). Every
// reader of them rounds them to bf16 anyway -- Z: the temporal conv forward
// (k_conv_x3 one-plane) and the weight gradient's Q (k_wgrad_bf16); dU: the
// data gradient (k_conv_x3 one-plane, stride-2 phases included) and the weight
// gradient's P -- so the results are bit-identical to fp32 storage and half
// the bytes move; the bias / BN gradients use the fp32 sums of the producing
// passes. The tensors keep their fp32-sized buffers (the first half holds the
// bf16 data). Producers: the fused spatial forward's epilogues (so C_in >= 16)
// and the BN2 + ReLU backward pass. (STGCN_AB_ACT_FP32 build: fp32 storage, A/B only)
bool act_bf16(const stgcn_desc_t *d) {
  constexpr bool off = STGCN_AB_ACT_FP32 != 0 || STGCN_AB_GENERIC_CONV != 0;
  // Stride-2 blocks at odd V keep fp32: their weight gradient (k_wgrad_bf16<9,V,2>)
  // staged bf16 pairs by registers slower than fp32 (cfg5 2.19 -> 2.66 ms per
  // step), more than the strided forward and data-gradient phases gained; at even
  // V it stages them by LDS-DMA (STGCN_AB_S2_ACT_FP32 build: fp32 there, A/B only).
  const bool s2 = d->stride == 2 && d->V % 2 == 0 && STGCN_AB_S2_ACT_FP32 == 0;
  if (off || !fused_sp(d) || residual(d) || (d->stride != 1 && !s2)) return false;
  ConvGemmParams p = conv_base(d, nullptr);  // the temporal conv forward and data gradient
  p.C = d->C_out;
  p.R = d->C_out;
  p.NQ = 9;
  p.s_in = d->stride;
  if (!conv_b1_supported(p)) return false;
  WgradParams w = make_wgrad_taps(d, nullptr, nullptr, nullptr);
  return w.bf16 == 1;
}
bool z_bf16(const stgcn_desc_t *d) { return act_bf16(d); }
bool du_bf16(const stgcn_desc_t *d) { return act_bf16(d); }

// dZ (the gradient at the SpatialConv output) stored in bf16 on the bf16 path's
// non-residual blocks whose dW' reads the kept bf16 G: its readers round dZ to
// bf16 anyway (k_sp_bwd_fused's H GEMM operand -- or, unfused, the H GEMM
// k_conv_bf16<1, .., IB> -- and k_wgrad_gemm_gk's P operand), so they see the
// same values at half the bytes (and the fused kernel's ring is 6 chunks deep
// instead of 4); the remaining reader, the bias-type sums sum_{n,t} dZ
// (k_sum_nt4_bf16), accumulates the bf16 values in fp64. Producer: the temporal
// data-gradient (one-plane k_conv_x3, bf16 epilogue store). The buffer keeps
// its fp32 size.
// Not the shipped default: measured in one A/B call (round 3) fp32 dZ ran cfg3
// 5415 vs 5285 and cfg5 2137 vs 2126 clips/s, so bf16 dZ is the STGCN_AB_DZ_BF16
// build only (A/B measurement).
bool dz_bf16(const stgcn_desc_t *d) {
  constexpr bool on = STGCN_AB_DZ_BF16 != 0;
  if (!on || !bf16(d) || residual(d) || !fused_sp(d)) return false;
  if (fused_spb(d) && d->V == 50) return false;  // (k_sp50_dx / _dA read fp32 dZ)
  if (!fused_spb(d)) {  // the unfused spatial backward: its H GEMM reads dZ (k_conv_bf16<.., IB>)
    ConvGemmParams h = conv_base(d, nullptr);
    h.C = d->C_out;
    h.R = d->K * d->C_in;
    h.NQ = 1;
    h.s_in = 1;
    if (!conv_bf16_supported(h)) return false;
  }
  ConvGemmParams p = conv_base(d, nullptr);  // the data gradient's launch(es)
  p.C = d->C_out;
  p.R = d->C_out;
  p.s_in = 1;
  p.NQ = d->stride == 1 ? 9 : 5;
  if (!conv_b1_supported(p)) return false;
  p.NQ = 4;
  return d->stride == 1 || conv_b1_supported(p);
}

}  // namespace

// Every GEMM launch of the block fits its LDS budget.
static bool geometry_supported(const stgcn_desc_t *d) {
  const int R = d->C_out, C = d->C_in, K = d->K;
  WgradParams w1 = make_wgrad_taps(d, nullptr, nullptr, nullptr);
  WgradParams w2 = make_wgrad(d, nullptr, 0, R, d->T, nullptr, 0, K * C, d->T, 1, 1, 0, nullptr);
  if (!(w1.bf16 || wgrad_taps_supported(w1)) || !(w2.bf16 || wgrad_supported(w2))) return false;
  ConvGemmParams p = conv_base(d, nullptr);
  p.NQ = 9;
  p.s_in = d->stride;
  p.R = R;
  p.C = R;
  if (!conv_gemm_supported(p)) return false;
  p.NQ = 1;
  p.s_in = 1;
  if (!conv_gemm_supported(p)) return false;
  if (projection(d)) {
    p.s_in = d->stride;  // the strided 1x1 projection
    p.R = R;
    p.C = C;
    WgradParams w3 = make_wgrad(d, nullptr, 0, R, d->T_out, nullptr, 0, C, d->T, 1, d->stride, 0,
                                nullptr);
    if (!conv_gemm_supported(p) || !(w3.bf16 || wgrad_sp_applies(w3) || wgrad_supported(w3)))
      return false;
  }
  return true;
}

// Residual block after the spatial conv (st_graphconv.py:75-80, :105):
//   Za = ReLU(BN2(Z)); y = ReLU(Conv9x1(Za) + bt + R(x)),
// R = x (identity) or Wr x + br with temporal stride (projection).
static int residual_fwd_tail(const stgcn_desc_t *d, const stgcn_fwd_args_t *a,
                             const FwdLayout &L, hipStream_t s) {
  const int N = d->N, C = d->C_in, R = d->C_out, T = d->T, To = d->T_out, V = d->V;
  float *mean2 = a->stats + 2 * C, *invstd2 = a->stats + 2 * C + R;
  HIP_TRY(launch_bn_finalize(L.s2, L.q2, R, (int64_t)N * T * V, d->eps, d->momentum,
                             d->training, a->rm2, a->rv2, mean2, invstd2, s));
  HIP_TRY(launch_bn_relu_fwd(a->Z, mean2, invstd2, a->g2, a->b2, a->Za, N, R, T * V, nullptr,
                             nullptr, Dropout(), s));
  const float *resid = a->x;
  if (projection(d)) {  // apply_residual: Conv2d(C_in, C_out, 1, stride (s,1)) (:27)
    ConvGemmParams p = conv_base(d, L.wpk);
    p.in = a->x;
    p.w = a->Wr;
    p.out = L.Rp;
    p.bias_r = a->br;
    p.in_bstride = (int64_t)C * T * V;
    p.out_bstride = (int64_t)R * To * V;
    p.w_sr = C;
    p.w_sc = 1;
    p.w_sq = 0;
    p.C = C;
    p.R = R;
    p.NQ = 1;
    p.s_in = d->stride;
    p.off = 0;
    p.s_out = 1;
    p.p_out = 0;
    p.M = To;
    p.T_src = T;
    p.T_dst = To;
    conv_tiles(p);
    HIP_TRY(launch_conv_gemm(p, s));
    resid = L.Rp;
  }
  ConvGemmParams p = conv_base(d, L.wpk);
  p.in = a->Za;
  p.w = a->Wt;
  p.out = a->y;
  p.bias_r = a->bWt;
  p.res = resid;
  p.relu_out = 1;
  p.drop = make_dropout(d, a->dropout_p, a->seed);
  if (d->training && a->y_stats) {  // next block's BN1 statistics from the epilogue
    HIP_TRY(hipMemsetAsync(a->y_stats, 0, y_stats_bytes(R), s));
    p.stat_sum = a->y_stats;
    p.stat_sq = a->y_stats + R;
  }
  p.in_bstride = (int64_t)R * T * V;
  p.out_bstride = (int64_t)R * To * V;
  p.w_sr = (int64_t)R * 9;
  p.w_sc = 9;
  p.w_sq = 1;
  p.C = R;
  p.R = R;
  p.NQ = 9;
  p.s_in = d->stride;
  p.off = -d->pad;
  p.s_out = 1;
  p.p_out = 0;
  p.M = To;
  p.T_src = T;
  p.T_dst = To;
  conv_tiles(p);
  HIP_TRY(launch_conv_gemm(p, s));
  if (d->training && a->y_stats)  // (ABI 7: max y after the sums, the next block's bound)
    HIP_TRY(launch_absmax(a->y, (int64_t)N * R * To * V,
                          reinterpret_cast<unsigned *>(a->y_stats + 5 * R), s));
  return STGCN_OK;
}

extern "C" {

int stgcn_abi_version(void) { return STGCN_ABI_VERSION; }

const char *stgcn_last_error(void) { return g_err.c_str(); }

static bool geometry_supported(const stgcn_desc_t *d);

int stgcn_check_desc(const stgcn_desc_t *d) {
  if (!d) return fail(STGCN_E_INVALID, "null descriptor");
  if (d->N <= 0 || d->C_in <= 0 || d->C_out <= 0 || d->T <= 0 || d->V <= 0 || d->K <= 0)
    return fail(STGCN_E_INVALID, "non-positive dimension");
  if ((d->flags & ~(STGCN_F_RESIDUAL | STGCN_F_BF16 | STGCN_F_F32X3 | STGCN_F_F16X2 |
                    STGCN_F_NO_G)) != 0)
    return fail(STGCN_E_UNSUPPORTED, "unknown flags");
  if ((d->flags & STGCN_F_NO_G) && !(d->flags & STGCN_F_F16X2))
    return fail(STGCN_E_INVALID, "STGCN_F_NO_G needs STGCN_F_F16X2");
  if ((d->flags & STGCN_F_BF16) && (d->flags & STGCN_F_F32X3))
    return fail(STGCN_E_INVALID, "STGCN_F_BF16 and STGCN_F_F32X3 are exclusive");
  if ((d->flags & STGCN_F_F16X2) && !(d->flags & STGCN_F_F32X3))
    return fail(STGCN_E_INVALID, "STGCN_F_F16X2 needs STGCN_F_F32X3");
  if (d->gamma != 9 || d->pad != 4)
    return fail(STGCN_E_UNSUPPORTED, "only gamma=9, pad=4 (the reference default)");
  if (d->stride != 1 && d->stride != 2) return fail(STGCN_E_UNSUPPORTED, "stride must be 1 or 2");
  if (d->T_out != (d->T + 2 * d->pad - d->gamma) / d->stride + 1)
    return fail(STGCN_E_INVALID, "T_out inconsistent with T, stride, pad");
  if (d->V > kTileCols) return fail(STGCN_E_UNSUPPORTED, "V > 256");
  if (d->K * d->V * d->V > 8192) return fail(STGCN_E_UNSUPPORTED, "K*V*V > 8192");
  if ((int64_t)d->N * d->K * d->C_in * d->T * d->V > INT32_MAX ||
      (int64_t)d->N * d->C_out * d->T * d->V > INT32_MAX)
    return fail(STGCN_E_UNSUPPORTED, "tensor too large for 32-bit element indexing");
  if (!geometry_supported(d))
    return fail(STGCN_E_UNSUPPORTED, "tile geometry exceeds LDS for this V / channel count");
  return STGCN_OK;
}

int stgcn_block_plan(const stgcn_desc_t *d, uint32_t *plan) {
  int rc = stgcn_check_desc(d);
  if (rc) return rc;
  if (!plan) return fail(STGCN_E_INVALID, "null plan pointer");
  uint32_t f = 0;
  if (fold_w(d)) f |= STGCN_PLAN_FOLD;
  if (fused_sp(d)) f |= STGCN_PLAN_SP_FWD_FUSED;
  if (fused_spb(d) || fold_spb(d)) f |= STGCN_PLAN_SP_BWD_FUSED;
  if (act_bf16(d)) f |= STGCN_PLAN_ACT_BF16;
  if (!fold_w(d) && !fused_sp(d)) {  // the spatial dW' GEMM of the unfolded block
    WgradParams w = make_wgrad(d, nullptr, 0, d->C_out, d->T, nullptr, 0, d->K * d->C_in, d->T,
                               1, 1, 0, nullptr);
    if (w.bf16 == 3) f |= STGCN_PLAN_WSP_SPLIT;
  }
  if (f32x3(d)) {
    ConvGemmParams p = conv_base(d, nullptr);  // the temporal conv forward (capi stgcn_block_fwd)
    p.C = fold_w(d) ? d->C_in : d->C_out;
    p.R = d->C_out;
    p.NQ = 9;
    p.s_in = d->stride;
    if (conv_x3_supported(p)) f |= STGCN_PLAN_TCONV_SPLIT;
    WgradParams w = make_wgrad_taps(d, nullptr, nullptr, nullptr, fold_w(d) ? d->C_in : 0);
    if (w.bf16 == 3) f |= STGCN_PLAN_TWGRAD_SPLIT;
  }
  if (f16x2_tw(d)) f |= STGCN_PLAN_F16X2;
  if (fold_bna(d)) f |= STGCN_PLAN_FOLD_NO_G;
  if (x_from_u(d)) f |= STGCN_PLAN_X_FROM_U;
  *plan = f;
  return STGCN_OK;
}

size_t stgcn_fwd_workspace_bytes(const stgcn_desc_t *d) {
  if (stgcn_check_desc(d) != STGCN_OK) return 0;
  return fwd_layout(d, nullptr).total;
}

size_t stgcn_keep_g_bytes(const stgcn_desc_t *d) {
  if (stgcn_check_desc(d) != STGCN_OK) return 0;
  if (fused_sp(d)) return sp_keep_g_bytes(d->N, d->C_in, d->T, d->V, d->K);
  // (no G: only the forward's max |x| for the backward's weight gradient)
  if (fold_bna(d)) return sizeof(unsigned) * kAmaxWords;
  // (f16x2: + one word after G, its max |G| for the backward's weight gradient)
  return sizeof(float) * (size_t)d->N * d->K * d->C_in * d->T * d->V +
         (f16x2_tw(d) ? sizeof(unsigned) * kAmaxWords : 0);
}

size_t stgcn_fold_prep_bytes(const stgcn_desc_t *d) {
  if (stgcn_check_desc(d) != STGCN_OK || !prep_applies(d)) return 0;
  return prep_layout(d, nullptr).total;
}

int stgcn_fold_prep(int nblocks, const stgcn_desc_t *descs, const stgcn_fold_weights_t *weights,
                    void *const *prep, void *stream) {
  if (nblocks < 0 || (nblocks > 0 && (!descs || !weights || !prep)))
    return fail(STGCN_E_INVALID, "null fold_prep argument");
  std::vector<FoldPrepSpec> sp;
  std::vector<PackJob> pk;
  for (int i = 0; i < nblocks; ++i) {
    const stgcn_desc_t *d = descs + i;
    int rc = stgcn_check_desc(d);
    if (rc) return rc;
    if (!prep_applies(d)) continue;  // (stgcn_fold_prep_bytes == 0: not a folded block)
    const stgcn_fold_weights_t &w = weights[i];
    if (!prep[i] || !w.A || !w.W || !w.bW || !w.Wt || !w.bWt)
      return fail(STGCN_E_INVALID, "null fold_prep weights / buffer of a folded block");
    const PrepLayout P = prep_layout(d, prep[i]);
    FoldPrepSpec b{};
    b.A = w.A;
    b.W = w.W;
    b.bW = w.bW;
    b.Wt = w.Wt;
    b.bWt = w.bWt;
    b.R = d->C_out;
    b.C = d->C_in;
    b.V = d->V;
    b.T = d->T;
    b.To = d->T_out;
    b.stride = d->stride;
    b.bZ = P.bZ;
    b.Wc = P.Wc;
    b.BT = P.BT;
    b.fscr_f = P.fscr_f;
    b.fscr_b = P.fscr_b;
    b.bq = P.bq;
    b.f64 = P.f64;
    b.amax = P.amax;
    sp.push_back(b);
    // the split-plane packs of the forward and data-gradient GEMMs (with max |Wc|)
    ConvGemmParams f = fold_fwd_wparams(d, P.Wc);
    f.wpk = reinterpret_cast<float *>(P.wpk_f);
    f.amax_w = P.amax;
    pk.push_back(conv_x3_pack_job(f, fold_fwd_npl(d)));
    for (int ph = 0; ph < (d->stride == 1 ? 1 : 2); ++ph) {
      ConvGemmParams g = fold_dgrad_wparams(d, P.Wc, ph);
      g.wpk = reinterpret_cast<float *>(P.wpk_d[ph]);
      g.amax_w = P.amax;
      pk.push_back(conv_x3_pack_job(g, fold_dgrad_npl(d)));
    }
  }
  if (sp.empty()) return STGCN_OK;
  hipStream_t s = (hipStream_t)stream;
  HIP_TRY(launch_fold_prep(sp.data(), (int)sp.size(), s));
  HIP_TRY(launch_pack_jobs(pk.data(), (int)pk.size(), s));
  return STGCN_OK;
}

size_t stgcn_bwd_workspace_bytes(const stgcn_desc_t *d) {
  if (stgcn_check_desc(d) != STGCN_OK) return 0;
  return bwd_layout(d, nullptr).total;
}

int stgcn_block_fwd(const stgcn_desc_t *d, const stgcn_fwd_args_t *a, void *workspace,
                    size_t workspace_bytes, void *stream) {
  int rc = stgcn_check_desc(d);
  if (rc) return rc;
  const bool res = residual(d);
  // ABI 8: x from the previous block's U (STGCN_PLAN_X_FROM_U); y null: statistics only
  const bool xu = a && a->prev_U;
  const bool ystats_only = a && !a->y && a->y_stats && d->training && !res && a->dropout_p == 0.f;
  // ABI 9: y and y_stats both null: no output pass (stgcn_head_fwd_u pools from U)
  const bool no_out = a && !a->y && !a->y_stats && d->training && !res && a->dropout_p == 0.f;
  if (!a || (!a->x && !xu) || !a->A || !a->W || !a->bW || !a->Wt || !a->bWt || !a->g1 ||
      !a->b1 || !a->g2 || !a->b2 || (!a->y && !ystats_only && !no_out) || !a->Z ||
      (!res && !a->U) ||
      !a->stats)
    return fail(STGCN_E_INVALID, "null tensor argument");
  if (res && (!a->Za || (projection(d) && (!a->Wr || !a->br))))
    return fail(STGCN_E_INVALID, "residual block: null Za / projection weights");
  if (!a->rm1 || !a->rv1 || !a->rm2 || !a->rv2)
    return fail(STGCN_E_INVALID, "null running-stat buffer");
  if (xu && (!x_from_u(d) || !a->x_stats || !a->prev_stats || !a->prev_g2 || !a->prev_b2 ||
             ((uintptr_t)a->prev_U & 15) != 0))
    return fail(STGCN_E_INVALID,
                "prev_U input: needs STGCN_PLAN_X_FROM_U, x_stats, prev_stats / prev_g2 / "
                "prev_b2 and a 16-byte aligned prev_U");
  const FwdLayout L = fwd_layout(d, workspace);
  if (!workspace || workspace_bytes < L.total)
    return fail(STGCN_E_INVALID, "workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const int N = d->N, C = d->C_in, R = d->C_out, T = d->T, To = d->T_out, V = d->V, K = d->K;
  float *mean1 = a->stats, *invstd1 = a->stats + C;
  float *mean2 = a->stats + 2 * C, *invstd2 = a->stats + 2 * C + R;

  // (folded training forward with the previous block's statistics: nothing in the
  // workspace's fp64 area accumulates -- BN2 goes to per-tile partials -- except
  // the f16x2 max |G| / |Wc| words, which the BN1 finalize zeroes: no memset)
  const bool stat_parts = fold_stat_parts(d) && L.s2part;
  const bool no_memset = stat_parts && a->x_stats;
  if (!no_memset) HIP_TRY(hipMemsetAsync(workspace, 0, L.dbl_bytes, s));
  // BN1 statistics of the block input (st_graphconv.py:98)
  // (the caller may hand over the previous block's y statistics: x_stats)
  const double *xs1 = L.s1, *xq1 = L.q1;
  const bool bna = fold_bna(d);
  const unsigned *xmax = L.amax;  // (bna: max |x|, the fp16 operand bound's input)
  if (d->training && a->x_stats) {
    xs1 = a->x_stats;
    xq1 = a->x_stats + C;
    xmax = reinterpret_cast<const unsigned *>(a->x_stats + 5 * C);  // (ABI 7: after the sums)
  } else if (d->training) {
    HIP_TRY(launch_bn_stats(a->x, N, C, T * V, L.s1, L.q1, s, bna ? L.amax : nullptr));
  } else if (bna) {
    HIP_TRY(launch_absmax(a->x, (int64_t)N * C * T * V, L.amax, s));
  }
  HIP_TRY(launch_bn_finalize(xs1, xq1, C, (int64_t)N * T * V, d->eps, d->momentum, d->training,
                             a->rm1, a->rv1, mean1, invstd1, s, no_memset ? L.amax : nullptr,
                             no_memset ? 2 * kAmaxWords : 0));
  // (the folded block: G only; W' rides on the temporal conv's weights)
  const bool fold = fold_w(d);
  // (ABI 7: the folded block's weight-only operands from stgcn_fold_prep)
  const bool pre = fold && a->prep && prep_applies(d);
  const PrepLayout P = pre ? prep_layout(d, a->prep) : PrepLayout{};
  // Spatial graph conv (st_graphconv.py:139-152) in the form (1).
  if (!pre) HIP_TRY(launch_bias_rv(a->A, a->bW, L.biasZ, K, R, V, s));
  const float *Gfold = nullptr;
  const float *Wz = a->W;
  if (K > 1) {
    HIP_TRY(launch_pack_w(a->W, L.Wpk, K, R, C, s));
    Wz = L.Wpk;
  }
  // (residual block: SpatialConv sees ReLU(BN1(x)), st_graphconv.py:72-74)
  if (fused_sp(d)) {
    // bf16 path: BN1 + joint contraction + W' GEMM in one kernel; G kept in bf16
    // for the backward when the caller asks (stgcn_keep_g_bytes)
    PrevBn pv;  // (x = ReLU(BN2_prev(prev_U)) formed on staging)
    if (xu) {
      pv.mean = a->prev_stats;
      pv.invstd = a->prev_stats + C;
      pv.g = a->prev_g2;
      pv.b = a->prev_b2;
    }
    HIP_TRY(launch_sp_fwd_bf16(xu ? a->prev_U : a->x, mean1, invstd1, a->g1, a->b1, a->A, a->W,
                               L.biasZ, L.wpk, a->Z, z_bf16(d) ? 1 : 0,
                               reinterpret_cast<__bf16 *>(a->G),
                               (res && d->training) ? L.s2 : nullptr,
                               (res && d->training) ? L.q2 : nullptr, N, C, R, T, V, K, res, s,
                               xu ? &pv : nullptr));
  } else if (!bna) {
  float *G = a->G ? a->G : L.G;  // kept for the backward when the caller asks
  PrevBn pv;  // (x = ReLU(BN2_prev(prev_U)) formed on load)
  if (xu) {
    pv.mean = a->prev_stats;
    pv.invstd = a->prev_stats + C;
    pv.g = a->prev_g2;
    pv.b = a->prev_b2;
  }
  HIP_TRY(launch_gather_fwd(xu ? a->prev_U : a->x, mean1, invstd1, a->g1, a->b1, a->A, G, N, C,
                            T, V, K, res, s, f16x2(d) ? L.amax : nullptr,  // (f16x2: max |G|)
                            xu ? &pv : nullptr));
  Gfold = G;
  if (!fold) {
    ConvGemmParams p = conv_base(d, L.wpk);
    p.in = G;
    p.w = Wz;
    p.out = a->Z;
    p.bias_rv = L.biasZ;
    if (res && d->training) {  // BN2 of the residual block normalizes Z (:76)
      p.stat_sum = L.s2;
      p.stat_sq = L.q2;
    }
    p.in_bstride = (int64_t)K * C * T * V;
    p.out_bstride = (int64_t)R * T * V;
    p.w_sr = (int64_t)K * C;
    p.w_sc = 1;
    p.w_sq = 0;
    p.C = K * C;
    p.R = R;
    p.NQ = 1;
    p.s_in = 1;
    p.off = 0;
    p.s_out = 1;
    p.p_out = 0;
    p.M = T;
    p.T_src = T;
    p.T_dst = T;
    conv_tiles(p);
    HIP_TRY(launch_conv_gemm(p, s));
    // (the unfolded fp16-split block: max |Z| for the temporal GEMMs' operand
    // scale, one pass over Z -- tracking it in the spatial GEMM's epilogue cost
    // that kernel 65 registers, half its occupancy)
    if (f16x2_unfold(d)) HIP_TRY(launch_absmax(a->Z, (int64_t)N * R * T * V, L.amax, s));
  }
  }
  if (res) return residual_fwd_tail(d, a, L, s);
  // Temporal (9,1) conv, stride (s,1), pad (4,0), bias (st_graphconv.py:41-43,99),
  // with the BN2 batch statistics accumulated in the epilogue.
  {
    ConvGemmParams p = conv_base(d, L.wpk);
    p.in = a->Z;
    p.in_bf16 = z_bf16(d) ? 1 : 0;
    p.w = a->Wt;
    p.out = a->U;
    p.bias_r = a->bWt;
    if (d->training) {
      p.stat_sum = L.s2;
      p.stat_sq = L.q2;
    }
    p.in_bstride = (int64_t)R * T * V;
    p.out_bstride = (int64_t)R * To * V;
    p.w_sr = (int64_t)R * 9;
    p.w_sc = 9;
    p.w_sq = 1;
    p.C = R;
    p.R = R;
    if (fold) {  // U = sum_q Wc_q G[s t + q - 4] + BT[o, t, v]  (kernels_fold.hip)
      float *Wc = fold_wc_in_z(d) ? a->Z : L.Wc;  // (kept for the backward)
      const float *BT = L.BT;
      const unsigned *amax_wc = L.amax + kAmaxWords;
      if (pre) {  // (formed for the whole stack by stgcn_fold_prep)
        Wc = P.Wc;
        BT = P.BT;
        amax_wc = P.amax;
        p.wpk = reinterpret_cast<float *>(P.wpk_f);
        p.wpk_ready = 1;
      } else {
        HIP_TRY(launch_fold_fwd(a->Wt, a->W, a->bWt, L.biasZ, R, C, V, T, To, d->stride, Wc, L.bq,
                                L.BT, L.fscr, s));
        if (f16x2(d)) HIP_TRY(launch_absmax(Wc, (int64_t)R * C * 9, L.amax + kAmaxWords, s));
      }
      if (f16x2(d)) {  // the fp16 splits' operand scales: max |G| (gather), max |Wc|
        p.f16x2 = 1;
        p.amax_in = L.amax;
        p.amax_w = amax_wc;
        if (a->G)  // (the kept G carries its bound to the backward)
          p.amax_keep = reinterpret_cast<unsigned *>(a->G + (size_t)N * C * T * V);
      }
      p.in = Gfold;
      p.res = BT;
      if (bna) {  // x in, BN1 in the loader, A in the epilogue (G never formed)
        p.in = a->x;
        p.bna = 1;
        p.amax_in = xmax;
        p.sA = a->A;
        p.mean1 = mean1;
        p.invstd1 = invstd1;
        p.g1 = a->g1;
        p.b1 = a->b1;
        // (the kept "G" buffer holds only max |x|, for the backward's weight gradient)
        p.amax_keep = a->G ? reinterpret_cast<unsigned *>(a->G) : nullptr;
      }
      p.w = Wc;
      p.bias_r = nullptr;
      p.res_shared = 1;
      p.in_bstride = (int64_t)C * T * V;
      p.w_sr = (int64_t)C * 9;
      p.C = C;
    } else if (f16x2_unfold(d)) {  // fp16 splits: max |Z| (spatial epilogue), max |Wt|
      HIP_TRY(launch_absmax(a->Wt, (int64_t)R * R * 9, L.amax + kAmaxWords, s));
      p.f16x2 = 1;
      p.amax_in = L.amax;
      p.amax_w = L.amax + kAmaxWords;
      if (a->G)  // (the kept G carries max |Z| to the backward's weight gradient)
        p.amax_keep = reinterpret_cast<unsigned *>(a->G + (size_t)N * K * C * T * V);
    }
    p.NQ = 9;
    p.s_in = d->stride;
    p.off = -d->pad;
    p.s_out = 1;
    p.p_out = 0;
    p.M = To;
    p.T_src = T;
    p.T_dst = To;
    p.w4 = fwd_w4(d) ? 1 : 0;
    conv_tiles(p);
    // (the folded forward on k_conv_x3: BN2 statistics as per-tile partials)
    if (stat_parts) p.stat_part = L.s2part;
    HIP_TRY(launch_conv_gemm(p, s));
  }
  // BN2 (st_graphconv.py:100) + ReLU (:105)
  double *ys = (d->training && a->y_stats) ? a->y_stats : nullptr;
  if (stat_parts)  // (zeroes y_stats on the way)
    HIP_TRY(launch_bn_finalize_parts(L.s2part, fold_stat_tiles(d), R, (int64_t)N * To * V, d->eps,
                                     d->momentum, d->training, a->rm2, a->rv2, mean2, invstd2, s,
                                     ys, kAmaxWords));
  else
    HIP_TRY(launch_bn_finalize(L.s2, L.q2, R, (int64_t)N * To * V, d->eps, d->momentum,
                               d->training, a->rm2, a->rv2, mean2, invstd2, s));
  const Dropout ydrop = make_dropout(d, a->dropout_p, a->seed);
  // (ABI 5: y_stats holds 5 * C_out sums; the last three -- over the ReLU mask --
  // feed the next block's deferred-dx chain, meaningless under dropout; ABI 7:
  // then max y in STGCN_STATS_AMAX_WORDS words, the next block's operand bound;
  // ABI 8, y null: only these -- k_bn_relu_stats; ABI 9, y and y_stats null:
  // nothing -- the consumer forms ReLU(BN2(U)) itself)
  if (!a->y && !ys) return STGCN_OK;
  if (ys && !stat_parts) HIP_TRY(hipMemsetAsync(ys, 0, y_stats_bytes(R), s));
  HIP_TRY(launch_bn_relu_fwd(a->U, mean2, invstd2, a->g2, a->b2, a->y, N, R, To * V, ys,
                             ys ? ys + R : nullptr, ydrop, s,
                             (ys && !ydrop.thresh) ? ys + 2 * R : nullptr,
                             ys ? reinterpret_cast<unsigned *>(ys + 5 * R) : nullptr));
  return STGCN_OK;
}

int stgcn_block_bwd(const stgcn_desc_t *d, const stgcn_bwd_args_t *a, void *workspace,
                    size_t workspace_bytes, void *stream) {
  int rc = stgcn_check_desc(d);
  if (rc) return rc;
  const bool res = residual(d);
  // ABI 8: x null after a forward from prev_U -- the fused folded backward (or the
  // bf16 spatial backward in prev mode) reads prev_U (deferred dx) and the kept
  // G, nothing else reads x
  const bool xnull = a && !a->x;
  if (xnull && (!x_from_u(d) || !a->G))
    return fail(STGCN_E_INVALID, "x null: needs STGCN_PLAN_X_FROM_U and the kept G");
  if (!a || (!a->dy && !a->dy_nc) || (!a->x && !xnull) || !a->Z || (!res && !a->U) || !a->stats || !a->A || !a->W ||
      !a->bW || !a->Wt || !a->g1 || !a->b1 || !a->g2 || !a->b2 || !a->dA || !a->dW || !a->dbW ||
      !a->dWt || !a->dbWt || !a->dg1 || !a->db1 || !a->dg2 || !a->db2 || (d->need_dx && !a->dx))
    return fail(STGCN_E_INVALID, "null tensor argument");
  if (res && (!a->Za || !a->y || (projection(d) && (!a->Wr || !a->dWr || !a->dbr))))
    return fail(STGCN_E_INVALID, "residual block: null Za / y / projection tensors");
  if (res && a->dy_sums)
    return fail(STGCN_E_INVALID, "dy_sums applies to the non-residual block only");
  // ABI 10: dy as one value per (clip, channel): the three ReLU + BN2 backward
  // passes of the non-residual block (not the residual block's ReLU backward, nor
  // the frame-wise dU A pass of the block without G)
  if (a->dy_nc && (res || (cols_sums(d) && fold_bna(d))))
    return fail(STGCN_E_UNSUPPORTED, "dy_nc: this block's backward needs the full dy");
  const Dropout drop = make_dropout(d, a->dropout_p, a->seed);
  if (drop.thresh && a->dy_sums)
    return fail(STGCN_E_INVALID, "dy_sums cannot be combined with dropout");
  if (!d->training && (a->dy_sums || a->prev_sums))
    return fail(STGCN_E_INVALID, "stack chaining applies to training mode only");
  if (a->dy_coef && (!a->dy_sums || res || drop.thresh))
    return fail(STGCN_E_INVALID, "dy_coef needs dy_sums, a non-residual block, no dropout");
  const BwdLayout L = bwd_layout(d, workspace);
  if (!workspace || workspace_bytes < L.total)
    return fail(STGCN_E_INVALID, "workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const int N = d->N, C = d->C_in, R = d->C_out, T = d->T, To = d->T_out, V = d->V, K = d->K;
  const float *mean1 = a->stats, *invstd1 = a->stats + C;
  const float *mean2 = a->stats + 2 * C, *invstd2 = a->stats + 2 * C + R;
  // deferred dx (ABI 5; below)
  const bool defer = d->need_dx && d->training && !res && a->prev_g2 && a->prev_b2 &&
                     a->prev_sums && a->prev_U && a->prev_stats && a->x_stats && a->dx_coef &&
                     a->dx_deferred &&
                     (fused_spb(d) || fold_spb(d) || spatial_dx_prev_supported(N, C, T, V, K));
  if (xnull && !defer)
    return fail(STGCN_E_INVALID,
                "x null: the backward must defer dx (prev_U, prev_stats, prev_g2 / prev_b2, "
                "prev_sums, x_stats, dx_coef, dx_deferred)");

  HIP_TRY(hipMemsetAsync(workspace, 0, L.dbl_bytes, s));
  // (Tq's fp64 re-layout goes straight into launch_fold_sdz's scratch slot in
  // this call's workspace -- never into the prep buffer, which holds only the
  // step's weight-only operands and may be shared by concurrent backwards)
  double *tqT = nullptr;
  if (cols_sums(d)) tqT = fold_sdz_tq_slot(L.f64scr, R, C);
  if (!res) {
    // ReLU + BN2 backward -> dU, dgamma2, dbeta2, d(temporal bias); the
    // reduction comes from the next block when it was chained (dy_sums)
    const double *sg = L.sg, *sgu = L.sgu;
    if (a->dy_sums) {
      sg = a->dy_sums;
      sgu = a->dy_sums + R;
    } else {
      HIP_TRY(launch_bn_relu_bwd_reduce(a->dy, a->U, mean2, invstd2, a->g2, a->b2, N, R, To * V,
                                        L.sg, L.sgu, drop, s, a->dy_nc));
    }
    // (with the clip-chunk sums of dU: sum_{n,t} dZ follows from them per tap,
    // no pass over dZ)
    if (cols_sums(d) && fold_bna(d)) {  // + dU A (the weight gradient's P) in dZ's buffer
      HIP_TRY(launch_bn_relu_bwd_apply_fr(a->dy, a->U, mean2, invstd2, a->g2, a->b2, sg, sgu,
                                          L.dU, L.dZ, L.sdu, N, R, To, V, d->training, drop,
                                          a->dy_coef, L.fcs, L.amax, L.amax + 2 * kAmaxWords,
                                          a->A, s));
      HIP_TRY(launch_fold_tq(L.fcs, apply_cols_chunks(N), R, T, To, V, d->stride, L.ftq, tqT,
                             s));
    } else if (cols_sums(d)) {
      HIP_TRY(launch_bn_relu_bwd_apply_cols(a->dy, a->U, mean2, invstd2, a->g2, a->b2, sg, sgu,
                                            L.dU, L.sdu, N, R, To * V, d->training, drop, s,
                                            du_bf16(d) ? 1 : 0, a->dy_coef, L.fcs,
                                            f16x2_tw(d) ? L.amax : nullptr,  // (f16x2: max |dU|)
                                            a->dy_nc));
      HIP_TRY(launch_fold_tq(L.fcs, apply_cols_chunks(N), R, T, To, V, d->stride, L.ftq, tqT,
                             s));
    } else {
      HIP_TRY(launch_bn_relu_bwd_apply(a->dy, a->U, mean2, invstd2, a->g2, a->b2, sg, sgu, L.dU,
                                       L.sdu, N, R, To * V, d->training, drop, s,
                                       du_bf16(d) ? 1 : 0, a->dy_coef, a->dy_nc));
    }
    HIP_TRY(launch_bn_grads_out(sg, sgu, L.sdu, R, a->dg2, a->db2, a->dbWt, s));
  } else {
    // residual block: final ReLU backward -> dU (= d(conv out) = d(residual));
    // temporal and projection bias grads are its per-channel sums
    HIP_TRY(launch_relu_bwd(a->dy, a->y, L.dU, L.sdu, N, R, To * V, drop.thresh ? drop.scale : 1.f,
                            s));
    HIP_TRY(launch_bn_grads_out(L.sdu, L.sdu, nullptr, R, a->dbWt, a->dbr ? a->dbr : a->dbWt,
                                nullptr, s));
  }

  // dZ in bf16 where every reader takes it (needs the kept G: k_wgrad_gemm_gk)
  const bool dzb = dz_bf16(d) && a->G != nullptr;
  // Deferred dx (ABI 5): the BN1 backward apply of this block is folded into the
  // previous block's ReLU+BN2 backward apply (launch_bn_relu_bwd_apply with
  // dy_coef). The spatial backward then reads the previous block's U in place of
  // x (PrevBn: x rebuilt, that block's mask / uhat sums), dx receives dxhat, and
  // launch_chain_coef forms dg1 / db1, the coefficients and the previous block's
  // ReLU+BN2 sums: dx never makes its own HBM round trip.
  PrevBn pvb;
  if (defer) {
    pvb.mean = a->prev_stats;
    pvb.invstd = a->prev_stats + C;
    pvb.g = a->prev_g2;
    pvb.b = a->prev_b2;
    pvb.s1 = L.s1;
    pvb.s2 = L.s2;
  }
  const float *xin = defer ? a->prev_U : a->x;
  if (a->dx_deferred) *a->dx_deferred = defer ? 1 : 0;
  if (fold_w(d)) {
    // The folded block (kernels_fold.hip): Wc_q = Wt_q W'; the data gradient
    // with Wc gives H = W'^T dZ directly (C_in channels), the weight gradient
    // over G gives dWc, and dWt, dW', sum_{n,t} dZ follow from dWc and the dU sums.
    // (ABI 7: the weight-only operands from stgcn_fold_prep, same step)
    const bool pre = a->prep && prep_applies(d);
    const PrepLayout P = pre ? prep_layout(d, a->prep) : PrepLayout{};
    const float *Wc = a->Z;  // (left there by the forward)
    const float *bZ = L.bZ, *fscr = L.fscr;
    double *f64scr = L.f64scr;
    const unsigned *amax_wc = L.amax + kAmaxWords;
    if (pre) {
      Wc = P.Wc;
      bZ = P.bZ;
      fscr = P.fscr_b;
      f64scr = P.f64;
      amax_wc = P.amax;
    } else {
      if (!fold_wc_in_z(d)) {
        HIP_TRY(launch_fold_w(a->Wt, a->W, R, C, L.Wc, L.fscr, s));
        Wc = L.Wc;
      }
      HIP_TRY(launch_bias_rv(a->A, a->bW, L.bZ, K, R, V, s));
      HIP_TRY(launch_fold_prep_bwd(a->Wt, a->W, R, C, L.fscr, s));
    }
    if (fold_spb(d)) {  // dbW and the bias part of dA first: the data gradient adds to dA;
      // BN1's sd from the dU sums (fp64, exact against the cancellation in sum dxhat)
      HIP_TRY(launch_fold_sdz(f64scr, a->Wt, Wc, L.ftq, R, C, V, L.SdZ, L.SdH, s, pre, tqT));
      HIP_TRY(launch_fold_small_sd(L.SdZ, a->A, a->bW, R, V, a->dbW, a->dA, L.SdH, C, L.sd, s));
    }
    if (f16x2_dgrad(d) && !pre)  // the fp16 splits' operand scales: max |dU| (apply pass), max |Wc|
      HIP_TRY(launch_absmax(Wc, (int64_t)R * C * 9, L.amax + kAmaxWords, s));
    {
      ConvGemmParams p = conv_base(d, L.wpk);
      p.in = L.dU;
      p.out = L.H;
      if (f16x2_dgrad(d)) {
        p.f16x2 = 1;
        p.amax_in = L.amax;
        p.amax_w = amax_wc;
      }
      if (fold_spb(d)) {  // dxhat -> dx; BN1 / chain sums and dA from the tile (H on chip)
        p.spb = 1;
        p.out = d->need_dx ? a->dx : nullptr;
        p.sx = xin;
        p.sA = a->A;
        p.mean1 = mean1;
        p.invstd1 = invstd1;
        p.g1 = a->g1;
        p.b1 = a->b1;
        if (defer) p.prev = pvb;
        p.sd = L.sd;
        p.sd_given = 1;
        p.sdn = L.sdn;
        p.dA = a->dA;
      }
      // (deterministic dA: every workgroup's partial in its own slot, summed below)
      int64_t dparts = 0;
      const int dnpl = f16x2_dgrad(d) ? 2 : 3;
      auto dA_slots = [&](ConvGemmParams &q) {
        q.dA_part = nullptr;  // (no slots: fp32 atomics into dA)
        if (!fold_spb(d) || !L.dApart) return;
        const int rows = conv_x3_tile_rows(q, dnpl);
        const int64_t nb = (int64_t)N * q.n_mtiles * ((q.R + rows - 1) / rows);
        if (dparts + nb > L.dA_cap) return;
        q.dA_part = L.dApart + dparts * V * V;
        dparts += nb;
      };
      p.in_bstride = (int64_t)R * To * V;
      p.out_bstride = (int64_t)C * T * V;
      p.w_sr = 9;
      p.w_sc = (int64_t)C * 9;
      p.C = R;
      p.R = C;
      p.T_src = To;
      p.T_dst = T;
      p.s_in = 1;
      if (d->stride == 1) {
        p.w = Wc + 8;
        p.w_sq = -1;
        p.NQ = 9;
        p.off = -4;
        p.s_out = 1;
        p.p_out = 0;
        p.M = T;
        if (pre) {
          p.wpk = reinterpret_cast<float *>(P.wpk_d[0]);
          p.wpk_ready = 1;
        }
        conv_tiles(p);
        dA_slots(p);
        HIP_TRY(launch_conv_gemm(p, s));
      } else {
        for (int ph = 0; ph < 2; ++ph) {
          p.w = Wc + (ph == 0 ? 8 : 7);
          p.w_sq = -2;
          p.NQ = ph == 0 ? 5 : 4;
          p.off = ph == 0 ? -2 : -1;
          p.s_out = 2;
          p.p_out = ph;
          p.M = ph == 0 ? (T + 1) / 2 : T / 2;
          if (pre) {
            p.wpk = reinterpret_cast<float *>(P.wpk_d[ph]);
            p.wpk_ready = 1;
          }
          if (p.M <= 0) continue;
          conv_tiles(p);
          dA_slots(p);
          HIP_TRY(launch_conv_gemm(p, s));
        }
      }
      HIP_TRY(launch_dA_reduce(L.dApart, dparts, V * V, L.dAlvl, a->dA, s));
    }
    if (fold_bna(d)) {  // dWc = sum (dU A) BN1(x): Q = x with BN1 at staging, P = dU A
      const unsigned *xmax = reinterpret_cast<const unsigned *>(a->G);  // (the forward's max |x|)
      if (!xmax) {
        HIP_TRY(launch_absmax(a->x, (int64_t)N * C * T * V, L.amax + 3 * kAmaxWords, s));
        xmax = L.amax + 3 * kAmaxWords;
      }
      WgradParams w = make_wgrad_taps(d, L.dZ, a->x, L.slab, C);
      if (w.bf16 != 3) return fail(STGCN_E_HIP, "bna weight gradient: no split plan");
      w.f16x2 = 1;
      w.amax_p = L.amax + 2 * kAmaxWords;
      w.amax_q = xmax;
      w.q_mean = mean1;
      w.q_invstd = invstd1;
      w.q_g = a->g1;
      w.q_b = a->b1;
      HIP_TRY(launch_wgrad_taps(w, s));
      HIP_TRY(launch_fold_grads(L.slab, w.S, fscr, bZ, L.ftq, R, C, V, L.dWc, a->dWt, a->dW, s));
    } else {
    const float *G = a->G;  // kept fp32 G (f16x2: its max |G| follows it), else recomputed
    const unsigned *amax_g = G ? reinterpret_cast<const unsigned *>(G + (size_t)N * C * T * V)
                               : L.amax + 2 * kAmaxWords;
    if (!G) {
      HIP_TRY(launch_gather_fwd(a->x, mean1, invstd1, a->g1, a->b1, a->A, L.G, N, C, T, V, K,
                                res, s, f16x2(d) ? L.amax + 2 * kAmaxWords : nullptr));
      G = L.G;
    }
    WgradParams w = make_wgrad_taps(d, L.dU, G, L.slab, C);
    if (f16x2(d) && w.bf16 == 3) {  // max |dU| (apply pass), max |G|
      w.f16x2 = 1;
      w.amax_p = L.amax;
      w.amax_q = amax_g;
    }
    HIP_TRY(launch_wgrad_taps(w, s));
    HIP_TRY(launch_fold_grads(L.slab, w.S, fscr, bZ, L.ftq, R, C, V, L.dWc, a->dWt, a->dW, s));
    }
  } else {
  // Temporal conv data-gradient: dZ = conv^T(dU)
  {
    ConvGemmParams p = conv_base(d, L.wpk);
    p.in = L.dU;
    p.in_bf16 = du_bf16(d) ? 1 : 0;
    p.out = L.dZ;
    p.out_bf16 = dzb ? 1 : 0;
    p.in_bstride = (int64_t)R * To * V;
    p.out_bstride = (int64_t)R * T * V;
    p.w_sr = 9;
    p.w_sc = (int64_t)R * 9;
    p.C = R;
    p.R = R;
    p.T_src = To;
    p.T_dst = T;
    p.s_in = 1;
    if (d->stride == 1) {
      p.w = a->Wt + 8;
      p.w_sq = -1;
      p.NQ = 9;
      p.off = -4;
      p.s_out = 1;
      p.p_out = 0;
      p.M = T;
      conv_tiles(p);
      HIP_TRY(launch_conv_gemm(p, s));
    } else {
      for (int ph = 0; ph < 2; ++ph) {
        p.w = a->Wt + (ph == 0 ? 8 : 7);
        p.w_sq = -2;
        p.NQ = ph == 0 ? 5 : 4;
        p.off = ph == 0 ? -2 : -1;
        p.s_out = 2;
        p.p_out = ph;
        p.M = ph == 0 ? (T + 1) / 2 : T / 2;
        if (p.M <= 0) continue;
        conv_tiles(p);
        HIP_TRY(launch_conv_gemm(p, s));
      }
    }
  }
  // Temporal conv weight-gradient: dWt[co][ci][q] = sum dU[co] * Z[ci](shifted)
  {
    WgradParams w = make_wgrad_taps(d, L.dU, res ? a->Za : a->Z, L.slab);
    w.q_bf16 = z_bf16(d) ? 1 : 0;
    w.p_bf16 = du_bf16(d) ? 1 : 0;
    if (f16x2_unfold(d) && w.bf16 == 3) {  // fp16 splits: max |dU| (apply pass), max |Z|
      if (!cols_sums(d))  // (the apply pass without the column sums forms no max |dU|)
        HIP_TRY(launch_absmax(L.dU, (int64_t)N * R * To * V, L.amax, s));
      const unsigned *zmax =
          a->G ? reinterpret_cast<const unsigned *>(a->G + (size_t)N * K * C * T * V) : nullptr;
      if (!zmax) {  // (no kept G: a pass over Z)
        HIP_TRY(launch_absmax(a->Z, (int64_t)N * R * T * V, L.amax + 3 * kAmaxWords, s));
        zmax = L.amax + 3 * kAmaxWords;
      }
      w.f16x2 = 1;
      w.amax_p = L.amax;
      w.amax_q = zmax;
    }
    HIP_TRY(launch_wgrad_taps(w, s));
    HIP_TRY(launch_slab_reduce(L.slab, w.S, (int64_t)R * R * 9, a->dWt, 0, R, 1, R, s));
  }
  if (res) {
    // BN2 + ReLU backward over Z (residual block, st_graphconv.py:76-77): dZ in place
    HIP_TRY(launch_bn_relu_bwd_reduce(L.dZ, a->Z, mean2, invstd2, a->g2, a->b2, N, R, T * V,
                                      L.sg, L.sgu, Dropout(), s));
    HIP_TRY(launch_bn_relu_bwd_apply(L.dZ, a->Z, mean2, invstd2, a->g2, a->b2, L.sg, L.sgu,
                                     L.dZ, L.sdu, N, R, T * V, d->training, Dropout(), s));
    HIP_TRY(launch_bn_grads_out(L.sg, L.sgu, nullptr, R, a->dg2, a->db2, nullptr, s));
  }
  // Spatial conv backward. Recompute G = f(BN1(x)) A^T (f = ReLU in the
  // residual block), then
  //   dW' = dZ G^T (split-K), H_k = W_k^T dZ, dxhat = sum_k H_k A_k,
  //   dA = sum H_k^T f(BN1(x)) + bias part, dbW = sum dZ rowsum(A_k).
  if (fused_sp(d) && a->G) {
    // the bf16 G kept by the fused forward (k_sp_fwd_bf16) -> k_wgrad_gemm_gk
    WgradParams w{};
    w.P = L.dZ;
    w.Q = a->G;
    w.slab = L.slab;
    w.p_bstride = (int64_t)R * T * V;
    w.R = R;
    w.C = K * C;
    w.NQ = 1;
    w.s_in = 1;
    w.M = T;
    w.T_src = T;
    w.V = V;
    w.N = N;
    w.p_bf16 = dzb ? 1 : 0;
    plan_wgrad_gk(w, T);
    HIP_TRY(launch_wgrad_gk(w, s));
    HIP_TRY(launch_slab_reduce(L.slab, w.S, (int64_t)R * K * C, a->dW, 1, R, K, C, s));
  } else {
    const float *G = fused_sp(d) ? nullptr : a->G;  // kept fp32 G, else recomputed
    if (!G) {
      HIP_TRY(launch_gather_fwd(a->x, mean1, invstd1, a->g1, a->b1, a->A, L.G, N, C, T, V, K,
                                res, s));
      G = L.G;
    }
    WgradParams w = make_wgrad(d, L.dZ, (int64_t)R * T * V, R, T, G, (int64_t)K * C * T * V,
                               K * C, T, 1, 1, 0, L.slab);
    HIP_TRY(launch_wgrad(w, s));
    HIP_TRY(launch_slab_reduce(L.slab, w.S, (int64_t)R * K * C, a->dW, 1, R, K, C, s));
  }
  if (!cols_sums(d)) HIP_TRY(launch_sum_nt(L.dZ, N, R, T, V, L.SdZ, s, dzb ? 1 : 0));
  }
  // sum_{n,t} dZ: from the temporal weight and the per-tap dU sums on the
  // non-residual block (dZ = conv^T(dU)); the residual block's dZ passes BN2
  // (the fused folded backward did both before its data gradient)
  if (!fold_spb(d)) {
    if (cols_sums(d))
      HIP_TRY(launch_fold_sdz(L.f64scr, a->Wt, nullptr, L.ftq, R, C, V, L.SdZ, nullptr, s));
    HIP_TRY(launch_spatial_small(L.SdZ, a->A, a->bW, K, R, V, a->dbW, a->dA, s));
  }
  if (fold_spb(d)) {
    // (done in the folded block's data gradient: kernels_x3.hip spb_epilogue)
  } else if (fused_spb(d)) {
    // H = W'^T dZ, dx = sum_k H_k A_k, dA, BN1 sums in one kernel (H stays on chip)
    HIP_TRY(launch_sp_bwd_fused(L.dZ, xin, mean1, invstd1, a->g1, a->b1, a->A, a->W, L.wpk,
                                a->dx, a->dA, L.sd, L.sdn, N, C, R, T, V, K, d->need_dx, res,
                                f32x3(d), s, defer ? &pvb : nullptr, dzb ? 1 : 0));
  } else {
  // Clip slices (spatial_bwd_slice): the H GEMM and the joint kernel run on ns
  // clips at a time, so the slice of H they hand over (and the dZ / x / dx
  // slices around it) stay within the 256 MiB Infinity Cache: H is written and
  // read back on-die instead of through HBM (the buffer is reused per slice).
  const float *Wz = a->W;
  if (K > 1) {
    HIP_TRY(launch_pack_w(a->W, L.Wpk, K, R, C, s));
    Wz = L.Wpk;
  }
  const int NSL = spatial_bwd_slice(d);
  int64_t sparts = 0;  // (deterministic dA: the joint kernel's workgroup partials, if it takes them)
  for (int n0 = 0; n0 < N; n0 += NSL) {
  const int ns = std::min(NSL, N - n0);
  const int64_t xo = (int64_t)n0 * C * T * V;
  if (!fold_w(d)) {  // (the folded block's data gradient wrote H)
    // H = W'^T dZ for all partitions in one GEMM (rows k*C_in + ci of H are
    // the channels of H_k): dZ is read once instead of K times
    ConvGemmParams p = conv_base(d, L.wpk);
    p.N = ns;
    p.in_bf16 = dzb ? 1 : 0;  // (element offsets: the bf16 kernel halves them)
    p.in = dzb ? reinterpret_cast<const float *>(reinterpret_cast<const __bf16 *>(L.dZ) +
                                                 (int64_t)n0 * R * T * V)
               : L.dZ + (int64_t)n0 * R * T * V;
    p.w = Wz;
    p.out = L.H;
    p.in_bstride = (int64_t)R * T * V;
    p.out_bstride = (int64_t)K * C * T * V;
    p.w_sr = 1;
    p.w_sc = (int64_t)K * C;
    p.w_sq = 0;
    p.C = R;
    p.R = K * C;
    p.NQ = 1;
    p.s_in = 1;
    p.off = 0;
    p.s_out = 1;
    p.p_out = 0;
    p.M = T;
    p.T_src = T;
    p.T_dst = T;
    conv_tiles(p);
    HIP_TRY(launch_conv_gemm(p, s));
  }
  int64_t np = 0;
  HIP_TRY(launch_spatial_dx(L.H, xin + xo, mean1, invstd1, a->g1, a->b1, a->A,
                            a->dx ? a->dx + xo : nullptr, a->dA, L.sd, L.sdn, ns, C, T, V, K,
                            d->need_dx, res, bf16(d) ? 1 : 0, s, defer ? &pvb : nullptr,
                            L.dApart ? L.dApart + sparts * K * V * V : nullptr,
                            L.dA_cap - sparts, &np));
  sparts += np;
  }
  HIP_TRY(launch_dA_reduce(L.dApart, sparts, K * V * V, L.dAlvl, a->dA, s));
  }
  if (defer) {
    HIP_TRY(launch_chain_coef(L.sd, L.sdn, mean1, invstd1, a->g1, L.s1, L.s2, a->x_stats, C,
                              (int64_t)N * T * V, a->dg1, a->db1, a->dx_coef, a->prev_sums, s));
    return STGCN_OK;
  }
  HIP_TRY(launch_bn_grads_out(L.sd, L.sdn, nullptr, C, a->dg1, a->db1, nullptr, s));
  // residual path gradient (added to dx after the BN1 backward)
  const float *add = nullptr;
  if (res && !projection(d)) add = L.dU;  // identity: d(res) = dU
  if (projection(d)) {
    // dWr[co][ci] = sum dU[co](m) x[ci](s*m)
    WgradParams w = make_wgrad(d, L.dU, (int64_t)R * To * V, R, To, a->x, (int64_t)C * T * V, C,
                               T, 1, d->stride, 0, L.slab);
    HIP_TRY(launch_wgrad(w, s));
    HIP_TRY(launch_slab_reduce(L.slab, w.S, (int64_t)R * C, a->dWr, 0, R, 1, C, s));
    if (d->need_dx) {  // Rg[ci](s*m) = sum_co Wr[co][ci] dU[co](m); other frames 0
      HIP_TRY(hipMemsetAsync(L.Rg, 0, sizeof(float) * (size_t)N * C * T * V, s));
      ConvGemmParams p = conv_base(d, L.wpk);
      p.in = L.dU;
      p.w = a->Wr;
      p.out = L.Rg;
      p.in_bstride = (int64_t)R * To * V;
      p.out_bstride = (int64_t)C * T * V;
      p.w_sr = 1;
      p.w_sc = C;
      p.w_sq = 0;
      p.C = R;
      p.R = C;
      p.NQ = 1;
      p.s_in = 1;
      p.off = 0;
      p.s_out = d->stride;
      p.p_out = 0;
      p.M = To;
      p.T_src = To;
      p.T_dst = T;
      conv_tiles(p);
      HIP_TRY(launch_conv_gemm(p, s));
      add = L.Rg;
    }
  }
  if (d->need_dx) {
    const bool chain = d->training && a->prev_g2 && a->prev_b2 && a->prev_sums;
    const bool chain_u = chain && a->prev_U && a->prev_stats;
    if (chain) HIP_TRY(hipMemsetAsync(a->prev_sums, 0, sizeof(double) * 2 * C, s));
    HIP_TRY(launch_bn1_bwd_apply(a->dx, a->x, mean1, invstd1, a->g1, L.sd, L.sdn, add, N, C,
                                 T * V, (int64_t)N * T * V, d->training,
                                 chain ? a->prev_g2 : nullptr, chain ? a->prev_b2 : nullptr,
                                 chain ? a->prev_sums : nullptr, chain_u ? a->prev_U : nullptr,
                                 chain_u ? a->prev_stats : nullptr,
                                 chain_u ? a->prev_stats + C : nullptr, s));
  }
  return STGCN_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Measurement entry points (bench.py roofline): run ONE of the block's GEMM
// kernels `iters` times on the caller's stream between two hipEvents, with the
// exact launch parameters stgcn_block_fwd / _bwd use for this descriptor.
//   which 0: temporal (9,1) conv forward      (k_conv_gemm<9>)
//         1: temporal conv data-gradient      (k_conv_gemm<9> or <5>+<4>)
//         2: temporal conv weight-gradient    (k_wgrad<9>, slab reduce excluded)
//         3: spatial channel GEMM Z = W' G    (k_conv_gemm<1>; with the fused bf16
//            spatial forward: that kernel, joint contraction FLOPs included)
//         4: spatial backward dZ -> dx, dA, BN1 sums (k_sp_bwd_fused where it
//            applies, else the stacked H GEMM + the joint kernel; H GEMM and
//            joint contraction FLOPs)
//         5: the stacked H GEMM of the unfused spatial backward alone
//            (V = 50 fused: its dx kernel k_sp50_dx alone)
//         6: the joint kernel of the unfused spatial backward alone
//            (V = 50 fused: its dA kernel k_sp50_dA alone)
//            (k_spatial_bwd5 / _bwd6 / _bwd3: dx, dA, BN1 sums from H)
//         (5 and 6 fail with STGCN_E_UNSUPPORTED where k_sp_bwd_fused<25> runs)
// flops = the algorithmic FLOPs of one launch (SURVEY.md §8d terms).
// ---------------------------------------------------------------------------
namespace {
struct TimedPlan {
  ConvGemmParams cp[2];
  int ncp = 0;
  WgradParams wp{};
  bool wgrad = false;
  // which 3 on the fused bf16 spatial forward (k_sp_fwd_bf16 / k_sp_fwd_wide)
  bool spf = false;
  const float *x = nullptr, *st = nullptr, *A = nullptr, *W = nullptr, *biasZ = nullptr;
  void *wpk = nullptr;
  float *Z = nullptr;
  __bf16 *Gk = nullptr;
  // which 4: the spatial backward (5: its H GEMM only, 6: its joint kernel only)
  bool spb = false, spb_gemm = true, spb_joint = true;
  const float *dZ = nullptr;
  float *H = nullptr, *dx = nullptr, *dA = nullptr;
  double *sd = nullptr;
  // f16x2: the operands whose max |x| the fp16 splits scale by (computed once
  // before the timed launches, as the block does before its GEMMs)
  unsigned *amax = nullptr;
  const float *ax[2] = {nullptr, nullptr};
  int64_t an[2] = {0, 0};
  size_t bytes = 0;
  double flops = 0;
};

TimedPlan plan_timed(const stgcn_desc_t *d, int which, void *scratch) {
  TimedPlan P;
  Carve c(scratch);
  const int N = d->N, C = d->C_in, R = d->C_out, T = d->T, To = d->T_out, V = d->V, K = d->K;
  // (the folded block: the temporal GEMMs run over C_in channels on the G side)
  const bool fold = fold_w(d);
  const int CZ = fold ? C : R;
  const double tflops = 2.0 * 9 * R * (double)CZ * To * V * N;
  float *wpk = c.take<float>(wpk_floats(d));
  if (f16x2_tw(d) && which <= 2) P.amax = c.take<unsigned>(2 * kAmaxWords);
  if (which == 0) {
    ConvGemmParams p = conv_base(d, wpk);
    p.in = c.take<float>((size_t)N * CZ * T * V);
    p.w = c.take<float>((size_t)R * CZ * 9);
    p.out = c.take<float>((size_t)N * R * To * V);
    p.bias_r = c.take<float>(R);
    p.stat_sum = c.take<double>(R);
    p.stat_sq = c.take<double>(R);
    p.in_bstride = (int64_t)R * T * V;
    p.out_bstride = (int64_t)R * To * V;
    p.w_sr = (int64_t)R * 9;
    p.w_sc = 9;
    p.w_sq = 1;
    p.C = R;
    p.R = R;
    p.NQ = 9;
    p.s_in = d->stride;
    p.off = -d->pad;
    p.s_out = 1;
    p.p_out = 0;
    p.M = To;
    p.T_src = T;
    p.T_dst = To;
    p.in_bf16 = z_bf16(d) ? 1 : 0;
    if (fold) {
      p.bias_r = nullptr;
      p.res = c.take<float>((size_t)R * To * V);
      p.res_shared = 1;
      p.in_bstride = (int64_t)C * T * V;
      p.w_sr = (int64_t)C * 9;
      p.C = C;
    }
    if (P.amax) {
      p.f16x2 = 1;
      p.amax_in = P.amax;
      p.amax_w = P.amax + kAmaxWords;
      P.ax[0] = p.in;
      P.an[0] = (int64_t)N * CZ * T * V;
      P.ax[1] = p.w;
      P.an[1] = (int64_t)R * CZ * 9;
    }
    p.w4 = fwd_w4(d) ? 1 : 0;
    if (fold_bna(d)) {  // x in: BN1 in the loader, the joint contraction in the epilogue
      p.bna = 1;
      p.sA = c.take<float>((size_t)V * V);
      float *st = c.take<float>((size_t)4 * C);
      p.mean1 = st;
      p.invstd1 = st + C;
      p.g1 = st + 2 * C;
      p.b1 = st + 3 * C;
    }
    conv_tiles(p);
    P.cp[P.ncp++] = p;
    // (bna: + the joint contraction 2 K C_out T V^2 of the spatial forward, now here)
    P.flops = tflops + (fold_bna(d) ? 2.0 * K * R * (double)To * V * V * N : 0.0);
  } else if (which == 1) {
    ConvGemmParams p = conv_base(d, wpk);
    p.in = c.take<float>((size_t)N * R * To * V);
    p.in_bf16 = du_bf16(d) ? 1 : 0;
    const float *w = c.take<float>((size_t)R * CZ * 9);
    p.out = c.take<float>((size_t)N * CZ * T * V);
    p.out_bf16 = dz_bf16(d) ? 1 : 0;  // (the stack keeps G, so dZ is bf16 there)
    p.in_bstride = (int64_t)R * To * V;
    p.out_bstride = (int64_t)CZ * T * V;
    p.w_sr = 9;
    p.w_sc = (int64_t)CZ * 9;
    p.C = R;
    p.R = CZ;
    p.T_src = To;
    p.T_dst = T;
    p.s_in = 1;
    if (P.amax && f16x2_dgrad(d)) {
      p.f16x2 = 1;
      p.amax_in = P.amax;
      p.amax_w = P.amax + kAmaxWords;
      P.ax[0] = p.in;
      P.an[0] = (int64_t)N * R * To * V;
      P.ax[1] = w;
      P.an[1] = (int64_t)R * CZ * 9;
    }
    if (fold_spb(d)) {  // the fused SpatialConv backward epilogue and its operands
      p.spb = 1;
      p.sx = c.take<float>((size_t)N * C * T * V);
      p.sA = c.take<float>((size_t)V * V);
      float *st = c.take<float>((size_t)4 * C);
      p.mean1 = st;
      p.invstd1 = st + C;
      p.g1 = st + 2 * C;
      p.b1 = st + 3 * C;
      double *sd = c.take<double>((size_t)2 * C);
      p.sd = sd;
      p.sdn = sd + C;
      p.dA = c.take<float>((size_t)V * V);
    }
    if (d->stride == 1) {
      p.w = w ? w + 8 : nullptr;
      p.w_sq = -1;
      p.NQ = 9;
      p.off = -4;
      p.s_out = 1;
      p.p_out = 0;
      p.M = T;
      conv_tiles(p);
      P.cp[P.ncp++] = p;
    } else {
      for (int ph = 0; ph < 2; ++ph) {
        p.w = w ? w + (ph == 0 ? 8 : 7) : nullptr;
        p.w_sq = -2;
        p.NQ = ph == 0 ? 5 : 4;
        p.off = ph == 0 ? -2 : -1;
        p.s_out = 2;
        p.p_out = ph;
        p.M = ph == 0 ? (T + 1) / 2 : T / 2;
        conv_tiles(p);
        if (p.M > 0) P.cp[P.ncp++] = p;
      }
    }
    // (fused: + the joint contractions dxhat = H A and dA = H^T BN1(x))
    P.flops = tflops + (fold_spb(d) ? 4.0 * K * C * (double)T * V * V * N : 0.0);
  } else if (which == 2) {
    const float *dU = c.take<float>((size_t)N * R * To * V);
    const float *Z = c.take<float>((size_t)N * CZ * T * V);
    WgradParams w = make_wgrad_taps(d, dU, Z, nullptr, CZ);
    w.q_bf16 = z_bf16(d) ? 1 : 0;
    w.p_bf16 = du_bf16(d) ? 1 : 0;
    w.slab = c.take<float>((size_t)w.S * R * CZ * 9);
    if (P.amax && w.bf16 == 3) {
      w.f16x2 = 1;
      w.amax_p = P.amax;
      w.amax_q = P.amax + kAmaxWords;
      P.ax[0] = dU;
      P.an[0] = (int64_t)N * R * To * V;
      P.ax[1] = Z;
      P.an[1] = (int64_t)N * CZ * T * V;
    }
    if (fold_bna(d) && w.bf16 == 3) {  // P = dU A, Q = x with BN1 at staging
      // (taken whether or not scratch is given: the size query must match)
      float *st = c.take<float>((size_t)4 * C);
      w.q_mean = st;
      w.q_invstd = st + C;
      w.q_g = st + 2 * C;
      w.q_b = st + 3 * C;
    }
    P.wp = w;
    P.wgrad = true;
    P.flops = tflops;
  } else if (which >= 4) {
    P.spb = true;
    P.spb_gemm = which != 6 && !fold;  // (folded: the data gradient wrote H)
    P.spb_joint = which != 5;
    P.wpk = wpk;
    P.x = c.take<float>((size_t)N * C * T * V);
    P.st = c.take<float>((size_t)4 * C);
    P.A = c.take<float>((size_t)K * V * V);
    P.W = c.take<float>((size_t)K * R * C);
    P.dZ = c.take<float>((size_t)N * R * T * V);
    P.dx = c.take<float>((size_t)N * C * T * V);
    P.dA = c.take<float>((size_t)K * V * V);
    P.sd = c.take<double>((size_t)2 * C);
    if (!fused_spb(d)) {
      P.H = c.take<float>((size_t)N * K * C * T * V);
    }
    if (!fused_spb(d) && !fold) {
      ConvGemmParams p = conv_base(d, wpk);
      p.in = P.dZ;
      p.in_bf16 = dz_bf16(d) ? 1 : 0;
      p.w = c.take<float>((size_t)R * K * C);  // (the packed W' of the block)
      p.out = P.H;
      p.in_bstride = (int64_t)R * T * V;
      p.out_bstride = (int64_t)K * C * T * V;
      p.w_sr = 1;
      p.w_sc = (int64_t)K * C;
      p.w_sq = 0;
      p.C = R;
      p.R = K * C;
      p.NQ = 1;
      p.s_in = 1;
      p.off = 0;
      p.s_out = 1;
      p.p_out = 0;
      p.M = T;
      p.T_src = T;
      p.T_dst = T;
      conv_tiles(p);
      P.cp[P.ncp++] = p;
    }
    P.flops = (P.spb_gemm ? 2.0 * K * C * (double)R * T * V * N : 0.0) +
              (P.spb_joint ? 4.0 * K * C * (double)T * V * V * N : 0.0);
    if (fused_spb50(d) && which >= 5)  // k_sp50_dx / _dA: each its H GEMM + its contraction
      P.flops = 2.0 * K * C * (double)R * T * V * N + 2.0 * K * C * (double)T * V * V * N;
  } else if (fused_sp(d)) {
    // the forward's fused spatial kernel (G kept in bf16 as in the stack)
    P.spf = true;
    P.wpk = wpk;
    P.x = c.take<float>((size_t)N * C * T * V);
    P.st = c.take<float>((size_t)4 * C);
    P.A = c.take<float>((size_t)K * V * V);
    P.W = c.take<float>((size_t)K * R * C);
    P.biasZ = c.take<float>((size_t)R * V);
    P.Z = c.take<float>((size_t)N * R * T * V);
    P.Gk = reinterpret_cast<__bf16 *>(c.take<char>(sp_keep_g_bytes(N, C, T, V, K)));
    P.flops = 2.0 * K * C * (double)R * T * V * N + 2.0 * K * C * (double)T * V * V * N;
  } else {
    ConvGemmParams p = conv_base(d, wpk);
    p.in = c.take<float>((size_t)N * K * C * T * V);
    p.w = c.take<float>((size_t)R * K * C);
    p.out = c.take<float>((size_t)N * R * T * V);
    p.bias_rv = c.take<float>((size_t)R * V);
    p.in_bstride = (int64_t)K * C * T * V;
    p.out_bstride = (int64_t)R * T * V;
    p.w_sr = (int64_t)K * C;
    p.w_sc = 1;
    p.w_sq = 0;
    p.C = K * C;
    p.R = R;
    p.NQ = 1;
    p.s_in = 1;
    p.off = 0;
    p.s_out = 1;
    p.p_out = 0;
    p.M = T;
    p.T_src = T;
    p.T_dst = T;
    conv_tiles(p);
    P.cp[P.ncp++] = p;
    P.flops = 2.0 * K * C * (double)R * T * V * N;
  }
  P.bytes = c.off;
  return P;
}
}  // namespace

extern "C" {

size_t stgcn_time_kernel_bytes(const stgcn_desc_t *d, int which) {
  if (stgcn_check_desc(d) != STGCN_OK || which < 0 || which > 6) return 0;
  if (which >= 5 && fused_spb(d) && !fused_spb50(d)) return 0;
  if ((which == 3 || which == 5) && fold_w(d)) return 0;  // (no spatial / H GEMM there)
  if (which >= 4 && fold_spb(d)) return 0;  // (inside the data gradient, which 1)
  return plan_timed(d, which, nullptr).bytes;
}

int stgcn_time_kernel(const stgcn_desc_t *d, int which, void *scratch, size_t scratch_bytes,
                      int iters, void *stream, float *avg_ms, double *flops) {
  int rc = stgcn_check_desc(d);
  if (rc) return rc;
  if (which < 0 || which > 6 || iters <= 0 || !avg_ms || !flops)
    return fail(STGCN_E_INVALID, "bad timing request");
  if (which >= 5 && fused_spb(d) && !fused_spb50(d))
    return fail(STGCN_E_UNSUPPORTED, "the spatial backward is one fused kernel here (which 4)");
  if ((which == 3 || which == 5) && fold_w(d))
    return fail(STGCN_E_UNSUPPORTED, "the folded block has no spatial / H GEMM");
  if (which >= 4 && fold_spb(d))
    return fail(STGCN_E_UNSUPPORTED, "the folded block's spatial backward runs inside its data "
                                     "gradient (which 1)");
  TimedPlan P = plan_timed(d, which, scratch);
  if (!scratch || scratch_bytes < P.bytes) return fail(STGCN_E_INVALID, "scratch too small");
  hipStream_t s = (hipStream_t)stream;
  auto launch = [&]() -> hipError_t {
    if (P.wgrad) return launch_wgrad_taps(P.wp, s);
    if (P.spb) {
      const int C = d->C_in;
      if (fused_spb(d))
        return launch_sp_bwd_fused(P.dZ, P.x, P.st, P.st + C, P.st + 2 * C, P.st + 3 * C, P.A,
                                   P.W, P.wpk, P.dx, P.dA, P.sd, P.sd + C, d->N, C, d->C_out,
                                   d->T, d->V, d->K, 1, residual(d) ? 1 : 0, f32x3(d), s,
                                   nullptr, dz_bf16(d) ? 1 : 0,
                                   P.spb_gemm && P.spb_joint ? 0 : (P.spb_gemm ? 1 : 2));
      if (P.spb_gemm) {
        hipError_t e = launch_conv_gemm(P.cp[0], s);
        if (e != hipSuccess || !P.spb_joint) return e;
      }
      return launch_spatial_dx(P.H, P.x, P.st, P.st + C, P.st + 2 * C, P.st + 3 * C, P.A, P.dx,
                               P.dA, P.sd, P.sd + C, d->N, C, d->T, d->V, d->K, 1,
                               residual(d) ? 1 : 0, bf16(d) ? 1 : 0, s);
    }
    if (P.spf) {
      const int C = d->C_in;
      return launch_sp_fwd_bf16(P.x, P.st, P.st + C, P.st + 2 * C, P.st + 3 * C, P.A, P.W,
                                P.biasZ, P.wpk, P.Z, z_bf16(d) ? 1 : 0, P.Gk, nullptr, nullptr, d->N, C, d->C_out,
                                d->T, d->V, d->K, residual(d) ? 1 : 0, s);
    }
    for (int i = 0; i < P.ncp; ++i) {
      hipError_t e = launch_conv_gemm(P.cp[i], s);
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  };
  if (P.amax) {  // the f16x2 operand scales (not timed)
    HIP_TRY(hipMemsetAsync(P.amax, 0, 2 * kAmaxWords * sizeof(unsigned), s));
    for (int i = 0; i < 2; ++i)
      if (P.ax[i]) HIP_TRY(launch_absmax(P.ax[i], P.an[i], P.amax + i * kAmaxWords, s));
  }
  HIP_TRY(launch());  // warm-up
  hipEvent_t e0, e1;
  HIP_TRY(hipEventCreate(&e0));
  HIP_TRY(hipEventCreate(&e1));
  HIP_TRY(hipEventRecord(e0, s));
  for (int i = 0; i < iters; ++i) HIP_TRY(launch());
  HIP_TRY(hipEventRecord(e1, s));
  HIP_TRY(hipEventSynchronize(e1));
  float ms = 0.f;
  HIP_TRY(hipEventElapsedTime(&ms, e0, e1));
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  *avg_ms = ms / iters;
  *flops = P.flops;
  return STGCN_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// SpatialConv on its own (st_graphconv.py:139-152), ABI 4: the block's
// spatial kernels with BatchNorm replaced by the identity (mean 0, invstd 1,
// gamma 1, beta 0: (x - 0) * 1 * 1 + 0 == x exactly in fp32).
//   fwd: G = x A_k^T (joint contraction), out = W' G + sum_k bW_k rowsum(A_k)
//   bwd: dW' = dout G^T, H = W'^T dout, dx = sum_k H_k A_k,
//        dA = sum H_k^T x + bias part, dbW = sum dout rowsum(A_k)
// ---------------------------------------------------------------------------
namespace {

// A block descriptor with the spatial shape (stride 1; the temporal fields
// only satisfy the planner).
stgcn_desc_t spatial_as_block(const stgcn_spatial_desc_t *sd) {
  stgcn_desc_t d{};
  d.N = sd->N;
  d.C_in = sd->C_in;
  d.C_out = sd->C_out;
  d.T = sd->T;
  d.T_out = sd->T;
  d.V = sd->V;
  d.K = sd->K;
  d.gamma = 9;
  d.stride = 1;
  d.pad = 4;
  d.eps = 1e-5f;
  d.momentum = 0.1f;
  d.training = 1;
  d.need_dx = 1;
  d.flags = sd->flags & STGCN_F_BF16;
  return d;
}

struct SpatialLayout {
  float *ident;  // [4][C_in]: mean 0 | invstd 1 | gamma 1 | beta 0
  double *sd, *sdn, *SdZ;
  float *G, *H, *Wpk, *biasZ, *wpk, *slab;
  size_t total;
};

SpatialLayout spatial_layout(const stgcn_desc_t *d, void *ws, bool backward) {
  Carve c(ws);
  SpatialLayout L{};
  const int R = d->C_out, C = d->C_in, K = d->K;
  L.ident = c.take<float>((size_t)4 * C);
  L.G = c.take<float>((size_t)d->N * K * C * nT(d));
  L.Wpk = c.take<float>((size_t)R * K * C);
  L.wpk = c.take<float>(wpk_floats(d));
  if (!backward) {
    L.biasZ = c.take<float>((size_t)R * d->V);
  } else {
    L.sd = c.take<double>(C);
    L.sdn = c.take<double>(C);
    L.SdZ = c.take<double>((size_t)R * d->V);
    L.H = c.take<float>((size_t)d->N * K * C * nT(d));
    WgradParams w = make_wgrad(d, nullptr, 0, R, d->T, nullptr, 0, K * C, d->T, 1, 1, 0, nullptr);
    L.slab = c.take<float>((size_t)w.S * R * K * C);
  }
  L.total = c.off;
  return L;
}

int spatial_check(const stgcn_spatial_desc_t *sd, stgcn_desc_t *d) {
  if (!sd) return fail(STGCN_E_INVALID, "null descriptor");
  if (sd->flags & ~STGCN_F_BF16) return fail(STGCN_E_UNSUPPORTED, "unknown spatial flags");
  *d = spatial_as_block(sd);
  return stgcn_check_desc(d);
}

hipError_t fill_identity_bn(float *ident, int C, hipStream_t s) {
  hipError_t e = hipMemsetD32Async((hipDeviceptr_t)ident, 0u, (size_t)C, s);  // mean 0
  if (e == hipSuccess)  // invstd 1, gamma 1
    e = hipMemsetD32Async((hipDeviceptr_t)(ident + C), 0x3f800000u, (size_t)2 * C, s);
  if (e == hipSuccess) e = hipMemsetD32Async((hipDeviceptr_t)(ident + 3 * C), 0u, (size_t)C, s);
  return e;
}

}  // namespace

extern "C" {

size_t stgcn_spatial_workspace_bytes(const stgcn_spatial_desc_t *sd, int backward) {
  stgcn_desc_t d;
  if (spatial_check(sd, &d) != STGCN_OK) return 0;
  return spatial_layout(&d, nullptr, backward != 0).total;
}

int stgcn_spatial_fwd(const stgcn_spatial_desc_t *sd, const float *x, const float *A,
                      const float *W, const float *bW, float *out, void *workspace,
                      size_t workspace_bytes, void *stream) {
  stgcn_desc_t dd;
  int rc = spatial_check(sd, &dd);
  if (rc) return rc;
  const stgcn_desc_t *d = &dd;
  if (!x || !A || !W || !bW || !out) return fail(STGCN_E_INVALID, "null tensor argument");
  const SpatialLayout L = spatial_layout(d, workspace, false);
  if (!workspace || workspace_bytes < L.total) return fail(STGCN_E_INVALID, "workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const int N = d->N, C = d->C_in, R = d->C_out, T = d->T, V = d->V, K = d->K;
  HIP_TRY(fill_identity_bn(L.ident, C, s));
  HIP_TRY(launch_bias_rv(A, bW, L.biasZ, K, R, V, s));
  const float *Wz = W;
  if (K > 1) {
    HIP_TRY(launch_pack_w(W, L.Wpk, K, R, C, s));
    Wz = L.Wpk;
  }
  HIP_TRY(launch_gather_fwd(x, L.ident, L.ident + C, L.ident + 2 * C, L.ident + 3 * C, A, L.G, N,
                            C, T, V, K, 0, s));
  ConvGemmParams p = conv_base(d, L.wpk);
  p.in = L.G;
  p.w = Wz;
  p.out = out;
  p.bias_rv = L.biasZ;
  p.in_bstride = (int64_t)K * C * T * V;
  p.out_bstride = (int64_t)R * T * V;
  p.w_sr = (int64_t)K * C;
  p.w_sc = 1;
  p.w_sq = 0;
  p.C = K * C;
  p.R = R;
  p.NQ = 1;
  p.s_in = 1;
  p.off = 0;
  p.s_out = 1;
  p.p_out = 0;
  p.M = T;
  p.T_src = T;
  p.T_dst = T;
  conv_tiles(p);
  HIP_TRY(launch_conv_gemm(p, s));
  return STGCN_OK;
}

int stgcn_spatial_bwd(const stgcn_spatial_desc_t *sd, const float *dout, const float *x,
                      const float *A, const float *W, const float *bW, float *dx, float *dA,
                      float *dW, float *dbW, void *workspace, size_t workspace_bytes,
                      void *stream) {
  stgcn_desc_t dd;
  int rc = spatial_check(sd, &dd);
  if (rc) return rc;
  const stgcn_desc_t *d = &dd;
  if (!dout || !x || !A || !W || !bW || !dA || !dW || !dbW)
    return fail(STGCN_E_INVALID, "null tensor argument");
  const SpatialLayout L = spatial_layout(d, workspace, true);
  if (!workspace || workspace_bytes < L.total) return fail(STGCN_E_INVALID, "workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const int N = d->N, C = d->C_in, R = d->C_out, T = d->T, V = d->V, K = d->K;
  HIP_TRY(fill_identity_bn(L.ident, C, s));
  HIP_TRY(hipMemsetAsync(L.sd, 0, sizeof(double) * C, s));
  HIP_TRY(hipMemsetAsync(L.sdn, 0, sizeof(double) * C, s));
  HIP_TRY(hipMemsetAsync(L.SdZ, 0, sizeof(double) * R * V, s));
  const float *mean = L.ident, *invstd = L.ident + C, *g = L.ident + 2 * C, *b = L.ident + 3 * C;
  HIP_TRY(launch_gather_fwd(x, mean, invstd, g, b, A, L.G, N, C, T, V, K, 0, s));
  {
    WgradParams w = make_wgrad(d, dout, (int64_t)R * T * V, R, T, L.G, (int64_t)K * C * T * V,
                               K * C, T, 1, 1, 0, L.slab);
    HIP_TRY(launch_wgrad(w, s));
    HIP_TRY(launch_slab_reduce(L.slab, w.S, (int64_t)R * K * C, dW, 1, R, K, C, s));
  }
  HIP_TRY(launch_sum_nt(dout, N, R, T, V, L.SdZ, s));
  HIP_TRY(launch_spatial_small(L.SdZ, A, bW, K, R, V, dbW, dA, s));
  const float *Wz = W;
  if (K > 1) {
    HIP_TRY(launch_pack_w(W, L.Wpk, K, R, C, s));
    Wz = L.Wpk;
  }
  ConvGemmParams p = conv_base(d, L.wpk);
  p.in = dout;
  p.w = Wz;
  p.out = L.H;
  p.in_bstride = (int64_t)R * T * V;
  p.out_bstride = (int64_t)K * C * T * V;
  p.w_sr = 1;
  p.w_sc = (int64_t)K * C;
  p.w_sq = 0;
  p.C = R;
  p.R = K * C;
  p.NQ = 1;
  p.s_in = 1;
  p.off = 0;
  p.s_out = 1;
  p.p_out = 0;
  p.M = T;
  p.T_src = T;
  p.T_dst = T;
  conv_tiles(p);
  HIP_TRY(launch_conv_gemm(p, s));
  // dx = sum_k H_k A_k (BatchNorm identity: dx is dxhat; sd/sdn unused)
  HIP_TRY(launch_spatial_dx(L.H, x, mean, invstd, g, b, A, dx, dA, L.sd, L.sdn, N, C, T, V, K,
                            dx != nullptr, 0, bf16(d) ? 1 : 0, s));
  return STGCN_OK;
}

}  // extern "C"

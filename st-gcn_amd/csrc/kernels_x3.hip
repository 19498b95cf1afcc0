// fp32 temporal-conv GEMMs on the bf16 matrix cores by exact operand splitting
// (STGCN_F_F32X3) — gfx950 only.
//
// gfx950 runs fp32 MFMA (v_mfma_f32_32x32x2_f32) at 157 TF/s and bf16 MFMA
// (v_mfma_f32_32x32x16_bf16) at 2.5 PF/s. Every fp32 value splits EXACTLY into
// three bf16 (round-to-nearest-even at each step):
//   h = bf16(x),  m = bf16(x - h),  l = bf16(x - h - m),   x == h + m + l
// (x - h and x - h - m are exact fp32 differences; the last residual holds at
// most 7 significant bits, so l is exact). A product then expands into nine
// bf16 x bf16 products, each exact in the fp32 accumulator's input; the six
// with weight >= 2^-16 are kept:
//   a*b ~= ah*bh + ah*bm + am*bh + ah*bl + am*bm + al*bh
// The three dropped terms (am*bl, al*bm, al*bl) are below 2^-23 |a||b| — the
// size of one fp32 rounding — so each output carries fp32-GEMM error (fp32
// accumulation as in v_mfma_f32_32x32x2_f32), and the block is gated at the
// fp32 tolerance (1e-5 rel-to-max vs fp64). Six bf16 MFMAs
// (6 x 32 cycles) replace the eight fp32 MFMAs (8 x 64 cycles) of one
// 32x32x16 step: a 2.67x higher ceiling, 417 TF/s of fp32 work.
//
// k_conv_x3<NQ, TG, V>: the ConvGemmParams GEMM (internal.h) for the stride-1
// temporal conv forward (NQ = 9) and data-gradient (NQ = 9; stride-2 phases
// NQ = 5 / 4). Tile = 64 rows x FT*V columns as in k_tconv / k_conv_bf16 (same
// epilogue). Workgroup = 8 waves, two per SIMD: wave w computes rows
// (w&1)*32..+31 of column tiles ((w>>1)&1)*4 + (w>>2)*2 + {0,1}, with the h*h
// products and the five small cross terms in separate accumulators. Chunk =
// 16 channels = one k-step per tap; a chunk runs in NQ/TG steps of TG taps.
//   Weights: pre-split by k_pack_conv_w_x3 into [chunk][tap group][plane][tap]
//            [octet][64 rows][8] bf16 (6 KiB per tap), moved per step by
//            16-byte LDS-DMA, double-buffered.
//   Window:  [position][plane*2 + octet] 16-byte slots, pitch 7 slots (odd:
//            ds_read_b128 of 16 consecutive positions is conflict-free),
//            double-buffered; chunk c+1 is loaded as fp32 dwords (coalesced
//            along positions) in chunk c's first step, split and written in its
//            last one. Staging is dealt evenly over the 8 waves (no wave-
//            dependent branches: they would make the compiler copy and wait).
// One barrier per step; weights prefetched two steps ahead where LDS allows.
// LDS: 3 x TG x 6 KiB + 2 x SPAN x 112 B (142.6 KiB at V = 18, NQ = 9): one
// workgroup per CU, two waves per SIMD.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "device_common.h"
#include "internal.h"

// k_wgrad_x3: first k-step carrying the next item's LDS writes (>= KSTEPS: after the k-steps)
constexpr int kWgWriteStart = 1;

namespace stgcn {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef int int4v __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ floatx16 mfma_x(bf16x8_t a, bf16x8_t b, floatx16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));
typedef float f2v __attribute__((ext_vector_type(2)));
// fp16 operands carried in the same 16-byte fragment registers (NPL = 2)
__device__ __forceinline__ floatx16 mfma_h(bf16x8_t a, bf16x8_t b, floatx16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8_t, a),
                                                __builtin_bit_cast(f16x8_t, b), c, 0, 0, 0);
}
// the plane products of one MFMA: bf16 (NPL = 1, 3) or fp16 (NPL = 2)
template <int NPL>
__device__ __forceinline__ floatx16 mfma_p(bf16x8_t a, bf16x8_t b, floatx16 c) {
  if constexpr (NPL == 2)
    return mfma_h(a, b, c);
  else
    return mfma_x(a, b, c);
}

__host__ __device__ __forceinline__ unsigned pk2(float a, float b) {
  const bf16x2_t v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(unsigned, v);
}
__device__ __forceinline__ float lo_f(unsigned w) { return __builtin_bit_cast(float, w << 16); }
__device__ __forceinline__ float hi_f(unsigned w) {
  return __builtin_bit_cast(float, w & 0xffff0000u);
}

__host__ __device__ __forceinline__ unsigned pkh2(float a, float b) {
  typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
  const h2_t v = {(_Float16)a, (_Float16)b};
  return __builtin_bit_cast(unsigned, v);
}
__device__ __forceinline__ float lo_h(unsigned w) {
  return (float)__builtin_bit_cast(_Float16, (unsigned short)(w & 0xffffu));
}
__device__ __forceinline__ float hi_h(unsigned w) {
  return (float)__builtin_bit_cast(_Float16, (unsigned short)(w >> 16));
}
// 2-way fp16 split of two (scaled) floats: x = h + l to 2^-22 (RNE twice)
__device__ __forceinline__ void splith2(float a, float b, unsigned &h, unsigned &l) {
  h = pkh2(a, b);
  l = pkh2(a - lo_h(h), b - hi_h(h));
}

// Power-of-two operand scale of the fp16 splits: max |x| (float bits in *amax)
// maps into [2^13, 2^14), so h <= 2^14 < 65504 and every element keeps 22
// significant bits down to 2^-24 (fp16's subnormal step) in scaled units; the
// exponent is clamped to +-100 (0 / denormal / inf maxima). Returns the scale's
// exponent (scale = 2^se).
__device__ __forceinline__ int f16x2_se(const unsigned *amax) {
  const int e = (int)((amax ? amax_read(amax) : 0x3f800000u) >> 23) & 0xff;
  const int se = e == 0 ? 0 : 140 - e;
  return se < -100 ? -100 : (se > 100 ? 100 : se);
}
__device__ __forceinline__ float pow2f(int e) { return __builtin_bit_cast(float, (unsigned)(e + 127) << 23); }

// exact 3-way split of two floats into packed (h, m, l) bf16 pairs
__device__ __forceinline__ void split2(float a, float b, unsigned &h, unsigned &m, unsigned &l) {
  h = pk2(a, b);
  const float ra = a - lo_f(h), rb = b - hi_f(h);
  m = pk2(ra, rb);
  l = pk2(ra - lo_f(m), rb - hi_f(m));
}

// Waits until at most NA VMEM operations are in flight, naming the 16 window
// staging registers (so no consumer of them is scheduled above the wait).
#define X3_ST8(k)                                                                         \
  "+v"(st[k][0]), "+v"(st[k][1]), "+v"(st[k][2]), "+v"(st[k][3]), "+v"(st[k][4]),       \
      "+v"(st[k][5]), "+v"(st[k][6]), "+v"(st[k][7])
template <int NA>
__device__ __forceinline__ void wait_img(float (&st)[2][8]) {
  asm volatile("s_waitcnt vmcnt(%16)" : X3_ST8(0), X3_ST8(1) : "n"(NA) : "memory");
}
template <int NA>
__device__ __forceinline__ void wait_img(float (&st)[3][8]) {
  asm volatile("s_waitcnt vmcnt(%24)" : X3_ST8(0), X3_ST8(1), X3_ST8(2) : "n"(NA) : "memory");
}
template <int NA>
__device__ __forceinline__ void wait_img(float (&st)[4][8]) {
  asm volatile("s_waitcnt vmcnt(%32)"
               : X3_ST8(0), X3_ST8(1), X3_ST8(2), X3_ST8(3)
               : "n"(NA)
               : "memory");
}
#undef X3_ST8

// NW = 8: two row halves of 32 MR rows (waves w, w ^ 1), ROWS = 64 MR, one
// workgroup per CU (fp32 splits) or two (bf16). NW = 4 (the fp16-split stride-1
// forward, x3_w4): one 64-row half, ROWS = 32 MR = 64, each wave 64 rows x two
// column tiles (the 128-row wave shape), LDS <= 80 KiB: TWO workgroups per CU,
// whose barriers, DMA waits, window staging, prologue and epilogue are
// independent -- each covers the other's with its MFMAs.
template <int NQ, int TG, int V, int SIN, int MR, int NPL, int NW = 8>
struct ConvX3Geo {
  static_assert(NW == 8 || (NW == 4 && MR == 2 && NPL == 2), "4-wave tiles: 64 rows, fp16 splits");
  static constexpr int NT = NW * 64;              // threads per workgroup
  static constexpr int RH = NW == 8 ? 2 : 1;      // row halves
  static constexpr int ROWS = 32 * MR * RH;       // output rows per workgroup
  static constexpr int CK = 16;                   // channels per chunk (one k-step)
  static constexpr int FT = kTileCols / V;
  static constexpr int NCOLS = FT * V;
  static constexpr int SPAN = (SIN * (FT - 1) + NQ) * V;  // window positions
  static constexpr int SLOTS = 2 * NPL + 1;       // (plane, octet) slots + 1 pad (odd)
  // stride-2 windows: FPAD spare slots after every frame. A 16-lane group of a
  // B-fragment read spans two output frames, i.e. input frames 2 apart, and
  // with the plain pitch those rows land on the same banks (2-way on every
  // read; the stride-2 forward measured 1.26 conflict cycles per LDS-active
  // cycle). The pads (bank model over every column tile and tap: 2.0 -> 1.06)
  // are taken where the LDS plan stays the same; V = 25 has no such pad.
  static constexpr int FPAD = SIN != 2 ? 0
                              : V == 18 ? (NPL == 2 ? 3 : NPL == 3 ? 1 : 0)
                              : V == 50 ? (NPL == 1 ? 5 : NPL == 2 ? 3 : 1)
                                        : 0;
  static constexpr int FP = V * SLOTS + FPAD;     // slots per window frame
  static constexpr int IMG = (SPAN / V) * FP * 16;  // window bytes
  static constexpr int NG = NQ / TG;              // steps per chunk
  static constexpr int WST = NPL * TG * 2 * ROWS * 16;  // packed weight bytes per step
  static constexpr int WDMA = WST / 1024;         // 1 KiB DMA pieces per step
  // LDS plan, first that fits: window double-buffered with a 3-step weight ring
  // (prefetch distance 2), double-buffered with a 2-step ring, or a single
  // window (written between two barriers) with a 3- or 2-step ring
  // (NPL = 1: two workgroups per CU)
  static constexpr int BUDGET = (NPL == 1 || NW == 4) ? 80 * 1024 : 160 * 1024;
  static constexpr int PLAN = 3 * WST + 2 * IMG <= BUDGET   ? 0
                              : 2 * WST + 2 * IMG <= BUDGET ? 1
                              : 3 * WST + IMG <= BUDGET     ? 2
                                                            : 3;
  static constexpr int NWIN = PLAN <= 1 ? 2 : 1;
  static constexpr int NWB = (PLAN == 0 || PLAN == 2) ? 3 : 2;
  static constexpr int PD = NWB - 1;
  static constexpr int EPI = MR == 1 ? (64 * kEpiPitch + 64 * V) * 4 : (ROWS * kEpiPitch + ROWS * V) * 4;
  static constexpr int MAIN = NWB * WST + NWIN * IMG;
  static constexpr int LDS = MAIN > EPI ? MAIN : EPI;
  static constexpr int NIT = SPAN * 2;            // (position, octet) staging items
  static constexpr int IPT = (NIT + NT - 1) / NT;  // staging items per thread
  static_assert(IPT >= 2 && IPT <= 4, "wait_img overloads");
  static constexpr int DPW = (WDMA + NW - 1) / NW;  // DMA pieces per wave and step (max)
  static constexpr int DPWMIN = WDMA / NW;          // ... issued by every wave
  // vmcnt allowance at step g's barrier (DMA(s) must have landed): the VMEM
  // operations every wave issued after DMA(s) in steady state — the pieces of
  // the PD-1 later weight steps and the window loads of the chunk-start steps
  // among the PD steps before s (fewer before that: the wait is conservative).
  // In a tile's last PD-1 steps fewer weight steps follow: the kernel waits
  // for everything there (vmcnt(0)).
  // A step's weight DMA pieces and (chunk start) window loads are issued tap by
  // tap (tap q: DMA pieces i with i % TG == q, then window loads [img_lo(q),
  // img_lo(q + 1)) of the IPT * 8), not as one burst after the barrier (+0.5%
  // cfg2 step, profiles/r6k_bench_spread_ab.txt)
  static constexpr int img_lo(int q) { return q * IPT * 8 / TG; }
  // window loads issued after a step's last DMA piece (that of tap min(DPW, TG) - 1)
  static constexpr int img_tail() { return IPT * 8 - img_lo((DPW < TG ? DPW : TG) - 1); }
  static constexpr int wait_n(int g) {
    int n = (PD - 1) * DPWMIN;
    for (int k = 1; k <= PD; ++k)
      if (((g - k) % NG + NG) % NG == 0) n += k == PD ? img_tail() : IPT * 8;
    return n;
  }
  static_assert(NQ % TG == 0, "whole tap groups");
  static_assert(LDS <= BUDGET, "LDS budget");
  static_assert(MR == 2 || 4096 + 4 * 2 * 64 * 16 * 4 <= LDS, "epilogue hand-over fits");
  static_assert((ROWS * kEpiPitch + ROWS * V) * 4 <= LDS, "row-major epilogue image fits");
};

// ---------------------------------------------------------------------------
// The folded block's SpatialConv backward fused into its data gradient's
// epilogue (capi.hip fold_spb; the backward of st_graphconv.py:148-150 with
// K = 1, V = 18 -- north star: the spatial and temporal halves in one kernel,
// A pinned in LDS / registers, H never in HBM). The tile's accumulators hold
// H = sum_q Wc_q^T dU (rows = input channels c, columns = 14 frames x 18
// joints; frame t = s_out m + p_out covers the stride-2 phases too). In halves
// of 64 rows (MR = 2: the waves of row half h hand their accumulators over):
//   1. H -> LDS image; the tile's x rows (deferred dx: the previous block's U)
//      -> LDS by 4-byte LDS-DMA (column offsets per lane, OOB -> 0);
//   2. row pass, item = (row, frame), three lanes per item (6 output joints
//      each, their 6 columns of A held in 108 registers, so a 16-byte LDS read
//      of H feeds 24 FMAs instead of 4 of A^T), 21 items per wave: dxhat[w] =
//      sum_v H[v] A[v][w], x rebuilt as k_spatial_bwd5's row pass does (prev
//      mode: ReLU(BN2_prev(U)), its mask and uhat), BN1(x) written back over x,
//      the BN1 sums sd += dxhat, sdn += dxhat (x - mu) invstd (prev: s1, s2)
//      combined over the item's lanes and added per row in LDS (fp64), dxhat
//      stored (consecutive lanes: consecutive 24-byte pieces of a row);
//   3. dA partials: thread = (6-joint v block, 6-joint w block, 1/56 of the
//      (row, frame) pairs), 36 register accumulators over both halves;
// then the partials meet in LDS and each dA entry is summed in a fixed order
// and added atomically (as k_spatial_bwd5 does), and the per-row sums go out
// with one fp64 atomic per row and statistic. Arithmetic per element is that of
// k_spatial_bwd5 (fp32, sums in fp64), so the results match it.
// ---------------------------------------------------------------------------
constexpr int kSpbAt = 18 * 20;  // A transposed, rows padded to 20 (16-byte aligned)
// H and x images of one 64-row half + A^T
// image pitch: 272 = 16 mod 64 banks (conflict-free 8-byte reads across rows)
constexpr int kSpbPitch = 272;
constexpr int kSpbRowTab = 2 * 64 * 8;  // per-row parameters [MR * 64][8] (MR <= 2)
constexpr int kSpbLds = (2 * 64 * kSpbPitch + kSpbAt + kSpbRowTab) * 4 + 2 * 64 * 4 * 8;

// MR = 1: the tile's x rows were loaded into registers during the main loop's
// last chunk (xpre[4 i + k]: row wave + 8 i, compacted column k * 64 + lane --
// the LDS-DMA pattern below), so only their LDS writes remain here
template <int MR>
__device__ __forceinline__ void spb_epilogue(const ConvGemmParams &p, floatx16 (&acc)[4],
                                             float *smem, int n, int r0, int m0, int mi,
                                             int nj0, const float *xpre) {
  constexpr int V = 18, FT = kTileCols / V, NCOLS = FT * V, P = kSpbPitch;
  constexpr int NSUB = 56;   // threads per (v block, w block) combination of dA
  constexpr int NSLOT = 21;  // row-pass items per wave (lanes 3 s + jb; lane 63 idle)
  float *const Himg = smem, *const Ximg = smem + 64 * P, *const At = smem + 2 * 64 * P;
  float *const rtab = At + kSpbAt;                                      // [MR * 64][8]
  double *const rsum = reinterpret_cast<double *>(rtab + kSpbRowTab);  // [MR][64][4]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int C = p.R, T = p.T_dst;
  const int nvf = min(FT, p.M - m0);  // valid frame slots of the tile
  // x DMA: compacted column j = k * 64 + lane of a row -> float offset in a channel
  unsigned coff[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int j = k * 64 + lane, mf = j / V, w = j - mf * V;
    const int t = p.s_out * (m0 + mf) + p.p_out;
    coff[k] = (j < NCOLS && mf < nvf && t < T) ? (unsigned)(t * V + w) : kOOB;
  }
  const int64_t cT = (int64_t)T * V;  // floats per channel
  const uint64_t xsrc = reinterpret_cast<uint64_t>(p.sx + (int64_t)n * C * cT);
  const int64_t xbytes = (int64_t)C * cT * 4;
  const int4v rsx = {(int)(uint32_t)xsrc, (int)((xsrc >> 32) & 0xffff),
                     (int)(xbytes > 0x7fffffff ? 0x7fffffff : xbytes), 0x00020000};
  const bool pv = p.prev.mean != nullptr;
  const int combo = tid / NSUB, sub = tid - combo * NSUB;
  const int vb = combo / 3, wb = combo - (combo / 3) * 3;
  // The per-row parameters (thread tid < MR * 64: row tid), loaded here, before
  // any of the epilogue's stores (vmcnt counts stores and loads in one in-order
  // counter: a load waited for after a store waits for that store too), and
  // written to LDS once the main loop's buffers are free
  float rp[8];  // mu, invstd, a = invstd g, beta; prev: mu, invstd, a, beta
  {
    const int c = r0 + tid;
    const bool rok = tid < MR * 64 && c < C, pok = pv && rok;
    const int cc = rok ? c : 0;  // (a valid address either way)
    const float *pm = pv ? p.prev.mean : p.mean1, *pi = pv ? p.prev.invstd : p.invstd1;
    const float *pg = pv ? p.prev.g : p.g1, *pbb = pv ? p.prev.b : p.b1;
    const float mu = p.mean1[cc], is = p.invstd1[cc], g = p.g1[cc], be = p.b1[cc];
    const float qmu = pm[cc], qis = pi[cc], qg = pg[cc], qb = pbb[cc];
    rp[0] = rok ? mu : 0.f;
    rp[1] = rok ? is : 0.f;
    rp[2] = rok ? is * g : 0.f;
    rp[3] = rok ? be : 0.f;
    rp[4] = pok ? qmu : 0.f;
    rp[5] = pok ? qis : 1.f;
    rp[6] = pok ? qis * qg : 1.f;
    rp[7] = pok ? qb : 0.f;
  }
  static_assert(kSpbAt <= 512, "one A^T element per thread");
  float sa = 0.f;  // A^T element tid
  if (tid < kSpbAt) {
    const int w = tid / 20, v = tid - w * 20;
    sa = v < V ? p.sA[v * V + w] : 0.f;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) asm volatile("" : "+v"(rp[i]));
  asm volatile("" : "+v"(sa));
  f2v dacc[18];  // (v, w pair) of this thread's 6 x 6 block
#pragma unroll
  for (int i = 0; i < 18; ++i) dacc[i] = (f2v){0.f, 0.f};
  // row pass lanes: item slot sl of the wave's 21, joint block jb (output joints 6 jb ..)
  const int jb = lane % 3, sl = lane / 3;
  const bool lact = lane < 3 * NSLOT;
  const bool need_s0 = !p.sd_given;  // (uniform)

#pragma unroll
  for (int h = 0; h < MR; ++h) {
    __syncthreads();  // every wave is done with the main loop's buffers / the last half
    // (the x rows' DMA first: its latency runs under the H image and table writes)
    asm volatile("s_nop 4" ::: "memory");  // descriptor SGPRs -> buffer_load
    for (int rr = wave; rr < (MR == 1 ? 0 : 64); rr += 8) {
      const int c = r0 + h * 64 + rr;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const unsigned voff = (c < C && coff[k] != kOOB) ? ((unsigned)(c * cT) + coff[k]) * 4u : kOOB;
        const unsigned m0v = (unsigned)reinterpret_cast<uintptr_t>(Ximg + rr * P + k * 64);
        unsigned keep;
        asm volatile(
            "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
            "buffer_load_dword %2, %3, 0 offen lds\n\ts_mov_b32 m0, %0"
            : "=&s"(keep)
            : "s"(m0v), "v"(voff), "s"(rsx)
            : "memory");
      }
    }
    if (MR == 1 || mi == h) {
#pragma unroll
      for (int rb = 0; rb < MR; ++rb)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc_to_img<P>(Himg, acc[rb * 2 + j], MR == 2 ? rb * 32 : mi * 32, (nj0 + j) * 32);
    }
    if (h == 0) {  // A^T[w][v], the row table, zeroed row sums
      if (tid < kSpbAt) At[tid] = sa;
      if (tid < MR * 64) {
        *reinterpret_cast<float4 *>(rtab + tid * 8) = make_float4(rp[0], rp[1], rp[2], rp[3]);
        *reinterpret_cast<float4 *>(rtab + tid * 8 + 4) = make_float4(rp[4], rp[5], rp[6], rp[7]);
      }
      for (int i = tid; i < MR * 64 * 4; i += 512) rsum[i] = 0.0;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if constexpr (MR == 1) {  // the prefetched x rows (landed: vmcnt(0) above)
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int k = 0; k < 4; ++k) Ximg[(wave + 8 * i) * P + k * 64 + lane] = xpre[4 * i + k];
    }
    __syncthreads();
    {  // dxhat, BN1(x) in place, the BN1 / chain sums, dxhat stores
      f2v a6[V][3];  // A[v][6 jb + 2 j2 + {0, 1}] (joint pairs: packed FMA)
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        const float *ac = At + (jb * 6 + j) * 20;
        float av[V];
#pragma unroll
        for (int v4 = 0; v4 < 16; v4 += 4) {
          const float4 q = *reinterpret_cast<const float4 *>(ac + v4);
          av[v4] = q.x;
          av[v4 + 1] = q.y;
          av[v4 + 2] = q.z;
          av[v4 + 3] = q.w;
        }
        const float2 q = *reinterpret_cast<const float2 *>(ac + 16);
        av[16] = q.x;
        av[17] = q.y;
#pragma unroll
        for (int v = 0; v < V; ++v) a6[v][j >> 1][j & 1] = av[v];
      }
      const float *rt = rtab + h * 64 * 8;
      for (int it0 = wave * NSLOT; it0 < 64 * FT; it0 += 8 * NSLOT) {
        const int it = it0 + sl;
        const int rr = it / FT, f = it - rr * FT;
        const bool ok = lact && it < 64 * FT && f < nvf;
        float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
        if (ok) {
          const float4 q0 = *reinterpret_cast<const float4 *>(rt + rr * 8);
          const float4 q1 = *reinterpret_cast<const float4 *>(rt + rr * 8 + 4);
          const float mu = q0.x, is = q0.y, a = q0.z, be = q0.w;
          const float pmu = q1.x, pis = q1.y, pa = q1.z, pb = q1.w;
          const int c = r0 + h * 64 + rr;
          const float *hr = Himg + rr * P + f * V;
          float hv[V];
#pragma unroll
          for (int i = 0; i < V / 2; ++i) {
            const float2 a2 = *reinterpret_cast<const float2 *>(hr + 2 * i);
            hv[2 * i] = a2.x;
            hv[2 * i + 1] = a2.y;
          }
          float d[6];
#pragma unroll
          for (int j2 = 0; j2 < 3; ++j2) {  // dxhat[w] = sum_v H[v] A[v][w], v in order
            f2v acc2 = (f2v){0.f, 0.f};
#pragma unroll
            for (int v = 0; v < V; ++v)
              acc2 = __builtin_elementwise_fma((f2v){hv[v], hv[v]}, a6[v][j2], acc2);
            d[2 * j2] = acc2.x;
            d[2 * j2 + 1] = acc2.y;
          }
          float *xr = Ximg + rr * P + f * V + jb * 6;
          float xs[6];
#pragma unroll
          for (int i = 0; i < 3; ++i) {
            const float2 x2 = *reinterpret_cast<const float2 *>(xr + 2 * i);
            xs[2 * i] = x2.x;
            xs[2 * i + 1] = x2.y;
          }
#pragma unroll
          for (int e = 0; e < 6; ++e) {
            float xx = xs[e], uh = 0.f;
            bool pm = false;
            if (pv) {  // the previous block's output x = ReLU(BN2(U)) as its output pass formed it
              const float t = (xx - pmu) * pa + pb;
              uh = (xx - pmu) * pis;
              pm = t > 0.f;
              xx = pm ? t : 0.f;
            }
            const float bn = (xx - mu) * a + be;
            if (need_s0) s0 += d[e];
            s1 = fmaf(d[e], (xx - mu) * is, s1);
            if (pm) {
              s2 += d[e];
              s3 = fmaf(d[e], uh, s3);
            }
            xs[e] = c < C ? bn : 0.f;
          }
#pragma unroll
          for (int i = 0; i < 3; ++i)
            *reinterpret_cast<float2 *>(xr + 2 * i) = make_float2(xs[2 * i], xs[2 * i + 1]);
          if (p.out && c < C) {
            float *dst = p.out + ((int64_t)n * C + c) * cT +
                         (int64_t)(p.s_out * (m0 + f) + p.p_out) * V + jb * 6;
#pragma unroll
            for (int i = 0; i < 3; ++i)
              *reinterpret_cast<float2 *>(dst + 2 * i) = make_float2(d[2 * i], d[2 * i + 1]);
          }
        }
        // the item's three lanes -> lane jb = 0 (fp32, as one 18-joint frame
        // sum), then the row's LDS sums in fp64; only the sums in use (sd comes
        // from the fp64 dU sums on the folded block: p.sd_given)
        auto red3 = [&](float v) {
          return v + (__shfl_down(v, 1, 64) + __shfl_down(v, 2, 64));
        };
        s1 = red3(s1);
        if (need_s0) s0 = red3(s0);
        if (pv) {
          s2 = red3(s2);
          s3 = red3(s3);
        }
        if (ok && jb == 0) {
          double *rs = rsum + (h * 64 + rr) * 4;
          if (need_s0) atomicAdd(rs, (double)s0);
          atomicAdd(rs + 1, (double)s1);
          if (pv) {
            atomicAdd(rs + 2, (double)s2);
            atomicAdd(rs + 3, (double)s3);
          }
        }
      }
    }
    __syncthreads();  // BN1(x) and H images complete (and this half's row sums)
    // dA partials over this half's (row, frame) pairs: thread = (v block, w block,
    // 1 / 56 of the pairs); after the last half the partials meet in LDS (over
    // the H image) and each entry is summed over its 56 threads in a fixed order
    if (combo < 9) {
      // (a fixed 16 pairs per thread, unrolled so the LDS reads run ahead; frames
      // >= nvf add nothing: their x image columns are zero -- OOB DMA, no row pass)
      static_assert((64 * FT) % NSUB == 0, "whole pair rounds");
#pragma unroll 4
      for (int q = sub; q < 64 * FT; q += NSUB) {
        const int rr = q / FT, f = q - rr * FT;
        const float *hr = Himg + rr * P + f * V + vb * 6;
        const float *xr = Ximg + rr * P + f * V + wb * 6;
        float hv[6];
        f2v xv[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          const float2 a2 = *reinterpret_cast<const float2 *>(hr + 2 * i);
          const float2 b2 = *reinterpret_cast<const float2 *>(xr + 2 * i);
          hv[2 * i] = a2.x;
          hv[2 * i + 1] = a2.y;
          xv[i] = (f2v){b2.x, b2.y};
        }
#pragma unroll
        for (int i = 0; i < 6; ++i)
#pragma unroll
          for (int j = 0; j < 3; ++j)
            dacc[i * 3 + j] = __builtin_elementwise_fma((f2v){hv[i], hv[i]}, xv[j], dacc[i * 3 + j]);
      }
    }
  }
  // the BN1 / chain sums: one fp64 atomic per row and statistic (rsum complete:
  // the barrier after the last row pass)
  if (tid < MR * 64) {
    const int c = r0 + tid;
    if (c < C) {
      const double *rs = rsum + tid * 4;
      if (!p.sd_given) atomicAdd(p.sd + c, rs[0]);
      atomicAdd(p.sdn + c, rs[1]);
      if (pv) {
        atomicAdd(p.prev.s1 + c, rs[2]);
        atomicAdd(p.prev.s2 + c, rs[3]);
      }
    }
  }
  __syncthreads();  // the images are read
  constexpr int PP = 37;  // partial pitch (odd: conflict-free column reads)
  float *part = smem;
  if (combo < 9) {
#pragma unroll
    for (int i = 0; i < 18; ++i) {
      part[(combo * NSUB + sub) * PP + 2 * i] = dacc[i].x;
      part[(combo * NSUB + sub) * PP + 2 * i + 1] = dacc[i].y;
    }
  }
  __syncthreads();
  if (tid < V * V) {  // (four interleaved chains: 14 dependent LDS reads, not 56)
    const int v = tid / V, w = tid - (tid / V) * V;
    const int cb = (v / 6) * 3 + w / 6, i = (v % 6) * 6 + (w % 6);
    const float *pc = part + cb * NSUB * PP + i;
    float s4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < NSUB; k += 4)
#pragma unroll
      for (int u = 0; u < 4; ++u) s4[u] += pc[(k + u) * PP];
    const float sum = (s4[0] + s4[1]) + (s4[2] + s4[3]);
    if (p.dA_part)  // (deterministic: launch_dA_reduce adds the partials in order)
      p.dA_part[(int64_t)blockIdx.x * (V * V) + tid] = sum;
    else
      atomicAdd(p.dA + tid, sum);
  }
}

// ---------------------------------------------------------------------------
// The folded block's forward without G (capi.hip fold_bna; north star N1: the
// SpatialConv joint contraction inside the temporal conv kernel). With one
// adjacency partition the joint contraction commutes with the folded conv's
// channel and tap mixing (st_graphconv.py:99, :148-150):
//   U[o,t,v] = sum_q sum_c Wc[o,c,q] G[c,t',v] + BT[o,t,v]
//            = sum_w A[v][w] U'[o,t,w] + BT[o,t,v],
//   U'[o,t,w] = sum_q sum_c Wc[o,c,q] xhat[c,t',w],   xhat = BN1(x) (0 in padded frames),
// so the window loader reads x and applies BN1 per channel (a [mu | a | be] table
// in LDS) before the fp16 split, and the epilogue contracts each (row, frame) of
// the tile with A (rows of A in LDS, 18 fp32 fma per output, fixed order) before
// the bias table, the BN2 statistics and the stores: G never exists.
// fp16 operand bound: |xhat| <= max_c |a_c| (M + |mu_c|) + |be_c|, M = max |x|.
// ---------------------------------------------------------------------------
constexpr int kBnaAr = 18 * 20;  // A[v][w], rows padded to 20 floats

__host__ __device__ constexpr int bna_cpad(int C) { return (C + 15) & ~15; }
// (+ 8 floats: block_max_all's scratch)
__host__ __device__ constexpr int bna_extra_bytes(int C) { return (3 * bna_cpad(C) + kBnaAr + 8) * 4; }

__device__ __forceinline__ int f16x2_se_bits(unsigned bits) {
  const int e = (int)(bits >> 23) & 0xff;
  const int se = e == 0 ? 0 : 140 - e;
  return se < -100 ? -100 : (se > 100 ? 100 : se);
}

// Block-wide max of m >= 0 (NT threads; red: NT / 64 floats of LDS); every
// thread gets the result (two barriers)
template <int NT>
__device__ __forceinline__ float block_max_all(float m, float *red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  float b = red[0];
#pragma unroll
  for (int i = 1; i < NT / 64; ++i) b = fmaxf(b, red[i]);
  __syncthreads();
  return b;
}

// |BN1(x)| bound of channel c (0 past C): |a| (M + |mu|) + |be|
__device__ __forceinline__ float bn1_bound(const ConvGemmParams &p, int c, float M, float &mu,
                                           float &a, float &be) {
  mu = a = be = 0.f;
  if (c >= p.C) return 0.f;
  mu = p.mean1[c];
  a = p.invstd1[c] * p.g1[c];
  be = p.b1[c];
  return fabsf(a) * (M + fabsf(mu)) + fabsf(be);
}

// The tile's output rows x frames in the row-major LDS image (acc_to_img),
// each (row, frame) replaced by its joint contraction with A: out[v] =
// sum_w A[v][w] in[w] (fp32 fma in w order). ar: A rows padded to 20.
template <int ROWS>
__device__ __forceinline__ void bna_contract(float *img, const float *ar) {
  constexpr int V = 18, FT = kTileCols / V, NPAIR = ROWS * FT, S = (NPAIR + 511) / 512;
  static_assert(S % 2 == 0, "pairs of (row, frame) items per packed fma");
  constexpr int S2 = S / 2;
  // items s and s + S2 of this thread side by side in one float2 (v_pk_fma_f32:
  // two outputs per instruction)
  f2v in[S2][V];
  int base[S];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int q = threadIdx.x + 512 * s, r = q % ROWS, f = q / ROWS;
    base[s] = q < NPAIR ? r * kEpiPitch + f * V : -1;
  }
#pragma unroll
  for (int s = 0; s < S2; ++s) {
    const float *s0 = img + (base[s] >= 0 ? base[s] : 0);
    const float *s1 = img + (base[s + S2] >= 0 ? base[s + S2] : 0);
#pragma unroll
    for (int i = 0; i < V / 2; ++i) {
      const float2 t0 = *reinterpret_cast<const float2 *>(s0 + 2 * i);
      const float2 t1 = *reinterpret_cast<const float2 *>(s1 + 2 * i);
      in[s][2 * i] = (f2v){t0.x, t1.x};
      in[s][2 * i + 1] = (f2v){t0.y, t1.y};
    }
  }
  // a few rows of A live at a time (fully unrolled, the compiler hoists every
  // row's LDS reads and spills); each output written in place as formed
#pragma unroll 3
  for (int v = 0; v < V; ++v) {
    float av[20];
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      const float4 t = *reinterpret_cast<const float4 *>(ar + v * 20 + 4 * i);
      av[4 * i] = t.x;
      av[4 * i + 1] = t.y;
      av[4 * i + 2] = t.z;
      av[4 * i + 3] = t.w;
    }
#pragma unroll
    for (int s = 0; s < S2; ++s) {
      f2v o = (f2v){av[0], av[0]} * in[s][0];
#pragma unroll
      for (int w = 1; w < V; ++w) o = __builtin_elementwise_fma((f2v){av[w], av[w]}, in[s][w], o);
      if (base[s] >= 0) img[base[s] + v] = o.x;
      if (base[s + S2] >= 0) img[base[s + S2] + v] = o.y;
    }
  }
}

// IB (NPL = 1 only): the input is stored in bf16 (p.in_bf16; a template switch so
// the staging code of the fp32-input kernels is unchanged)
// SPB (V = 18, NPL >= 2): the fused SpatialConv backward epilogue (spb_epilogue)
// BNA (V = 18, NPL = 2): the folded forward from x (BN1 in the loader, A in the
// epilogue; see bna_contract)
template <int NQ, int TG, int V, int SIN, int MR, int NPL, bool IB = false, bool SPB = false,
          bool BNA = false, int NW = 8>
__global__ __launch_bounds__(NW * 64, (NPL == 1 || NW == 4) ? 2 : 1) void k_conv_x3(ConvGemmParams p) {
  using G = ConvX3Geo<NQ, TG, V, SIN, MR, NPL, NW>;
  static_assert(!BNA || (V == 18 && NPL == 2 && !SPB), "bna: the folded fp16-split forward");
  static_assert(NW == 8 || (!SPB && !BNA && SIN == 1), "4-wave tiles: the plain stride-1 forward");
  static_assert(kBnaAr <= 512, "one A element per thread");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  char *lds = reinterpret_cast<char *>(smem);
  char *const wbuf0 = lds, *const win0 = lds + G::NWB * G::WST;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int half = wave >> 2;
  const int hi = lane >> 5, lo = lane & 31;
  int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int rt = bid % p.n_rtiles;
  bid /= p.n_rtiles;
  const int mt = bid % p.n_mtiles;
  const int n = bid / p.n_mtiles;
  const int r0 = rt * G::ROWS, m0 = mt * G::FT;
  const int cstride = p.T_src * V;
  const int g0 = (SIN * m0 + p.off) * V;
  const int nchunks = (p.C + G::CK - 1) / G::CK;
  const int nsteps = nchunks * G::NG;
  const char *wblk = reinterpret_cast<const char *>(p.wpk) + (int64_t)rt * nsteps * G::WST;
  const int mi = NW == 8 ? wave & 1 : 0;
  const int nj0 = NW == 8 ? ((wave >> 1) & 1) * 4 + half * 2 : wave * 2;

  // A fragment (plane 0, tap 0, octet hi, row block 0) and B fragments (tap 0,
  // plane 0, octet hi); wave rows mi*32*MR .. +32*MR-1 (MR 32-row blocks)
  const int ao = (hi * G::ROWS + mi * 32 * MR + lo) * 16;
  int bo[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = (nj0 + j) * 32 + lo;
    const int mf = col / V;
    const int cp = col < G::NCOLS ? SIN * mf * V + (col - mf * V) : 0;
    bo[j] = (cp * G::SLOTS + (cp / V) * G::FPAD + hi) * 16;
  }
  // window staging items (octet o, position pp), dealt over all 8 waves
  unsigned voff[G::IPT];
  int loff[G::IPT], ioct[G::IPT];
#pragma unroll
  for (int k = 0; k < G::IPT; ++k) {
    const int e = k * G::NT + tid;
    const int o = e / G::SPAN, pp = e - o * G::SPAN;
    const int g = g0 + pp;
    const bool ok = e < G::NIT && g >= 0 && g < cstride;
    voff[k] = ok ? (unsigned)(o * 8 * cstride + g) * 4u : kOOB;
    loff[k] = e < G::NIT ? (pp * G::SLOTS + (pp / V) * G::FPAD + o) * 16 : -1;
    ioct[k] = o;
  }
  // BNA: the BN1 table [mu | a | be] (Cp entries each) and the rows of A past
  // the kernel's own LDS plan, and the fp16 operand bound of BN1(x)
  const int Cp = nchunks * G::CK;
  float *const btab = smem + G::LDS / 4, *const arow = btab + 3 * Cp;
  // (loaded here into registers, written to LDS after the prologue's DMA is
  // issued, so the two latencies overlap; Cp <= 512 and kBnaAr <= 512: one
  // channel and one A element per thread)
  float t_mu = 0.f, t_a = 0.f, t_be = 0.f, t_ar = 0.f, t_bm = 0.f;
  if constexpr (BNA) {
    const float M = __builtin_bit_cast(float, amax_read(p.amax_in));
    if (tid < Cp) t_bm = bn1_bound(p, tid, M, t_mu, t_a, t_be);
    if (tid < kBnaAr) {
      const int v = tid / 20, w = tid - v * 20;
      t_ar = w < 18 ? p.sA[v * 18 + w] : 0.f;
    }
  }
  float st[G::IPT][8];
  // Window loads as inline asm too (the compiler neither waits for them nor
  // counts them; a compiler-counted load here would make hipcc wait vmcnt(0)
  // -- including the weight DMA issued after it -- before the write). Their
  // completion is waited for by wait_img, which names every destination.
  // (NPL = 1 with p.in_bf16: the input is bf16 -- e.g. the spatial conv output Z
  // kept in bf16 -- loaded as zero-extended shorts at half the byte offsets)
  static_assert(!IB || NPL == 1, "bf16 input: one-plane kernels");
  constexpr bool inb = IB;
  // NPL = 2: the window's power-of-two scale (f16x2_se of max |in|)
  int in_se = NPL == 2 && !BNA ? f16x2_se(p.amax_in) : 0;  // (BNA: after the table)
  float in_scale = pow2f(in_se);
  if (NPL == 2 && p.amax_keep && blockIdx.x == 0 && tid < kAmaxSlots)  // (slot 0: the bound)
    p.amax_keep[tid * kAmaxStride] = tid == 0 ? amax_read(p.amax_in) : 0u;
  // window loads [e0, e1) of the IPT * 8 (item k, channel j: e = 8 k + j)
  auto load_img_part = [&](int chunk, int e0, int e1, float (&sx)[G::IPT][8]) {
    // chunk == nchunks (the pipeline's tail) has no channels: every load is OOB -> 0
    const int esz = inb ? 2 : 4;
    const int64_t rem = (int64_t)(p.C - chunk * G::CK) * cstride * esz;
    const uint64_t src = reinterpret_cast<uint64_t>(p.in) +
                         (uint64_t)(((int64_t)n * p.in_bstride + (int64_t)chunk * G::CK * cstride) * esz);
    const int4v rs = {(int)(uint32_t)src, (int)((src >> 32) & 0xffff),
                      (int)(rem > 0x7fffffff ? 0x7fffffff : (rem > 0 ? rem : 0)), 0x00020000};
    asm volatile("s_nop 4" ::: "memory");  // descriptor SGPRs -> buffer_load
    if constexpr (inb) {
#pragma unroll
      for (int k = 0; k < G::IPT; ++k)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (8 * k + j >= e0 && 8 * k + j < e1)
            asm volatile("buffer_load_ushort %0, %1, %2, 0 offen"
                         : "=v"(sx[k][j])
                         : "v"(voff[k] == kOOB ? kOOB : (voff[k] >> 1) + (unsigned)(j * cstride * 2)),
                           "s"(rs)
                         : "memory");
    } else {
#pragma unroll
      for (int k = 0; k < G::IPT; ++k)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (8 * k + j >= e0 && 8 * k + j < e1)
            asm volatile("buffer_load_dword %0, %1, %2, 0 offen"
                         : "=v"(sx[k][j])
                         : "v"(voff[k] + (unsigned)(j * cstride * 4)), "s"(rs)
                         : "memory");
    }
  };
  auto load_img = [&](int chunk) { load_img_part(chunk, 0, G::IPT * 8, st); };
  // SPB, MR = 1 (XPF): the epilogue's 64 x rows (its LDS-DMA pattern: row
  // wave + 8 i, compacted column k * 64 + lane, 0 outside the tile) loaded into
  // registers in place of the last chunk's (never read) zero window, so their
  // HBM latency runs under the last chunk's MFMAs instead of the epilogue
  constexpr bool XPF = SPB && MR == 1;
  constexpr int NXP = XPF ? 32 : 1;
  float xpre[NXP];
#pragma unroll
  for (int i = 0; i < NXP; ++i) xpre[i] = 0.f;
  auto load_x_part = [&](int e0, int e1) {
    if constexpr (XPF) {
      const int Cx = p.R, T = p.T_dst;
      const int64_t cT = (int64_t)T * V;
      const uint64_t xsrc = reinterpret_cast<uint64_t>(p.sx + (int64_t)n * Cx * cT);
      const int64_t xbytes = (int64_t)Cx * cT * 4;
      const int4v rsx = {(int)(uint32_t)xsrc, (int)((xsrc >> 32) & 0xffff),
                         (int)(xbytes > 0x7fffffff ? 0x7fffffff : xbytes), 0x00020000};
      const int nvf = min(G::FT, p.M - m0);
      asm volatile("s_nop 4" ::: "memory");  // descriptor SGPRs -> buffer_load
#pragma unroll
      for (int e = 0; e < 32; ++e)
        if (e >= e0 && e < e1) {
          const int i = e >> 2, k = e & 3;
          const int j = k * 64 + lane, mf = j / V, w = j - mf * V;
          const int t = p.s_out * (m0 + mf) + p.p_out;
          const int c = r0 + wave + 8 * i;
          const bool ok = j < G::NCOLS && mf < nvf && t < T && c < Cx;
          const unsigned voff = ok ? ((unsigned)(c * cT) + (unsigned)(t * V + w)) * 4u : kOOB;
          asm volatile("buffer_load_dword %0, %1, %2, 0 offen"
                       : "=v"(xpre[e])
                       : "v"(voff), "s"(rsx)
                       : "memory");
        }
    }
  };
  auto write_img = [&](char *win, int chunk, float (&sx)[G::IPT][8]) {
    // (BNA: chunk nchunks is the pipeline's zero tail, never read: any table row)
    const int cch = min(chunk, nchunks - 1) * G::CK;
#pragma unroll
    for (int k = 0; k < G::IPT; ++k)
      if (NPL == 1 && loff[k] >= 0) {  // bf16 operands: one rounded plane
        uint4 h;
        if constexpr (inb) {  // already bf16 (zero-extended shorts)
          const auto u = [&](int j) { return __builtin_bit_cast(unsigned, sx[k][j]); };
          h.x = u(0) | (u(1) << 16);
          h.y = u(2) | (u(3) << 16);
          h.z = u(4) | (u(5) << 16);
          h.w = u(6) | (u(7) << 16);
        } else {
          h.x = pk2(sx[k][0], sx[k][1]);
          h.y = pk2(sx[k][2], sx[k][3]);
          h.z = pk2(sx[k][4], sx[k][5]);
          h.w = pk2(sx[k][6], sx[k][7]);
        }
        *reinterpret_cast<uint4 *>(win + loff[k]) = h;
      } else if (NPL == 2 && loff[k] >= 0) {  // fp16 (h, l) planes of the scaled input
        const float sc = in_scale;
        float xv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) xv[j] = sx[k][j];
        if constexpr (BNA) {  // BN1 of the item's 8 channels; 0 in padded frames
          const float *tb = btab + cch + ioct[k] * 8;
          float mu[8], a[8], be[8];
#pragma unroll
          for (int h4 = 0; h4 < 2; ++h4) {
            const float4 m4 = *reinterpret_cast<const float4 *>(tb + 4 * h4);
            const float4 a4 = *reinterpret_cast<const float4 *>(tb + Cp + 4 * h4);
            const float4 b4 = *reinterpret_cast<const float4 *>(tb + 2 * Cp + 4 * h4);
            mu[4 * h4] = m4.x; mu[4 * h4 + 1] = m4.y; mu[4 * h4 + 2] = m4.z; mu[4 * h4 + 3] = m4.w;
            a[4 * h4] = a4.x; a[4 * h4 + 1] = a4.y; a[4 * h4 + 2] = a4.z; a[4 * h4 + 3] = a4.w;
            be[4 * h4] = b4.x; be[4 * h4 + 1] = b4.y; be[4 * h4 + 2] = b4.z; be[4 * h4 + 3] = b4.w;
          }
          const bool live = voff[k] != kOOB;
#pragma unroll
          for (int j = 0; j < 8; ++j) xv[j] = live ? (xv[j] - mu[j]) * a[j] + be[j] : 0.f;
        }
        uint4 h, l;
        splith2(xv[0] * sc, xv[1] * sc, h.x, l.x);
        splith2(xv[2] * sc, xv[3] * sc, h.y, l.y);
        splith2(xv[4] * sc, xv[5] * sc, h.z, l.z);
        splith2(xv[6] * sc, xv[7] * sc, h.w, l.w);
        *reinterpret_cast<uint4 *>(win + loff[k]) = h;
        *reinterpret_cast<uint4 *>(win + loff[k] + 32) = l;
      } else if (loff[k] >= 0) {
        uint4 h, m, l;
        split2(sx[k][0], sx[k][1], h.x, m.x, l.x);
        split2(sx[k][2], sx[k][3], h.y, m.y, l.y);
        split2(sx[k][4], sx[k][5], h.z, m.z, l.z);
        split2(sx[k][6], sx[k][7], h.w, m.w, l.w);
        *reinterpret_cast<uint4 *>(win + loff[k]) = h;
        *reinterpret_cast<uint4 *>(win + loff[k] + 32) = m;
        *reinterpret_cast<uint4 *>(win + loff[k] + 64) = l;
      }
  };
  // Weight DMA as inline asm: hipcc treats an LDS-DMA builtin as a pending LDS
  // write and waits for it (vmcnt) before the next ds_read of ANY buffer, which
  // would drain the prefetch every step. Its completion is counted by hand
  // (the s_waitcnt before each step's barrier).
  const uint64_t wsrc = reinterpret_cast<uint64_t>(wblk);
  const int4v rsw = {(int)(uint32_t)wsrc, (int)((wsrc >> 32) & 0xffff), nsteps * G::WST,
                     0x00020000};
  const unsigned lds0 = (unsigned)reinterpret_cast<uintptr_t>(wbuf0);
  // (qq >= 0: only the pieces i % TG == qq, issued with tap qq)
  auto dma_w = [&](int step, int buf, int qq = -1) {
#pragma unroll
    for (int i = 0; i < G::DPW; ++i) {
      const int d = i * NW + wave;
      if (d < G::WDMA && (qq < 0 || i % TG == qq)) {
        const unsigned voffw = (unsigned)(step * G::WST + d * 1024 + lane * 16);
        const unsigned m0v = lds0 + (unsigned)(buf * G::WST + d * 1024);
        unsigned keep;
        asm volatile(
            "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
            "buffer_load_dwordx4 %2, %3, 0 offen lds\n\ts_mov_b32 m0, %0"
            : "=&s"(keep)
            : "s"(m0v), "v"(voffw), "s"(rsw)
            : "memory");
      }
    }
  };

  // acc: the h*h products; acl: the five small cross terms (<= 2^-8 of acc),
  // accumulated apart so their roundings stay 2^-8 smaller; summed at the end.
  // Tile (row block rb, column tile j) -> acc[rb*2 + j] (MR = 1: acc[2..3] are
  // the hand-over registers of the stride-2 epilogue)
  // (NPL = 1: plain bf16 operands, acc only)
  // (NW = 4: every product in acc -- one fp32 chain per tile, small products
  // first within a tap; the 64 registers of acl would spill the 4-wave kernel)
  constexpr bool kOneAcc = NW == 4;
  constexpr int NACL = NPL >= 2 && !kOneAcc ? 2 * MR : 1;
  floatx16 acc[4], acl[NACL];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[j][i] = 0.f;
#pragma unroll
  for (int j = 0; j < NACL; ++j)
#pragma unroll
    for (int i = 0; i < 16; ++i) acl[j][i] = 0.f;

  struct Frag {
    bf16x8_t a[NPL][MR], b[NPL][2];
  };
  auto ld = [&](const char *wa, const char *win, int qq, int q, Frag &f) {
#pragma unroll
    for (int pl = 0; pl < NPL; ++pl)
#pragma unroll
      for (int rb = 0; rb < MR; ++rb)
        f.a[pl][rb] = *reinterpret_cast<const bf16x8_t *>(
            wa + (pl * TG + qq) * 2 * G::ROWS * 16 + rb * 32 * 16);
#pragma unroll
    for (int pl = 0; pl < NPL; ++pl)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        f.b[pl][j] =
            *reinterpret_cast<const bf16x8_t *>(win + bo[j] + (q * G::FP + 2 * pl) * 16);
  };
  // the six products (plane of A, plane of B) of one tap over the MR x 2 tiles
  // (NPL = 1: the one product)
  // (NPL = 2: the three fp16 products hh, hl, lh)
  auto mm = [&](const Frag &f) {
    constexpr int PA[6] = {0, 0, 1, 0, 1, 2}, PB[6] = {0, 1, 0, 2, 1, 0};
    constexpr int NPROD = NPL == 3 ? 6 : (NPL == 2 ? 3 : 1);
#pragma unroll
    for (int t = 0; t < NPROD; ++t)
#pragma unroll
      for (int rb = 0; rb < MR; ++rb)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          if (t == 0)
            acc[rb * 2 + j] = mfma_p<NPL>(f.a[0][rb], f.b[0][j], acc[rb * 2 + j]);
          else
            acl[(rb * 2 + j) % NACL] = mfma_p<NPL>(f.a[PA[t] % NPL][rb], f.b[PB[t] % NPL][j],
                                                   acl[(rb * 2 + j) % NACL]);
        }
  };

  // MR = 1: two fragment sets (tap qq of a step in f[qq % 2]); MR = 2: one,
  // refilled in place (tap2)
  constexpr int NF = MR == 1 ? 2 : 1;
  Frag f[NF];
#pragma unroll
  for (int d = 0; d < G::PD; ++d)
    if (d < nsteps) dma_w(d, d);
  load_img(0);
  if constexpr (BNA) {  // the BN1 table, A's rows, the operand bound
    if (tid < Cp) {
      btab[tid] = t_mu;
      btab[Cp + tid] = t_a;
      btab[2 * Cp + tid] = t_be;
    }
    if (tid < kBnaAr) arow[tid] = t_ar;
    const float bound = block_max_all<512>(t_bm, arow + kBnaAr);  // (barriers inside)
    in_se = f16x2_se_bits(__builtin_bit_cast(unsigned, bound));
    in_scale = pow2f(in_se);
  }
  // MR = 1: tap qq's MFMAs (fragment set fm) with the NEXT tap's fragment reads
  // (set fl from weights wl / window wn, tap ql, window frame qn) interleaved
  constexpr int NR1 = NPL * (MR + 2), NM1 = (NPL == 3 ? 6 : (NPL == 2 ? 3 : 1)) * 2 * MR;
  constexpr int NI1 = NR1 < NM1 ? NR1 : NM1;
  auto mm_ld1 = [&](const Frag &fm, const char *wl, const char *wn, int ql, int qn, Frag &fl) {
    ld(wl, wn, ql, qn, fl);
    mm(fm);
#pragma unroll
    for (int i = 0; i < NI1; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
    }
    if constexpr (NM1 > NI1) __builtin_amdgcn_sched_group_barrier(0x008, NM1 - NI1, 0);
    if constexpr (NR1 > NI1) __builtin_amdgcn_sched_group_barrier(0x100, NR1 - NI1, 0);
    __builtin_amdgcn_sched_barrier(0);
  };
  // MR = 2: one fragment set, refilled in place for the next tap as its planes
  // retire (48 instead of 96 fragment registers live). Product order per tap:
  // mm, lh, hl, mh, hm, hh -- the first (a1 x b1) uses neither plane-0
  // fragment, which are the last ones refilled. tap2(nx, wl, wn, ql, qn): the
  // MFMAs of the tap in f[0], refilled (nx) with tap ql / window frame qn
  auto grp = [&](int pa, int pb) {
    Frag &fr = f[0];
#pragma unroll
    for (int rb = 0; rb < MR; ++rb)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if ((pa == 0 && pb == 0) || kOneAcc)
          acc[rb * 2 + j] =
              mfma_p<NPL>(fr.a[pa % NPL][rb], fr.b[pb % NPL][j], acc[rb * 2 + j]);
        else
          acl[(rb * 2 + j) % NACL] =
              mfma_p<NPL>(fr.a[pa % NPL][rb], fr.b[pb % NPL][j], acl[(rb * 2 + j) % NACL]);
      }
  };
  auto lda = [&](const char *wl, int qq, int pl) {
#pragma unroll
    for (int rb = 0; rb < MR; ++rb)
      f[0].a[pl][rb] = *reinterpret_cast<const bf16x8_t *>(
          wl + (pl * TG + qq) * 2 * G::ROWS * 16 + rb * 32 * 16);
  };
  auto ldb = [&](const char *wn, int q, int pl) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
      f[0].b[pl][j] = *reinterpret_cast<const bf16x8_t *>(wn + bo[j] + (q * G::FP + 2 * pl) * 16);
  };
  auto tap2 = [&](bool nx, const char *wl, const char *wn, int ql, int qn) {
    if constexpr (NPL == 2) {
      // fp16 (h, l): products lh, hl, hh; plane 1 of A / B refilled as it retires
      grp(1, 0);
      if (nx) lda(wl, ql, 1);
      __builtin_amdgcn_sched_barrier(0);
      grp(0, 1);
      if (nx) ldb(wn, qn, 1);
      __builtin_amdgcn_sched_barrier(0);
      grp(0, 0);
      if (nx) {
        lda(wl, ql, 0);
        ldb(wn, qn, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    } else {
      grp(1, 1);
      __builtin_amdgcn_sched_barrier(0);
      grp(2, 0);
      if (nx) lda(wl, ql, 2);
      __builtin_amdgcn_sched_barrier(0);
      grp(0, 2);
      if (nx) ldb(wn, qn, 2);
      __builtin_amdgcn_sched_barrier(0);
      grp(1, 0);
      if (nx) lda(wl, ql, 1);
      __builtin_amdgcn_sched_barrier(0);
      grp(0, 1);
      if (nx) ldb(wn, qn, 1);
      __builtin_amdgcn_sched_barrier(0);
      grp(0, 0);
      if (nx) {
        lda(wl, ql, 0);
        ldb(wn, qn, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  wait_img<0>(st);
  write_img(win0, 0, st);
  for (int c = 0; c < nchunks; ++c) {
    const char *win = win0 + (G::NWIN == 2 ? (c & 1) * G::IMG : 0);
#pragma unroll
    for (int g = 0; g < G::NG; ++g) {
      const int s = c * G::NG + g;
      // step s's weights: each wave waits for its own DMA pieces (issued PD
      // steps earlier; later pieces and window loads stay in flight), then the
      // barrier publishes them and chunk c's window (written in the previous
      // chunk's last step)
      if (XPF && c + 1 == nchunks && s + G::PD - 1 < nsteps)  // (32 x loads, not IPT * 8)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::wait_n(g) + (g >= 1 ? 32 - G::IPT * 8 : 0))
                     : "memory");
      else if (s + G::PD - 1 < nsteps)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::wait_n(g)) : "memory");
      else  // a tile's last steps: fewer weight steps were issued after DMA(s)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      const char *wa = wbuf0 + (s % G::NWB) * G::WST + ao;
      ld(wa, win, 0, g * TG, f[0]);  // tap 0's fragment reads
      // (VMEM issue after this step's first fragment reads: a compiler wait
      // placed before those reads then finds no load of ours in flight)
#pragma unroll
      for (int qq = 0; qq < TG; ++qq) {
        const bool nx = qq + 1 < TG;
        // this tap's share of the step's VMEM issue: the next weights' DMA
        // pieces and (first step) chunk c+1's window loads (unconditional:
        // chunk == nchunks loads zeros and is never read; XPF loads the
        // epilogue's x rows in its place)
        if (s + G::PD < nsteps) dma_w(s + G::PD, (s + G::PD) % G::NWB, qq);
        if (g == 0) {
          if (XPF && c + 1 == nchunks)
            load_x_part(qq * 32 / TG, (qq + 1) * 32 / TG);
          else
            load_img_part(c + 1, G::img_lo(qq), G::img_lo(qq + 1), st);
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (MR == 1) {
          if (nx)  // tap qq+1's fragment reads among tap qq's MFMAs
            mm_ld1(f[qq % NF], wa, win, qq + 1, g * TG + qq + 1, f[(qq + 1) % NF]);
          else
            mm(f[qq % NF]);
          __builtin_amdgcn_sched_barrier(0);
        } else {
          tap2(nx, wa, win, qq + 1, g * TG + qq + 1);
        }
      }
      if (g == G::NG - 1 && !(XPF && c + 1 == nchunks)) {
        // issued after the loads (step g = 0): the weight pieces of steps 1..NG-1
        wait_img<(G::NG - 1) * G::DPWMIN>(st);
        if (G::NWIN == 1)  // single window: every wave is done reading chunk c's
          asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        write_img(win0 + (G::NWIN == 2 ? ((c + 1) & 1) * G::IMG : 0), c + 1, st);
      }
    }
  }
  if constexpr (NPL == 3) {
#pragma unroll
    for (int j = 0; j < 2 * MR; ++j) acc[j] += acl[j];
  } else if constexpr (NPL == 2) {  // undo the operand scales (powers of two: exact)
    const float ia = pow2f(-in_se), iw = pow2f(-f16x2_se(p.amax_w));
#pragma unroll
    for (int j = 0; j < 2 * MR; ++j) acc[j] = (kOneAcc ? acc[j] : acc[j] + acl[j]) * ia * iw;
  }
  if constexpr (SPB) {
    static_assert(V == 18 && SIN == 1 && NPL >= 2, "the folded block's data gradient");
    if constexpr (XPF) {  // (no consumer of xpre above the wait for its loads)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
      for (int i = 0; i < NXP; ++i) asm volatile("" : "+v"(xpre[i]));
    }
    spb_epilogue<MR>(p, acc, smem, n, r0, m0, mi, nj0, xpre);
    return;
  }
  if (p.s_out == 1) {
    // row-major epilogue through LDS: every wave writes its two tiles, then all
    // 512 threads store whole 16-byte row pieces (device_common.h)
    __syncthreads();  // every wave is done with the buffers
#pragma unroll
    for (int rb = 0; rb < MR; ++rb)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc_to_img(smem, acc[rb * 2 + j], mi * 32 * MR + rb * 32, (nj0 + j) * 32);
    __syncthreads();
    if constexpr (BNA) {  // U' -> U = A U' per (row, frame), in place
      bna_contract<G::ROWS>(smem, arow);
      __syncthreads();
    }
    // (one-plane bf16 path: the output may be stored in bf16, p.out_bf16 -- the
    // data gradient dZ of capi.hip dz_bf16)
    conv_tile_store_rows<V, G::NCOLS, G::NT, G::ROWS, NPL == 1, NPL != 1>(
        p, smem, smem + G::ROWS * kEpiPitch, n, r0, m0);
    return;
  }
  // (MR >= 2: never -- 128-row tiles are launched for s_out == 1 only)
  if constexpr (MR == 1) {
    // hand-over: waves 4-7 give their two column tiles to waves 0-3 (same rows,
    // next two tiles), which run the shared 4-wave epilogue
    float *ho = smem + 1024 + (wave & 3) * 2 * 64 * 16;
    __syncthreads();  // every wave is done with the buffers
    if (half == 1) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i = 0; i < 16; ++i) ho[(j * 16 + i) * 64 + lane] = acc[j][i];
    }
    __syncthreads();
    if (half == 0) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[2 + j][i] = ho[(j * 16 + i) * 64 + lane];
      conv_tile_epilogue<V, G::NCOLS, false, NPL == 1, NPL != 1>(p, acc, n, r0, m0, smem);
    } else if (p.stat_sum) {
      __syncthreads();  // the epilogue's one barrier (statistics)
    }
  }
}

// Packs w[r*w_sr + c*w_sc + q*w_sq] split into three bf16 planes:
// wpk[rt][chunk][tap group][plane][tap in group][octet][ROWS][8] (ROWS = 64 or
// 128 rows per tile; zero padded rows and channels), so one step's weights are
// one contiguous run.
__global__ void k_pack_conv_w_x3(const float *w, __bf16 *wpk, int R, int C, int NQ, int TG,
                                 int nch, int rows, int npl, int64_t w_sr, int64_t w_sc,
                                 int64_t w_sq, int64_t total, const unsigned *amax_w) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  // (the fp16 planes' operand scale: read once per wave, before any lane leaves)
  const int se = npl == 2 ? f16x2_se_bits(amax_w ? amax_read_wave(amax_w) : 0x3f800000u) : 0;
  if (idx >= total) return;
  const int jj = (int)(idx & 7);
  int64_t t = idx >> 3;
  const int rl = (int)(t % rows);
  t /= rows;
  const int o = (int)(t & 1);
  t >>= 1;
  const int qq = (int)(t % TG);
  t /= TG;
  const int pl = (int)(t % npl);
  t /= npl;
  const int NG = NQ / TG;
  const int g = (int)(t % NG);
  t /= NG;
  const int ch = (int)(t % nch);
  const int rt = (int)(t / nch);
  const int r = rt * rows + rl, c = ch * 16 + o * 8 + jj, q = g * TG + qq;
  float v = 0.f;
  if (r < R && c < C) v = w[(int64_t)r * w_sr + (int64_t)c * w_sc + (int64_t)q * w_sq];
  if (npl == 2) {  // fp16 (h, l) of the power-of-two-scaled weight
    const float vs = v * pow2f(se);
    const _Float16 h = (_Float16)vs;
    const _Float16 l = (_Float16)(vs - (float)h);
    reinterpret_cast<_Float16 *>(wpk)[idx] = pl == 0 ? h : l;
    return;
  }
  const __bf16 h = (__bf16)v;
  const float r1 = v - (float)h;
  const __bf16 m = (__bf16)r1;
  const __bf16 l = (__bf16)(r1 - (float)m);
  wpk[idx] = pl == 0 ? h : (pl == 1 ? m : l);
}

// The pack of several weight tensors in one launch (stgcn_fold_prep: every
// folded block's forward and data-gradient weights once per step). Same layout
// and arithmetic as k_pack_conv_w_x3, but one thread per run of 8 channels
// (one 16-byte piece of every plane: unit u = (rt, chunk, tap group, tap in
// group, octet, row), its npl pieces npl * 8 elements apart... written whole)
// and 32-bit index arithmetic (a job packs < 2^31 elements): the per-element
// form spent most of its time on 64-bit divisions. Job i covers units
// [start[i], start[i] + total / (8 npl)) of the concatenated jobs, its start a
// multiple of the 256-thread block (one job per block: the operand scale is
// read once per wave).
struct PackJobs {
  PackJob j[kPackJobs];
  int64_t start[kPackJobs + 1];
  int n;
};

__global__ __launch_bounds__(256) void k_pack_conv_w_x3_multi(PackJobs js) {
  const int64_t gi = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int k = 0;  // (uniform: job starts are multiples of the block)
  while (k + 1 < js.n && gi >= js.start[k + 1]) ++k;
  const PackJob &q = js.j[k];
  const int se = q.npl == 2 ? f16x2_se_bits(q.amax_w ? amax_read_wave(q.amax_w) : 0x3f800000u) : 0;
  const int npl = q.npl, rows = q.rows, TG = q.TG, NG = q.NQ / q.TG;
  const int units = (int)(q.total / (8 * npl));
  const int u0 = (int)(gi - js.start[k]);
  if (u0 >= units) return;
  int t = u0;
  const int rl = t % rows;
  t /= rows;
  const int o = t & 1;
  t >>= 1;
  const int qq = t % TG;
  t /= TG;
  const int g = t % NG;
  t /= NG;
  const int ch = t % q.nch;
  const int rt = t / q.nch;
  const int r = rt * rows + rl, c0 = ch * 16 + o * 8, tap = g * TG + qq;
  float v[8];
  const bool rok = r < q.R;
  const float *src = q.w + (int64_t)(rok ? r : 0) * q.w_sr + (int64_t)tap * q.w_sq;
#pragma unroll
  for (int jj = 0; jj < 8; ++jj)
    v[jj] = (rok && c0 + jj < q.C) ? src[(int64_t)(c0 + jj) * q.w_sc] : 0.f;
  // element index of plane 0's piece; plane pl is pl * TG * 2 * rows * 8 further
  const int64_t base = ((((int64_t)(rt * q.nch + ch) * NG + g) * npl * TG + qq) * 2 + o) *
                           rows * 8 + (int64_t)rl * 8;
  const int64_t pstride = (int64_t)TG * 2 * rows * 8;
  if (npl == 2) {  // fp16 (h, l) of the power-of-two-scaled weight
    const float sc = pow2f(se);
    unsigned hw[4], lw[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
      const float a = v[2 * i] * sc, b = v[2 * i + 1] * sc;
      const _Float16 ha = (_Float16)a, hb = (_Float16)b;
      const h2_t hv = {ha, hb}, lv = {(_Float16)(a - (float)ha), (_Float16)(b - (float)hb)};
      hw[i] = __builtin_bit_cast(unsigned, hv);
      lw[i] = __builtin_bit_cast(unsigned, lv);
    }
    _Float16 *out = reinterpret_cast<_Float16 *>(q.wpk);
    *reinterpret_cast<uint4 *>(out + base) = make_uint4(hw[0], hw[1], hw[2], hw[3]);
    *reinterpret_cast<uint4 *>(out + base + pstride) = make_uint4(lw[0], lw[1], lw[2], lw[3]);
    return;
  }
  __bf16 pv[3][8];
#pragma unroll
  for (int jj = 0; jj < 8; ++jj) {
    const __bf16 h = (__bf16)v[jj];
    const float r1 = v[jj] - (float)h;
    const __bf16 m = (__bf16)r1;
    pv[0][jj] = h;
    pv[1][jj] = m;
    pv[2][jj] = (__bf16)(r1 - (float)m);
  }
  __bf16 *out = reinterpret_cast<__bf16 *>(q.wpk);
#pragma unroll
  for (int pl = 0; pl < 3; ++pl)  // (npl = 1: h; npl = 3: h, m, l)
    if (pl < npl) {
      unsigned w4[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bf16x2_t pr = {pv[pl][2 * i], pv[pl][2 * i + 1]};
        w4[i] = __builtin_bit_cast(unsigned, pr);
      }
      *reinterpret_cast<uint4 *>(out + base + pl * pstride) = make_uint4(w4[0], w4[1], w4[2], w4[3]);
    }
}

static int x3_tg(int NQ) { return NQ == 9 ? 3 : NQ; }

bool conv_x3_supported(const ConvGemmParams &p) {
  if (p.C < 16) return false;
  if (p.V != 18 && p.V != 25) return false;
  if (p.FT != kTileCols / p.V) return false;
  if (p.s_in == 2) return p.NQ == 9;  // stride-2 forward
  return p.s_in == 1 && (p.NQ == 9 || p.NQ == 5 || p.NQ == 4);
}

bool conv_x3_bna_supported(const ConvGemmParams &p) {
  if (p.V != 18 || p.NQ != 9 || p.s_out != 1 || p.spb || !conv_x3_supported(p)) return false;
  if (bna_cpad(p.C) > 512) return false;  // (the kernel sets one table channel per thread)
  // the largest plan of the forward instances (128-row tiles, stride 2) + the table
  constexpr int lds = ConvX3Geo<9, 3, 18, 2, 2, 2>::LDS;
  return lds + bna_extra_bytes(p.C) <= 160 * 1024;
}

size_t conv_x3_wpk_bytes(const ConvGemmParams &p) {
  return (size_t)p.n_rtiles * ((p.C + 15) / 16) * 3 * p.NQ * 16 * 64 * 2;
}

// 128-row tiles (two 32-row blocks per wave: half the weight and window
// staging per MFMA, half the window re-reads over the row tiles) for the
// 9-tap launches with a whole number of them and unit output stride
// (STGCN_AB_X3_MR1 build: 64-row tiles everywhere, A/B measurement only)
static bool x3_wide_rows(const ConvGemmParams &p) {
  constexpr bool off = STGCN_AB_X3_MR1 != 0;
  return !off && p.NQ == 9 && p.s_out == 1 && p.R % 128 == 0;
}
// 4-wave 64-row tiles, two workgroups per CU (ConvX3Geo NW = 4): the fp16-split
// stride-1 forward where the caller marked it (p.w4: capi.hip fwd_w4), up to 128
// output rows (at 256 the second read of each window per 128 rows costs what
// the overlap gains: L8 0.668 vs 0.654 ms, profiles/r6b_kbench_w4.txt). Decides
// the packed weight layout (64-row tiles) and the kernel alike.
static bool x3_w4(const ConvGemmParams &p, int npl) {
  constexpr bool off = STGCN_AB_X3_NOW4 != 0;
  return !off && p.w4 && npl == 2 && !p.spb && !p.bna && p.NQ == 9 && p.s_in == 1 &&
         p.s_out == 1 && (p.V == 18 || p.V == 25) && p.R <= 128;
}
template <int V>
static void launch_cx_w4(const ConvGemmParams &p, int nblk, hipStream_t s) {
  using G = ConvX3Geo<9, 3, V, 1, 2, 2, 4>;
  hipLaunchKernelGGL((k_conv_x3<9, 3, V, 1, 2, 2, false, false, false, 4>), dim3(nblk),
                     dim3(G::NT), G::LDS, s, p);
}

template <int NQ, int V, int SIN, int MR, int NPL>
static bool launch_cx_if(const ConvGemmParams &p, int nblk, hipStream_t s) {
  if (p.V != V || p.s_in != SIN) return false;
  constexpr int TG = NQ == 9 ? 3 : NQ;
  constexpr int lds = ConvX3Geo<NQ, TG, V, SIN, MR, NPL>::LDS;
  if constexpr (V == 18 && SIN == 1 && NPL >= 2) {
    if (p.spb) {  // the folded block's data gradient with the SpatialConv backward
      constexpr int lds_spb = lds > kSpbLds ? lds : kSpbLds;
      hipLaunchKernelGGL((k_conv_x3<NQ, TG, V, SIN, MR, NPL, false, true>), dim3(nblk), dim3(512),
                         lds_spb, s, p);
      return true;
    }
  }
  if constexpr (V == 18 && NPL == 2 && NQ == 9) {
    if (p.bna) {  // the folded forward from x (BN1 in the loader, A in the epilogue)
      const int lds_bna = lds + bna_extra_bytes(p.C);
      if (lds_bna > 160 * 1024) return false;
      hipLaunchKernelGGL((k_conv_x3<NQ, TG, V, SIN, MR, NPL, false, false, true>), dim3(nblk),
                         dim3(512), lds_bna, s, p);
      return true;
    }
  }
  if constexpr (NPL == 1) {
    if (p.in_bf16) {
      hipLaunchKernelGGL((k_conv_x3<NQ, TG, V, SIN, MR, NPL, true>), dim3(nblk), dim3(512), lds, s,
                         p);
      return true;
    }
  }
  hipLaunchKernelGGL((k_conv_x3<NQ, TG, V, SIN, MR, NPL>), dim3(nblk), dim3(512), lds, s, p);
  return true;
}

template <int NQ, int MR, int NPL>
static bool launch_cx_v(const ConvGemmParams &p, int nblk, hipStream_t s) {
  if (launch_cx_if<NQ, 18, 1, MR, NPL>(p, nblk, s) || launch_cx_if<NQ, 25, 1, MR, NPL>(p, nblk, s))
    return true;
  if constexpr (NPL == 1)
    if (launch_cx_if<NQ, 50, 1, MR, NPL>(p, nblk, s)) return true;
  if constexpr (NQ == 9) {
    if (launch_cx_if<NQ, 18, 2, MR, NPL>(p, nblk, s) || launch_cx_if<NQ, 25, 2, MR, NPL>(p, nblk, s))
      return true;
    if constexpr (NPL == 1) return launch_cx_if<NQ, 50, 2, MR, NPL>(p, nblk, s);
  }
  return false;
}

// npl = 3: fp32 as exact 3-way splits (STGCN_F_F32X3); npl = 1: bf16 operands
// (STGCN_F_BF16), the same pipeline with one plane and two workgroups per CU
// The pack job of a launch_conv_planes call (same layout, same scales)
// rows per workgroup tile of a launch_conv_x3 launch (its grid: N x n_mtiles x
// ceil(R / rows) workgroups)
int conv_x3_tile_rows(const ConvGemmParams &p, int npl) {
  return npl >= 2 && x3_wide_rows(p) && !x3_w4(p, npl) ? 128 : 64;
}

static PackJob pack_job(const ConvGemmParams &p, int npl) {
  const bool w4 = x3_w4(p, npl);
  const bool wide = npl >= 2 && x3_wide_rows(p) && !w4;
  const int rows = wide ? 128 : 64;
  PackJob j{};
  j.w = p.w;
  j.wpk = p.wpk;
  j.R = p.R;
  j.C = p.C;
  j.NQ = p.NQ;
  j.TG = x3_tg(p.NQ);
  j.nch = (p.C + 15) / 16;
  j.rows = rows;
  j.npl = npl;
  j.w_sr = p.w_sr;
  j.w_sc = p.w_sc;
  j.w_sq = p.w_sq;
  j.total = (int64_t)((p.R + rows - 1) / rows) * j.nch * npl * p.NQ * 2 * rows * 8;
  j.amax_w = p.amax_w;
  return j;
}

size_t conv_x3_pack_bytes(const ConvGemmParams &p, int npl) {
  return (size_t)pack_job(p, npl).total * 2;
}

PackJob conv_x3_pack_job(const ConvGemmParams &p, int npl) { return pack_job(p, npl); }

hipError_t launch_pack_jobs(const PackJob *jobs, int n, hipStream_t s) {
  for (int i0 = 0; i0 < n; i0 += kPackJobs) {
    PackJobs js{};
    js.n = std::min(kPackJobs, n - i0);
    js.start[0] = 0;
    for (int k = 0; k < js.n; ++k) {
      js.j[k] = jobs[i0 + k];
      const int64_t units = js.j[k].total / (8 * js.j[k].npl);  // (threads of job k)
      js.start[k + 1] = js.start[k] + (units + 255) / 256 * 256;
    }
    const int64_t tot = js.start[js.n];
    if (tot > 0)
      hipLaunchKernelGGL(k_pack_conv_w_x3_multi, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s,
                         js);
  }
  return hipGetLastError();
}

static hipError_t launch_conv_planes(const ConvGemmParams &p0, int npl, hipStream_t s) {
  const bool w4 = x3_w4(p0, npl);
  const bool wide = npl >= 2 && x3_wide_rows(p0) && !w4;
  ConvGemmParams p = p0;
  const int rows = wide ? 128 : 64;
  p.n_rtiles = (p.R + rows - 1) / rows;
  const int nch = (p.C + 15) / 16;
  if (!p.wpk_ready) {  // (else packed by stgcn_fold_prep, pack_job's layout)
    const int64_t total = (int64_t)p.n_rtiles * nch * npl * p.NQ * 2 * rows * 8;
    hipLaunchKernelGGL(k_pack_conv_w_x3, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s,
                       p.w, reinterpret_cast<__bf16 *>(p.wpk), p.R, p.C, p.NQ, x3_tg(p.NQ), nch,
                       rows, npl, p.w_sr, p.w_sc, p.w_sq, total, p.amax_w);
  }
  const int nblk = p.N * p.n_mtiles * p.n_rtiles;
  bool done = false;
  if (w4) {
    if (p.V == 18)
      launch_cx_w4<18>(p, nblk, s);
    else
      launch_cx_w4<25>(p, nblk, s);
    done = true;
  } else if (wide && npl == 2) {
    done = launch_cx_v<9, 2, 2>(p, nblk, s);
  } else if (wide) {
    done = launch_cx_v<9, 2, 3>(p, nblk, s);
  } else if (npl == 2) {
    switch (p.NQ) {
      case 4: done = launch_cx_v<4, 1, 2>(p, nblk, s); break;
      case 5: done = launch_cx_v<5, 1, 2>(p, nblk, s); break;
      case 9: done = launch_cx_v<9, 1, 2>(p, nblk, s); break;
    }
  } else if (npl == 3) {
    switch (p.NQ) {
      case 4: done = launch_cx_v<4, 1, 3>(p, nblk, s); break;
      case 5: done = launch_cx_v<5, 1, 3>(p, nblk, s); break;
      case 9: done = launch_cx_v<9, 1, 3>(p, nblk, s); break;
    }
  } else {
    switch (p.NQ) {
      case 4: done = launch_cx_v<4, 1, 1>(p, nblk, s); break;
      case 5: done = launch_cx_v<5, 1, 1>(p, nblk, s); break;
      case 9: done = launch_cx_v<9, 1, 1>(p, nblk, s); break;
    }
  }
  return done ? hipGetLastError() : hipErrorInvalidValue;
}

hipError_t launch_conv_x3(const ConvGemmParams &p, hipStream_t s) {
  if (!conv_x3_supported(p) || !p.wpk) return hipErrorInvalidValue;
  if (p.f16x2 && (!p.amax_in || !p.amax_w)) return hipErrorInvalidValue;
  if (p.spb && (p.V != 18 || p.s_in != 1 || p.FT != kTileCols / 18 || !p.sx || !p.sA ||
                !p.mean1 || !p.invstd1 || !p.g1 || !p.b1 || !p.sd || !p.sdn || !p.dA))
    return hipErrorInvalidValue;
  if (p.bna && (!p.f16x2 || !conv_x3_bna_supported(p) || !p.sA || !p.mean1 || !p.invstd1 ||
                !p.g1 || !p.b1))
    return hipErrorInvalidValue;
  return launch_conv_planes(p, p.f16x2 ? 2 : 3, s);
}

// The bf16 temporal-conv GEMMs (9 taps; stride-2 data-gradient phases 5 / 4) on
// the one-plane k_conv_x3 (STGCN_AB_OLD_BF16CONV build: k_conv_bf16, A/B only)
bool conv_b1_supported(const ConvGemmParams &p) {
  constexpr bool off = STGCN_AB_OLD_BF16CONV != 0;
  if (off || p.C < 16) return false;
  if (p.V != 18 && p.V != 25 && p.V != 50) return false;
  if (p.FT != kTileCols / p.V) return false;
  if (p.s_in == 2) return p.NQ == 9;
  return p.s_in == 1 && (p.NQ == 9 || p.NQ == 5 || p.NQ == 4);
}

hipError_t launch_conv_b1(const ConvGemmParams &p, hipStream_t s) {
  if (!conv_b1_supported(p) || !p.wpk) return hipErrorInvalidValue;
  return launch_conv_planes(p, 1, s);
}

}  // namespace stgcn

namespace stgcn {

// ---------------------------------------------------------------------------
// k_wgrad_x3<V, SIN>: the temporal-conv weight gradient (WgradParams, NQ = 9,
// off = -4, stride SIN = 1 or 2) in fp32 via the same exact 3-way bf16 splits, six products per
// fp32 product, h*h and cross terms in separate accumulators:
//   slab[split][r][c*9 + q] = sum_{items of split} sum_{m,v} P[n,r,m,v] Q[n,c,SIN*m+q-4,v]
// Output tile 64 rows x 32 channels x 9 taps; 8 waves = (row half) x (tap
// group: taps 0-2, 3-4, 5-6, 7-8; waves w and w+4 share a SIMD, so every SIMD
// carries 5 or 4 taps). Work item = (clip, FT = 4 frames of P); each split
// takes a contiguous run of items (consecutive frame tiles: the Q halo of the
// next item is L2-hot). Reduction index = (frame, joint) with the joint axis
// padded to Vp = round4(V) (P's pad positions are 0). k-step = 16 positions:
// lane half h takes 4-groups 2s, 2s+1 of frame half h: A = one ds_read_b128 per
// plane, B per tap = two ds_read_b64 per plane (row pitches 8 mod 16 / 4 mod 8
// elements: conflict-free). Images: 3 planes each of P [64][KP] and Q
// [32][QF*Vp], double-buffered at stride 1 (157.5 KiB at V = 18; one buffer and
// a second barrier at stride 2); the next item is loaded
// into registers (4-joint groups, fp32 dwords) under this item's MFMAs, split
// and written after them; one barrier per item.
// ---------------------------------------------------------------------------
template <int V, int SIN, int NPL = 3, int MR = 1>
struct WgX3Geo {
  static constexpr int ROWS = 64 * MR;  // output rows per tile (MR = 2: NPL = 2 only)
  static constexpr int Vp = (V + 3) & ~3;
  static constexpr int G4 = Vp / 4;
  static constexpr int FT = 4;
  static constexpr int KP = FT * Vp;
  static constexpr int KSTEPS = KP / 16;
  static constexpr int HF = FT / 2;
  static constexpr int PPITCH = KP + 8;
  static constexpr int QF = SIN * (FT - 1) + 9;
  static constexpr int QP0 = QF * Vp;
  static constexpr int QPITCH = QP0 % 8 == 0 ? QP0 + 4 : QP0;
  static constexpr int CB = 32;
  static constexpr int PPL = ROWS * PPITCH * 2;  // bytes per P plane
  static constexpr int QPL = CB * QPITCH * 2;  // bytes per Q plane
  static constexpr int BUF = NPL * (PPL + QPL);
  // double-buffered where it fits (stride 1; NPL = 2: stride 2 too); else one
  // buffer written between two barriers (stride 2, three planes: 15 Q frames)
  static constexpr int NBUF = 2 * BUF <= 160 * 1024 ? 2 : 1;
  static constexpr int LDS = NBUF * BUF;
  // (the epilogue's slab tile [ROWS][CB][9] reuses the staging LDS; the launch
  // allocates at least that much -- one workgroup per CU either way)
  static constexpr int TILE = ROWS * CB * 9 * 4;
  static constexpr int LDSK = LDS > TILE ? LDS : TILE;
  static constexpr int PG = FT * G4;  // 4-joint groups per P row
  static constexpr int QG = QF * G4;  // ... per Q row
  static constexpr int NGRP = ROWS * PG + CB * QG;
  static constexpr int GPT = (NGRP + 511) / 512;
  static_assert(KP % 16 == 0 && PPITCH % 16 == 8 && QPITCH % 8 == 4, "conflict-free pitches");
  static_assert(PPL % 16 == 0 && QPL % 16 == 0, "plane alignment");
  static_assert(LDS <= 160 * 1024, "LDS budget");
};

// NPL = 2: fp32 as 2-way fp16 splits of the power-of-two-scaled operands (P and
// Q by the f16x2_se scales of p.amax_p / p.amax_q, undone on the slab values),
// three products hh, hl, lh. MR = 2 (NPL = 2, R % 128 == 0): 128-row tiles, each
// wave two 32-row blocks sharing its Q fragments (half the Q image traffic per
// flop: the kernel is bound by the L2 -> LDS staging, not the matrix rate), one
// accumulator per block (the three products summed in one fp32 chain, small
// ones first)
// QBN (NPL = 2, the folded block without G, capi.hip fold_bna): Q is the block
// input x and BN1 is applied while staging it (a [mu, a, be] row per channel of
// the tile in LDS past the plan; 0 in padded frames), P is dU A, so
//   sum_{t,w} (dU A)[o,t,w] BN1(x)[c,t',w] = sum_{t,v} dU[o,t,v] G[c,t',v] = dWc;
// Q's fp16 bound is |BN1(x)| <= max_c |a_c| (M + |mu_c|) + |be_c|, M = max |x|.
template <int V, int SIN, int NPL = 3, int MR = 1, bool QBN = false>
__global__ __launch_bounds__(512, 1) void k_wgrad_x3(WgradParams p) {
  using G = WgX3Geo<V, SIN, NPL, MR>;
  static_assert(MR == 1 || NPL == 2, "128-row tiles on the fp16 splits only");
  static_assert(!QBN || NPL == 2, "BN1 staging: the fp16 splits");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  char *lds = reinterpret_cast<char *>(smem);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hi = lane >> 5, lo = lane & 31;
  int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int jt = bid % p.n_jtiles;
  bid /= p.n_jtiles;
  const int rt = bid % p.n_rtiles;
  const int split = bid / p.n_rtiles;
  const int r0 = rt * G::ROWS, c0 = jt * G::CB;
  // QBN: [CB + 1][4] = (mu, a, be, 0) of channels c0.., then the identity (0, 1, 0)
  // that P's groups use (the transform runs branch-free on every group)
  float *const qtab = smem + G::LDS / 4;
  int q_se = NPL == 2 ? f16x2_se(p.amax_q) : 0;
  if constexpr (QBN) {
    const float M = __builtin_bit_cast(float, amax_read(p.amax_q));
    float bm = 0.f;
    for (int c = tid; c < p.C; c += 512) {
      const float a = p.q_invstd[c] * p.q_g[c];
      bm = fmaxf(bm, fabsf(a) * (M + fabsf(p.q_mean[c])) + fabsf(p.q_b[c]));
    }
    if (tid <= G::CB) {
      const int c = c0 + tid;
      const bool ok = tid < G::CB && c < p.C;
      *reinterpret_cast<float4 *>(qtab + 4 * tid) =
          tid == G::CB ? make_float4(0.f, 1.f, 0.f, 0.f)
                       : make_float4(ok ? p.q_mean[c] : 0.f, ok ? p.q_invstd[c] * p.q_g[c] : 0.f,
                                     ok ? p.q_b[c] : 0.f, 0.f);
    }
    q_se = f16x2_se_bits(
        __builtin_bit_cast(unsigned, block_max_all<512>(bm, qtab + 4 * (G::CB + 1))));
  }
  const int p_se = NPL == 2 ? f16x2_se(p.amax_p) : 0;
  const float p_scale = pow2f(p_se), q_scale = pow2f(q_se);
  const int mi = wave & 1, tq = wave >> 1;
  const int q0 = tq ? 1 + 2 * tq : 0;
  const int total = p.N * p.n_mtiles;
  const int per = (total + p.S - 1) / p.S;
  const int it0 = split * per, it1 = min(total, it0 + per);
  const int MV = p.M * V, TV = p.T_src * V;

  // staging groups of this thread: P (row, frame, joint group) or Q (channel, ...)
  int grow[G::GPT], gfr[G::GPT], gv0[G::GPT], gl[G::GPT];
  bool isq[G::GPT];
#pragma unroll
  for (int k = 0; k < G::GPT; ++k) {
    int e = k * 512 + tid;
    isq[k] = e >= G::ROWS * G::PG;
    if (isq[k]) e -= G::ROWS * G::PG;
    const int per_row = isq[k] ? G::QG : G::PG;
    const int row = e / per_row, g = e - row * per_row;
    grow[k] = row;
    gfr[k] = g / G::G4;
    gv0[k] = (g % G::G4) * 4;
    const bool live = isq[k] ? row < G::CB : true;
    // LDS byte offset within a plane (-1: no group)
    gl[k] = (!live || (isq[k] && e >= G::CB * G::QG)) ? -1
            : isq[k] ? (row * G::QPITCH + gfr[k] * G::Vp + gv0[k]) * 2
                     : (row * G::PPITCH + gfr[k] * G::Vp + gv0[k]) * 2;
  }
  float st[G::GPT][4];
  unsigned qval = 0;  // QBN: bit 2k + j = pair j of staging group k lies inside the clip
  auto load_item = [&](int item) __attribute__((always_inline)) {
    if constexpr (QBN) qval = 0;
    const int n = item / p.n_mtiles, m0 = (item - n * p.n_mtiles) * G::FT;
    const __amdgpu_buffer_rsrc_t rp = make_rsrc(p.P + (int64_t)n * p.p_bstride, p.p_bstride);
    const __amdgpu_buffer_rsrc_t rq = make_rsrc(p.Q + (int64_t)n * p.q_bstride, p.q_bstride);
#pragma unroll
    for (int k = 0; k < G::GPT; ++k) {
      unsigned base;
      if (isq[k]) {
        const int c = c0 + grow[k], t = SIN * m0 + p.off + gfr[k];
        const bool ok = gl[k] >= 0 && c < p.C && t >= 0 && t < p.T_src;
        base = ok ? (unsigned)(c * TV + t * V + gv0[k]) * 4u : kOOB;
      } else {
        const int r = r0 + grow[k], m = m0 + gfr[k];
        const bool ok = gl[k] >= 0 && r < p.R && m < p.M;
        base = ok ? (unsigned)(r * MV + m * V + gv0[k]) * 4u : kOOB;
      }
      // P / Q split of the staging groups falls on wave boundaries (64 * PG is a
      // multiple of 64): a wave-uniform descriptor choice (no waterfall loop)
      const bool q_k = __builtin_amdgcn_readfirstlane((int)isq[k]) != 0;
      const __amdgpu_buffer_rsrc_t rs = q_k ? rq : rp;
      // two 8-byte loads per 4-joint group (V even: pairs never straddle a
      // frame; pad pairs read 0 through an OOB offset)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const unsigned off = gv0[k] + 2 * j < V ? base + 8u * j : kOOB;
        if constexpr (QBN)  // (P's groups: always live; their zeros pass the identity)
          qval |= (!q_k || (base != kOOB && gv0[k] + 2 * j < V)) ? 1u << (2 * k + j) : 0u;
        const auto v2 = __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 0);
        st[k][2 * j] = __builtin_bit_cast(float, (unsigned)v2[0]);
        st[k][2 * j + 1] = __builtin_bit_cast(float, (unsigned)v2[1]);
      }
    }
  };
  static_assert(V % 2 == 0 && (G::ROWS * G::PG) % 64 == 0, "pair loads, uniform P/Q waves");
  // splits and writes staging groups [K0, K1) of the loaded item
  auto write_part = [&](char *buf, auto k0_c, auto k1_c) __attribute__((always_inline)) {
    constexpr int K0 = decltype(k0_c)::value, K1 = decltype(k1_c)::value;
#pragma unroll
    for (int k = K0; k < K1; ++k)
      if (gl[k] >= 0) {
        char *dst = buf + (isq[k] ? NPL * G::PPL : 0) + gl[k];
        const int pl = isq[k] ? G::QPL : G::PPL;
        if constexpr (NPL == 2) {
          const float sc = isq[k] ? q_scale : p_scale;
          float xv[4] = {st[k][0], st[k][1], st[k][2], st[k][3]};
          if constexpr (QBN) {  // BN1(x) of a Q group's channel, 0 outside the clip
            // (the P / Q split of the groups falls on wave boundaries: a scalar branch)
            if (__builtin_amdgcn_readfirstlane((int)isq[k]) != 0) {
              const float4 t = *reinterpret_cast<const float4 *>(qtab + 4 * grow[k]);
#pragma unroll
              for (int e = 0; e < 4; ++e)
                xv[e] = (qval >> (2 * k + e / 2)) & 1u ? (xv[e] - t.x) * t.y + t.z : 0.f;
            }
          }
          uint2 h, l;
          splith2(xv[0] * sc, xv[1] * sc, h.x, l.x);
          splith2(xv[2] * sc, xv[3] * sc, h.y, l.y);
          *reinterpret_cast<uint2 *>(dst) = h;
          *reinterpret_cast<uint2 *>(dst + pl) = l;
        } else {
          uint2 h, m, l;
          split2(st[k][0], st[k][1], h.x, m.x, l.x);
          split2(st[k][2], st[k][3], h.y, m.y, l.y);
          *reinterpret_cast<uint2 *>(dst) = h;
          *reinterpret_cast<uint2 *>(dst + pl) = m;
          *reinterpret_cast<uint2 *>(dst + 2 * pl) = l;
        }
      }
  };
  auto write_item = [&](char *buf) __attribute__((always_inline)) {
    // (in parts of three groups: one loop over all of them is not unrolled at every
    // instance -- the staging registers then go to scratch memory)
    using std::integral_constant;
    constexpr int Q = G::GPT;
    static_assert(Q <= 12, "write_item parts");
    write_part(buf, integral_constant<int, 0>{}, integral_constant<int, (Q < 3 ? Q : 3)>{});
    if constexpr (Q > 3)
      write_part(buf, integral_constant<int, 3>{}, integral_constant<int, (Q < 6 ? Q : 6)>{});
    if constexpr (Q > 6)
      write_part(buf, integral_constant<int, 6>{}, integral_constant<int, (Q < 9 ? Q : 9)>{});
    if constexpr (Q > 9)
      write_part(buf, integral_constant<int, 9>{}, integral_constant<int, Q>{});
  };

  // lane bases (elements) of the A (P) and B (Q) fragments in plane 0
  const int pa = (mi * 32 + lo) * G::PPITCH + hi * G::HF * G::Vp;
  const int qb = lo * G::QPITCH + hi * SIN * G::HF * G::Vp + q0 * G::Vp;

  auto run = [&](auto nt_c) __attribute__((always_inline)) {
    constexpr int NT = decltype(nt_c)::value;
    floatx16 acc[MR == 1 ? NT : 1], acl[MR == 1 ? NT : 1], acm[MR][MR == 2 ? NT : 1];
    if constexpr (MR == 1) {
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[t][i] = acl[t][i] = 0.f;
    } else {
#pragma unroll
      for (int mb = 0; mb < MR; ++mb)
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int i = 0; i < 16; ++i) acm[mb][t][i] = 0.f;
    }
    struct Frag {
      bf16x8_t a[MR][NPL], b[NPL][NT];
    };
    auto ld = [&](const char *buf, int s, Frag &f) __attribute__((always_inline)) {
      const __bf16 *P = reinterpret_cast<const __bf16 *>(buf) + pa + 8 * s;
      const int ga = 2 * s, gb = 2 * s + 1;
      const int oa = SIN * (ga / G::G4) * G::Vp + (ga % G::G4) * 4;
      const int ob = SIN * (gb / G::G4) * G::Vp + (gb % G::G4) * 4;
      const __bf16 *Q = reinterpret_cast<const __bf16 *>(buf + NPL * G::PPL) + qb;
#pragma unroll
      for (int pl = 0; pl < NPL; ++pl) {
#pragma unroll
        for (int mb = 0; mb < MR; ++mb)
          f.a[mb][pl] = *reinterpret_cast<const bf16x8_t *>(P + pl * (G::PPL / 2) + mb * 64 * G::PPITCH);
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const __bf16 *Qp = Q + pl * (G::QPL / 2) + t * G::Vp;
          const bf16x4_t b0 = *reinterpret_cast<const bf16x4_t *>(Qp + oa);
          const bf16x4_t b1 = *reinterpret_cast<const bf16x4_t *>(Qp + ob);
          f.b[pl][t] = __builtin_shufflevector(b0, b1, 0, 1, 2, 3, 4, 5, 6, 7);
        }
      }
    };
    auto mm = [&](const Frag &f) __attribute__((always_inline)) {
      if constexpr (MR == 2) {
#pragma unroll
        for (int mb = 0; mb < MR; ++mb)
#pragma unroll
          for (int t = 0; t < NT; ++t) {
            acm[mb][t] = mfma_p<NPL>(f.a[mb][1], f.b[0][t], acm[mb][t]);
            acm[mb][t] = mfma_p<NPL>(f.a[mb][0], f.b[1][t], acm[mb][t]);
            acm[mb][t] = mfma_p<NPL>(f.a[mb][0], f.b[0][t], acm[mb][t]);
          }
        return;
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = mfma_p<NPL>(f.a[0][0], f.b[0][t], acc[t]);
#pragma unroll
      for (int t = 0; t < NT; ++t) acl[t] = mfma_p<NPL>(f.a[0][0], f.b[1][t], acl[t]);
#pragma unroll
      for (int t = 0; t < NT; ++t) acl[t] = mfma_p<NPL>(f.a[0][1], f.b[0][t], acl[t]);
      if constexpr (NPL == 3) {
#pragma unroll
        for (int t = 0; t < NT; ++t) acl[t] = mfma_x(f.a[0][0], f.b[2 % NPL][t], acl[t]);
#pragma unroll
        for (int t = 0; t < NT; ++t) acl[t] = mfma_x(f.a[0][1], f.b[1][t], acl[t]);
#pragma unroll
        for (int t = 0; t < NT; ++t) acl[t] = mfma_x(f.a[0][2 % NPL], f.b[0][t], acl[t]);
      }
    };
    Frag f[2];
    for (int it = it0; it < it1; ++it) {
      const char *cur = lds + (G::NBUF == 2 ? ((it - it0) & 1) * G::BUF : 0);
      char *nxt = lds + (G::NBUF == 2 ? ((it - it0 + 1) & 1) * G::BUF : 0);
      // next item (the last iteration reloads its own item into the idle buffer:
      // unconditional, so no register copies across the loop)
      load_item(it + 1 < it1 ? it + 1 : it);
      ld(cur, 0, f[0]);
#pragma unroll
      for (int s = 0; s < G::KSTEPS; ++s) {
        if (s + 1 < G::KSTEPS) ld(cur, s + 1, f[(s + 1) & 1]);
        mm(f[s & 1]);
        if constexpr (G::NBUF == 2 && kWgWriteStart < G::KSTEPS) {
          // double buffer: the next item's split + LDS writes ride in the MFMA
          // shadow of k-steps WSTART.. (the loads were issued at the item start)
          using std::integral_constant;
          constexpr int W0 = kWgWriteStart, NP = G::KSTEPS - W0, Q = G::GPT;
          static_assert(W0 >= 1 && NP >= 1 && NP <= 4, "write parts");
          if (s == W0)
            write_part(nxt, integral_constant<int, 0>{}, integral_constant<int, Q / NP>{});
          else if (NP >= 2 && s == W0 + 1)
            write_part(nxt, integral_constant<int, Q / NP>{}, integral_constant<int, 2 * Q / NP>{});
          else if (NP >= 3 && s == W0 + 2)
            write_part(nxt, integral_constant<int, 2 * Q / NP>{},
                       integral_constant<int, 3 * Q / NP>{});
          else if (NP >= 4 && s == W0 + 3)
            write_part(nxt, integral_constant<int, 3 * Q / NP>{}, integral_constant<int, Q>{});
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (G::NBUF == 1) {
        __syncthreads();  // every wave is done reading the buffer
        write_item(nxt);
      } else if constexpr (kWgWriteStart >= G::KSTEPS) {
        write_item(nxt);
      }
      __syncthreads();
    }
    // the tile [ROWS][CB channels][9 taps] through LDS (the staging buffers are
    // free after the last item's barrier), then whole 16-byte pieces of each
    // row's CB * 9 contiguous slab floats: 4-byte stores at a 36-byte stride
    // (per tap and channel) measured ~6x the slab's bytes in HBM writes
    float *tile = reinterpret_cast<float *>(lds);
    static_assert(G::TILE <= G::LDSK && G::LDSK <= 160 * 1024, "slab tile LDS");
#pragma unroll
    for (int mb = 0; mb < MR; ++mb)
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int rl = mb * 64 + mi * 32 + (i & 3) + 8 * (i >> 2) + 4 * hi;
          float v;
          if constexpr (MR == 2)
            v = acm[mb][t][i] * pow2f(-p_se) * pow2f(-q_se);
          else
            v = NPL == 2 ? (acc[t][i] + acl[t][i]) * pow2f(-p_se) * pow2f(-q_se)
                         : acc[t][i] + acl[t][i];
          tile[(rl * G::CB + lo) * 9 + q0 + t] = v;
        }
    __syncthreads();
    float *slab = p.slab + (int64_t)split * p.R * p.C * 9;
    const int ncw = min(G::CB, p.C - c0) * 9;  // valid floats of a tile row
    constexpr int RF = G::CB * 9;              // tile row pitch (floats)
    const bool v4 = (p.C % 4) == 0;            // (16-byte aligned slab rows)
    for (int e = tid; e < G::ROWS * (RF / 4); e += 512) {
      const int rl = e / (RF / 4), f = (e - rl * (RF / 4)) * 4;
      const int r = r0 + rl;
      if (r >= p.R || f >= ncw) continue;
      float *dst = slab + ((int64_t)r * p.C + c0) * 9 + f;
      const float *src = tile + rl * RF + f;
      if (v4 && f + 4 <= ncw) {
        *reinterpret_cast<float4 *>(dst) = *reinterpret_cast<const float4 *>(src);
      } else {
        for (int k = 0; k < 4 && f + k < ncw; ++k) dst[k] = src[k];
      }
    }
  };
  if (it0 < it1) {
    load_item(it0);
    write_item(lds);
  }
  __syncthreads();
  if (tq == 0)
    run(std::integral_constant<int, 3>{});
  else
    run(std::integral_constant<int, 2>{});
}

bool plan_wgrad_x3(WgradParams &w, bool f16x2) {
  if (w.V != 18 || (w.s_in != 1 && w.s_in != 2) || w.NQ != 9 || w.off != -4 || w.C < 16)
    return false;
  w.FT = WgX3Geo<18, 1>::FT;
  w.n_mtiles = (w.M + w.FT - 1) / w.FT;
  w.x3_mr = f16x2 && w.R % 128 == 0 ? 2 : 1;  // (128-row tiles: k_wgrad_x3<.., 2, 2>)
  w.n_rtiles = (w.R + 64 * w.x3_mr - 1) / (64 * w.x3_mr);
  w.n_jtiles = (w.C + WgX3Geo<18, 1>::CB - 1) / WgX3Geo<18, 1>::CB;
  const int tiles = w.n_rtiles * w.n_jtiles;
  w.S = std::max(1, std::min((256 + tiles - 1) / tiles, w.N * w.n_mtiles));
  w.bf16 = 3;
  return true;
}

hipError_t launch_wgrad_x3(const WgradParams &p0, hipStream_t s) {
  if (p0.bf16 != 3 || p0.V != 18 || (p0.s_in != 1 && p0.s_in != 2)) return hipErrorInvalidValue;
  const int nblk = p0.n_rtiles * p0.n_jtiles * p0.S;
  if (p0.f16x2 && p0.q_mean) {  // 2-way fp16 splits, Q = x with BN1 at staging (QBN)
    const WgradParams &p = p0;
    if (!p.amax_p || !p.amax_q || !p.q_invstd || !p.q_g || !p.q_b) return hipErrorInvalidValue;
    if (p.x3_mr == 2 && p.R % 128 != 0) return hipErrorInvalidValue;
    constexpr int ex = (4 * 33 + 8) * 4;  // the Q channel table + block_max_all's scratch
    if (p.s_in == 1 && p.x3_mr == 2)
      hipLaunchKernelGGL((k_wgrad_x3<18, 1, 2, 2, true>), dim3(nblk), dim3(512),
                         (WgX3Geo<18, 1, 2, 2>::LDSK + ex), s, p);
    else if (p.s_in == 1)
      hipLaunchKernelGGL((k_wgrad_x3<18, 1, 2, 1, true>), dim3(nblk), dim3(512),
                         (WgX3Geo<18, 1, 2>::LDSK + ex), s, p);
    else if (p.x3_mr == 2)
      hipLaunchKernelGGL((k_wgrad_x3<18, 2, 2, 2, true>), dim3(nblk), dim3(512),
                         (WgX3Geo<18, 2, 2, 2>::LDSK + ex), s, p);
    else
      hipLaunchKernelGGL((k_wgrad_x3<18, 2, 2, 1, true>), dim3(nblk), dim3(512),
                         (WgX3Geo<18, 2, 2>::LDSK + ex), s, p);
    return hipGetLastError();
  }
  if (p0.f16x2) {  // 2-way fp16 splits (NPL = 2)
    if (!p0.amax_p || !p0.amax_q) return hipErrorInvalidValue;
    const WgradParams &p = p0;
    if (p.x3_mr == 2 && p.R % 128 != 0) return hipErrorInvalidValue;
    if (p.s_in == 1 && p.x3_mr == 2)
      hipLaunchKernelGGL((k_wgrad_x3<18, 1, 2, 2>), dim3(nblk), dim3(512), (WgX3Geo<18, 1, 2, 2>::LDSK),
                         s, p);
    else if (p.s_in == 1)
      hipLaunchKernelGGL((k_wgrad_x3<18, 1, 2>), dim3(nblk), dim3(512), (WgX3Geo<18, 1, 2>::LDSK), s, p);
    else if (p.x3_mr == 2)
      hipLaunchKernelGGL((k_wgrad_x3<18, 2, 2, 2>), dim3(nblk), dim3(512), (WgX3Geo<18, 2, 2, 2>::LDSK),
                         s, p);
    else
      hipLaunchKernelGGL((k_wgrad_x3<18, 2, 2>), dim3(nblk), dim3(512), (WgX3Geo<18, 2, 2>::LDSK), s, p);
    return hipGetLastError();
  }
  const WgradParams &p = p0;
  if (p.x3_mr != 1) return hipErrorInvalidValue;  // (128-row tiles: fp16 splits only)
  if (p.s_in == 1) {
    constexpr int lds = WgX3Geo<18, 1>::LDSK;
    hipLaunchKernelGGL((k_wgrad_x3<18, 1>), dim3(nblk), dim3(512), lds, s, p);
  } else {
    constexpr int lds = WgX3Geo<18, 2>::LDSK;
    hipLaunchKernelGGL((k_wgrad_x3<18, 2>), dim3(nblk), dim3(512), lds, s, p);
  }
  return hipGetLastError();
}

}  // namespace stgcn

// The folded block (capi.hip fold_w): with one adjacency partition (K = 1) the
// SpatialConv channel GEMM W' is a 1x1 conv that the (9,1) temporal conv can
// absorb (st_graphconv.py:99 temporalConv(spatialConv(x)), :148-150):
//   U[o,t] = sum_q Wt_q (W' G[t'] + bZ)[o]  =  sum_q Wc_q G[t'] + BT[o,t],
//   Wc_q = Wt_q W'  (C_out x C_in per tap),  t' = s t + q - 4,
//   BT[o,t,v] = bt[o] + sum_{q : 0 <= t' < T} (Wt_q bZ)[o,v]
// (bZ = b' rowsum(A), the padded frames of Z carry no bias), so the temporal
// conv's MFMA GEMM reads G (C_in channels) and Z is never formed. Backward:
//   dWc_q = sum dU G[t']^T (the temporal weight-gradient kernel over C_in),
//   dWt_q = dWc_q W'^T + sum_v Tq[o,v] bZ[c,v],   dW' = sum_q Wt_q^T dWc_q,
//   H = W'^T dZ = sum_q Wc_q^T dU[..]  (the data gradient with Wc: dZ never formed),
//   sum_{n,t} dZ[c,v] = sum_q sum_o Wt[o,c,q] Tq[o,v],
// Tq[o,v] = sum over (n, t) with t' in range of dU[o,t,v] = the total minus the
// boundary frames where tap q reads padding. Small fp64-accumulating kernels
// here; the big GEMMs are the temporal conv kernels.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <initializer_list>
#include <vector>

#include "device_common.h"
#include "internal.h"

#define HIP_RET(expr)                  \
  do {                                 \
    hipError_t e_ = (expr);            \
    if (e_ != hipSuccess) return e_;   \
  } while (0)

namespace stgcn {

// The fold's small GEMMs on the fp32 matrix cores (v_mfma_f32_16x16x4_f32: a
// k-ordered fp32 fma chain per output, fixed order: deterministic).
//
// Operands are first re-laid by k_fold_tr as fp32 [plane q][row][k] with k
// contiguous and rows and k zero-padded to multiples of 32, so the GEMM's inner
// loop is pure loads + MFMAs: lane l (row l & 15, k-quad l >> 4) loads four
// consecutive k (16 bytes) per operand for four MFMAs, no conversions, no
// bounds selects.
//
// k_fold_gemm: block = nine waves = the nine taps q of one 16 x 16 output tile;
// each wave streams its whole K range (L2-resident operands) with the next
// 16-k group's loads in flight (no LDS staging, no split-K partials). Two kinds:
//   TAP: out[q](m, n) = sum_k A[q](m, k) B[q](n, k) + sum_v A2(q, m, v) B2(n, v)
//        (each wave writes its tap): Wc = Wt W', the bias products bq,
//        dWt = dWc W'^T + Tq bZ (the short A2 / B2 term read directly)
//   RED: out(m, n) = sum_q sum_k A[q](m, k) B[q](n, k) (the nine waves' tiles
//        summed in LDS in tap order, in fp64): dW' = sum_q Wt_q^T dWc_q and
//        sum_{n,t} dZ = sum_q Wt_q^T Tq.
// Up to three jobs share a launch (blockIdx.x runs over their tiles).
typedef float float16v __attribute__((ext_vector_type(16)));
typedef float float8v __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef double double4v __attribute__((ext_vector_type(4)));

__host__ __device__ inline int pad32(int x) { return (x + 31) & ~31; }

struct FoldJob {
  const float *A, *B;  // A[q aq + m am + k], B[q bq + n bn + k] (padded re-layouts)
  int64_t aq, am, bq, bn;
  const double *A2;    // TAP only (or null): A2[q a2q + m a2m + v] B2[n b2n + v], v < K2
  const float *B2;
  int64_t a2q, a2m, b2n;
  void *out;
  int64_t oq, om, on;  // out[q oq + m om + n on] (RED: q = 0)
  int o_dbl, red;
  int M, N, K, K2;
};

constexpr int kFoldJobs = 18;  // jobs per k_fold_gemm launch (the stack prep batches blocks)
struct FoldJobs {
  FoldJob j[kFoldJobs];
  int n;
  int tile0[kFoldJobs + 1];  // first tile of job i; tile0[n] = the grid
};

// One wave's K stream, fully unrolled for NG 16-k groups (straight-line code:
// the compiler's load counters stay exact; D groups in flight, pinned by
// sched_barrier: the scheduler would otherwise sink each prefetch next to its
// MFMAs). Lane: k = 16 i + 4 (l >> 4) + j for MFMA j of group i.
template <int NG>
__device__ __forceinline__ void f32_stream(const float *pa, const float *pb, floatx4 &acc) {
  constexpr int D = NG < 4 ? NG : 4;
  float4 a[D], b[D];
#pragma unroll
  for (int d = 0; d < D; ++d) {
    a[d] = *reinterpret_cast<const float4 *>(pa + 16 * d);
    b[d] = *reinterpret_cast<const float4 *>(pb + 16 * d);
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < NG; ++i) {
    const int d = i % D;
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[d].x, b[d].x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[d].y, b[d].y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[d].z, b[d].z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[d].w, b[d].w, acc, 0, 0, 0);
    if (i + D < NG) {
      a[d] = *reinterpret_cast<const float4 *>(pa + 16 * (i + D));
      b[d] = *reinterpret_cast<const float4 *>(pb + 16 * (i + D));
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

__device__ __forceinline__ void f32_stream_any(const float *pa, const float *pb, int ng,
                                               floatx4 &acc) {
  switch (ng) {
    case 4: f32_stream<4>(pa, pb, acc); return;
    case 8: f32_stream<8>(pa, pb, acc); return;
    case 16: f32_stream<16>(pa, pb, acc); return;
    default: break;
  }
  for (int i = 0; i < ng; i += 4) {  // (other K: chunks of up to four groups)
    if (ng - i >= 4) {
      f32_stream<4>(pa + 16 * i, pb + 16 * i, acc);
    } else {
      for (int k = i; k < ng; ++k) f32_stream<1>(pa + 16 * k, pb + 16 * k, acc);
    }
  }
}

// 16 x 16 output tiles (v_mfma_f32_16x16x4_f32, same rate as 32 x 32 x 2): a
// block is one CU's worth of waves, so the tile count sets how many CUs work;
// 32 x 32 tiles left three quarters of the chip idle on the 256-channel blocks
__global__ __launch_bounds__(576) void k_fold_gemm(FoldJobs js) {
  __shared__ float red[9][16 * 17];
  const int tile = blockIdx.x;
  int ji = 0;
  while (ji + 1 < js.n && tile >= js.tile0[ji + 1]) ++ji;
  const FoldJob &g = js.j[ji];
  const int t = tile - js.tile0[ji], ntn = (g.N + 15) >> 4;
  const int m0 = (t / ntn) * 16, n0 = (t % ntn) * 16;
  const int q = threadIdx.x >> 6, l = threadIdx.x & 63, r16 = l & 15, kq = l >> 4;
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  {
    const float *pa = g.A + q * g.aq + (int64_t)(m0 + r16) * g.am + 4 * kq;
    const float *pb = g.B + q * g.bq + (int64_t)(n0 + r16) * g.bn + 4 * kq;
    f32_stream_any(pa, pb, (g.K + 15) >> 4, acc);
  }
  if (g.A2) {  // (short: K2 = V; bounds-checked direct reads)
    const int m = m0 + r16, n = n0 + r16;
    const bool ok_m = m < g.M, ok_n = n < g.N;
    const double *a2 = g.A2 + q * g.a2q + (int64_t)min(m, g.M - 1) * g.a2m;
    const float *b2 = g.B2 + (int64_t)min(n, g.N - 1) * g.b2n;
    for (int k0 = 0; k0 < g.K2; k0 += 4) {
      const int k = k0 + kq, kc = min(k, g.K2 - 1);
      const float x = (float)a2[kc], y = b2[kc];
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(k < g.K2 && ok_m ? x : 0.f,
                                                 k < g.K2 && ok_n ? y : 0.f, acc, 0, 0, 0);
    }
  }
  // C/D: col = lane & 15, row = 4 (lane >> 4) + reg
  if (!g.red) {
    const int nn = n0 + r16;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int mm = m0 + 4 * kq + r;
      if (mm >= g.M || nn >= g.N) continue;
      const int64_t o = q * g.oq + mm * g.om + nn * g.on;
      if (g.o_dbl)
        reinterpret_cast<double *>(g.out)[o] = acc[r];
      else
        reinterpret_cast<float *>(g.out)[o] = acc[r];
    }
    return;
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) red[q][(4 * kq + r) * 17 + r16] = acc[r];
  __syncthreads();
  if (threadIdx.x >= 256) return;
  const int rr = threadIdx.x >> 4, cc = threadIdx.x & 15;
  const int mm = m0 + rr, nn = n0 + cc;
  if (mm >= g.M || nn >= g.N) return;
  double sum = 0.0;
#pragma unroll
  for (int w = 0; w < 9; ++w) sum += red[w][rr * 17 + cc];
  const int64_t o = mm * g.om + nn * g.on;
  if (g.o_dbl)
    reinterpret_cast<double *>(g.out)[o] = sum;
  else
    reinterpret_cast<float *>(g.out)[o] = (float)sum;
}

// (any number of jobs: kFoldJobs per launch)
static hipError_t fold_gemm_v(const FoldJob *jobs, int n, hipStream_t s) {
  for (int i0 = 0; i0 < n; i0 += kFoldJobs) {
    FoldJobs js{};
    js.n = 0;
    int tiles = 0;
    for (int i = i0; i < std::min(n, i0 + kFoldJobs); ++i) {
      const FoldJob &g = jobs[i];
      if (g.M <= 0 || g.N <= 0) return hipErrorInvalidValue;
      js.j[js.n] = g;
      js.tile0[js.n++] = tiles;
      tiles += ((g.M + 15) / 16) * ((g.N + 15) / 16);
    }
    js.tile0[js.n] = tiles;
    hipLaunchKernelGGL(k_fold_gemm, dim3(tiles), dim3(576), 0, s, js);
  }
  return hipGetLastError();
}

static hipError_t fold_gemm(std::initializer_list<FoldJob> jobs, hipStream_t s) {
  return fold_gemm_v(jobs.begin(), (int)jobs.size(), s);
}

// k_fold_tr: the padded fp32 re-layouts. A job reads src(q, o, i) =
// sum_{k < S} src[k sstride + q sq + o so + i si] (slabs summed in order in
// fp64, then rounded to fp32; q < nq,
// nq = 9 or 1) and writes outQ[q][o][i] (rows O -> Op = pad32(O), row stride
// Ip = pad32(I)) and / or outT[q][i][o] (rows Ip, row stride Op), zeros in the
// padding. Tile = OT o-rows x 16 i x nq taps, one element per thread (576
// threads; OT = 4 for nq = 9, 36 for nq = 1); up to three jobs per launch.
struct TrJob {
  const void *src;
  int s_dbl, S, nq, q_inner;  // q_inner: sq == 1 (the element order q, i, o)
  int64_t sstride, sq, so, si;
  int O, I;
  void *outQ, *outT;
  int o_dbl;    // outputs fp64 (else fp32)
  int tiles_i;  // tiles along i (pad32(I) / 16)
};

constexpr int kTrJobs = 16;  // jobs per k_fold_tr launch
struct TrJobs {
  TrJob j[kTrJobs];
  int n;
  int tile0[kTrJobs + 1];
};

__global__ __launch_bounds__(576) void k_fold_tr(TrJobs js) {
  __shared__ double tile[36 * 16 + 4];
  const int blk = blockIdx.x, tid = threadIdx.x;
  int ji = 0;
  while (ji + 1 < js.n && blk >= js.tile0[ji + 1]) ++ji;
  const TrJob &g = js.j[ji];
  const int t = blk - js.tile0[ji];
  const int nq = g.nq, OT = nq == 9 ? 4 : 36;
  const int o0 = (t / g.tiles_i) * OT, i0 = (t % g.tiles_i) * 16;
  const int Op = pad32(g.O), Ip = pad32(g.I);
  // element e = tid: (oo, ii, q) with the source's innermost index fastest
  int oo, ii, q;
  if (nq == 1) {
    oo = tid >> 4; ii = tid & 15; q = 0;
  } else if (g.q_inner) {
    oo = tid / 144; const int r = tid - oo * 144; ii = r / 9; q = r - ii * 9;
  } else {
    oo = tid / 144; const int r = tid - oo * 144; q = r >> 4; ii = r & 15;
  }
  const int o = o0 + oo, i = i0 + ii;
  double v = 0.0;
  if (o < g.O && i < g.I) {
    const int64_t at = q * g.sq + o * g.so + i * g.si;
    if (g.s_dbl) {
      v = reinterpret_cast<const double *>(g.src)[at];
    } else {
      const float *p = reinterpret_cast<const float *>(g.src) + at;
      int k = 0;
      // (sixteen loads in flight, summed in slab order: at S = 128 slabs -- the
      // 64-channel blocks' weight gradient -- four in flight left the launch
      // waiting 32 load latencies)
      for (; k + 16 <= g.S; k += 16) {
        float a[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) a[u] = p[(int64_t)(k + u) * g.sstride];
#pragma unroll
        for (int u = 0; u < 16; ++u) v += a[u];
      }
      for (; k + 4 <= g.S; k += 4) {
        const float a0 = p[k * g.sstride], a1 = p[(k + 1) * g.sstride],
                    a2 = p[(k + 2) * g.sstride], a3 = p[(k + 3) * g.sstride];
        v += a0;
        v += a1;
        v += a2;
        v += a3;
      }
      for (; k < g.S; ++k) v += p[k * g.sstride];
    }
  }
  const int slot = (q * OT + oo) * 16 + ii;  // tile[q][oo][ii]
  tile[slot + slot / 16 / 8] = v;           // (a pad word every 8 rows)
  __syncthreads();
  if (g.outQ) {  // [q][o][i]: runs of 16 i; the thread's own element order
    const int sq2 = tid / (OT * 16), a = (tid >> 4) % OT, b = tid & 15;
    const int s2 = (sq2 * OT + a) * 16 + b;
    const int64_t at = ((int64_t)sq2 * Op + o0 + a) * Ip + i0 + b;
    if (o0 + a < Op) {
      if (g.o_dbl)
        reinterpret_cast<double *>(g.outQ)[at] = tile[s2 + s2 / 16 / 8];
      else
        reinterpret_cast<float *>(g.outQ)[at] = (float)tile[s2 + s2 / 16 / 8];
    }
  }
  if (g.outT) {  // [q][i][o]: runs of OT o
    const int sq2 = tid / (OT * 16), a = (tid / OT) & 15, b = tid % OT;
    const int s2 = (sq2 * OT + b) * 16 + a;
    const int64_t at = ((int64_t)sq2 * Ip + i0 + a) * Op + o0 + b;
    if (o0 + b < Op) {
      if (g.o_dbl)
        reinterpret_cast<double *>(g.outT)[at] = tile[s2 + s2 / 16 / 8];
      else
        reinterpret_cast<float *>(g.outT)[at] = (float)tile[s2 + s2 / 16 / 8];
    }
  }
}

static TrJob tr_job(const void *src, int s_dbl, int S, int64_t sstride, int nq, int64_t sq,
                    int64_t so, int64_t si, int O, int I, float *outQ, float *outT,
                    double *outQd = nullptr, double *outTd = nullptr) {
  TrJob g{};
  g.src = src; g.s_dbl = s_dbl; g.S = S; g.sstride = sstride;
  g.nq = nq; g.sq = sq; g.so = so; g.si = si; g.q_inner = sq == 1;
  g.O = O; g.I = I; g.outQ = outQ; g.outT = outT;
  if (outQd || outTd) {
    g.o_dbl = 1;
    g.outQ = outQd;
    g.outT = outTd;
  }
  g.tiles_i = pad32(I) / 16;
  return g;
}

// (any number of jobs: kTrJobs per launch)
static hipError_t fold_tr_v(const TrJob *jobs, int n, hipStream_t s) {
  for (int i0 = 0; i0 < n; i0 += kTrJobs) {
    TrJobs js{};
    int tiles = 0;
    for (int i = i0; i < std::min(n, i0 + kTrJobs); ++i) {
      const TrJob &g = jobs[i];
      if ((g.nq != 1 && g.nq != 9) || g.O <= 0 || g.I <= 0) return hipErrorInvalidValue;
      js.j[js.n] = g;
      js.tile0[js.n++] = tiles;
      const int OT = g.nq == 9 ? 4 : 36;
      tiles += g.tiles_i * ((pad32(g.O) + OT - 1) / OT);
    }
    js.tile0[js.n] = tiles;
    hipLaunchKernelGGL(k_fold_tr, dim3(tiles), dim3(576), 0, s, js);
  }
  return hipGetLastError();
}

static hipError_t fold_tr(std::initializer_list<TrJob> jobs, hipStream_t s) {
  return fold_tr_v(jobs.begin(), (int)jobs.size(), s);
}

// Wt [R][R][9] (o, c, q) as the A operand WtQ[q][o][c] of Wc and bq; W' [R][C]
// (c, i) as W'T[i][c]; bZ [R][V] (c, v) as bZT[v][c]
size_t fold_fwd_scratch_floats(int R, int C, int V) {
  const int Rp = pad32(R);
  return (size_t)Rp * (9 * Rp + pad32(C) + pad32(V));
}

// Wc[o][i][q] = sum_c Wt[o][c][q] W'[c][i]  and  bq[q][o][v] = sum_c Wt[o][c][q] bZ[c][v]
static hipError_t fold_fwd_gemms(const float *Wt, const float *W, const float *bZ, int R, int C,
                                 int V, float *Wc, double *bq, float *scratch, hipStream_t s) {
  const int Rp = pad32(R), Cp = pad32(C);
  float *wtq = scratch, *wT = wtq + (size_t)9 * Rp * Rp, *bzT = wT + (size_t)Cp * Rp;
  const TrJob ja = tr_job(Wt, 0, 1, 0, 9, 1, (int64_t)R * 9, 9, R, R, wtq, nullptr);
  const TrJob jb = tr_job(W, 0, 1, 0, 1, 0, C, 1, R, C, nullptr, wT);
  if (bq)
    HIP_RET(fold_tr({ja, jb, tr_job(bZ, 0, 1, 0, 1, 0, V, 1, R, V, nullptr, bzT)}, s));
  else
    HIP_RET(fold_tr({ja, jb}, s));
  FoldJob w{};
  w.A = wtq; w.aq = (int64_t)Rp * Rp; w.am = Rp;
  w.B = wT; w.bn = Rp;
  w.out = Wc; w.oq = 1; w.om = (int64_t)C * 9; w.on = 9;
  w.M = R; w.N = C; w.K = R;
  if (!bq) return fold_gemm({w}, s);
  FoldJob b{};
  b.A = wtq; b.aq = (int64_t)Rp * Rp; b.am = Rp;
  b.B = bzT; b.bn = Rp;
  b.out = bq; b.o_dbl = 1; b.oq = (int64_t)R * V; b.om = V; b.on = 1;
  b.M = R; b.N = V; b.K = R;
  return fold_gemm({w, b}, s);
}

hipError_t launch_fold_w(const float *Wt, const float *W, int R, int C, float *Wc, float *scratch,
                         hipStream_t s) {
  return fold_fwd_gemms(Wt, W, nullptr, R, C, 0, Wc, nullptr, scratch, s);
}

// Boundary frames of the folded block: output frames t < nb0 and t >= tb1 read
// padding for some tap (slot t, resp. nb0 + t - tb1; at most 8 slots)
__device__ __forceinline__ int fold_slot_frame(int slot, int nb0, int tb1) {
  return slot < nb0 ? slot : tb1 + slot - nb0;
}

// BT[o][t][v] = bt[o] + sum_{q: 0 <= s t + q - 4 < T} Bq[q][o][v],
// Bq[q][o][v] = sum_c Wt[o][c][q] bZ[c][v] (small GEMM into `bq`, R * V * 9 doubles)
__global__ __launch_bounds__(256) void k_fold_bias(const double *bq, const float *bt, int R, int V,
                                                   int T, int To, int st, float *BT) {
  __shared__ double bs[9 * 256], full[256];  // (V <= 256, checked by the launcher)
  const int o = blockIdx.x, tid = threadIdx.x;
  for (int e = tid; e < 9 * V; e += 256) {
    const int q = e / V, v = e - q * V;
    bs[e] = bq[((int64_t)q * R + o) * V + v];
  }
  __syncthreads();
  const double b0 = bt[o];
  if (tid < V) {
    double a = b0;
#pragma unroll
    for (int q = 0; q < 9; ++q) a += bs[q * V + tid];
    full[tid] = a;
  }
  __syncthreads();
  float *dst = BT + (int64_t)o * To * V;
  for (int tv = tid; tv < To * V; tv += 256) {
    const int t = tv / V, v = tv - t * V, t0 = st * t - 4;
    double a;
    if (t0 >= 0 && t0 + 8 < T) {
      a = full[v];  // (interior frame: all nine taps)
    } else {
      a = b0;
      for (int q = 0; q < 9; ++q)
        if (t0 + q >= 0 && t0 + q < T) a += bs[q * V + v];
    }
    dst[tv] = (float)a;
  }
}

static hipError_t fold_bias_frames(const double *bq, const float *bt, int R, int V, int T, int To,
                                   int st, float *BT, hipStream_t s) {
  if (V > 256) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_fold_bias, dim3(R), dim3(256), 0, s, bq, bt, R, V, T, To, st, BT);
  return hipGetLastError();
}

// the forward's fold in three launches: the re-layouts, {Wc, bq}, the table BT
hipError_t launch_fold_fwd(const float *Wt, const float *W, const float *bt, const float *bZ, int R,
                           int C, int V, int T, int To, int st, float *Wc, double *bq, float *BT,
                           float *scratch, hipStream_t s) {
  HIP_RET(fold_fwd_gemms(Wt, W, bZ, R, C, V, Wc, bq, scratch, s));
  return fold_bias_frames(bq, bt, R, V, T, To, st, BT, s);
}

// Tq[q][o][v] = sum_t cs[o][t][v] over the frames t whose tap q reads inside
// [0, T) (all but a few boundary frames): the total minus those frames.
// cs holds nz clip-chunk partials ([nz][R][To][V], k_bn_relu_bwd_apply_cols).
// One launch, one block per output channel (R <= 512 blocks reading R nz To V
// doubles: a few microseconds).

// block = o; thread (phase ph, joint v): the total over the chunks' frames
// t = ph, ph + PH, ... (in chunk order) and the boundary frame ph (< nsl) summed
// over the clip chunks; LDS reduce; threads v < V form the nine taps. tqT (or
// null): Tq also as the fp64 re-layout launch_fold_sdz reads ([q][Vp][Rp], zero
// padded; blocks o >= R only write their padding column)
// (1024 threads: 56 frame phases at V = 18, so each thread's loads are few and
// all in flight -- the kernel is latency-bound with one block per channel)
constexpr int kTqThreads = 1024;
__global__ __launch_bounds__(kTqThreads) void k_fold_tq(const double *cs, int nz, int R, int V,
                                                        int T, int To, int st, int nb0, int tb1,
                                                        double *Tq, double *tqT) {
  __shared__ double ts[kTqThreads], bs[8 * 256];  // (boundary slots x joints, V <= 256)
  const int o = blockIdx.x, tid = threadIdx.x;
  const int Rp = pad32(R), Vp = pad32(V);
  if (o >= R) {  // (tqT's zero padding columns)
    for (int e = tid; e < 9 * Vp; e += kTqThreads) tqT[(int64_t)e * Rp + o] = 0.0;
    return;
  }
  const int PH = kTqThreads / V, ph = tid / V, v = tid - ph * V;
  const int nsl = nb0 + (To - tb1);
  const int64_t zs = (int64_t)R * To * V;
  double a = 0.0;
  if (ph < PH) {
    // (the (chunk, frame) pairs flattened, four loads in flight per round)
    const int nj = nz * To;
    auto at = [&](int j) {
      const int z = j / To, t = j - z * To;
      return cs[z * zs + ((int64_t)o * To + t) * V + v];
    };
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    int j = ph;
    for (; j + 3 * PH < nj; j += 4 * PH) {
      const double x0 = at(j), x1 = at(j + PH), x2 = at(j + 2 * PH), x3 = at(j + 3 * PH);
      a0 += x0;
      a1 += x1;
      a2 += x2;
      a3 += x3;
    }
    for (; j < nj; j += PH) a0 += at(j);
    a = (a0 + a1) + (a2 + a3);
    for (int sl = ph; sl < nsl; sl += PH) {
      const int t = fold_slot_frame(sl, nb0, tb1);
      double b = 0.0;
      for (int z = 0; z < nz; ++z) b += cs[z * zs + ((int64_t)o * To + t) * V + v];
      bs[sl * V + v] = b;
    }
  }
  ts[tid] = a;
  __syncthreads();
  if (tqT && tid >= V && tid < Vp)  // (padding rows)
    for (int q = 0; q < 9; ++q) tqT[((int64_t)q * Vp + tid) * Rp + o] = 0.0;
  if (tid >= V) return;
  double tot = 0.0;
  for (int p = 0; p < PH; ++p) tot += ts[p * V + tid];
  for (int q = 0; q < 9; ++q) {
    double r = tot;
    for (int sl = 0; sl < nsl; ++sl) {
      const int tt = st * fold_slot_frame(sl, nb0, tb1) + q - 4;
      if (tt < 0 || tt >= T) r -= bs[sl * V + tid];
    }
    Tq[((int64_t)q * R + o) * V + tid] = r;
    if (tqT) tqT[((int64_t)q * Vp + tid) * Rp + o] = r;
  }
}

void fold_slots(int T, int To, int st, int &nb0, int &tb1) {
  nb0 = std::min(To, (4 + st - 1) / st);                   // frames with s t - 4 < 0
  tb1 = std::max(nb0, std::min(To, (T - 4 + st - 1) / st));  // frames with s t + 4 >= T
}

// one launch (the frame totals are summed by the same blocks; one block per
// output channel reads its nz * To * V sums)
hipError_t launch_fold_tq(const double *cs, int nz, int R, int T, int To, int V, int st,
                          double *Tq, double *tqT, hipStream_t s) {
  if (V > 256) return hipErrorInvalidValue;  // (checked before any launch)
  int nb0, tb1;
  fold_slots(T, To, st, nb0, tb1);
  hipLaunchKernelGGL(k_fold_tq, dim3(tqT ? pad32(R) : R), dim3(kTqThreads), 0, s, cs, nz, R, V, T, To, st,
                     nb0, tb1, Tq, tqT);
  return hipGetLastError();
}

double *fold_sdz_tq_slot(double *scratch, int R, int C) {
  return scratch + (size_t)9 * pad32(R) * (pad32(R) + pad32(C));
}

// amax[0] = max(amax[0], max_i |x[i]|) as float bits (non-negative floats order
// as unsigned integers): one atomic per wave
__global__ __launch_bounds__(256) void k_absmax(const float *x, int64_t n, unsigned *amax) {
  float m = 0.f;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if ((reinterpret_cast<uintptr_t>(x) & 15) == 0) {
    const int64_t n4 = n / 4;
    for (int64_t i = i0; i < n4; i += stride) {
      const float4 v = reinterpret_cast<const float4 *>(x)[i];
      m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    }
    for (int64_t i = n4 * 4 + i0; i < n; i += stride) m = fmaxf(m, fabsf(x[i]));
  } else {
    for (int64_t i = i0; i < n; i += stride) m = fmaxf(m, fabsf(x[i]));
  }
  block_amax<256>(m, amax);
}

hipError_t launch_absmax(const float *x, int64_t n, unsigned *amax, hipStream_t s) {
  const int64_t blocks = std::min<int64_t>(2048, std::max<int64_t>(1, (n / 4 + 255) / 256));
  hipLaunchKernelGGL(k_absmax, dim3((unsigned)blocks), dim3(256), 0, s, x, n, amax);
  return hipGetLastError();
}

// The backward's re-layouts (scratch: [WtT | W'c]): WtT[q][c][o] (A of dW': rows
// c, k = o), W' [c][i] (B of dWt: rows c, k = i)
size_t fold_bwd_scratch_floats(int R, int C) {
  const int Rp = pad32(R);
  return (size_t)Rp * (9 * Rp + pad32(C));
}
size_t fold_dwc_floats(int R, int C) { return (size_t)18 * pad32(R) * pad32(C); }

hipError_t launch_fold_prep_bwd(const float *Wt, const float *W, int R, int C, float *scratch,
                                hipStream_t s) {
  const int Rp = pad32(R);
  float *wtT = scratch, *wd = wtT + (size_t)9 * Rp * Rp;
  return fold_tr({tr_job(Wt, 0, 1, 0, 9, 1, (int64_t)R * 9, 9, R, R, nullptr, wtT),
                  tr_job(W, 0, 1, 0, 1, 0, C, 1, R, C, wd, nullptr)},
                 s);
}

// The folded block's weight gradients from the slabs of dWc (the temporal weight
// gradient over C_in channels, [S][o][i][q]) and Tq: the slab sum re-laid as
// dWcQ[q][o][i] and dWcT[q][i][o], then one GEMM launch:
//   dWt[o][c][q] = sum_i dWc[o][i][q] W'[c][i] + sum_v Tq[q][o][v] bZ[c][v]
//   dW'[c][i]    = sum_{(o,q)} Wt[o][c][q] dWc[o][i][q]
hipError_t launch_fold_grads(const float *slab, int S, const float *scratch, const float *bZ,
                             const double *Tq, int R, int C, int V, float *dwc, float *dWt,
                             float *dW, hipStream_t s) {
  const int Rp = pad32(R), Cp = pad32(C);
  const float *wtT = scratch, *wd = wtT + (size_t)9 * Rp * Rp;
  float *dWcQ = dwc, *dWcT = dwc + (size_t)9 * Rp * Cp;
  HIP_RET(fold_tr({tr_job(slab, 0, S, (int64_t)R * C * 9, 9, 1, (int64_t)C * 9, 9, R, C, dWcQ,
                          dWcT)},
                  s));
  FoldJob a{};
  a.A = dWcQ; a.aq = (int64_t)Rp * Cp; a.am = Cp;
  a.B = wd; a.bn = Cp;
  a.A2 = Tq; a.a2q = (int64_t)R * V; a.a2m = V;
  a.B2 = bZ; a.b2n = V;
  a.K2 = V;
  a.out = dWt; a.oq = 1; a.om = (int64_t)R * 9; a.on = 9;
  a.M = R; a.N = R; a.K = C;
  FoldJob b{};
  b.A = wtT; b.aq = (int64_t)Rp * Rp; b.am = Rp;
  b.B = dWcT; b.bq = (int64_t)Cp * Rp; b.bn = Rp;
  b.out = dW; b.om = C; b.on = 1; b.red = 1;
  b.M = R; b.N = C; b.K = R;
  return fold_gemm({a, b}, s);
}

// The dU-sum reductions on the fp64 matrix cores (v_mfma_f64_16x16x4_f64, 16 x 16
// tiles, nine waves = taps summed in LDS in tap order), from fp64 re-layouts:
//   SdZ[c][v] = sum_q sum_o Wt[o][c][q] Tq[q][o][v]   (= sum_{n,t} dZ[c,t,v])
//   SdH[c][v] = sum_q sum_o Wc[o][c][q] Tq[q][o][v]   (= sum_{n,t} H[c,t,v])
// Both feed sums that nearly cancel (BN2 makes sum_{t,v} dU = 0 per channel, so
// the bias gradients dbW, db1 are small against their terms): fp64 throughout.
struct Red64Job {
  const double *A, *B;  // A[q aq + m am + k], B[q bq + n bn + k] (k < K, padded to 16)
  int64_t aq, am, bq, bn;
  double *out;          // out[m om + n]
  int64_t om;
  int M, N, K;
};

struct Red64Jobs {
  Red64Job j[2];
  int n;
  int tile0[3];
};

template <int NG>
__device__ __forceinline__ void f64_stream(const double *pa, const double *pb, double4v &acc) {
  constexpr int D = NG < 4 ? NG : 4;
  double4v a[D], b[D];
#pragma unroll
  for (int d = 0; d < D; ++d) {
    a[d] = *reinterpret_cast<const double4v *>(pa + 16 * d);
    b[d] = *reinterpret_cast<const double4v *>(pb + 16 * d);
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < NG; ++i) {
    const int d = i % D;
#pragma unroll
    for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[d][j], b[d][j], acc, 0, 0, 0);
    if (i + D < NG) {
      a[d] = *reinterpret_cast<const double4v *>(pa + 16 * (i + D));
      b[d] = *reinterpret_cast<const double4v *>(pb + 16 * (i + D));
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

__global__ __launch_bounds__(576) void k_fold_red64(Red64Jobs js) {
  __shared__ double red[9][16 * 17];
  const int tile = blockIdx.x;
  const int ji = (js.n > 1 && tile >= js.tile0[1]) ? 1 : 0;
  const Red64Job &g = js.j[ji];
  const int t = tile - js.tile0[ji], ntn = (g.N + 15) >> 4;
  const int m0 = (t / ntn) * 16, n0 = (t % ntn) * 16;
  const int q = threadIdx.x >> 6, l = threadIdx.x & 63, r16 = l & 15, kq = (l >> 4) * 4;
  double4v acc = {0.0, 0.0, 0.0, 0.0};
  const double *pa = g.A + q * g.aq + (int64_t)(m0 + r16) * g.am + kq;
  const double *pb = g.B + q * g.bq + (int64_t)(n0 + r16) * g.bn + kq;
  // lane: k = 16 i + 4 (l >> 4) + j for MFMA j of group i (straight-line streams)
  const int ng = (g.K + 15) >> 4;
  if (ng == 4) {
    f64_stream<4>(pa, pb, acc);
  } else if (ng == 8) {
    f64_stream<8>(pa, pb, acc);
  } else if (ng == 16) {
    f64_stream<16>(pa, pb, acc);
  } else {
    for (int i = 0; i < ng; i += 4) {
      if (ng - i >= 4) {
        f64_stream<4>(pa + 16 * i, pb + 16 * i, acc);
      } else {
        for (int k = i; k < ng; ++k) f64_stream<1>(pa + 16 * k, pb + 16 * k, acc);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) red[q][((l >> 4) + 4 * r) * 17 + r16] = acc[r];
  __syncthreads();
  if (threadIdx.x >= 256) return;
  const int rr = threadIdx.x >> 4, cc = threadIdx.x & 15;
  const int mm = m0 + rr, nn = n0 + cc;
  if (mm >= g.M || nn >= g.N) return;
  double s = 0.0;
#pragma unroll
  for (int w = 0; w < 9; ++w) s += red[w][rr * 17 + cc];
  g.out[mm * g.om + nn] = s;
}

// doubles of launch_fold_sdz's scratch: WtT, WcT, TqT as fp64 [q][row][o]
size_t fold_sdz_scratch_doubles(int R, int C, int V) {
  return (size_t)9 * pad32(R) * (pad32(R) + pad32(C) + pad32(V));
}

// SdZ (and, with Wc, SdH); Wt [R][R][9], Wc [R][C][9] (o, c, q), Tq [9][R][V]
hipError_t launch_fold_sdz(double *scratch, const float *Wt, const float *Wc, const double *Tq,
                           int R, int C, int V, double *SdZ, double *SdH, hipStream_t s, bool pre,
                           const double *tq_re) {
  const int Rp = pad32(R), Cp = pad32(C), Vp = pad32(V);
  double *wtT = scratch, *wcT = wtT + (size_t)9 * Rp * Rp;
  const double *tqT = tq_re ? tq_re : wcT + (size_t)9 * Cp * Rp;
  const TrJob jt = tr_job(Wt, 0, 1, 0, 9, 1, (int64_t)R * 9, 9, R, R, nullptr, nullptr, nullptr, wtT);
  (void)Tq;  // (its re-layout tqT [q][Vp][Rp]: written by k_fold_tq, fold_sdz_tq_slot)
  if (pre) {
    // (the weight re-layouts were formed by launch_fold_prep)
  } else if (Wc) {
    HIP_RET(fold_tr({jt, tr_job(Wc, 0, 1, 0, 9, 1, (int64_t)C * 9, 9, R, C, nullptr, nullptr,
                                nullptr, wcT)},
                    s));
  } else {
    HIP_RET(fold_tr({jt}, s));
  }
  Red64Jobs js{};
  Red64Job z{};
  z.A = wtT; z.aq = (int64_t)Rp * Rp; z.am = Rp;
  z.B = tqT; z.bq = (int64_t)Vp * Rp; z.bn = Rp;
  z.out = SdZ; z.om = V;
  z.M = R; z.N = V; z.K = R;
  js.j[0] = z;
  js.n = 1;
  const int tz = ((R + 15) / 16) * ((V + 15) / 16);
  js.tile0[1] = tz;
  int tiles = tz;
  if (Wc && SdH) {
    Red64Job h = z;
    h.A = wcT; h.aq = (int64_t)Cp * Rp;
    h.out = SdH;
    h.M = C;
    js.j[1] = h;
    js.n = 2;
    tiles += ((C + 15) / 16) * ((V + 15) / 16);
  }
  js.tile0[js.n] = tiles;
  hipLaunchKernelGGL(k_fold_red64, dim3(tiles), dim3(576), 0, s, js);
  return hipGetLastError();
}

// k_spatial_small (K = 1: dbW, the bias part of dA from SdZ) and BN1's sd of the
// folded block (db1: sum_{n,t,v} of the BN1-output gradient,
// sd[c] = sum_v SdH[c][v] sum_w A[v][w], since dxhat[c,t,w] = sum_v A[v][w] H[c,t,v])
// in one launch: block 0 the first, blocks 1.. the second
__global__ __launch_bounds__(256) void k_fold_small_sd(const double *SdZ, const float *A,
                                                       const float *bW, int R, int V, float *dbW,
                                                       float *dA, const double *SdH, int C,
                                                       double *sd) {
  __shared__ double rs[256], part[256];
  const int tid = threadIdx.x;
  for (int v = tid; v < V; v += 256) {
    double ra = 0.0;
    for (int w = 0; w < V; ++w) ra += (double)A[v * V + w];
    rs[v] = ra;
  }
  __syncthreads();
  if (blockIdx.x > 0) {  // sd
    const int c = (blockIdx.x - 1) * blockDim.x + tid;
    if (c >= C) return;
    double a = 0.0;
    for (int v = 0; v < V; ++v) a += SdH[(int64_t)c * V + v] * rs[v];
    sd[c] = a;
    return;
  }
  // k_spatial_small, K = 1
  for (int co = tid; co < R; co += 256) {
    double acc = 0.0;
    for (int v = 0; v < V; ++v) acc += SdZ[co * V + v] * rs[v];
    dbW[co] = (float)acc;
  }
  const int P = 256 / V;
  const int v = tid % V, j = tid / V;
  double acc = 0.0;
  if (j < P)
    for (int co = j; co < R; co += P) acc += (double)bW[co] * SdZ[co * V + v];
  part[tid] = acc;
  __syncthreads();
  if (tid < V) {
    double t = 0.0;
    for (int jj = 0; jj < P; ++jj) t += part[jj * V + tid];
    rs[tid] = t;  // (rowsums no longer needed: block 0 only)
  }
  __syncthreads();
  for (int i = tid; i < V * V; i += 256) dA[i] = (float)rs[i / V];
}

hipError_t launch_fold_small_sd(const double *SdZ, const float *A, const float *bW, int R, int V,
                                float *dbW, float *dA, const double *SdH, int C, double *sd,
                                hipStream_t s) {
  if (V > 128) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_fold_small_sd, dim3(1 + (C + 255) / 256), dim3(256), 0, s, SdZ, A, bW, R, V,
                     dbW, dA, SdH, C, sd);
  return hipGetLastError();
}


// ---------------------------------------------------------------------------
// stgcn_fold_prep (capi.hip): the weight-only operands of every folded block of
// a stack in a dozen launches per training step instead of ~11 small launches
// per block in each block's forward and backward. Every job is the one the
// block would run itself (same kernels, same operand layouts, same order of
// arithmetic), batched over the blocks by job tables in the kernel arguments.
// ---------------------------------------------------------------------------
constexpr int kPrepJobs = 16;

struct BiasRvJob {
  const float *A, *bW;
  float *out;
  int R, V, blk0;  // first block of the job
};
struct BiasRvJobs {
  BiasRvJob j[kPrepJobs];
  int n, blk1;  // blk1 = total blocks
};

// bZ[co][v] = bW[co] rowsum(A)[v] (K = 1: the folded block), as k_bias_rv
__global__ void k_bias_rv_multi(BiasRvJobs js) {
  int k = 0;
  while (k + 1 < js.n && (int)blockIdx.x >= js.j[k + 1].blk0) ++k;
  const BiasRvJob &q = js.j[k];
  const int idx = ((int)blockIdx.x - q.blk0) * blockDim.x + threadIdx.x;
  if (idx >= q.R * q.V) return;
  const int co = idx / q.V, v = idx - co * q.V;
  double ra = 0.0;
  for (int w = 0; w < q.V; ++w) ra += q.A[(int64_t)v * q.V + w];
  q.out[idx] = (float)((double)q.bW[co] * ra);
}

struct BiasJob {
  const double *bq;
  const float *bt;
  float *BT;
  int R, V, T, To, st, blk0;
};
struct BiasJobs {
  BiasJob j[kPrepJobs];
  int n;
};

// k_fold_bias over several blocks (block = one output channel of one job)
__global__ __launch_bounds__(256) void k_fold_bias_multi(BiasJobs js) {
  int k = 0;
  while (k + 1 < js.n && (int)blockIdx.x >= js.j[k + 1].blk0) ++k;
  const BiasJob &q = js.j[k];
  __shared__ double bs[9 * 256], full[256];
  const int o = (int)blockIdx.x - q.blk0, tid = threadIdx.x, V = q.V, R = q.R;
  for (int e = tid; e < 9 * V; e += 256) {
    const int qq = e / V, v = e - qq * V;
    bs[e] = q.bq[((int64_t)qq * R + o) * V + v];
  }
  __syncthreads();
  const double b0 = q.bt[o];
  if (tid < V) {
    double a = b0;
#pragma unroll
    for (int qq = 0; qq < 9; ++qq) a += bs[qq * V + tid];
    full[tid] = a;
  }
  __syncthreads();
  float *dst = q.BT + (int64_t)o * q.To * V;
  for (int tv = tid; tv < q.To * V; tv += 256) {
    const int t = tv / V, v = tv - t * V, t0 = q.st * t - 4;
    double a;
    if (t0 >= 0 && t0 + 8 < q.T) {
      a = full[v];
    } else {
      a = b0;
      for (int qq = 0; qq < 9; ++qq)
        if (t0 + qq >= 0 && t0 + qq < q.T) a += bs[qq * V + v];
    }
    dst[tv] = (float)a;
  }
}

struct AmaxJob {
  const float *x;
  int64_t n;
  unsigned *amax;
};
struct AmaxJobs {
  AmaxJob j[kPrepJobs];
  int n;
};

// max |x| of each job into its kAmaxSlots words: job = blockIdx.y, the job's
// kAmaxSlots workgroups each store their own slot (no atomics: nothing to zero)
__global__ __launch_bounds__(256) void k_absmax_multi(AmaxJobs js) {
  const AmaxJob &q = js.j[blockIdx.y];
  float m = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < q.n; i += (int64_t)gridDim.x * 256)
    m = fmaxf(m, fabsf(q.x[i]));
  __shared__ float wmax[4];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0)
    q.amax[blockIdx.x * kAmaxStride] =
        __builtin_bit_cast(unsigned, fmaxf(fmaxf(wmax[0], wmax[1]), fmaxf(wmax[2], wmax[3])));
}

hipError_t launch_fold_prep(const FoldPrepSpec *sp, int n, hipStream_t s) {
  for (int i = 0; i < n; ++i)
    if (sp[i].V > 256 || sp[i].V <= 0 || sp[i].R <= 0 || sp[i].C <= 0) return hipErrorInvalidValue;
  // 1. bZ of every block
  for (int i0 = 0; i0 < n; i0 += kPrepJobs) {
    BiasRvJobs js{};
    int blk = 0;
    for (int i = i0; i < std::min(n, i0 + kPrepJobs); ++i) {
      js.j[js.n] = {sp[i].A, sp[i].bW, sp[i].bZ, sp[i].R, sp[i].V, blk};
      blk += (sp[i].R * sp[i].V + 255) / 256;
      ++js.n;
    }
    js.blk1 = blk;
    hipLaunchKernelGGL(k_bias_rv_multi, dim3(blk), dim3(256), 0, s, js);
  }
  // 2. the re-layouts of Wt, W', bZ: the forward's fold GEMM operands
  //    (fold_fwd_gemms), the backward's (launch_fold_prep_bwd) and the fp64 Wt of
  //    launch_fold_sdz
  std::vector<TrJob> tr;
  std::vector<FoldJob> fg;
  for (int i = 0; i < n; ++i) {
    const FoldPrepSpec &b = sp[i];
    const int R = b.R, C = b.C, V = b.V, Rp = pad32(R), Cp = pad32(C);
    float *wtq = b.fscr_f, *wT = wtq + (size_t)9 * Rp * Rp, *bzT = wT + (size_t)Cp * Rp;
    tr.push_back(tr_job(b.Wt, 0, 1, 0, 9, 1, (int64_t)R * 9, 9, R, R, wtq, nullptr));
    tr.push_back(tr_job(b.W, 0, 1, 0, 1, 0, C, 1, R, C, nullptr, wT));
    tr.push_back(tr_job(b.bZ, 0, 1, 0, 1, 0, V, 1, R, V, nullptr, bzT));
    float *wtT = b.fscr_b, *wd = wtT + (size_t)9 * Rp * Rp;
    tr.push_back(tr_job(b.Wt, 0, 1, 0, 9, 1, (int64_t)R * 9, 9, R, R, nullptr, wtT));
    tr.push_back(tr_job(b.W, 0, 1, 0, 1, 0, C, 1, R, C, wd, nullptr));
    tr.push_back(tr_job(b.Wt, 0, 1, 0, 9, 1, (int64_t)R * 9, 9, R, R, nullptr, nullptr, nullptr,
                        b.f64));
    FoldJob w{};
    w.A = wtq; w.aq = (int64_t)Rp * Rp; w.am = Rp;
    w.B = wT; w.bn = Rp;
    w.out = b.Wc; w.oq = 1; w.om = (int64_t)C * 9; w.on = 9;
    w.M = R; w.N = C; w.K = R;
    FoldJob q{};
    q.A = wtq; q.aq = (int64_t)Rp * Rp; q.am = Rp;
    q.B = bzT; q.bn = Rp;
    q.out = b.bq; q.o_dbl = 1; q.oq = (int64_t)R * V; q.om = V; q.on = 1;
    q.M = R; q.N = V; q.K = R;
    fg.push_back(w);
    fg.push_back(q);
  }
  HIP_RET(fold_tr_v(tr.data(), (int)tr.size(), s));
  // 3. Wc = Wt W' and the bias products bq (fold_fwd_gemms)
  HIP_RET(fold_gemm_v(fg.data(), (int)fg.size(), s));
  // 4. the per-frame bias tables, the fp64 Wc re-layout of launch_fold_sdz, max |Wc|
  for (int i0 = 0; i0 < n; i0 += kPrepJobs) {
    BiasJobs js{};
    AmaxJobs am{};
    int blk = 0;
    for (int i = i0; i < std::min(n, i0 + kPrepJobs); ++i) {
      js.j[js.n++] = {sp[i].bq, sp[i].bWt, sp[i].BT, sp[i].R, sp[i].V, sp[i].T, sp[i].To,
                      sp[i].stride, blk};
      blk += sp[i].R;
      am.j[am.n++] = {sp[i].Wc, (int64_t)sp[i].R * sp[i].C * 9, sp[i].amax};
    }
    hipLaunchKernelGGL(k_fold_bias_multi, dim3(blk), dim3(256), 0, s, js);
    hipLaunchKernelGGL(k_absmax_multi, dim3(kAmaxSlots, am.n), dim3(256), 0, s, am);
  }
  tr.clear();
  for (int i = 0; i < n; ++i) {
    const FoldPrepSpec &b = sp[i];
    const int R = b.R, C = b.C, Rp = pad32(R);
    tr.push_back(tr_job(b.Wc, 0, 1, 0, 9, 1, (int64_t)C * 9, 9, R, C, nullptr, nullptr, nullptr,
                        b.f64 + (size_t)9 * Rp * Rp));
  }
  HIP_RET(fold_tr_v(tr.data(), (int)tr.size(), s));
  return hipGetLastError();
}

}  // namespace stgcn

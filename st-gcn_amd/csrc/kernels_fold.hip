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

#include "device_common.h"
#include "internal.h"

#define HIP_RET(expr)                  \
  do {                                 \
    hipError_t e_ = (expr);            \
    if (e_ != hipSuccess) return e_;   \
  } while (0)

namespace stgcn {

// The fold's small GEMMs on the fp64 matrix cores (v_mfma_f64_16x16x4_f64;
// operands float or double converted exactly, fp64 products and accumulation
// in a fixed order: deterministic). Two shapes cover them:
//
// k_fold_tapgemm: out[m][n][q] = sum_k A[m][k][q] B[k][n] (+ sum_v A2[q][m][v] B2[v][n])
//   for all nine taps q in ONE block: the A rows are contiguous 9-tap runs
//   (coalesced), the B tile is shared by the taps. Wc = Wt W', dWt = dWc W'^T
//   (+ the Tq bZ bias term) and the bias products bq.
// k_fold_koq: out[m][n] = sum_o sum_q A[o][m][q] B[o][n][q]: K = (o, q), split
//   over o in slabs summed in a fixed order afterwards. dW' = sum_q Wt_q^T dWc_q
//   and sum_{n,t} dZ = sum_q Wt_q^T Tq.
// Tiles of 32 x 32 per block, wave = one 16 x 16 MFMA tile (per tap).
typedef double double4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ double ld_fd(const void *p, int dbl, int64_t i) {
  return dbl ? reinterpret_cast<const double *>(p)[i] : (double)reinterpret_cast<const float *>(p)[i];
}

struct TapGemm {
  const void *A;
  int a_dbl;
  int64_t am, ak, aq;  // A[m am + k ak + q aq]
  const float *B;
  int64_t bk, bn;      // B[k bk + n bn]
  const double *A2;    // (or null) A2[q a2q + m a2m + v], v < K2
  int64_t a2q, a2m;
  const float *B2;     // B2[v b2k + n b2n]
  int64_t b2k, b2n;
  void *out;
  int o_dbl;
  int64_t om, on, oq;  // out[m om + n on + q oq]
  int M, N, K, K2;
  double *part;        // [S][M][N][9] split-K partials (summed by k_tap_sum)
  int kper;            // k per split (a multiple of the chunk)
};

// One block = 32 x 32 outputs x 9 taps over the k range of split blockIdx.z;
// the next chunk's operands are loaded into registers while this chunk's MFMAs run.
__global__ __launch_bounds__(256) void k_fold_tapgemm(TapGemm g) {
  constexpr int KC = 8;
  // (rows of 33: the staging writes walk q fastest, 33 doubles apart, so
  // consecutive lanes hit different banks; 32 would put all nine taps on one)
  __shared__ double As[KC][9][33], Bs[KC][32];
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int wm = (w & 1) * 16, wn = (w >> 1) * 16;
  const int m0 = blockIdx.y * 32, n0 = blockIdx.x * 32;
  const int Ktot = g.K + (g.A2 ? g.K2 : 0);
  const int kb = blockIdx.z * g.kper, ke = min(Ktot, kb + g.kper);
  double4v acc[9];
#pragma unroll
  for (int q = 0; q < 9; ++q) acc[q] = (double4v){0.0, 0.0, 0.0, 0.0};
  double ra[9], rb;
  auto load = [&](int k0) {
#pragma unroll
    for (int r = 0; r < 9; ++r) {  // A: q fastest, then k, then m (9-tap runs)
      const int e = r * 256 + tid;
      const int q = e % 9, t = e / 9, kk = t % KC, mm = t / KC;
      const int k = k0 + kk, m = m0 + mm;
      double v = 0.0;
      if (m < g.M && k < ke) {
        if (k < g.K)
          v = ld_fd(g.A, g.a_dbl, m * g.am + k * g.ak + q * g.aq);
        else
          v = g.A2[q * g.a2q + m * g.a2m + (k - g.K)];
      }
      ra[r] = v;
    }
    const int kk = tid >> 5, nn = tid & 31, k = k0 + kk, n = n0 + nn;
    rb = 0.0;
    if (n < g.N && k < ke) rb = k < g.K ? g.B[k * g.bk + n * g.bn] : g.B2[(k - g.K) * g.b2k + n * g.b2n];
  };
  if (kb < ke) load(kb);
  for (int k0 = kb; k0 < ke; k0 += KC) {
    __syncthreads();  // the previous chunk's reads are done
#pragma unroll
    for (int r = 0; r < 9; ++r) {
      const int e = r * 256 + tid;
      const int q = e % 9, t = e / 9;
      As[t % KC][q][t / KC] = ra[r];
    }
    Bs[tid >> 5][tid & 31] = rb;
    __syncthreads();
    if (k0 + KC < ke) load(k0 + KC);  // in flight under this chunk's MFMAs
#pragma unroll
    for (int ks = 0; ks < KC; ks += 4) {
      // A operand: lane l holds A[row l & 15][k l >> 4]; B: B[k l >> 4][col l & 15]
      const double b = Bs[ks + (l >> 4)][wn + (l & 15)];
#pragma unroll
      for (int q = 0; q < 9; ++q)
        acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(As[ks + (l >> 4)][q][wm + (l & 15)], b,
                                                      acc[q], 0, 0, 0);
    }
  }
  // C/D: col = lane & 15, row = (lane >> 4) + 4 * reg
  const int n = n0 + wn + (l & 15);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int m = m0 + wm + (l >> 4) + 4 * r;
    if (m >= g.M || n >= g.N) continue;
    double *dst = g.part + (((int64_t)blockIdx.z * g.M + m) * g.N + n) * 9;
#pragma unroll
    for (int q = 0; q < 9; ++q) dst[q] = acc[q][r];
  }
}

// out[m om + n on + q oq] = sum_s part[s][m][n][q] (fixed order), float or double
__global__ void k_tap_sum(TapGemm g, int S) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t tot = (int64_t)g.M * g.N * 9;
  if (i >= tot) return;
  const int q = (int)(i % 9);
  const int64_t mn = i / 9;
  const int n = (int)(mn % g.N), m = (int)(mn / g.N);
  double a = 0.0;
  for (int z = 0; z < S; ++z) a += g.part[(int64_t)z * tot + i];
  const int64_t o = m * g.om + n * g.on + q * g.oq;
  if (g.o_dbl)
    reinterpret_cast<double *>(g.out)[o] = a;
  else
    reinterpret_cast<float *>(g.out)[o] = (float)a;
}

// split-K over <= 4 slabs so the grid fills the chip (part: 4 * 9 * M * N doubles)
static hipError_t tapgemm(TapGemm g, double *part, hipStream_t s) {
  const int tiles = ((g.M + 31) / 32) * ((g.N + 31) / 32);
  const int Ktot = g.K + (g.A2 ? g.K2 : 0);
  const int chunks = (Ktot + 7) / 8;
  const int S = std::max(1, std::min(std::min(4, (256 + tiles - 1) / tiles), chunks));
  g.kper = (chunks + S - 1) / S * 8;
  g.part = part;
  hipLaunchKernelGGL(k_fold_tapgemm, dim3((g.N + 31) / 32, (g.M + 31) / 32, S), dim3(256), 0, s, g);
  const int64_t tot = (int64_t)g.M * g.N * 9;
  hipLaunchKernelGGL(k_tap_sum, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, g, S);
  return hipGetLastError();
}

struct KoqGemm {
  const float *A;
  int64_t a_o, a_m, a_q;  // A[o a_o + m a_m + q a_q]
  const void *B;
  int b_dbl;
  int64_t b_o, b_n, b_q;  // B[o b_o + n b_n + q b_q]
  double *part;           // [S][M][N] partial sums over o-slices
  int M, N, O, per;       // o in [s per, min(O, (s + 1) per)) for split s = blockIdx.z
};

__global__ __launch_bounds__(256) void k_fold_koq(KoqGemm g) {
  constexpr int KO = 4;  // o per chunk: 36 k = 9 MFMA k-steps
  __shared__ double As[KO * 9][33], Bs[KO * 9][33];  // (33: conflict-free staging writes)
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int wm = (w & 1) * 16, wn = (w >> 1) * 16;
  const int m0 = blockIdx.y * 32, n0 = blockIdx.x * 32;
  const int o_begin = blockIdx.z * g.per, o_end = min(g.O, o_begin + g.per);
  double4v acc = {0.0, 0.0, 0.0, 0.0};
  constexpr int NE = (KO * 9 * 32 + 255) / 256;  // elements per thread and operand
  double ra[NE], rb[NE];
  auto load = [&](int o0) {  // q fastest, then m / n, then o
#pragma unroll
    for (int r = 0; r < NE; ++r) {
      const int e = r * 256 + tid;
      const int q = e % 9, t = e / 9, mm = t % 32, oo = t / 32;
      const int o = o0 + oo, m = m0 + mm, n = n0 + mm;
      const bool ok = e < KO * 9 * 32 && o < o_end;
      ra[r] = ok && m < g.M ? (double)g.A[o * g.a_o + m * g.a_m + q * g.a_q] : 0.0;
      rb[r] = ok && n < g.N ? ld_fd(g.B, g.b_dbl, o * g.b_o + n * g.b_n + q * g.b_q) : 0.0;
    }
  };
  if (o_begin < o_end) load(o_begin);
  for (int o0 = o_begin; o0 < o_end; o0 += KO) {
    __syncthreads();
#pragma unroll
    for (int r = 0; r < NE; ++r) {
      const int e = r * 256 + tid;
      if (e < KO * 9 * 32) {
        const int q = e % 9, t = e / 9, mm = t % 32, oo = t / 32;
        As[oo * 9 + q][mm] = ra[r];
        Bs[oo * 9 + q][mm] = rb[r];
      }
    }
    __syncthreads();
    if (o0 + KO < o_end) load(o0 + KO);  // in flight under this chunk's MFMAs
#pragma unroll
    for (int ks = 0; ks < KO * 9; ks += 4)
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(As[ks + (l >> 4)][wm + (l & 15)],
                                                 Bs[ks + (l >> 4)][wn + (l & 15)], acc, 0, 0, 0);
  }
  const int n = n0 + wn + (l & 15);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int m = m0 + wm + (l >> 4) + 4 * r;
    if (m < g.M && n < g.N) g.part[((int64_t)blockIdx.z * g.M + m) * g.N + n] = acc[r];
  }
}

// dst[i] = sum_{z < Z} part[z * n + i] (fixed order), as float or double
__global__ void k_sum_parts(const double *part, int Z, int64_t n, float *dstf, double *dstd) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double a = 0.0;
  for (int z = 0; z < Z; ++z) a += part[(int64_t)z * n + i];
  if (dstf) dstf[i] = (float)a;
  else dstd[i] = a;
}

size_t fold_part_doubles(int R, int C, int V) {
  return (size_t)36 * R * std::max(std::max(R, C), V);
}

// slabs of the o-split: enough blocks to fill the chip, at least 8 o per slab
static int koq_splits(int M, int N, int O) {
  const int tiles = ((M + 31) / 32) * ((N + 31) / 32);
  return std::max(1, std::min(std::min((256 + tiles - 1) / tiles, (O + 7) / 8), 9));
}

// part must hold koq_splits(M, N, O) * M * N doubles (the callers' fold part buffer
// holds 9 R max(C, V) >= that); the result goes to dstf (float) or dstd
static hipError_t koq(KoqGemm g, double *part, float *dstf, double *dstd, hipStream_t s) {
  const int S = koq_splits(g.M, g.N, g.O);
  g.per = (g.O + S - 1) / S;
  g.part = part;
  hipLaunchKernelGGL(k_fold_koq, dim3((g.N + 31) / 32, (g.M + 31) / 32, S), dim3(256), 0, s, g);
  const int64_t n = (int64_t)g.M * g.N;
  hipLaunchKernelGGL(k_sum_parts, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, part, S, n,
                     dstf, dstd);
  return hipGetLastError();
}

// Wc[o][i][q] = sum_c Wt[o][c][q] W'[c][i]   (W' = SpatialConv.W, C_out x C_in)
hipError_t launch_fold_w(const float *Wt, const float *W, int R, int C, float *Wc, double *part,
                         hipStream_t s) {
  TapGemm g{};
  g.A = Wt; g.am = (int64_t)R * 9; g.ak = 9; g.aq = 1;
  g.B = W; g.bk = C; g.bn = 1;
  g.out = Wc; g.om = (int64_t)C * 9; g.on = 9; g.oq = 1;
  g.M = R; g.N = C; g.K = R;
  return tapgemm(g, part, s);
}

// Boundary frames of the folded block: output frames t < nb0 and t >= tb1 read
// padding for some tap (slot t, resp. nb0 + t - tb1; at most 8 slots)
__device__ __forceinline__ int fold_slot_frame(int slot, int nb0, int tb1) {
  return slot < nb0 ? slot : tb1 + slot - nb0;
}

// BT[o][t][v] = bt[o] + sum_{q: 0 <= s t + q - 4 < T} Bq[q][o][v],
// Bq[q][o][v] = sum_c Wt[o][c][q] bZ[c][v] (small GEMM into `bq`, R * V * 9 doubles)
__global__ void k_fold_bias(const double *bq, const float *bt, int R, int V, int T, int To, int st,
                            float *BT) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)R * To * V) return;
  const int v = (int)(idx % V);
  const int64_t ot = idx / V;
  const int t = (int)(ot % To), o = (int)(ot / To);
  const int t0 = st * t - 4;
  double a = bt[o];
#pragma unroll
  for (int q = 0; q < 9; ++q)
    if (t0 + q >= 0 && t0 + q < T) a += bq[((int64_t)q * R + o) * V + v];
  BT[idx] = (float)a;
}

hipError_t launch_fold_bias(const float *Wt, const float *bt, const float *bZ, int R, int V, int T,
                            int To, int st, double *bq, float *BT, double *part, hipStream_t s) {
  // bq[q][o][v] = sum_c Wt[o][c][q] bZ[c][v]
  TapGemm g{};
  g.A = Wt; g.am = (int64_t)R * 9; g.ak = 9; g.aq = 1;
  g.B = bZ; g.bk = V; g.bn = 1;
  g.out = bq; g.o_dbl = 1; g.om = V; g.on = 1; g.oq = (int64_t)R * V;
  g.M = R; g.N = V; g.K = R;
  HIP_RET(tapgemm(g, part, s));
  const int64_t n = (int64_t)R * To * V;
  hipLaunchKernelGGL(k_fold_bias, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, bq, bt, R, V,
                     T, To, st, BT);
  return hipGetLastError();
}

// Tq[q][o][v] = sum_t cs[o][t][v] over the frames t whose tap q reads inside
// [0, T) (all but a few boundary frames): the total minus those frames.
// cs holds nz clip-chunk partials ([nz][R][To][V], k_bn_relu_bwd_apply_cols).
// Two steps: k_fold_tot sums frame blocks of 16 (grid R x nz x blocks, one
// partial per block and joint, fixed order), k_fold_tq adds the partials and
// subtracts the boundary frames per tap.
constexpr int kTotFrames = 16;

__global__ __launch_bounds__(256) void k_fold_tot(const double *cs, int R, int V, int To,
                                                  double *part) {
  __shared__ double ts[256];
  const int o = blockIdx.x, z = blockIdx.y, tb = blockIdx.z, tid = threadIdx.x;
  const int PH = 256 / V, ph = tid / V, v = tid - ph * V;
  const double *c = cs + ((int64_t)z * R + o) * To * V;
  double a = 0.0;
  if (ph < PH)
    for (int t = tb * kTotFrames + ph; t < min(To, (tb + 1) * kTotFrames); t += PH)
      a += c[(int64_t)t * V + v];
  ts[tid] = a;
  __syncthreads();
  if (tid >= V) return;
  double tot = 0.0;
  for (int p = 0; p < PH; ++p) tot += ts[p * V + tid];
  part[(((int64_t)o * gridDim.y + z) * gridDim.z + tb) * V + tid] = tot;
}

// block = o; thread (phase ph, joint v): partial totals over the frame-block
// partials k = ph, ph + PH, ..., and the boundary frame ph (< nsl) summed over
// the clip chunks; LDS reduce; threads v < V form the nine taps
__global__ __launch_bounds__(256) void k_fold_tq(const double *cs, const double *part, int np,
                                                 int nz, int R, int V, int T, int To, int st,
                                                 int nb0, int tb1, double *Tq) {
  __shared__ double ts[256], bs[8 * 256];  // (boundary slots x joints, V <= 256)
  const int o = blockIdx.x, tid = threadIdx.x;
  const int PH = 256 / V, ph = tid / V, v = tid - ph * V;
  const int nsl = nb0 + (To - tb1);
  const int64_t zs = (int64_t)R * To * V;
  double a = 0.0;
  if (ph < PH) {
    for (int k = ph; k < np; k += PH) a += part[((int64_t)o * np + k) * V + v];
    for (int sl = ph; sl < nsl; sl += PH) {
      const int t = fold_slot_frame(sl, nb0, tb1);
      double b = 0.0;
      for (int z = 0; z < nz; ++z) b += cs[z * zs + ((int64_t)o * To + t) * V + v];
      bs[sl * V + v] = b;
    }
  }
  ts[tid] = a;
  __syncthreads();
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
  }
}

void fold_slots(int T, int To, int st, int &nb0, int &tb1) {
  nb0 = std::min(To, (4 + st - 1) / st);                   // frames with s t - 4 < 0
  tb1 = std::max(nb0, std::min(To, (T - 4 + st - 1) / st));  // frames with s t + 4 >= T
}

int fold_tot_blocks(int To) { return (To + kTotFrames - 1) / kTotFrames; }

// part: R * nz * fold_tot_blocks(To) * V doubles
hipError_t launch_fold_tq(const double *cs, int nz, int R, int T, int To, int V, int st,
                          double *part, double *Tq, hipStream_t s) {
  if (V > 256) return hipErrorInvalidValue;  // (checked before any launch)
  int nb0, tb1;
  fold_slots(T, To, st, nb0, tb1);
  const int ntb = fold_tot_blocks(To);
  hipLaunchKernelGGL(k_fold_tot, dim3(R, nz, ntb), dim3(256), 0, s, cs, R, V, To, part);
  hipLaunchKernelGGL(k_fold_tq, dim3(R), dim3(256), 0, s, cs, part, nz * ntb, nz, R, V, T, To, st,
                     nb0, tb1, Tq);
  return hipGetLastError();
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

__global__ void k_slab_reduce_f64(const float *slab, int S, int64_t n, double *dst) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double a = 0.0;
  for (int k = 0; k < S; ++k) a += slab[(int64_t)k * n + i];
  dst[i] = a;
}

// The folded block's weight gradients from dWc (slab of the temporal weight
// gradient over C_in channels) and Tq:
//   dWt[o][c][q] = sum_i dWc[o][i][q] W'[c][i] + sum_v Tq[q][o][v] bZ[c][v]
//   dW'[c][i]    = sum_{(o,q)} Wt[o][c][q] dWc[o][i][q]
// part: fold_part_doubles(R, C, V) doubles (split-K slabs)
hipError_t launch_fold_grads(const float *slab, int S, const float *Wt, const float *W,
                             const float *bZ, const double *Tq, int R, int C, int V,
                             double *dWc, double *part, float *dWt, float *dW, hipStream_t s) {
  const int64_t n = (int64_t)R * C * 9;
  hipLaunchKernelGGL(k_slab_reduce_f64, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, slab,
                     S, n, dWc);
  {
    TapGemm g{};
    g.A = dWc; g.a_dbl = 1; g.am = (int64_t)C * 9; g.ak = 9; g.aq = 1;
    g.B = W; g.bk = 1; g.bn = C;
    g.A2 = Tq; g.a2q = (int64_t)R * V; g.a2m = V;
    g.B2 = bZ; g.b2k = 1; g.b2n = V;
    g.K2 = V;
    g.out = dWt; g.om = (int64_t)R * 9; g.on = 9; g.oq = 1;
    g.M = R; g.N = R; g.K = C;
    HIP_RET(tapgemm(g, part, s));
  }
  KoqGemm g{};
  g.A = Wt; g.a_o = (int64_t)R * 9; g.a_m = 9; g.a_q = 1;
  g.B = dWc; g.b_dbl = 1; g.b_o = (int64_t)C * 9; g.b_n = 9; g.b_q = 1;
  g.M = R; g.N = C; g.O = R;
  return koq(g, part, dW, nullptr, s);
}

// SdZ[c][v] = sum_q sum_o Wt[o][c][q] Tq[q][o][v]  (= sum_{n,t} dZ[c,t,v]; Wt is
// the temporal weight [R][C][9] with C = its input channels, the Z channels);
// part: fold_part_doubles(R, C, V) doubles
hipError_t launch_fold_sdz(const float *Wt, const double *Tq, int R, int C, int V, double *part,
                           double *SdZ, hipStream_t s) {
  KoqGemm g{};
  g.A = Wt; g.a_o = (int64_t)C * 9; g.a_m = 9; g.a_q = 1;
  g.B = Tq; g.b_dbl = 1; g.b_o = V; g.b_n = 1; g.b_q = (int64_t)R * V;
  g.M = C; g.N = V; g.O = R;
  return koq(g, part, nullptr, SdZ, s);
}

}  // namespace stgcn

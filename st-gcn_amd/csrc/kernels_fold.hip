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

#include "internal.h"

#define HIP_RET(expr)                  \
  do {                                 \
    hipError_t e_ = (expr);            \
    if (e_ != hipSuccess) return e_;   \
  } while (0)

namespace stgcn {

// out[z][m][n] = sum_{k < K} A[z][m][k] B[z][k][n] + sum_{k < K2} A2[z][m][k] B2[k][n]
// (element offsets from the strides, z = blockIdx.z adds a_z / b_z / a2_z /
// o_z). fp64 accumulation; operands and output float or double (run-time
// flags). Block = 256 threads (4 waves) on a 32 x 32 output tile, thread = 4 x 4
// outputs; K in 64-deep chunks staged in LDS ([k][m] and [k][n]); wave w takes
// k-steps w*16 .. w*16+15 of each chunk, and the four partial tiles are summed
// in a fixed order through LDS at the end (deterministic).
struct SmallGemm {
  const void *A, *B, *A2, *B2;
  void *out;
  int M, N, K, K2;
  int a_dbl, b_dbl, a2_dbl, b2_dbl, o_dbl;
  int64_t am, ak, bk, bn, om, on;
  int64_t a2m, a2k, b2k, b2n;
  int64_t a_z, b_z, a2_z, o_z;
};

__device__ __forceinline__ double ld_fd(const void *p, int dbl, int64_t i) {
  return dbl ? reinterpret_cast<const double *>(p)[i] : (double)reinterpret_cast<const float *>(p)[i];
}

__global__ __launch_bounds__(256) void k_small_gemm(SmallGemm g) {
  // 32 x 32 output tile; wave w takes k-steps w*16 .. +15 of every 64-deep
  // chunk (thread = 4 x 4 outputs), the four partial tiles summed in LDS at the end
  __shared__ __attribute__((aligned(16))) double sm[2 * 64 * 32];
  double(*As)[32] = reinterpret_cast<double(*)[32]>(sm);            // [k][m]
  double(*Bs)[32] = reinterpret_cast<double(*)[32]>(sm + 64 * 32);  // [k][n]
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int tm = l >> 3, tn = l & 7;
  const int m0 = blockIdx.y * 32, n0 = blockIdx.x * 32;
  const int64_t z = blockIdx.z;
  double acc[4][4] = {};
  auto run = [&](const void *A, const void *B, int adbl, int bdbl, int K, int64_t am, int64_t ak,
                 int64_t bk, int64_t bn, int64_t aoff, int64_t boff) {
    for (int k0 = 0; k0 < K; k0 += 64) {
      __syncthreads();
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const int e = r * 256 + tid;
        {  // A: consecutive threads take consecutive k of one row
          const int kk = e & 63, mm = e >> 6;
          const int m = m0 + mm, k = k0 + kk;
          As[kk][mm] = (m < g.M && k < K) ? ld_fd(A, adbl, aoff + m * am + k * ak) : 0.0;
        }
        {
          const int nn = e & 31, kk = e >> 5;
          const int k = k0 + kk, n = n0 + nn;
          Bs[kk][nn] = (k < K && n < g.N) ? ld_fd(B, bdbl, boff + k * bk + n * bn) : 0.0;
        }
      }
      __syncthreads();
#pragma unroll 4
      for (int kk = w * 16; kk < w * 16 + 16; ++kk) {
        double a[4], b[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          a[i] = As[kk][tm * 4 + i];
          b[i] = Bs[kk][tn * 4 + i];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] += a[i] * b[j];
      }
    }
  };
  run(g.A, g.B, g.a_dbl, g.b_dbl, g.K, g.am, g.ak, g.bk, g.bn, z * g.a_z, z * g.b_z);
  if (g.A2) run(g.A2, g.B2, g.a2_dbl, g.b2_dbl, g.K2, g.a2m, g.a2k, g.b2k, g.b2n, z * g.a2_z, 0);
  // partial tiles of waves 1-3 -> LDS, wave 0 sums in fixed order and stores
  __syncthreads();
  if (w > 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) sm[((w - 1) * 64 + l) * 16 + i * 4 + j] = acc[i][j];
  }
  __syncthreads();
  if (w > 0) return;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + tm * 4 + i;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + tn * 4 + j;
      double v = acc[i][j];
#pragma unroll
      for (int p = 0; p < 3; ++p) v += sm[(p * 64 + l) * 16 + i * 4 + j];
      if (m >= g.M || n >= g.N) continue;
      const int64_t o = z * g.o_z + m * g.om + n * g.on;
      if (g.o_dbl)
        reinterpret_cast<double *>(g.out)[o] = v;
      else
        reinterpret_cast<float *>(g.out)[o] = (float)v;
    }
  }
}

static hipError_t small_gemm(const SmallGemm &g, int nz, hipStream_t s) {
  hipLaunchKernelGGL(k_small_gemm, dim3((g.N + 31) / 32, (g.M + 31) / 32, nz), dim3(256), 0, s, g);
  return hipGetLastError();
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

// Wc[o][i][q] = sum_c Wt[o][c][q] W'[c][i]   (W' = SpatialConv.W, C_out x C_in)
hipError_t launch_fold_w(const float *Wt, const float *W, int R, int C, float *Wc, hipStream_t s) {
  SmallGemm g{};
  g.A = Wt; g.am = (int64_t)R * 9; g.ak = 9; g.a_z = 1;
  g.B = W; g.bk = C; g.bn = 1;
  g.out = Wc; g.om = (int64_t)C * 9; g.on = 9; g.o_z = 1;
  g.M = R; g.N = C; g.K = R;
  return small_gemm(g, 9, s);
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
                            int To, int st, double *bq, float *BT, hipStream_t s) {
  SmallGemm g{};
  g.A = Wt; g.am = (int64_t)R * 9; g.ak = 9; g.a_z = 1;
  g.B = bZ; g.bk = V; g.bn = 1;
  g.out = bq; g.o_dbl = 1; g.om = V; g.on = 1; g.o_z = (int64_t)R * V;
  g.M = R; g.N = V; g.K = R;
  HIP_RET(small_gemm(g, 9, s));
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
//   dW'[c][i]    = sum_q sum_o Wt[o][c][q] dWc[o][i][q]
// (the tap sum of dW' as per-tap partial products in `part`, 9 R max(C, V)
// doubles, summed in fixed order)
hipError_t launch_fold_grads(const float *slab, int S, const float *Wt, const float *W,
                             const float *bZ, const double *Tq, int R, int C, int V,
                             double *dWc, double *part, float *dWt, float *dW, hipStream_t s) {
  const int64_t n = (int64_t)R * C * 9;
  hipLaunchKernelGGL(k_slab_reduce_f64, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, slab,
                     S, n, dWc);
  {
    SmallGemm g{};
    g.A = dWc; g.a_dbl = 1; g.am = (int64_t)C * 9; g.ak = 9; g.a_z = 1;
    g.B = W; g.bk = 1; g.bn = C;
    g.A2 = Tq; g.a2_dbl = 1; g.a2m = V; g.a2k = 1; g.a2_z = (int64_t)R * V;
    g.B2 = bZ; g.b2k = 1; g.b2n = V;
    g.K2 = V;
    g.out = dWt; g.om = (int64_t)R * 9; g.on = 9; g.o_z = 1;
    g.M = R; g.N = R; g.K = C;
    HIP_RET(small_gemm(g, 9, s));
  }
  {
    SmallGemm g{};
    g.A = Wt; g.am = 9; g.ak = (int64_t)R * 9; g.a_z = 1;
    g.B = dWc; g.b_dbl = 1; g.bk = (int64_t)C * 9; g.bn = 9; g.b_z = 1;
    g.out = part; g.o_dbl = 1; g.om = C; g.on = 1; g.o_z = (int64_t)R * C;
    g.M = R; g.N = C; g.K = R;
    HIP_RET(small_gemm(g, 9, s));
    const int64_t m = (int64_t)R * C;
    hipLaunchKernelGGL(k_sum_parts, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, part, 9, m,
                       dW, nullptr);
  }
  return hipGetLastError();
}

// SdZ[c][v] = sum_q sum_o Wt[o][c][q] Tq[q][o][v]  (= sum_{n,t} dZ[c,t,v]; Wt is
// the temporal weight [R][C][9] with C = its input channels, the Z channels)
hipError_t launch_fold_sdz(const float *Wt, const double *Tq, int R, int C, int V, double *part,
                           double *SdZ, hipStream_t s) {
  SmallGemm g{};
  g.A = Wt; g.am = 9; g.ak = (int64_t)C * 9; g.a_z = 1;
  g.B = Tq; g.b_dbl = 1; g.bk = V; g.bn = 1; g.b_z = (int64_t)R * V;
  g.out = part; g.o_dbl = 1; g.om = V; g.on = 1; g.o_z = (int64_t)C * V;
  g.M = C; g.N = V; g.K = R;
  HIP_RET(small_gemm(g, 9, s));
  const int64_t m = (int64_t)C * V;
  hipLaunchKernelGGL(k_sum_parts, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, part, 9, m,
                     nullptr, SdZ);
  return hipGetLastError();
}

}  // namespace stgcn

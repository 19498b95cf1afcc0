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

// The fold's small GEMMs as single launches on the fp64 matrix cores
// (v_mfma_f64_16x16x4_f64; operands float or double, converted exactly, fp64
// products and accumulation in a fixed order, so the results are deterministic):
//   out(m, n) = sum_{k < K} A(m, k) B(k, n) + sum_{k < K2} A2(m, k) B2(k, n)
// Every operand index is a two-level mixed-radix map per dimension,
//   idx(x) = (x / d) * s1 + (x % d) * s0,
// so the nine taps ride in M or K of ONE GEMM (no per-tap launches and no
// per-tap partial sums): e.g. Wc[o][i][q] = sum_c Wt[o][c][q] W'[c][i] is the
// (9 R) x C x R GEMM with m = 9 o + q.
// Block = 256 threads on a 64 x 64 output tile (wave = 32 x 32 = 2 x 2 MFMA
// tiles), K in chunks of 16 staged as fp64 in LDS.
struct Map {
  int d = 1;
  int64_t s1 = 0, s0 = 0;
  __host__ __device__ int64_t operator()(int x) const {
    return d == 1 ? (int64_t)x * s1 : (int64_t)(x / d) * s1 + (int64_t)(x % d) * s0;
  }
};
struct Gemm64 {
  const void *A, *B, *A2, *B2;
  void *out;
  int M, N, K, K2;
  int a_dbl, b_dbl, a2_dbl, b2_dbl, o_dbl;
  Map am, ak, bk, bn, a2m, a2k, b2k, b2n, om, on;
};

__device__ __forceinline__ double ld_fd(const void *p, int dbl, int64_t i) {
  return dbl ? reinterpret_cast<const double *>(p)[i] : (double)reinterpret_cast<const float *>(p)[i];
}

typedef double double4v __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_gemm_f64(Gemm64 g) {
  constexpr int KC = 16, TP = 64 + 1;  // chunk depth, LDS pitch (doubles)
  __shared__ double As[KC][TP], Bs[KC][TP];
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int m0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
  const int wm = (w & 1) * 32, wn = (w >> 1) * 32;
  double4v acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (double4v){0.0, 0.0, 0.0, 0.0};
  const int Ktot = g.K + (g.A2 ? g.K2 : 0);
  for (int k0 = 0; k0 < Ktot; k0 += KC) {
    __syncthreads();  // the previous chunk's reads are done
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int e = r * 256 + tid;
      const int kk = e & (KC - 1), mm = e >> 4;  // A: 16 consecutive k of a row
      const int k = k0 + kk, m = m0 + mm, n = n0 + mm;
      double a = 0.0, b = 0.0;
      if (k < g.K) {
        if (m < g.M) a = ld_fd(g.A, g.a_dbl, g.am(m) + g.ak(k));
        if (n < g.N) b = ld_fd(g.B, g.b_dbl, g.bk(k) + g.bn(n));
      } else if (k < Ktot) {
        const int k2 = k - g.K;
        if (m < g.M) a = ld_fd(g.A2, g.a2_dbl, g.a2m(m) + g.a2k(k2));
        if (n < g.N) b = ld_fd(g.B2, g.b2_dbl, g.b2k(k2) + g.b2n(n));
      }
      As[kk][mm] = a;
      Bs[kk][mm] = b;
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < KC; ks += 4) {
      // A operand: lane l holds A[row l & 15][k l >> 4]; B: B[k l >> 4][col l & 15]
      double a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = As[ks + (l >> 4)][wm + i * 16 + (l & 15)];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = Bs[ks + (l >> 4)][wn + j * 16 + (l & 15)];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  }
  // C/D: col = lane & 15, row = (lane >> 4) + 4 * reg
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm + i * 16 + (l >> 4) + 4 * r, n = n0 + wn + j * 16 + (l & 15);
        if (m >= g.M || n >= g.N) continue;
        const int64_t o = g.om(m) + g.on(n);
        if (g.o_dbl)
          reinterpret_cast<double *>(g.out)[o] = acc[i][j][r];
        else
          reinterpret_cast<float *>(g.out)[o] = (float)acc[i][j][r];
      }
}

static hipError_t gemm64(const Gemm64 &g, hipStream_t s) {
  hipLaunchKernelGGL(k_gemm_f64, dim3((g.N + 63) / 64, (g.M + 63) / 64), dim3(256), 0, s, g);
  return hipGetLastError();
}

static Map mp(int64_t s1) {
  Map m;
  m.s1 = s1;
  return m;
}
static Map mp(int d, int64_t s1, int64_t s0) {
  Map m;
  m.d = d;
  m.s1 = s1;
  m.s0 = s0;
  return m;
}

// Wc[o][i][q] = sum_c Wt[o][c][q] W'[c][i]   (W' = SpatialConv.W, C_out x C_in);
// one (9 R) x C x R GEMM, m = 9 o + q
hipError_t launch_fold_w(const float *Wt, const float *W, int R, int C, float *Wc, hipStream_t s) {
  Gemm64 g{};
  g.A = Wt; g.am = mp(9, (int64_t)R * 9, 1); g.ak = mp(9);
  g.B = W; g.bk = mp(C); g.bn = mp(1);
  g.out = Wc; g.om = mp(9, (int64_t)C * 9, 1); g.on = mp(9);
  g.M = 9 * R; g.N = C; g.K = R;
  return gemm64(g, s);
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
  // bq[q][o][v]: one (9 R) x V x R GEMM, m = q R + o
  Gemm64 g{};
  g.A = Wt; g.am = mp(R, 1, (int64_t)R * 9); g.ak = mp(9);
  g.B = bZ; g.bk = mp(V); g.bn = mp(1);
  g.out = bq; g.o_dbl = 1; g.om = mp(R, (int64_t)R * V, V); g.on = mp(1);
  g.M = 9 * R; g.N = V; g.K = R;
  HIP_RET(gemm64(g, s));
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
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) atomicMax(amax, __builtin_bit_cast(unsigned, m));
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
//                  ((9 R) x R GEMM over K = C_in, plus the K2 = V bias term)
//   dW'[c][i]    = sum_{(o,q)} Wt[o][c][q] dWc[o][i][q]   (R x C GEMM over K = 9 R)
// (part: unused, kept for the caller's workspace layout)
hipError_t launch_fold_grads(const float *slab, int S, const float *Wt, const float *W,
                             const float *bZ, const double *Tq, int R, int C, int V,
                             double *dWc, double *part, float *dWt, float *dW, hipStream_t s) {
  (void)part;
  const int64_t n = (int64_t)R * C * 9;
  hipLaunchKernelGGL(k_slab_reduce_f64, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, slab,
                     S, n, dWc);
  {
    Gemm64 g{};
    g.A = dWc; g.a_dbl = 1; g.am = mp(9, (int64_t)C * 9, 1); g.ak = mp(9);
    g.B = W; g.bk = mp(1); g.bn = mp(C);
    g.A2 = Tq; g.a2_dbl = 1; g.a2m = mp(9, V, (int64_t)R * V); g.a2k = mp(1);
    g.B2 = bZ; g.b2k = mp(1); g.b2n = mp(V);
    g.K2 = V;
    g.out = dWt; g.om = mp(9, (int64_t)R * 9, 1); g.on = mp(9);
    g.M = 9 * R; g.N = R; g.K = C;
    HIP_RET(gemm64(g, s));
  }
  {
    Gemm64 g{};
    g.A = Wt; g.am = mp(9); g.ak = mp(9, (int64_t)R * 9, 1);
    g.B = dWc; g.b_dbl = 1; g.bk = mp(9, (int64_t)C * 9, 1); g.bn = mp(9);
    g.out = dW; g.om = mp(C); g.on = mp(1);
    g.M = R; g.N = C; g.K = 9 * R;
    HIP_RET(gemm64(g, s));
  }
  return hipGetLastError();
}

// SdZ[c][v] = sum_q sum_o Wt[o][c][q] Tq[q][o][v]  (= sum_{n,t} dZ[c,t,v]; Wt is
// the temporal weight [R][C][9] with C = its input channels, the Z channels):
// one C x V GEMM over K = 9 R (k = 9 o + q). (part: unused)
hipError_t launch_fold_sdz(const float *Wt, const double *Tq, int R, int C, int V, double *part,
                           double *SdZ, hipStream_t s) {
  (void)part;
  Gemm64 g{};
  g.A = Wt; g.am = mp(9); g.ak = mp(9, (int64_t)C * 9, 1);
  g.B = Tq; g.b_dbl = 1; g.bk = mp(9, V, (int64_t)R * V); g.bn = mp(1);
  g.out = SdZ; g.o_dbl = 1; g.om = mp(V); g.on = mp(1);
  g.M = C; g.N = V; g.K = 9 * R;
  return gemm64(g, s);
}

}  // namespace stgcn

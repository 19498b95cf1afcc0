// Training-step ops around the block stack: the
// classification head (global average pool over (T, V) + Linear + cross
// entropy, lightning_model.py:105-107, :202) and a multi-tensor Adam step
// (lightning_model.py:196-197, torch.optim.Adam semantics), gfx950 only.
// Both are launch-bound, not FLOP-bound: the head is 5 small kernels instead
// of torch's ~12, Adam is ONE launch over every parameter tensor.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>

#include "../../include/stgcn_hip.h"
#include "device_common.h"

namespace stgcn {
void set_last_error(const std::string &msg);  // capi.hip (stgcn_last_error)
}

namespace {

using stgcn::wave_sumf;

int fail(int code, const std::string &m) {
  stgcn::set_last_error(m);
  return code;
}

#define HIP_TRY2(expr)                                                                     \
  do {                                                                                     \
    hipError_t e_ = (expr);                                                                \
    if (e_ != hipSuccess)                                                                  \
      return fail(STGCN_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));        \
  } while (0)

// ---------------------------------------------------------------------------
// Adam. Per element, in fp32, in torch's order (optim/adam.py _multi_tensor_adam /
// _single_tensor_adam, weight_decay folded into the gradient as in torch):
//   g  = grad + wd * p
//   m  = lerp(m, g, 1 - beta1)          (m + w (g - m) for w < 0.5)
//   v  = v * beta2;  v = v + ((1 - beta2) * g) * g
//   p  = p + (-lr / bc1) * (m / (sqrt(v) / sqrt(bc2) + eps))
// with bc1 = 1 - beta1^step, bc2 = 1 - beta2^step computed in double on the
// host and rounded to float like torch's scalar arguments.
// ---------------------------------------------------------------------------
constexpr int kAdamChunk = 2048;  // elements per block (256 threads x 8)

struct AdamScalars {
  float lerp_w, beta2, one_minus_beta2, neg_step_size, bc2_sqrt, eps, wd;
};

// the element loop of both launch forms (one function: the same instructions)
__device__ __forceinline__ void adam_block(const stgcn_adam_tensor_t *tab,
                                           const int64_t *chunk_start, int ntensors,
                                           const AdamScalars &s) {
#pragma clang fp contract(off)
  // tensor of this block: the last t with chunk_start[t] <= blockIdx.x
  const int64_t b = blockIdx.x;
  int lo = 0, hi = ntensors - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (chunk_start[mid] <= b) lo = mid; else hi = mid - 1;
  }
  const stgcn_adam_tensor_t t = tab[lo];
  const int64_t base = (b - chunk_start[lo]) * kAdamChunk;
  for (int i = threadIdx.x; i < kAdamChunk; i += 256) {
    const int64_t e = base + i;
    if (e >= t.numel) break;
    // (every operation rounded on its own -- no fma contraction, whose choices
    // differed between the two kernels -- as torch's unfused CPU loop rounds)
    float p = t.param[e];
    float g = t.grad[e];
    if (s.wd != 0.f) g = g + s.wd * p;
    float m = t.exp_avg[e];
    m = m + s.lerp_w * (g - m);
    float v = t.exp_avg_sq[e] * s.beta2;
    v = v + (s.one_minus_beta2 * g) * g;
    const float denom = sqrtf(v) / s.bc2_sqrt + s.eps;
    p = p + s.neg_step_size * (m / denom);
    t.exp_avg[e] = m;
    t.exp_avg_sq[e] = v;
    t.param[e] = p;
  }
}

__global__ __launch_bounds__(256) void k_adam(const stgcn_adam_tensor_t *tab,
                                              const int64_t *chunk_start, int ntensors,
                                              AdamScalars s) {
  adam_block(tab, chunk_start, ntensors, s);
}

// The device-step form (stgcn_adam_step_dev, ABI 11): k_adam_tick advances the
// step count, then every block forms the scalars from it exactly as
// stgcn_adam_step does on the host (double, rounded to float) -- thread 0 into
// LDS -- and runs k_adam's element loop.
__global__ void k_adam_tick(float *step) { *step = *step + 1.f; }

__global__ __launch_bounds__(256) void k_adam_dev(const stgcn_adam_tensor_t *tab,
                                                  const int64_t *chunk_start, int ntensors,
                                                  const float *step, double lr, double beta1,
                                                  double beta2, double eps, double wd) {
  __shared__ AdamScalars sh;
  if (threadIdx.x == 0) {
    const double t = (double)*step;
    const double bc1 = 1.0 - pow(beta1, t), bc2 = 1.0 - pow(beta2, t);
    AdamScalars sc;
    sc.lerp_w = (float)(1.0 - beta1);
    sc.beta2 = (float)beta2;
    sc.one_minus_beta2 = (float)(1.0 - beta2);
    sc.neg_step_size = (float)(-(lr / bc1));
    sc.bc2_sqrt = (float)sqrt(bc2);
    sc.eps = (float)eps;
    sc.wd = (float)wd;
    sh = sc;
  }
  __syncthreads();
  const AdamScalars s = sh;
  adam_block(tab, chunk_start, ntensors, s);
}

// ---------------------------------------------------------------------------
// Head. y: (N, C, L) block output (L = T*V), W: (classes, C), b: (classes),
// labels: int64 (N). pooled (N, C), logits (N, classes), lossv (N) per-clip
// losses, loss (1) = mean.
// ---------------------------------------------------------------------------
// pooled[n][c] = mean_l y[n][c][l]: one wave per (n, c) row, 4 rows per block
__global__ __launch_bounds__(256) void k_head_pool(const float *y, float *pooled, int64_t rows,
                                                   int L) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float *src = y + row * L;
  float s = 0.f;
  for (int l = lane; l < L; l += 64) s += src[l];
  s = wave_sumf(s);
  if (lane == 0) pooled[row] = s / (float)L;
}

// ABI 9: the same mean over y = ReLU(BN2(U)) formed on load from the last
// block's pre-BN2 tensor U (its y is never written): the element arithmetic of
// k_bn_relu_fwd (kernels.hip bn_relu_fwd_body), the summation order of
// k_head_pool, so pooled is bit-identical to pooling the written y
__global__ __launch_bounds__(256) void k_head_pool_u(const float *U, const float *mean,
                                                     const float *invstd, const float *g,
                                                     const float *b, float *pooled, int64_t rows,
                                                     int C, int L) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const int c = (int)(row % C);
  const float mu = mean[c], a = invstd[c] * g[c], be = b[c];
  const float *src = U + row * L;
  float s = 0.f;
  for (int l = lane; l < L; l += 64) {
    const float t = (src[l] - mu) * a + be;
    s += t > 0.f ? t : 0.f;
  }
  s = wave_sumf(s);
  if (lane == 0) pooled[row] = s / (float)L;
}

// one block per clip: logits = pooled W^T + b, per-clip CE loss (log-sum-exp)
__global__ __launch_bounds__(256) void k_head_fc_ce(const float *pooled, const float *W,
                                                    const float *bias, const int64_t *labels,
                                                    float *logits, float *lossv, int C,
                                                    int classes) {
  extern __shared__ float sh[];  // [C] pooled row, [classes] logits, [8] reduction
  float *pr = sh, *lg = sh + C, *red = lg + classes;
  const int n = blockIdx.x, tid = threadIdx.x;
  for (int c = tid; c < C; c += 256) pr[c] = pooled[(int64_t)n * C + c];
  __syncthreads();
  for (int j = tid; j < classes; j += 256) {
    const float *w = W + (int64_t)j * C;
    float a = 0.f;
    for (int c = 0; c < C; ++c) a = fmaf(pr[c], w[c], a);
    a += bias[j];
    lg[j] = a;
    logits[(int64_t)n * classes + j] = a;
  }
  __syncthreads();
  float mx = -INFINITY;
  for (int j = tid; j < classes; j += 256) mx = fmaxf(mx, lg[j]);
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  if ((tid & 63) == 0) red[tid >> 6] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float se = 0.f;
  for (int j = tid; j < classes; j += 256) se += expf(lg[j] - mx);
  se = wave_sumf(se);
  if ((tid & 63) == 0) red[4 + (tid >> 6)] = se;
  __syncthreads();
  if (tid == 0) {
    const float tot = (red[4] + red[5]) + (red[6] + red[7]);
    const int64_t y = labels[n];
    lossv[n] = (y >= 0 && y < classes) ? (logf(tot) + mx) - lg[y] : NAN;  // bad label: NaN
  }
}

// loss = mean_n lossv[n] (fixed order: deterministic)
__global__ void k_head_loss_mean(const float *lossv, float *loss, int N) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    double s = 0.0;
    for (int n = 0; n < N; ++n) s += lossv[n];
    loss[0] = (float)(s / N);
  }
}

// dlogits[n][j] = (softmax_j - [j == y_n]) * dloss / N; dpooled[n][c] = sum_j dlogits W[j][c]
__global__ __launch_bounds__(256) void k_head_bwd_rows(const float *logits, const float *W,
                                                       const int64_t *labels, const float *dloss,
                                                       float *dlogits, float *dpooled, int N,
                                                       int C, int classes) {
  extern __shared__ float sh[];  // [classes] dlogits, [8]
  float *dl = sh, *red = sh + classes;
  const int n = blockIdx.x, tid = threadIdx.x;
  const float *lg = logits + (int64_t)n * classes;
  float mx = -INFINITY;
  for (int j = tid; j < classes; j += 256) mx = fmaxf(mx, lg[j]);
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  if ((tid & 63) == 0) red[tid >> 6] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  float se = 0.f;
  for (int j = tid; j < classes; j += 256) se += expf(lg[j] - mx);
  se = wave_sumf(se);
  if ((tid & 63) == 0) red[4 + (tid >> 6)] = se;
  __syncthreads();
  const float tot = (red[4] + red[5]) + (red[6] + red[7]);
  const float scale = dloss[0] / (float)N;
  const int64_t y = labels[n];
  for (int j = tid; j < classes; j += 256) {
    const float d = (expf(lg[j] - mx) / tot - (j == y ? 1.f : 0.f)) * scale;
    dl[j] = d;
    dlogits[(int64_t)n * classes + j] = d;
  }
  __syncthreads();
  for (int c = tid; c < C; c += 256) {
    float a = 0.f;
    for (int j = 0; j < classes; ++j) a = fmaf(dl[j], W[(int64_t)j * C + c], a);
    dpooled[(int64_t)n * C + c] = a;
  }
}

// dW[j][c] = sum_n dlogits[n][j] pooled[n][c]; db[j] = sum_n dlogits[n][j]
__global__ __launch_bounds__(256) void k_head_wgrad(const float *dlogits, const float *pooled,
                                                    float *dW, float *db, int N, int C,
                                                    int classes) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (int64_t)classes * (C + 1)) return;
  const int j = (int)(idx / (C + 1)), c = (int)(idx % (C + 1));
  float a = 0.f;
  if (c < C) {
    for (int n = 0; n < N; ++n) a = fmaf(dlogits[(int64_t)n * classes + j], pooled[(int64_t)n * C + c], a);
    dW[(int64_t)j * C + c] = a;
  } else {
    for (int n = 0; n < N; ++n) a += dlogits[(int64_t)n * classes + j];
    db[j] = a;
  }
}

// dy[n][c][l] = dpooled[n][c] / L (the avg-pool backward), float4 stores when L % 4 == 0
__global__ __launch_bounds__(256) void k_head_bcast(const float *dpooled, float *dy, int64_t rows,
                                                    int L) {
  const int64_t row = blockIdx.x;
  if (row >= rows) return;
  const float v = dpooled[row] / (float)L;
  float *dst = dy + row * L;
  for (int l = threadIdx.x; l < L; l += 256) dst[l] = v;
}

// the per-row value k_head_bcast writes at every position (same arithmetic)
__global__ __launch_bounds__(256) void k_head_dync(const float *dpooled, float *dy_nc, int64_t rows,
                                                   int L) {
  const int64_t row = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (row < rows) dy_nc[row] = dpooled[row] / (float)L;
}

}  // namespace

extern "C" {

size_t stgcn_adam_table_bytes(int ntensors) {
  if (ntensors <= 0) return 0;
  return (size_t)ntensors * sizeof(stgcn_adam_tensor_t) + (size_t)(ntensors + 1) * sizeof(int64_t);
}

int stgcn_adam_build_table(const stgcn_adam_tensor_t *tensors, int ntensors, void *host_table,
                           size_t table_bytes, int64_t *total_chunks) {
  if (!tensors || ntensors <= 0 || !host_table || !total_chunks)
    return fail(STGCN_E_INVALID, "adam: null argument or no tensors");
  if (table_bytes < stgcn_adam_table_bytes(ntensors))
    return fail(STGCN_E_INVALID, "adam: table buffer too small");
  auto *tab = reinterpret_cast<stgcn_adam_tensor_t *>(host_table);
  auto *cs = reinterpret_cast<int64_t *>(reinterpret_cast<char *>(host_table) +
                                         (size_t)ntensors * sizeof(stgcn_adam_tensor_t));
  int64_t chunks = 0;
  for (int i = 0; i < ntensors; ++i) {
    const stgcn_adam_tensor_t &t = tensors[i];
    if (!t.param || !t.grad || !t.exp_avg || !t.exp_avg_sq || t.numel <= 0)
      return fail(STGCN_E_INVALID,
                  "adam: tensor " + std::to_string(i) + " has a null pointer or numel <= 0");
    tab[i] = t;
    cs[i] = chunks;
    chunks += (t.numel + kAdamChunk - 1) / kAdamChunk;
  }
  cs[ntensors] = chunks;
  if (chunks > INT32_MAX) return fail(STGCN_E_UNSUPPORTED, "adam: too many elements");
  *total_chunks = chunks;
  return STGCN_OK;
}

int stgcn_adam_step(const void *dev_table, int ntensors, int64_t total_chunks, double lr,
                    double beta1, double beta2, double eps, double weight_decay, int64_t step,
                    void *stream) {
  if (!dev_table || ntensors <= 0 || total_chunks <= 0 || step <= 0)
    return fail(STGCN_E_INVALID, "adam: bad table / chunk count / step");
  // scalars as torch forms them: Python doubles, rounded to float at the kernel
  const double bc1 = 1.0 - std::pow(beta1, (double)step);
  const double bc2 = 1.0 - std::pow(beta2, (double)step);
  AdamScalars sc;
  sc.lerp_w = (float)(1.0 - beta1);
  sc.beta2 = (float)beta2;
  sc.one_minus_beta2 = (float)(1.0 - beta2);
  sc.neg_step_size = (float)(-(lr / bc1));
  sc.bc2_sqrt = (float)std::sqrt(bc2);
  sc.eps = (float)eps;
  sc.wd = (float)weight_decay;
  const auto *tab = reinterpret_cast<const stgcn_adam_tensor_t *>(dev_table);
  const auto *cs = reinterpret_cast<const int64_t *>(reinterpret_cast<const char *>(dev_table) +
                                                     (size_t)ntensors * sizeof(stgcn_adam_tensor_t));
  hipLaunchKernelGGL(k_adam, dim3((unsigned)total_chunks), dim3(256), 0, (hipStream_t)stream, tab,
                     cs, ntensors, sc);
  HIP_TRY2(hipGetLastError());
  return STGCN_OK;
}

int stgcn_adam_step_dev(const void *dev_table, int ntensors, int64_t total_chunks, double lr,
                        double beta1, double beta2, double eps, double weight_decay, float *step,
                        void *stream) {
  if (!dev_table || ntensors <= 0 || total_chunks <= 0 || !step)
    return fail(STGCN_E_INVALID, "adam: bad table / chunk count / step pointer");
  const auto *tab = reinterpret_cast<const stgcn_adam_tensor_t *>(dev_table);
  const auto *cs = reinterpret_cast<const int64_t *>(reinterpret_cast<const char *>(dev_table) +
                                                     (size_t)ntensors * sizeof(stgcn_adam_tensor_t));
  hipLaunchKernelGGL(k_adam_tick, dim3(1), dim3(1), 0, (hipStream_t)stream, step);
  hipLaunchKernelGGL(k_adam_dev, dim3((unsigned)total_chunks), dim3(256), 0, (hipStream_t)stream,
                     tab, cs, ntensors, step, lr, beta1, beta2, eps, weight_decay);
  HIP_TRY2(hipGetLastError());
  return STGCN_OK;
}

int stgcn_head_fwd(const stgcn_head_desc_t *d, const float *y, const float *W, const float *bias,
                   const int64_t *labels, float *pooled, float *logits, float *lossv, float *loss,
                   void *stream) {
  if (!d || d->N <= 0 || d->C <= 0 || d->L <= 0 || d->classes <= 0)
    return fail(STGCN_E_INVALID, "head: bad descriptor");
  if (!y || !W || !bias || !labels || !pooled || !logits || !lossv || !loss)
    return fail(STGCN_E_INVALID, "head: null tensor argument");
  if ((size_t)(d->C + d->classes + 8) * sizeof(float) > 64 * 1024)
    return fail(STGCN_E_UNSUPPORTED, "head: C + classes too large");
  hipStream_t s = (hipStream_t)stream;
  const int64_t rows = (int64_t)d->N * d->C;
  hipLaunchKernelGGL(k_head_pool, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, y, pooled,
                     rows, d->L);
  hipLaunchKernelGGL(k_head_fc_ce, dim3(d->N), dim3(256),
                     (size_t)(d->C + d->classes + 8) * sizeof(float), s, pooled, W, bias, labels,
                     logits, lossv, d->C, d->classes);
  hipLaunchKernelGGL(k_head_loss_mean, dim3(1), dim3(64), 0, s, lossv, loss, d->N);
  HIP_TRY2(hipGetLastError());
  return STGCN_OK;
}

int stgcn_head_fwd_u(const stgcn_head_desc_t *d, const float *U, const float *stats2,
                     const float *g2, const float *b2, const float *W, const float *bias,
                     const int64_t *labels, float *pooled, float *logits, float *lossv,
                     float *loss, void *stream) {
  if (!d || d->N <= 0 || d->C <= 0 || d->L <= 0 || d->classes <= 0)
    return fail(STGCN_E_INVALID, "head: bad descriptor");
  if (!U || !stats2 || !g2 || !b2 || !W || !bias || !labels || !pooled || !logits || !lossv ||
      !loss)
    return fail(STGCN_E_INVALID, "head: null tensor argument");
  if ((size_t)(d->C + d->classes + 8) * sizeof(float) > 64 * 1024)
    return fail(STGCN_E_UNSUPPORTED, "head: C + classes too large");
  hipStream_t s = (hipStream_t)stream;
  const int64_t rows = (int64_t)d->N * d->C;
  hipLaunchKernelGGL(k_head_pool_u, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, U, stats2,
                     stats2 + d->C, g2, b2, pooled, rows, d->C, d->L);
  hipLaunchKernelGGL(k_head_fc_ce, dim3(d->N), dim3(256),
                     (size_t)(d->C + d->classes + 8) * sizeof(float), s, pooled, W, bias, labels,
                     logits, lossv, d->C, d->classes);
  hipLaunchKernelGGL(k_head_loss_mean, dim3(1), dim3(64), 0, s, lossv, loss, d->N);
  HIP_TRY2(hipGetLastError());
  return STGCN_OK;
}

int stgcn_head_bwd(const stgcn_head_desc_t *d, const float *pooled, const float *logits,
                   const float *W, const int64_t *labels, const float *dloss, float *dlogits,
                   float *dpooled, float *dy, float *dW, float *dbias, void *stream) {
  if (!d || d->N <= 0 || d->C <= 0 || d->L <= 0 || d->classes <= 0)
    return fail(STGCN_E_INVALID, "head: bad descriptor");
  if (!pooled || !logits || !W || !labels || !dloss || !dlogits || !dpooled || !dy || !dW ||
      !dbias)
    return fail(STGCN_E_INVALID, "head: null tensor argument");
  hipStream_t s = (hipStream_t)stream;
  const int64_t rows = (int64_t)d->N * d->C;
  hipLaunchKernelGGL(k_head_bwd_rows, dim3(d->N), dim3(256),
                     (size_t)(d->classes + 8) * sizeof(float), s, logits, W, labels, dloss,
                     dlogits, dpooled, d->N, d->C, d->classes);
  const int64_t nw = (int64_t)d->classes * (d->C + 1);
  hipLaunchKernelGGL(k_head_wgrad, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, s, dlogits,
                     pooled, dW, dbias, d->N, d->C, d->classes);
  hipLaunchKernelGGL(k_head_bcast, dim3((unsigned)rows), dim3(256), 0, s, dpooled, dy, rows,
                     d->L);
  HIP_TRY2(hipGetLastError());
  return STGCN_OK;
}

int stgcn_head_bwd_nc(const stgcn_head_desc_t *d, const float *pooled, const float *logits,
                      const float *W, const int64_t *labels, const float *dloss, float *dlogits,
                      float *dpooled, float *dy_nc, float *dW, float *dbias, void *stream) {
  if (!d || d->N <= 0 || d->C <= 0 || d->L <= 0 || d->classes <= 0)
    return fail(STGCN_E_INVALID, "head: bad descriptor");
  if (!pooled || !logits || !W || !labels || !dloss || !dlogits || !dpooled || !dy_nc || !dW ||
      !dbias)
    return fail(STGCN_E_INVALID, "head: null tensor argument");
  hipStream_t s = (hipStream_t)stream;
  const int64_t rows = (int64_t)d->N * d->C;
  hipLaunchKernelGGL(k_head_bwd_rows, dim3(d->N), dim3(256),
                     (size_t)(d->classes + 8) * sizeof(float), s, logits, W, labels, dloss,
                     dlogits, dpooled, d->N, d->C, d->classes);
  const int64_t nw = (int64_t)d->classes * (d->C + 1);
  hipLaunchKernelGGL(k_head_wgrad, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, s, dlogits,
                     pooled, dW, dbias, d->N, d->C, d->classes);
  hipLaunchKernelGGL(k_head_dync, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, s, dpooled,
                     dy_nc, rows, d->L);
  HIP_TRY2(hipGetLastError());
  return STGCN_OK;
}

}  // extern "C"

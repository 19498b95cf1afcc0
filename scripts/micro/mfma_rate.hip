// fp64 / fp32 MFMA issue rate on gfx950: 8 waves per SIMD (2048 blocks of 256
// threads... ), each wave 4 independent accumulators x ITER MFMAs.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int ITER = 1024;
__global__ __launch_bounds__(256) void k64(double *out, double a) {
  d4 c[4] = {};
  double x = a + threadIdx.x, y = a * 0.5;
  for (int i = 0; i < ITER; ++i)
#pragma unroll
    for (int u = 0; u < 4; ++u) c[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, c[u], 0, 0, 0);
  out[blockIdx.x * 256 + threadIdx.x] = c[0][0] + c[1][1] + c[2][2] + c[3][3];
}
__global__ __launch_bounds__(256) void k32(float *out, float a) {
  f4 c[4] = {};
  float x = a + threadIdx.x, y = a * 0.5f;
  for (int i = 0; i < ITER; ++i)
#pragma unroll
    for (int u = 0; u < 4; ++u) c[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(x, y, c[u], 0, 0, 0);
  out[blockIdx.x * 256 + threadIdx.x] = c[0][0] + c[1][1] + c[2][2] + c[3][3];
}
__global__ __launch_bounds__(64) void k64dep(double *out, double a) {
  d4 c = {};
  double x = a + threadIdx.x, y = a * 0.5;
  for (int i = 0; i < ITER; ++i) c = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, c, 0, 0, 0);
  out[blockIdx.x * 64 + threadIdx.x] = c[0];
}
int main() {
  const int blocks = 256 * 8;
  double *o;
  hipMalloc(&o, sizeof(double) * blocks * 256);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int rep = 0; rep < 2; ++rep) {
    float ms;
    hipEventRecord(e0);
    k64<<<blocks, 256>>>(o, 1.0);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    double fl = (double)blocks * 4 * ITER * 4 * 16 * 16 * 4 * 2;
    printf("f64 16x16x4: %.2f ms  %.1f TF/s\n", ms, fl / ms / 1e9);
    hipEventRecord(e0);
    k32<<<blocks, 256>>>((float *)o, 1.0f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    printf("f32 16x16x4: %.2f ms  %.1f TF/s\n", ms, fl / ms / 1e9);
  }
  {
    float ms;
    hipEventRecord(e0);
    k64dep<<<256, 64>>>(o, 1.0);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    printf("f64 dependent chain: %.3f ms for %d MFMAs = %.1f ns each\n", ms, ITER, ms * 1e6 / ITER);
  }
  return 0;
}

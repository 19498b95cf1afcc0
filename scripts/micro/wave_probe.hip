// Probe: 64 blocks x 576 threads, each wave 128 x v_mfma_f32_32x32x2f32 on
// (a) register operands, (b) operands streamed from a 9 x 256 x 256 float
// array (k-contiguous rows, as k_fold_gemm reads them).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f16v __attribute__((ext_vector_type(16)));
typedef float f8v __attribute__((ext_vector_type(8)));
__global__ __launch_bounds__(576) void kreg(float *out, float s) {
  f16v acc = {};
  float x = s + threadIdx.x, y = s * 0.5f;
  for (int i = 0; i < 128; ++i) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(x, y, acc, 0, 0, 0);
  float t = 0;
  for (int r = 0; r < 16; ++r) t += acc[r];
  out[blockIdx.x * 576 + threadIdx.x] = t;
}
__global__ __launch_bounds__(576) void kmem(const float *A, const float *B, float *out, int K) {
  const int q = threadIdx.x >> 6, l = threadIdx.x & 63, r32 = l & 31, h = l >> 5;
  const int m0 = (blockIdx.x / 8) * 32, n0 = (blockIdx.x % 8) * 32;
  const float *pa = A + (size_t)q * 256 * 256 + (m0 + r32) * 256 + 8 * h;
  const float *pb = B + (n0 + r32) * 256 + 8 * h;
  f16v acc = {};
  for (int i = 0; i < K / 16; ++i) {
    f8v a = *reinterpret_cast<const f8v *>(pa + 16 * i);
    f8v b = *reinterpret_cast<const f8v *>(pb + 16 * i);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[j], b[j], acc, 0, 0, 0);
  }
  float t = 0;
  for (int r = 0; r < 16; ++r) t += acc[r];
  out[blockIdx.x * 576 + threadIdx.x] = t;
}
int main() {
  float *A, *B, *o;
  hipMalloc(&A, sizeof(float) * 9 * 256 * 256);
  hipMalloc(&B, sizeof(float) * 256 * 256);
  hipMalloc(&o, sizeof(float) * 64 * 576);
  hipMemset(A, 0, sizeof(float) * 9 * 256 * 256);
  hipMemset(B, 0, sizeof(float) * 256 * 256);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int rep = 0; rep < 3; ++rep) {
    float ms;
    hipEventRecord(e0);
    for (int i = 0; i < 10; ++i) kreg<<<64, 576>>>(o, 1.f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    printf("reg operands : %.2f us per launch\n", ms * 100);
    hipEventRecord(e0);
    for (int i = 0; i < 10; ++i) kmem<<<64, 576>>>(A, B, o, 256);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    printf("mem operands : %.2f us per launch\n", ms * 100);
  }
  return 0;
}

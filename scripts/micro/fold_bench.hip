// Micro-benchmark of the folded block's small GEMMs (kernels_fold.hip) at the
// cfg2 layer shapes: hipEvent time per launch of launch_fold_w / _bias /
// _grads / _sdz. Build: hipcc --offload-arch=gfx950 -O3 -std=c++17
//   scripts/micro/fold_bench.hip -o scripts/micro/fold_bench 
#include "../../st-gcn_amd/csrc/kernels_fold.hip"
#include <cstdio>
#include <vector>
#include <algorithm>

using namespace stgcn;

int main() {
  const int shapes[][2] = {{64, 64}, {128, 64}, {128, 128}, {256, 128}, {256, 256}};  // (R, C)
  const int V = 18;
  for (auto &sh : shapes) {
    const int R = sh[0], C = sh[1];
    const int S = std::max(1, 256 / (((R + 63) / 64) * ((C + 31) / 32)));  // (wgrad split-K slabs)
    float *Wt, *W, *Wc, *bZ, *dWt, *dW, *slab, *BT, *bt;
    float *fscr, *bscr;
    double *dscr, *SdH;
    double *bq, *Tq, *SdZ;
    float *dWc;
    hipMalloc(&Wt, sizeof(float) * R * R * 9);
    hipMalloc(&W, sizeof(float) * R * C);
    hipMalloc(&Wc, sizeof(float) * R * C * 9);
    hipMalloc(&bZ, sizeof(float) * R * V);
    hipMalloc(&bt, sizeof(float) * R);
    hipMalloc(&BT, sizeof(float) * R * 300 * V);
    hipMalloc(&dWt, sizeof(float) * R * R * 9);
    hipMalloc(&dW, sizeof(float) * R * C);
    hipMalloc(&slab, sizeof(float) * S * R * C * 9);
    hipMalloc(&bq, sizeof(double) * 9 * R * V);
    hipMalloc(&Tq, sizeof(double) * 9 * R * V);
    hipMalloc(&dWc, sizeof(float) * fold_dwc_floats(R, C));
    hipMalloc(&fscr, sizeof(float) * fold_fwd_scratch_floats(R, C, V));
    hipMalloc(&bscr, sizeof(float) * fold_bwd_scratch_floats(R, C));
    hipMalloc(&dscr, sizeof(double) * fold_sdz_scratch_doubles(R, C, V));
    hipMalloc(&SdH, sizeof(double) * C * V);
    hipMalloc(&SdZ, sizeof(double) * R * V);
    hipMemset(Wt, 0, sizeof(float) * R * R * 9);
    hipMemset(W, 0, sizeof(float) * R * C);
    hipMemset(slab, 0, sizeof(float) * S * R * C * 9);
    hipMemset(Tq, 0, sizeof(double) * 9 * R * V);
    hipMemset(bZ, 0, sizeof(float) * R * V);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto time = [&](const char *name, auto fn) {
      fn();
      hipDeviceSynchronize();
      hipEventRecord(e0, 0);
      for (int i = 0; i < 20; ++i) fn();
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      printf("R=%3d C=%3d %-10s %8.1f us\n", R, C, name, ms * 1000 / 20);
    };
    time("fold_fwd", [&] { launch_fold_fwd(Wt, W, bt, bZ, R, C, V, 300, 300, 1, Wc, bq, BT, fscr, 0); });
    time("fold_w", [&] { launch_fold_w(Wt, W, R, C, Wc, fscr, 0); });
    time("prep_bwd", [&] { launch_fold_prep_bwd(Wt, W, R, C, bscr, 0); });
    time("fold_grads", [&] { launch_fold_grads(slab, S, bscr, bZ, Tq, R, C, V, dWc, dWt, dW, 0); });
    time("fold_sdz", [&] { launch_fold_sdz(dscr, Wt, Wc, Tq, R, C, V, SdZ, SdH, 0); });
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) printf("error %s\n", hipGetErrorString(e));
  }
  return 0;
}

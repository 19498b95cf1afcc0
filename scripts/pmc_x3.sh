#!/bin/bash
# MFMA busy fraction and effective clock of the temporal-conv GEMM kernels
# (fp32 MFMA vs the bf16x3 split) at the cfg2 L8 shape: one PMC pass per mode.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for mode in 0 1; do
  KB_SHAPES=${KB_SHAPES:-5} KB_WHICH=0 KB_X3=$mode timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace \
    --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES \
    -d gpurun_out/pmc_x3_$mode -o run --output-format csv -- python3 scripts/kbench.py 5 \
    > gpurun_out/pmc_x3_$mode.log 2>&1
  rc=$?; echo "mode $mode rc=$rc"; [ $rc -eq 0 ] || exit $rc
done

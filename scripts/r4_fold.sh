#!/bin/bash
# Round-4 fold GEMM + f16x2 data-gradient check: fold micro-bench trace, the full
# GPU suite, the f16x2 suites on the f16dg variant (f16x2 data gradient), and a
# step profile per mode.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-fold}
mkdir -p $OUT
(cd scripts/micro && timeout -k 10 120 rocprofv3 --kernel-trace -d ../../$OUT/fb -o out -- ./fold_bench > /dev/null) || exit 1
timeout -k 10 500 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/ > $OUT/tests.log 2>&1
echo "default: $(tail -1 $OUT/tests.log)"
STGCN_LIB_VARIANT=f16dg timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread \
  -m gpu tests/test_gpu_f16x2.py tests/test_gpu_stack.py tests/test_gpu_f32x3.py > $OUT/tests_f16dg.log 2>&1
echo "f16dg: $(tail -1 $OUT/tests_f16dg.log)"
TAG=${TAG:-fold}/step MODES=f16x2 bash scripts/r4_step.sh || exit 1
STGCN_LIB_VARIANT=f16dg TAG=${TAG:-fold}/step_dg MODES=f16x2 bash scripts/r4_step.sh || exit 1
echo done

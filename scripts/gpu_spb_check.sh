#!/bin/bash
# Fused spatial backward check: bf16 parity tests, then an A/B of cfg3 / cfg5
# against the unfused H GEMM + k_spatial_bwd5/6 pair (STGCN_UNFUSED_SPB).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_f32x3.py tests/test_gpu_stack.py tests/test_gpu_callers.py \
  -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/spb_pytest.log 2>&1
rc=$?; tail -n 15 gpurun_out/spb_pytest.log; [ $rc -eq 0 ] || exit $rc
for c in ${CFGS:-cfg2 cfg3}; do
  for v in fused unfused; do
    if [ $v = unfused ]; then export STGCN_UNFUSED_SPB=1; else unset STGCN_UNFUSED_SPB; fi
    timeout -k 10 200 python bench.py --config $c --steps 6 --warmup 2 --no-cpu-baseline \
      --no-roofline --no-alt --no-repeats > gpurun_out/spb_${c}_$v.json 2> gpurun_out/spb_${c}_$v.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/spb_${c}_$v.json')); print('$c $v', d['value'], d['ms_per_step'])"
  done
done

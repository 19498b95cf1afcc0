#!/bin/bash
# bf16 activation storage check: bf16 / stack / caller parity tests, then an A/B
# of cfg3 / cfg5 against fp32 storage (STGCN_ACT_FP32).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_stack.py tests/test_gpu_callers.py \
  -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/zb_pytest.log 2>&1
rc=$?; tail -n 5 gpurun_out/zb_pytest.log; [ $rc -eq 0 ] || exit $rc
for c in ${CFGS:-cfg3 cfg5}; do
  for v in bf16 fp32; do
    if [ $v = fp32 ]; then export STGCN_ACT_FP32=1; else unset STGCN_ACT_FP32; fi
    timeout -k 10 200 python bench.py --config $c --steps 6 --warmup 2 --no-cpu-baseline \
      --no-roofline --no-alt --no-repeats > gpurun_out/zb_${c}_$v.json 2> gpurun_out/zb_${c}_$v.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/zb_${c}_$v.json')); print('$c $v', d['value'], d['ms_per_step'], d['loss'])"
  done
done

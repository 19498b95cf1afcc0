#!/bin/bash
# x3 kernel change check: x3 + stack parity tests, per-layer kbench, cfg2 A/B
# of an env switch (AB_ENV, e.g. STGCN_X3_MR1=1) on the bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/x3c_${TAG:-x}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_f32x3.py tests/test_gpu_stack.py tests/test_gpu_block.py -x -q \
  --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -n 3 $OUT/pytest.log; [ $rc -eq 0 ] || { echo "STOP pytest rc=$rc"; exit $rc; }
KB_X3=1 timeout -k 10 200 python scripts/kbench.py 30 2>&1 | grep -v amdgpu > $OUT/kb.txt || exit 1
cat $OUT/kb.txt
for e in - ${AB_ENV:-}; do
  for rep in 1 2; do
    if [ "$e" = "-" ]; then
      r=$(timeout -k 10 300 python bench.py --no-cpu-baseline --no-alt --no-repeats 2>/dev/null) || exit 1
    else
      r=$(env $e timeout -k 10 300 python bench.py --no-cpu-baseline --no-alt --no-repeats 2>/dev/null) || exit 1
    fi
    echo "$e $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["kernel"], r["frac"], r["avg_launch_ms"], r["per_kind_tflops"])')"
  done
done

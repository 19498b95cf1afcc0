#!/bin/bash
# GPU parity tests, then one bench line per BASELINE config (cfg2 fp32, cfg3 / cfg5 bf16).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-x}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -n 5 gpurun_out/pytest_gpu.log
  if [ $rc -ne 0 ]; then echo "STOP pytest rc=$rc"; exit $rc; fi
fi
for c in ${CFGS:-cfg2 cfg3 cfg5}; do
  timeout -k 10 600 python bench.py --config $c --steps 10 --warmup 3 ${BENCH_ARGS:---no-cpu-baseline} \
    > gpurun_out/bench_${TAG}_$c.json 2> gpurun_out/bench_${TAG}_$c.err
  rc=$?; cat gpurun_out/bench_${TAG}_$c.json; echo "bench $c rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done

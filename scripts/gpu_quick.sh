#!/bin/bash
# Quick GPU check: GPU parity tests + cfg2/cfg3/cfg5 bench lines (no profiling).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-q}
OUT=gpurun_out/q_$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${K:+-k "$K"} \
  > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -n 5 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || { echo "STOP pytest rc=$rc"; exit $rc; }
for c in cfg2 cfg3 cfg5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $OUT/bench_$c.json 2> $OUT/bench_$c.err
  rc=$?; cat $OUT/bench_$c.json; [ $rc -eq 0 ] || { echo "STOP bench $c rc=$rc"; exit $rc; }
done

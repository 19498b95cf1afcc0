#!/bin/bash
# GPU tests + rocprofv3 kernel-trace stats of a short bench run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r1}
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -n 15 gpurun_out/pytest_gpu.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP pytest rc=$rc"; exit $rc; fi
fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv \
  -- python3 bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline > gpurun_out/prof_bench_$TAG.log 2>&1
rc=$?; tail -n 3 gpurun_out/prof_bench_$TAG.log; echo "prof rc=$rc"
find gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -3

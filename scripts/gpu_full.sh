#!/bin/bash
# Full round: GPU tests, bench (roofline + cpu baseline), rocprofv3 kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r1}
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -n 8 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP pytest rc=$rc"; exit $rc; fi
timeout -k 10 900 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; cat gpurun_out/bench_$TAG.json; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv \
  -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_bench_$TAG.log 2>&1
echo "prof rc=$?"

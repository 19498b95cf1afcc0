#!/bin/bash
# Kernel-time breakdown of the training step alone (13 steps: 3 warm-up + 10).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/step_${TAG:-x}
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv \
  -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --no-alt \
  ${BENCH_ARGS:-} > $OUT/bench.log 2>&1
rc=$?; echo "rc=$rc"; tail -1 $OUT/bench.log

#!/bin/bash
# Round evidence: rocprofv3 kernel stats of the cfg2 bench command and PMC
# FETCH_SIZE / WRITE_SIZE passes (separate runs, no tracing domains) for cfg2 and cfg3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-x}
OUT=gpurun_out/round_$TAG
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/stats_cfg2 -o run --output-format csv \
  -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/stats_cfg2.log 2>&1
rc=$?; echo "stats cfg2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
for c in cfg2 cfg3; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 -s KILL 300 rocprofv3 --pmc $ctr -d $OUT/pmc_${c}_$ctr -o run --output-format csv \
      -- python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-roofline \
      > $OUT/pmc_${c}_$ctr.log 2>&1
    rc=$?; echo "pmc $c $ctr rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done

#!/bin/bash
# Round evidence in one GPU call: all GPU parity tests, the default bench line
# (cfg2, CPU baseline), cfg3 / cfg5 lines, rocprofv3 kernel stats of the bench
# command, and separate FETCH_SIZE / WRITE_SIZE PMC passes (no tracing domains).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-x}
OUT=gpurun_out/ev_$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -n 3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || { echo "STOP pytest rc=$rc"; exit $rc; }
timeout -k 10 600 python bench.py > $OUT/bench_cfg2.json 2> $OUT/bench_cfg2.err
rc=$?; cat $OUT/bench_cfg2.json; [ $rc -eq 0 ] || { echo "STOP bench rc=$rc"; exit $rc; }
for c in cfg3 cfg5; do
  timeout -k 10 600 python bench.py --config $c --no-cpu-baseline > $OUT/bench_$c.json 2> $OUT/bench_$c.err
  rc=$?; [ $rc -eq 0 ] || { echo "STOP bench $c rc=$rc"; exit $rc; }
done
echo "benches done"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv \
  -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/stats_bench.log 2>&1
rc=$?; echo "stats rc=$rc"; [ $rc -eq 0 ] || exit $rc
# HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes) per config, then
# MFMA-busy cycles + the clock (SQ_VALU_MFMA_BUSY_CYCLES, GRBM_GUI_ACTIVE) on cfg2
for c in cfg2 cfg3 cfg5; do
  i=0
  for ctr in FETCH_SIZE WRITE_SIZE "SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    [ $i -eq 3 ] && [ $c != cfg2 ] && continue
    timeout -k 10 -s KILL 300 rocprofv3 --pmc $ctr -d $OUT/pmc_$c/p$i -o run --output-format csv \
      -- python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-roofline --no-alt --no-repeats > $OUT/pmc_${c}_p$i.log 2>&1
    rc=$?; echo "pmc $c $ctr rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done

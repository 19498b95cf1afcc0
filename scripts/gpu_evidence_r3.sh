#!/bin/bash
# Round-3 evidence, per config (cfg2 / cfg3 / cfg5), in two GPU calls:
#   STAGE=a: GPU parity tests, the three bench lines (each with its CPU
#            baseline), and a rocprofv3 --kernel-trace --stats summary of each
#            bench command;
#   STAGE=b: PMC passes per config (FETCH_SIZE / WRITE_SIZE / MFMA busy, one
#            counter group per run, no tracing domains), plus the source hash
#            of the tree they ran on (profiles/pmc_<tag>_<cfg>.json via
#            scripts/pmc_traffic.py afterwards).
# Every GPU step runs under its own time limit; the first failure ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-x}
STAGE=${STAGE:-a}
CFGS=${CFGS:-"cfg2 cfg3 cfg5"}
OUT=gpurun_out/ev_$TAG
mkdir -p $OUT
python3 -c "import bench; print(bench.source_sha16())" > $OUT/src_sha16.txt
if [ "$STAGE" = a ]; then
  if [ "${TESTS:-1}" = 1 ]; then
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
      > $OUT/pytest_gpu.log 2>&1
    rc=$?; tail -n 3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || { echo "STOP pytest rc=$rc"; exit $rc; }
  fi
  for c in $CFGS; do
    timeout -k 10 600 python3 bench.py --config $c > $OUT/bench_$c.json 2> $OUT/bench_$c.err
    rc=$?; cat $OUT/bench_$c.json; [ $rc -eq 0 ] || { echo "STOP bench $c rc=$rc"; exit $rc; }
  done
  for c in $CFGS; do
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/stats_$c -o run --output-format csv \
      -- python3 bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline \
      > $OUT/stats_bench_$c.json 2> $OUT/stats_bench_$c.err
    rc=$?; echo "stats $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
fi
if [ "$STAGE" = b ]; then
  for c in $CFGS; do
    i=0
    for ctr in FETCH_SIZE WRITE_SIZE "SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"; do
      i=$((i+1))
      timeout -k 10 -s KILL 300 rocprofv3 --pmc $ctr -d $OUT/pmc_$c/p$i -o run --output-format csv \
        -- python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-roofline \
        --no-alt --no-repeats > $OUT/pmc_${c}_p$i.log 2>&1
      rc=$?; echo "pmc $c $ctr rc=$rc"; [ $rc -eq 0 ] || exit $rc
    done
  done
fi
echo "stage $STAGE done"

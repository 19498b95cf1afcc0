#!/bin/bash
# Per-kernel step traces (rocprofv3 kernel trace of 10 bench steps, summarised
# per kernel by step_busy.py) of the configs in CFGS on the shipped library.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6s}
mkdir -p $OUT
for c in ${CFGS:-cfg2 cfg3 cfg5}; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/tr_$c -o run --output-format csv \
    -- python3 bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --no-alt \
    --no-repeats --no-sweep > $OUT/trb_$c.json 2> $OUT/trb_$c.err || { tail -5 $OUT/trb_$c.err; exit 1; }
  f=$(find $OUT/tr_$c -name "*kernel_trace.csv" | head -1)
  python3 scripts/step_busy.py $f 10 > $OUT/step_$c.txt 2>&1
  rm -rf $OUT/tr_$c
  head -3 $OUT/step_$c.txt
done

#!/bin/bash
# Per-kernel cfg2 step traces (rocprofv3 kernel trace, step_busy.py) of the
# shipped library and variant libraries (VARIANTS), one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6vs}
mkdir -p $OUT
for v in base ${VARIANTS:-}; do
  lv=""; [ $v = base ] || lv=$v
  STGCN_LIB_VARIANT=$lv timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/tr_$v -o run --output-format csv \
    -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --no-alt \
    --no-repeats --no-sweep --no-graph > $OUT/trb_$v.json 2> $OUT/trb_$v.err || { tail -5 $OUT/trb_$v.err; exit 1; }
  f=$(find $OUT/tr_$v -name "*kernel_trace.csv" | head -1)
  python3 scripts/step_busy.py $f 10 > $OUT/step_$v.txt 2>&1
  rm -rf $OUT/tr_$v
  echo "== $v"; head -14 $OUT/step_$v.txt
done

#!/bin/bash
# Per-step kernel breakdown (rocprofv3 kernel trace + step_busy.py) per f32 GEMM mode.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-step}
mkdir -p $OUT
for m in ${MODES:-bf16x3 f16x2}; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/tr_$m -o run --output-format csv \
    -- python3 bench.py --config ${CFG:-cfg2} --steps 10 --warmup 3 --no-cpu-baseline \
    --no-roofline --no-alt --no-repeats --no-sweep --f32-gemm $m > $OUT/trb_$m.json 2> $OUT/trb_$m.err || exit 1
  f=$(find $OUT/tr_$m -name "*kernel_trace.csv" | head -1)
  python3 scripts/step_busy.py $f 10 > $OUT/step_$m.txt 2>&1
  echo "== $m"; head -30 $OUT/step_$m.txt
done
echo done

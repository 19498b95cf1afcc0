#!/bin/bash
# Round 4: error diagnostics per GEMM mode, kernel timings (bf16x3 vs f16x2) and
# the cfg2 bench in both modes (no parity gate).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-perf}
mkdir -p $OUT
timeout -k 10 300 python scripts/diag_x3.py > $OUT/diag_errors.txt 2>&1 || exit 10
KB_X3=1 KB_WHICH=0,1,2 timeout -k 10 300 python scripts/kbench.py 20 > $OUT/kb_x3.txt 2>&1 || exit 11
KB_F16=1 KB_WHICH=0,1,2 timeout -k 10 300 python scripts/kbench.py 20 > $OUT/kb_f16.txt 2>&1 || exit 12
cat $OUT/kb_x3.txt $OUT/kb_f16.txt
for m in ${MODES:-bf16x3 f16x2}; do
  timeout -k 10 600 python3 bench.py --config cfg2 --no-cpu-baseline --f32-gemm $m > $OUT/bench_$m.json 2> $OUT/bench_$m.err || { tail -5 $OUT/bench_$m.err; exit 13; }
  python3 -c "import json;a=json.load(open('$OUT/bench_$m.json'));print('$m',a['value'],a['runs_clips_s'],a['roofline']['kernel'],a['roofline']['frac'],a.get('batch_sweep_clips_s'))"
done
echo done

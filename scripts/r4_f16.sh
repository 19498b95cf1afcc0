#!/bin/bash
# Round 4: fp16-split GEMMs (STGCN_F_F16X2) -- parity subset, kernel timings
# (bf16x3 vs f16x2), cfg2 bench in both modes, then the full GPU suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-f16}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_f16x2.py tests/test_gpu_f32x3.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest_f16.log 2>&1
rc=$?; tail -n 3 $OUT/pytest_f16.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $OUT/pytest_f16.log | head -30; exit $rc; }
KB_X3=1 KB_WHICH=0,1,2 timeout -k 10 300 python scripts/kbench.py 20 > $OUT/kb_x3.txt 2>&1 || exit 11
KB_F16=1 KB_WHICH=0,1,2 timeout -k 10 300 python scripts/kbench.py 20 > $OUT/kb_f16.txt 2>&1 || exit 12
cat $OUT/kb_x3.txt $OUT/kb_f16.txt
for m in bf16x3 f16x2; do
  timeout -k 10 600 python3 bench.py --config cfg2 --no-cpu-baseline --f32-gemm $m > $OUT/bench_$m.json 2> $OUT/bench_$m.err || { tail -5 $OUT/bench_$m.err; exit 13; }
  python3 -c "import json;a=json.load(open('$OUT/bench_$m.json'));print('$m',a['value'],a['runs_clips_s'],a['roofline']['kernel'],a['roofline']['frac'],a.get('batch_sweep_clips_s'))"
done
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?; tail -n 3 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -30; exit $rc; }
fi
echo done

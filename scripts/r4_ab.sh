#!/bin/bash
# Round-4 A/B: kernel timings (kbench) and the cfg2 bench on the shipped library
# and on one variant library (STGCN_LIB_VARIANT), then optionally the GPU tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ab}
VAR=${VAR:-f16x2}
mkdir -p $OUT
KB_X3=1 KB_WHICH=${KB_WHICH:-0,1} timeout -k 10 300 python scripts/kbench.py 20 > $OUT/kb_base.txt 2>&1 || exit 11
STGCN_LIB_VARIANT=$VAR KB_X3=1 KB_WHICH=${KB_WHICH:-0,1} timeout -k 10 300 python scripts/kbench.py 20 > $OUT/kb_$VAR.txt 2>&1 || exit 12
cat $OUT/kb_base.txt $OUT/kb_$VAR.txt
for c in ${BENCH:-cfg2}; do
  timeout -k 10 600 python3 bench.py --config $c --no-cpu-baseline > $OUT/bench_base_$c.json 2> $OUT/bench_base_$c.err || exit 13
  STGCN_LIB_VARIANT=$VAR timeout -k 10 600 python3 bench.py --config $c --no-cpu-baseline > $OUT/bench_${VAR}_$c.json 2> $OUT/bench_${VAR}_$c.err || exit 14
  python3 -c "import json;a=json.load(open('$OUT/bench_base_$c.json'));b=json.load(open('$OUT/bench_${VAR}_$c.json'));print('$c base',a['value'],'var',b['value'])"
done
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?; tail -n 3 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -30; exit $rc; }
fi
echo done

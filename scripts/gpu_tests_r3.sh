#!/bin/bash
# GPU parity tests (optionally a -k subset), then an optional quick bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/t_${TAG:-x}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  ${K:+-k "$K"} > $OUT/pytest.log 2>&1
rc=$?; tail -n 4 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $OUT/pytest.log | head -30; echo "STOP pytest rc=$rc"; exit $rc; }
for c in ${BENCH:-}; do
  timeout -k 10 600 python3 bench.py --config $c --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/bench_$c.json 2> $OUT/bench_$c.err
  rc=$?; python3 -c "import json;d=json.load(open('$OUT/bench_$c.json'));print('$c', d['value'], d['runs_clips_s'], d.get('roofline',{}).get('kernel'), d.get('roofline',{}).get('frac'))"; [ $rc -eq 0 ] || { tail -5 $OUT/bench_$c.err; exit $rc; }
done
echo "done"

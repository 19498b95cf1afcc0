#!/bin/bash
# Round-4 validation + bench: the full GPU suite, smoke(), the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-run}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/ > $OUT/tests.log 2>&1
echo "tests: $(tail -1 $OUT/tests.log)"
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
echo "smoke: $(tail -1 $OUT/smoke.log)"
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
[ -x scripts/micro/wave_probe ] && timeout -k 10 60 scripts/micro/wave_probe > $OUT/wave_probe.txt 2>&1
echo done

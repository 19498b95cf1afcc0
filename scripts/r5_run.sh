#!/bin/bash
# Round-5 iteration: the GPU suite, smoke(), a quick cfg2 bench and its per-step
# kernel breakdown (rocprofv3 kernel trace + step_busy.py). Every GPU step has
# its own time limit; the script stops at the first failing step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5}
mkdir -p $OUT
if [ -z "${NO_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu ${TESTS:-tests/} > $OUT/tests.log 2>&1
  rc=$?; echo "tests rc $rc: $(tail -1 $OUT/tests.log)"
  [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)" $OUT/tests.log | head -20; exit 1; }
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
  echo "smoke: $(tail -1 $OUT/smoke.log)"
fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python - $OUT/bench.json <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r=d.get("roofline",{})
print("bench", d["value"], d["ms_per_step"], "runs", d.get("runs_clips_s"), "frac", r.get("frac"), r.get("kernel"))
print("per_symbol", r.get("per_symbol_ms_per_step"))
PY
if [ -z "${NO_STEP:-}" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/tr -o run --output-format csv \
    -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --no-alt \
    --no-repeats --no-sweep ${BENCH_ARGS:-} > $OUT/trb.json 2> $OUT/trb.err || { tail -5 $OUT/trb.err; exit 1; }
  f=$(find $OUT/tr -name "*kernel_trace.csv" | head -1)
  python3 scripts/step_busy.py $f 10 > $OUT/step.txt 2>&1
  head -40 $OUT/step.txt
fi
echo done

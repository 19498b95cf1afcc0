#!/bin/bash
# Round-6 GPU call: optional GPU test suite, then a same-box A/B of the shipped
# library against variant libraries (VARIANTS="a b"): per-kernel times at the
# cfg2 layer shapes (scripts/kbench.py, f16x2) and short cfg2 bench runs,
# alternating so that clock drift hits every library alike.
# Env: TAG (output dir under gpurun_out), TESTS=1 (run pytest -m gpu first),
#      KB=0 (skip kbench), BENCH_CFGS ("cfg2" default), ROUNDS (bench rounds, 2)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r6}
mkdir -p $OUT
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    ${PYTEST_ARGS:-} > $OUT/tests.log 2>&1
  rc=$?
  tail -3 $OUT/tests.log
  # a failed assertion (1) still leaves the GPU usable; anything else ends the call
  [ $rc -le 1 ] || exit $rc
fi
if [ "${KB:-1}" = 1 ]; then
  for v in base ${VARIANTS:-}; do
    lv=""; [ $v = base ] || lv=$v
    echo "== kbench $v" | tee -a $OUT/kbench.txt
    STGCN_LIB_VARIANT=$lv KB_F16=1 KB_WHICH=${KB_WHICH:-0,1,2} KB_SHAPES=${KB_SHAPES:-0,1,2,3,4,5} \
      timeout -k 10 300 python scripts/kbench.py 10 >> $OUT/kbench.txt 2>&1 || exit 1
  done
fi
for r in $(seq 1 ${ROUNDS:-2}); do
  for cfg in ${BENCH_CFGS:-cfg2}; do
    for v in base ${VARIANTS:-}; do
      lv=""; [ $v = base ] || lv=$v
      STGCN_LIB_VARIANT=$lv timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 5 \
        --no-cpu-baseline --no-roofline --no-alt --no-sweep > $OUT/bench_${cfg}_${v}_$r.json \
        2> $OUT/bench_${cfg}_${v}_$r.err || { tail -5 $OUT/bench_${cfg}_${v}_$r.err; exit 1; }
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], sys.argv[4], d['value'], d['runs_clips_s'])" \
        $OUT/bench_${cfg}_${v}_$r.json $cfg $v $r | tee -a $OUT/bench_ab.txt
    done
  done
done

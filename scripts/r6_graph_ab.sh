#!/bin/bash
# Round-6 GPU call: the GPU test suite, then cfg2 / cfg3 / cfg5 bench lines in
# both step modes (HIP-graph replay, the N=1 default, and --no-graph eager),
# alternating, on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r6g}
mkdir -p $OUT
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > $OUT/tests.log 2>&1
  rc=$?; tail -n 2 $OUT/tests.log; [ $rc -le 1 ] || exit $rc
fi
for c in ${CFGS:-cfg2 cfg3 cfg5}; do
  for m in graph eager; do
    extra=""; [ $m = eager ] && extra="--no-graph"
    timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline \
      --no-roofline --no-alt --no-sweep $extra > $OUT/bench_${c}_$m.json 2> $OUT/bench_${c}_$m.err \
      || { tail -n 5 $OUT/bench_${c}_$m.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['value'], d['runs_clips_s'], d['loss'], d.get('step_mode'))" \
      $OUT/bench_${c}_$m.json $c $m | tee -a $OUT/bench_ab.txt
  done
done

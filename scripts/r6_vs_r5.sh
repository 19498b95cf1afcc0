#!/bin/bash
# Same-box A/B of the whole round-6 tree against the round-5 tree (git
# worktree of ec1183d built in .r5tree/, not committed): cfg2 / cfg3 / cfg5
# bench lines (20 timed steps after 5 warm-up), alternating, ROUNDS times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r6vs5}
mkdir -p $OUT
for r in $(seq 1 ${ROUNDS:-2}); do
  for c in ${CFGS:-cfg2 cfg3 cfg5}; do
    for t in r5 r6; do
      b=bench.py; [ $t = r5 ] && b=.r5tree/bench.py
      timeout -k 10 300 python $b --config $c --steps 20 --warmup 5 --no-cpu-baseline \
        --no-roofline --no-alt --no-sweep > $OUT/${t}_${c}_$r.json 2> $OUT/${t}_${c}_$r.err \
        || { tail -n 5 $OUT/${t}_${c}_$r.err; exit 1; }
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], sys.argv[4], d['value'], d['runs_clips_s'], d.get('step_mode', 'eager'))" \
        $OUT/${t}_${c}_$r.json $t $c $r | tee -a $OUT/ab.txt
    done
  done
done

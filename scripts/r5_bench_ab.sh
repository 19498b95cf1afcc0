#!/bin/bash
# Same-box A/B of whole training steps: bench.py (cfg2 unless BENCH_ARGS) on the
# shipped library and on each variant library (lib/libstgcn_hip_<v>.so).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r5bab}
mkdir -p $OUT
for v in base ${VARIANTS}; do
  if [ $v = base ]; then
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --no-alt --no-sweep ${BENCH_ARGS:-} > $OUT/b_$v.json 2> $OUT/b_$v.err || { tail -5 $OUT/b_$v.err; exit 1; }
  else
    STGCN_LIB_VARIANT=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --no-alt --no-sweep ${BENCH_ARGS:-} > $OUT/b_$v.json 2> $OUT/b_$v.err || { tail -5 $OUT/b_$v.err; exit 1; }
  fi
  python -c "import json,sys; d=json.loads(open('$OUT/b_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d.get('runs_clips_s'))"
done

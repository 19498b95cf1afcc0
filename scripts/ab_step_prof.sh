#!/bin/bash
# In-call A/B of library variants on one config: a short bench line per variant
# (time) and a rocprofv3 kernel trace of each (per-step kernel breakdown via
# scripts/collect_evidence.py step_text). VARIANTS="base v1 ..." CFG=cfg5
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/abp_${TAG:-x}
mkdir -p $OUT
for v in ${VARIANTS}; do
  if [ $v = base ]; then unset STGCN_LIB_VARIANT; else export STGCN_LIB_VARIANT=$v; fi
  timeout -k 10 300 python3 bench.py --config ${CFG:-cfg5} --steps 10 --warmup 3 --no-cpu-baseline \
    --no-roofline --no-alt > $OUT/bench_$v.json 2> $OUT/bench_$v.err || exit 1
  python3 -c "import json; d=json.load(open('$OUT/bench_$v.json')); print('$v', d['value'], d['ms_per_step'], d['runs_clips_s'])"
done
for v in ${VARIANTS}; do
  if [ $v = base ]; then unset STGCN_LIB_VARIANT; else export STGCN_LIB_VARIANT=$v; fi
  timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/tr_$v -o run --output-format csv \
    -- python3 bench.py --config ${CFG:-cfg5} --steps 10 --warmup 3 --no-cpu-baseline \
    --no-roofline --no-alt --no-repeats > $OUT/trb_$v.json 2> $OUT/trb_$v.err || exit 1
done
echo done

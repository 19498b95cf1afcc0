#!/bin/bash
# A/B of library variants (lib/libstgcn_hip_<v>.so, "base" = the in-tree build)
# on short bench runs of configs $CFGS.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for c in ${CFGS:-cfg3 cfg5}; do
  for v in base ${VARIANTS}; do
    if [ $v = base ]; then unset STGCN_LIB_VARIANT; else export STGCN_LIB_VARIANT=$v; fi
    timeout -k 10 200 python bench.py --config $c --steps 6 --warmup 2 --no-cpu-baseline \
      --no-roofline --no-alt > gpurun_out/abb_${c}_$v.json 2> gpurun_out/abb_${c}_$v.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/abb_${c}_$v.json')); print('$c $v', d['value'], d['ms_per_step'])"
  done
done

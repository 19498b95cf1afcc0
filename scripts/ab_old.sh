#!/bin/bash
# A/B of the committed library (lib/libstgcn_hip_old.so, built from HEAD) against
# the working tree's, and the working tree with fp32 activation storage.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in ${CFGS:-cfg3 cfg5 cfg2}; do
  for v in old base act32 old base; do
    unset STGCN_LIB_VARIANT STGCN_ACT_FP32
    [ $v = old ] && export STGCN_LIB_VARIANT=old
    [ $v = act32 ] && export STGCN_ACT_FP32=1
    timeout -k 10 200 python bench.py --config $c --steps 6 --warmup 2 --no-cpu-baseline \
      --no-roofline --no-alt --no-repeats > gpurun_out/abo_${c}_$v.json 2> gpurun_out/abo_${c}_$v.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/abo_${c}_$v.json')); print('$c $v', d['value'], d['ms_per_step'], d['loss'])"
  done
done

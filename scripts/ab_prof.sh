#!/bin/bash
# A/B kernel stats: rocprofv3 --kernel-trace --stats of short bench runs for the
# in-tree library ("new") and lib/libstgcn_hip_prev.so ("prev"), configs $CFGS.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for v in new prev; do
  if [ $v = prev ]; then export STGCN_LIB_VARIANT=prev; fi
  for c in ${CFGS:-cfg2 cfg3 cfg5}; do
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ab_${c}_$v -o run \
      --output-format csv -- python3 bench.py --config $c --steps 6 --warmup 2 \
      --no-cpu-baseline --no-roofline --no-alt > gpurun_out/ab_${c}_$v.log 2>&1 || exit 1
    grep '^{' gpurun_out/ab_${c}_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c $v', d['value'], d['ms_per_step'])"
  done
done

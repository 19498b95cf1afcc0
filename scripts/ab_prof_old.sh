#!/bin/bash
# Step-only kernel traces of cfg5 with the committed library (old) and the
# working tree's (fp32 activation storage), for a per-kernel comparison.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for v in ${VS:-old act32}; do
  unset STGCN_LIB_VARIANT STGCN_ACT_FP32
  [ $v = old ] && export STGCN_LIB_VARIANT=old
  [ $v = act32 ] && export STGCN_ACT_FP32=1
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/apo_${CFG:-cfg5}_$v -o run --output-format csv \
    -- python3 bench.py --config ${CFG:-cfg5} --steps 4 --warmup 2 --no-cpu-baseline --no-roofline --no-alt --no-repeats \
    > gpurun_out/apo_${CFG:-cfg5}_$v.log 2>&1 || exit 1
  echo "$v done"
done

#!/bin/bash
# rocprofv3 kernel stats of a short bench run per config (no roofline / cpu legs).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-x}
for c in ${CFGS:-cfg3 cfg5}; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_$c -o run \
    --output-format csv -- python3 bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline \
    --no-roofline > gpurun_out/prof_${TAG}_$c.log 2>&1
  rc=$?; echo "prof $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done

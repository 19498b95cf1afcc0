#!/bin/bash
# A/B PMC pass over a short bench run: ENVA vs ENVB (one counter set, no tracing domains).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmcab_${TAG:-x}
mkdir -p $OUT
SET=${SET:-"SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"}
for v in a b; do
  if [ $v = a ]; then E=${ENVA:-X_NONE=1}; else E=${ENVB:-X_NONE=1}; fi
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/t$v -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-roofline > $OUT/t$v.log 2>&1 || exit 1
done

#!/bin/bash
# Stall breakdown of the x3 kernels on the micro-bench: for each (which, shape)
# pair in PAIRS ("which:shape ..."), two PMC passes (SQ cycles/waits + MFMA busy,
# GRBM clock) over kbench with KB_X3=1. No tracing domains.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp KB_X3=1 KB_F16=${KB_F16:-0}
OUT=gpurun_out/pmcx_${TAG:-x}
mkdir -p $OUT
for pr in ${PAIRS:-2:1 0:1 0:5}; do
  w=${pr%%:*}; sh=${pr##*:}
  i=0
  for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
             "SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    KB_WHICH=$w KB_SHAPES=$sh timeout -k 10 -s KILL 120 rocprofv3 --pmc $set -d $OUT/w${w}s${sh}p$i -o run --output-format csv \
      -- python3 scripts/kbench.py 3 > $OUT/w${w}s${sh}p$i.log 2>&1
    rc=$?; echo "w$w s$sh pass $i rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $OUT/w${w}s${sh}p$i.log; exit $rc; fi
  done
done

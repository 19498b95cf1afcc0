#!/bin/bash
# Stall counters for the kernels matching KREGEX in a short bench run of CONFIG
# (two PMC passes, no tracing domains). Summary: scripts/pmc_stall.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmcb_${TAG:-x}
mkdir -p $OUT
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
           "SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 -s KILL 200 rocprofv3 --pmc $set --kernel-include-regex "${KREGEX}" -d $OUT/p$i -o run --output-format csv \
    -- python3 bench.py --config ${CONFIG:-cfg2} --steps 2 --warmup 1 --no-cpu-baseline --no-roofline --no-alt --no-repeats > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
done

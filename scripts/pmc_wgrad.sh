#!/bin/bash
# PMC counter passes (separate runs, no tracing domains) for one kernel type.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
W=${KB_WHICH:-2}
export KB_WHICH=$W KB_SHAPES=${KB_SHAPES:-1}
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES" \
           "SQ_INSTS_VALU_MFMA_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU" \
           "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set -d gpurun_out/pmc/p$i -o run --output-format csv -- python3 scripts/kbench.py 5 > gpurun_out/pmc/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc/p$i.log; exit $rc; fi
done

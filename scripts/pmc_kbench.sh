#!/bin/bash
# PMC counter passes (separate runs, no tracing) over the kernel micro-bench.
# env: KB_WHICH, KB_SHAPES (kbench selectors), TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmck_${TAG:-x}
mkdir -p $OUT
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VALU_MFMA_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM SQ_INSTS_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU" \
           "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 -s KILL 200 rocprofv3 --pmc $set -d $OUT/p$i -o run --output-format csv -- python3 scripts/kbench.py 3 > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
done

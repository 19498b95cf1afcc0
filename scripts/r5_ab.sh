#!/bin/bash
# A/B of library variants on the kernel micro-bench (stgcn_time_kernel, cfg2
# layer shapes, f16x2), then the default iteration script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r5ab}
mkdir -p $OUT
for v in base ${VARIANTS}; do
  echo "== $v"
  if [ $v = base ]; then
    KB_F16=1 KB_WHICH=${KB_WHICH:-0,1,2} timeout -k 10 200 python scripts/kbench.py 2>&1 | grep -v amdgpu.ids || exit 1
  else
    STGCN_LIB_VARIANT=$v KB_F16=1 KB_WHICH=${KB_WHICH:-0,1,2} timeout -k 10 200 python scripts/kbench.py 2>&1 | grep -v amdgpu.ids || exit 1
  fi
done > $OUT/ab.txt
cat $OUT/ab.txt
[ -n "${AB_ONLY:-}" ] && exit 0
bash scripts/r5_run.sh

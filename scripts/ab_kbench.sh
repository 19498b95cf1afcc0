#!/bin/bash
# A/B of library variants (lib/libstgcn_hip_<v>.so) on the kernel micro-bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in base ${VARIANTS}; do
  echo "== $v"
  if [ $v = base ]; then
    timeout -k 10 200 python scripts/kbench.py 2>&1 | grep -v amdgpu.ids || exit 1
  else
    STGCN_LIB_VARIANT=$v timeout -k 10 200 python scripts/kbench.py 2>&1 | grep -v amdgpu.ids || exit 1
  fi
done

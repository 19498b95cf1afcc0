#!/bin/bash
# GPU parity tests only (optionally a -k filter): one pytest process, hang-safe.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
K=${1:-}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  ${K:+-k "$K"} -s > gpurun_out/pytest_gpu.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|^\(|^\{" gpurun_out/pytest_gpu.log | tail -n 60
exit $rc

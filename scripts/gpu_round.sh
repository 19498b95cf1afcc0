#!/bin/bash
# One GPU-box session: smoke -> GPU parity tests -> short bench.
# Stops at the first crash / timeout (exit codes other than 0 and 1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STEPS=${STEPS:-5}
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 30 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
run smoke 400 python -c "import __graft_entry__ as g; g.smoke()"
run pytest_gpu 900 python -m pytest tests -m gpu -q -x
run bench 600 python bench.py --steps "$STEPS" --warmup 2

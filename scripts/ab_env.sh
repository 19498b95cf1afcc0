#!/bin/bash
# A/B of an environment switch on the bench: CONFIGS (default "cfg3 cfg5"),
# ENVS (space-separated VAR=VALUE settings; "-" = none), one bench line each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in ${CONFIGS:-cfg3 cfg5}; do
  for e in ${ENVS:--}; do
    if [ "$e" = "-" ]; then
      r=$(timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-roofline --no-alt --no-repeats 2>/dev/null) || exit 1
    else
      r=$(env $e timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-roofline --no-alt --no-repeats 2>/dev/null) || exit 1
    fi
    echo "$c $e $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done

#!/bin/bash
# Same-box A/B of the benched f16x2 step (G formed by k_gather4) against the
# G-free mode (f16x2-nog: BN1 in the forward GEMM's loader, A in its epilogue),
# both in the bench's step mode, ROUNDS times alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r6nog}
mkdir -p $OUT
for r in $(seq 1 ${ROUNDS:-2}); do
  for m in f16x2 f16x2-nog; do
    timeout -k 10 300 python bench.py --f32-gemm $m --steps 20 --warmup 5 --no-cpu-baseline \
      --no-roofline --no-alt --no-sweep > $OUT/$m.$r.json 2> $OUT/$m.$r.err || { tail -n 5 $OUT/$m.$r.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['value'], d['runs_clips_s'], d['step_mode'])" \
      $OUT/$m.$r.json $m $r | tee -a $OUT/ab.txt
  done
done

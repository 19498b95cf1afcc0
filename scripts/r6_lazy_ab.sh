set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r6c
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_stack.py -x -q --timeout 120 --timeout-method thread -k "lazy or bf16 or frozen or deferred" > $OUT/tests_stack.log 2>&1
rc=$?; tail -3 $OUT/tests_stack.log; [ $rc -le 1 ] || exit $rc
for r in 1 2; do
for cfg in cfg3 cfg5; do
  for mode in lazy nolazy; do
    extra=""; [ $mode = nolazy ] && extra="--no-lazy-links"
    timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --no-alt --no-sweep $extra > $OUT/b_${cfg}_${mode}_$r.json 2> $OUT/b_${cfg}_${mode}_$r.err || { tail -5 $OUT/b_${cfg}_${mode}_$r.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['value'], d['runs_clips_s'])" $OUT/b_${cfg}_${mode}_$r.json $cfg $mode | tee -a $OUT/ab.txt
  done
done
done

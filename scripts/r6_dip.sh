# First-timed-window dip: bench's graph mode at W = 5 and W = 40,
# eager at W = 5, twice each alternating, then the per-step window probe.
set -o pipefail
mkdir -p gpurun_out
F="--no-roofline --no-alt --no-cpu-baseline --no-sweep --steps 20"
for r in 1 2; do
  for v in "--warmup 5" "--warmup 40" "--warmup 5 --no-graph"; do
    timeout -k 10 240 python3 bench.py $F $v > gpurun_out/dip.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.load(open('gpurun_out/dip.json')); print(sys.argv[1], d['step_mode'], d['warmup'], d['value'], d['runs_clips_s'], flush=True)" "$r" >> gpurun_out/dip.txt
  done
done
WP_MODE=graph timeout -k 10 240 python3 -u scripts/window_probe.py >> gpurun_out/dip.txt 2>&1

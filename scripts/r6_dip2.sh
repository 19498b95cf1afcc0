# Window probe variants (host read of the loss after each window; no events)
# beside one bench line, same box.
set -o pipefail
mkdir -p gpurun_out
for v in "1 0" "0 0" "1 1" "0 1"; do
  set -- $v
  WP_ITEM=$1 WP_EVENTS=$2 WP_WINDOWS=5 timeout -k 10 240 python3 -u scripts/window_probe.py 2>/dev/null | sed 's/ | steps.*//' >> gpurun_out/dip2.txt || exit 1
done
timeout -k 10 240 python3 bench.py --no-roofline --no-alt --no-cpu-baseline --no-sweep --steps 20 --warmup 5 > gpurun_out/dip2.json 2>/dev/null || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/dip2.json')); print('bench', d['value'], d['runs_clips_s'])" >> gpurun_out/dip2.txt

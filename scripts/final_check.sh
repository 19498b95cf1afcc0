set -o pipefail
mkdir -p gpurun_out/fin
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/fin/pytest_gpu.txt 2>&1 || { tail -20 gpurun_out/fin/pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/fin/pytest_gpu.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin/smoke.txt 2>&1 || exit 1
tail -1 gpurun_out/fin/smoke.txt
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/fin/bench.json 2> gpurun_out/fin/bench.err || exit 1
cat gpurun_out/fin/bench.json

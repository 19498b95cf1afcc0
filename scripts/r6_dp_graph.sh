set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_dp_gpu.py tests/test_gpu_graph.py -x -v --timeout 300 --timeout-method thread > gpurun_out/dpg_pytest.txt 2>&1 || exit 1
for mode in "--dp-graph" ""; do
  STGCN_DIST_BACKEND=gloo OMP_NUM_THREADS=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29533 bench.py --gpus 2 --steps 10 --warmup 5 --batch 64 --no-roofline $mode >> gpurun_out/dpg_bench.txt 2>&1 || exit 1
done

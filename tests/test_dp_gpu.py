"""GPU: the multi-rank HIP data-parallel path (dp.GradAllReduce bucket views +
STGCNStack on the HIP library + FusedAdam) executed with world size 2 on the
box's one GPU, over gloo (tests/dp_gpu_worker.py documents the checks).

The ranks are started as child processes by torch.distributed.run before this
process touches the GPU (the file sorts before every other GPU test module and
this test makes no HIP call itself)."""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2])
def test_dp_two_ranks_on_hip(tmp_path, world):
    out = tmp_path / "dp.json"
    env = dict(os.environ, DP_OUT=str(out), OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={world}", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", os.path.join(ROOT, "tests", "dp_gpu_worker.py")]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = json.loads(out.read_text())
    print(res)
    assert res["bucket_views"] and res["buckets"] >= 2
    assert res["ranks_identical"]
    # every gradient (dA included: deterministic partials) at 1e-6 of the mean
    # of the per-shard gradients, and a re-run of a shard is bit-identical
    assert res["grad_err"] < 1e-6, res
    assert res["rerun_exact"], res
    # overlap: at least one bucket's all-reduce is issued before block 0's
    # backward has produced a gradient (block 0 runs last in backward)
    assert res["first_launch_pos"] < res["first_block0_grad_pos"], res
    assert res["launches_before_block0"] >= 1, res
    assert res["step_err"] < 1e-6, res


def test_graphed_dp_step_matches_eager(tmp_path):
    """train_ops.GraphedDPStep (bench.py's step mode at N > 1: forward +
    backward and Adam in two HIP graphs, the bucket all-reduces eager between
    them) against the eager DP step with the all-reduces issued from the
    backward hooks: loss, logits and every parameter equal after 5 steps on
    every rank (tests/dp_graph_worker.py)."""
    out = tmp_path / "dpg.json"
    env = dict(os.environ, DP_OUT=str(out), OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node=2", "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(ROOT, "tests", "dp_graph_worker.py")]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = json.loads(out.read_text())
    print(res)
    assert res["all_ranks_equal_eager"], res
    assert res["ranks_identical"] and res["bucket_views"], res


def test_bench_two_ranks_rehearsal():
    """bench.py's own N>1 branch (the one the driver launches per GPU over RCCL)
    run end to end with 2 ranks sharing the one GPU over gloo
    (STGCN_DIST_BACKEND=gloo): barrier + max-over-ranks timing, bucket-view
    all-reduce, FusedAdam, one JSON line from rank 0 with the whole-job value."""
    env = dict(os.environ, STGCN_DIST_BACKEND="gloo", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node=2", "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--batch", "8", "--no-roofline", "--no-repeats"]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    out = json.loads(lines[0])
    print(out)
    assert out["n_gpus"] == 2 and out["config"]["global_batch"] == 16
    assert out["config"]["parallelism"] == "dp2" and out["scaling"] == "weak"
    assert out["value"] > 0 and out["loss"] == out["loss"]  # finite, not NaN
    assert "cpu_baseline" not in out  # rank 0 at N=1 only
    assert out["step_mode"] == "eager"  # (--dp-graph: train_ops.GraphedDPStep)

"""Phase timing of the 2-rank step on one GPU over gloo (diagnostic for the
--dp-graph slowdown): per step, forward + backward, the
all-reduces (dp.synchronize) and Adam, each followed by a device synchronize,
eager and graphed (train_ops.GraphedDPStep's graphs replayed phase by phase)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402
from stgcn_loader import load  # noqa: E402

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("gloo")
pkg = load()
dev = torch.device("cuda", 0)
cfg = dict(bench.CONFIGS["cfg2"], f32_gemm="f16x2", N=64)
gen = torch.Generator().manual_seed(1 + rank)
x = torch.randn(cfg["N"], cfg["C"], cfg["T"], cfg["V"], generator=gen).to(dev)
y = torch.randint(0, cfg["classes"], (cfg["N"],), generator=gen).to(dev)


def setup():
    m = bench.build_model(pkg, cfg, dev)
    opt = pkg.FusedAdam(list(m.parameters()), lr=1e-3, capturable=True)
    dp = pkg.dp.GradAllReduce(m, world)

    def fwd_bwd():
        loss, _ = m.forward_loss(x, y)
        loss.backward()
        return loss
    return m, opt, dp, fwd_bwd


def timed(fn):
    torch.cuda.synchronize()
    t = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) * 1e3


for mode in ("eager", "graph"):
    m, opt, dp, fwd_bwd = setup()
    if mode == "graph":
        g = pkg.GraphedDPStep(fwd_bwd, dp, opt.step, warmup=2)
        phases = (g.graph_a.replay, dp.synchronize, g.graph_b.replay)
    else:
        def a():
            dp.zero_grad()
            fwd_bwd()
        phases = (a, dp.synchronize, opt.step)
    for i in range(8):
        dist.barrier()
        ts = [timed(f) for f in phases]
        if rank == 0 and i >= 2:
            print(f"{mode} step {i}: fwd+bwd {ts[0]:.1f} ms, all-reduce {ts[1]:.1f} ms, "
                  f"adam {ts[2]:.1f} ms", flush=True)
dist.barrier()
dist.destroy_process_group()

"""One rank of the graphed multi-rank step check (tests/test_dp_gpu.py).

Launched by torch.distributed.run with WORLD_SIZE ranks sharing the box's one
GPU over gloo (as tests/dp_gpu_worker.py). Each rank trains two copies of the
same STGCNStack (the benched f16x2 path, FusedAdam(capturable=True),
dp.GradAllReduce) on its own shard for 5 steps:
  * eager: the bucket all-reduces issued from the backward hooks (bench.py
    --no-graph at N > 1),
  * graphed: train_ops.GraphedDPStep (2 eager warm-up steps, capture, 3
    replays; the all-reduces eager between the two graphs; bench.py's default
    at N > 1),
and checks that the loss, the logits and every parameter are equal bit for
bit, and that all ranks hold the same parameters. Writes a JSON verdict to
$DP_OUT (rank 0).
"""
import contextlib
import io
import json
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from stgcn_loader import load  # noqa: E402


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    pkg = load()
    gr = pkg.graph
    A = gr.get_normalized_adjacency_matrices(0, 1, graph=gr.graph_for(18))
    N, T = 4, 64
    gen = torch.Generator().manual_seed(91)
    xs = torch.randn(world, N, 3, T, 18, generator=gen)
    ys = torch.randint(0, 60, (world, N), generator=gen)
    x, y = xs[rank].cuda(), ys[rank].cuda()

    def make():
        torch.manual_seed(0)
        with contextlib.redirect_stdout(io.StringIO()):
            m = pkg.STGCNStack(3, 60, A, f32_gemm="f16x2").cuda().train()
        opt = pkg.FusedAdam(list(m.parameters()), lr=1e-3, capturable=True)
        dp = pkg.dp.GradAllReduce(m, world, bucket_bytes=1 << 20)
        return m, opt, dp

    ma, opta, dpa = make()
    for _ in range(5):
        dpa.zero_grad()
        la, ga = ma.forward_loss(x, y)
        la.backward()
        dpa.synchronize()
        opta.step()

    mb, optb, dpb = make()

    def fwd_bwd():
        loss, logits = mb.forward_loss(x, y)
        loss.backward()
        return loss, logits

    g = pkg.GraphedDPStep(fwd_bwd, dpb, optb.step, warmup=2)
    for _ in range(3):
        lb, gb = g()
    torch.cuda.synchronize()
    equal = bool(torch.equal(la, lb) and torch.equal(ga, gb))
    diff = []
    for (ka, a), (kb, b) in zip(ma.state_dict().items(), mb.state_dict().items()):
        if ka != kb or not torch.equal(a, b):
            diff.append(ka)
    views = all(p.grad is dpb._view[p] for p in mb.parameters())
    flat = torch.cat([p.detach().reshape(-1) for p in mb.parameters()]).cpu()
    gathered = [torch.empty_like(flat) for _ in range(world)]
    dist.all_gather(gathered, flat)
    ok = torch.tensor([1 if equal and not diff else 0])
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if rank == 0:
        out = {"world": world, "all_ranks_equal_eager": bool(ok.item()),
               "rank0_loss_logits_equal": equal, "rank0_diff": diff[:8],
               "ranks_identical": all(torch.equal(gathered[0], t) for t in gathered[1:]),
               "bucket_views": views, "loss": float(lb)}
        with open(os.environ["DP_OUT"], "w") as f:
            json.dump(out, f)
        print(json.dumps(out), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

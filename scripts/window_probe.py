"""Per-window and per-step timing of the cfg2 bench step (diagnostic for the
graph step mode's first-timed-window dip). Builds the step as
bench.py does (W = 5 warm-up: 2 eager + capture + 3 replays in graph mode),
then times WP_WINDOWS windows of K = 20 steps exactly as bench.py brackets
them, with HIP events around every step of the first two windows.
WP_MODE: graph | eager; WP_SLEEP: seconds of host sleep before each window;
WP_ITEM=1: read the step's loss on the host after each window (as bench.py does
after its first); WP_EVENTS=0: no per-step events."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from stgcn_loader import load  # noqa: E402

mode = os.environ.get("WP_MODE", "graph")
slp = float(os.environ.get("WP_SLEEP", "0"))
nwin = int(os.environ.get("WP_WINDOWS", "6"))
item = os.environ.get("WP_ITEM", "0") == "1"
events = os.environ.get("WP_EVENTS", "1") == "1"
K, W = 20, 5
pkg = load()
dev = torch.device("cuda", 0)
cfg = dict(bench.CONFIGS["cfg2"], f32_gemm="f16x2")
model = bench.build_model(pkg, cfg, dev)
graph_on = mode == "graph"
opt = pkg.FusedAdam(list(model.parameters()), lr=1e-3, capturable=graph_on)
gen = torch.Generator(device="cpu").manual_seed(1)
x = torch.randn(cfg["N"], cfg["C"], cfg["T"], cfg["V"], generator=gen).to(dev)
labels = torch.randint(0, cfg["classes"], (cfg["N"],), generator=gen).to(dev)


def step():
    opt.zero_grad(set_to_none=True)
    loss, _ = model.forward_loss(x, labels)
    loss.backward()
    opt.step()
    return loss


run = step
if graph_on:
    run = pkg.GraphedStep(step, warmup=2)
    for _ in range(W - 2):
        run()
else:
    for _ in range(W):
        step()
torch.cuda.synchronize()
for w in range(nwin):
    if slp:
        time.sleep(slp)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(K + 1)] if w < 2 and events else None
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(K):
        if ev:
            ev[i].record()
        loss = run()
    if ev:
        ev[K].record()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if item:
        float(loss.item())
    line = f"{mode} sleep={slp} item={int(item)} events={int(events)} window {w}: {cfg['N'] * K / dt:.1f} clips/s, {dt / K * 1e3:.3f} ms/step"
    if ev:
        line += " | steps ms " + " ".join(f"{ev[i].elapsed_time(ev[i + 1]):.2f}" for i in range(K))
    print(line, flush=True)

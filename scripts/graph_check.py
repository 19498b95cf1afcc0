"""Loss per step of the cfg2 bench step three ways (eager with the host-step
Adam, eager with the device-step Adam, the HIP-graph replay of the latter):
the trajectories must agree (bench.py's step modes)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from stgcn_loader import load  # noqa: E402

pkg = load()
dev = torch.device("cuda", 0)
cfg = dict(bench.CONFIGS["cfg2"], f32_gemm="f16x2")
N = int(os.environ.get("GC_N", "32"))
cfg["N"] = N
steps = int(os.environ.get("GC_STEPS", "12"))
gen = torch.Generator().manual_seed(1)
x = torch.randn(N, cfg["C"], cfg["T"], cfg["V"], generator=gen).to(dev)
labels = torch.randint(0, cfg["classes"], (N,), generator=gen).to(dev)


def run(mode):
    model = bench.build_model(pkg, cfg, dev)
    opt = pkg.FusedAdam(list(model.parameters()), lr=1e-3, capturable=mode != "host")

    def step():
        opt.zero_grad(set_to_none=True)
        loss, _ = model.forward_loss(x, labels)
        loss.backward()
        opt.step()
        return loss
    out = []
    if mode == "graph":
        g = pkg.GraphedStep(step, warmup=2)
        # (the warm-up's two losses are not returned: report replays only)
        out += [float("nan")] * 2
        for _ in range(steps - 2):
            out.append(float(g()))
    else:
        for _ in range(steps):
            out.append(float(step()))
    return out


for mode in ("host", "device", "graph"):
    print(mode, " ".join(f"{v:.6f}" for v in run(mode)), flush=True)

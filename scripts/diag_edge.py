"""Diagnostic: per-tensor gradient errors of the cfg1 stack vs the fp64 oracle
under variants (masks / no masks, fused head / torch head, chained /
unchained), and V=18 blocks with an asymmetric A vs the fp64 oracle."""
import contextlib
import io
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import load_npz, rel_to_max  # noqa: E402
from oracle import ref_cpu  # noqa: E402
from stgcn_loader import load  # noqa: E402

pkg = load()
ref = load_npz("stack_cfg1_edge.npz")
A = torch.from_numpy(load_npz("adjacency.npz")["V18_s0_d1"])


def run(masks, head, chain, jitter=0.05):
    torch.manual_seed(0)
    with contextlib.redirect_stdout(io.StringIO()):
        model = pkg.STGCNStack(3, 2, A, use_edge_importance=masks, max_mask_jitter=jitter)
    p0, b0 = ref_cpu.init_stack_params(3, 2, A, seed=0, masks="jitter" if masks else None,
                                       max_mask_jitter=jitter)
    model = model.cuda().train()
    x = torch.from_numpy(ref["x"]).cuda().permute(0, 3, 1, 2).contiguous()
    lab = torch.from_numpy(ref["labels"]).cuda()
    if chain and head:
        loss, logits = model.forward_loss(x, lab)
    elif chain:
        logits = model.forward_nctv(x)
        loss = torch.nn.functional.cross_entropy(logits, lab)
    else:
        h = x
        for blk in model.conv:
            h = blk(h)
        logits = model.fc_layer(h.flatten(2).mean(dim=2))
        loss = torch.nn.functional.cross_entropy(logits, lab)
    loss.backward()
    torch.cuda.synchronize()

    def oracle(dtype):
        p = {k: v.clone().to(dtype).requires_grad_(True) for k, v in p0.items()}
        b = {k: (v.clone().to(dtype) if v.is_floating_point() else v.clone()) for k, v in b0.items()}
        lg = ref_cpu.Stack(p, b).forward(torch.from_numpy(ref["x"]), dtype=dtype)
        torch.nn.functional.cross_entropy(lg, torch.from_numpy(ref["labels"])).backward()
        return {k: v.grad for k, v in p.items()}
    g64, g32 = oracle(torch.float64), oracle(torch.float32)
    rows = []
    for k, v in model.named_parameters():
        if k.startswith("Masks") or k.endswith("temporalConv.bias"):
            continue
        w = g64[k].double().numpy()
        rows.append((k, rel_to_max(v.grad.cpu().double().numpy(), w),
                     rel_to_max(g32[k].double().numpy(), w)))
    worst = sorted(rows, key=lambda r: -r[1] / max(r[2], 1e-7))[:4]
    print(f"masks={masks} jitter={jitter} head={head} chain={chain}: worst",
          [(k, f"{e:.1e}", f"{f:.1e}") for k, e, f in worst])


for cfg in [(False, True, True), (True, True, True), (True, False, True), (True, False, False)]:
    run(*cfg)
run(True, False, False, jitter=0.0)

# block level, asymmetric A (V = 18, K = 1)
from test_gpu_block import _run_hip, _oracle  # noqa: E402
for case in [(128, 256, 2, 25), (256, 256, 1, 13), (64, 64, 1, 50), (3, 64, 1, 50)]:
    C_in, C_out, s, T = case
    torch.manual_seed(0)
    Am = A * (1 + 2 * (torch.rand(A.shape, generator=torch.Generator().manual_seed(5)) - 0.5) * 0.05)
    with contextlib.redirect_stdout(io.StringIO()):
        blk = pkg.SpatialTemporalConv(C_in, C_out, Am, 9, s, 4, dropout_rate=0)
    arrays = {"param." + k: v.detach().numpy() for k, v in blk.state_dict().items()}
    arrays["meta"] = np.array([C_in, C_out, s, 18, 0, 4, T, 0])
    x = torch.randn(4, C_in, T, 18, generator=torch.Generator().manual_seed(1))
    g = torch.randn(4, C_out, (T - 1) // s + 1, 18, generator=torch.Generator().manual_seed(2))
    arrays["x"], arrays["g"] = x.numpy(), g.numpy()
    for gemm in ("fp32", "f32x3"):
        got = _run_hip(pkg, arrays, x, g, gemm=gemm)
        want, floor = _oracle(arrays, got)
        errs = {k: rel_to_max(got[k].double().numpy(), v.detach().double().numpy())
                for k, v in want.items() if k in got and "num_batches" not in k}
        print("block", case, gemm, {k: f"{e:.1e}" for k, e in errs.items() if e > 1e-6})

"""Diagnostic: chained vs unchained stacks (dg2 = batch_n_2.weight grads) over
T and GEMM modes, plus unchained-vs-unchained repeatability."""
import contextlib
import io
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import rel_to_max  # noqa: E402
from stgcn_loader import load  # noqa: E402

pkg = load()
gr = pkg.graph
A = gr.get_normalized_adjacency_matrices(0, 1, graph=gr.graph_for(18))


def grads(model, x, lab, chained, head):
    model.zero_grad(set_to_none=True)
    if chained and head:
        loss, _ = model.forward_loss(x, lab)
    else:
        if chained:
            h = model.forward_nctv(x)
            out = h
        else:
            h = x
            for blk in model.conv:
                h = blk(h)
            out = model.fc_layer(h.flatten(2).mean(dim=2))
        loss = torch.nn.functional.cross_entropy(out, lab)
    loss.backward()
    torch.cuda.synchronize()
    return {k: p.grad.detach().cpu().double().clone() for k, p in model.named_parameters()}


for f32 in ("mfma", "bf16x3"):
    for T in (40, 300):
        for N in (4,):
            torch.manual_seed(3)
            with contextlib.redirect_stdout(io.StringIO()):
                m = pkg.STGCNStack(3, 400, A, f32_gemm=f32).cuda().train()
            sd = {k: v.clone() for k, v in m.state_dict().items()}
            x = torch.randn(N, 3, T, 18, generator=torch.Generator().manual_seed(4)).cuda()
            lab = torch.randint(0, 400, (N,), generator=torch.Generator().manual_seed(5)).cuda()
            res = {}
            for name, ch, hd in (("unch", False, False), ("unch2", False, False),
                                 ("chain", True, False), ("chain_head", True, True)):
                m.load_state_dict(sd)
                res[name] = grads(m, x, lab, ch, hd)
            for a, b in (("unch2", "unch"), ("chain", "unch"), ("chain_head", "unch")):
                e = {k: rel_to_max(res[a][k].numpy(), res[b][k].numpy())
                     for k in res[a] if k.endswith("batch_n_2.weight") or k.endswith("W.weight")}
                w = max(e.items(), key=lambda kv: kv[1])
                print(f"{f32} T={T} N={N} {a} vs {b}: worst {w[0]} {w[1]:.2e}; dg2:",
                      [f"{e[f'conv.{i}.batch_n_2.weight']:.1e}" for i in range(10)], flush=True)

"""GPU parity of the training-step ops through the
C-ABI: the fused head (avg-pool + Linear + cross entropy, lightning_model.py:
105-107, :202) against the same ops in torch on the CPU in fp64, and FusedAdam
against torch.optim.Adam on the CPU (the reference's optimizer,
lightning_model.py:196-197). Tolerances: head rel-to-max 1e-5 (fp32 sums in
a different order); Adam parameters within 2e-6 relative per element over 5
steps, moments within 1e-6 rel-to-max (the update is elementwise in torch's
op order; CPU and GPU may differ in fma contraction by an ulp, and moments
that cross 0 make per-element relative error meaningless)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import rel_to_max

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.mark.parametrize("N,C,T,V,classes", [(8, 256, 5, 18, 400), (16, 256, 7, 25, 60),
                                              (3, 64, 4, 50, 2), (5, 32, 1, 18, 7)])
def test_head_matches_torch(pkg, N, C, T, V, classes):
    g = torch.Generator().manual_seed(N * 31 + classes)
    y = torch.relu(torch.randn(N, C, T, V, generator=g))
    W = torch.randn(classes, C, generator=g) * 0.1
    b = torch.randn(classes, generator=g) * 0.1
    lab = torch.randint(0, classes, (N,), generator=g)
    # reference ops (lightning_model.py:105-107, :202) in fp64
    y64, W64, b64 = (t.double().requires_grad_(True) for t in (y, W, b))
    pooled = F.avg_pool2d(y64, (T, V)).view(N, C)
    logits64 = F.linear(pooled, W64, b64)
    loss64 = F.cross_entropy(logits64, lab)
    loss64.backward()
    yd, Wd, bd = (t.to(DEV).requires_grad_(True) for t in (y, W, b))
    loss, logits = pkg.train_ops.StgcnHeadFn.apply(yd, Wd, bd, lab.to(DEV))
    loss.backward()
    torch.cuda.synchronize()
    assert abs(loss.item() - loss64.item()) <= 1e-5 * abs(loss64.item())
    assert rel_to_max(logits.cpu().numpy(), logits64.detach().numpy()) < 1e-5
    for got, want in ((yd.grad, y64.grad), (Wd.grad, W64.grad), (bd.grad, b64.grad)):
        assert rel_to_max(got.cpu().numpy(), want.numpy()) < 1e-5


def test_head_in_stack_matches_torch_head(pkg):
    """forward_loss (fused head) == F.cross_entropy(forward_nctv(x)) on the
    same stack, and the same parameter gradients: tight for the head and the
    last block; the earlier blocks' gradients only within the stack's fp32
    conditioning (the 10-block stack amplifies a 1e-7 change of
    the last block's input gradient, here the head's summation order, to
    ~1e-3 on some BN-affine gradients, as it does for the reference itself)."""
    gr = pkg.graph
    A = gr.get_normalized_adjacency_matrices(0, 1, graph=gr.graph_for(18))
    torch.manual_seed(0)
    model = pkg.STGCNStack(3, 10, A).to(DEV)
    x = torch.randn(4, 3, 24, 18, generator=torch.Generator().manual_seed(1)).to(DEV)
    lab = torch.tensor([1, 5, 9, 0], device=DEV)
    loss_a, _ = model.forward_loss(x, lab)
    loss_a.backward()
    ga = {k: p.grad.clone() for k, p in model.named_parameters()}
    model.zero_grad(set_to_none=True)
    loss_b = F.cross_entropy(model.forward_nctv(x), lab)
    loss_b.backward()
    assert abs(loss_a.item() - loss_b.item()) < 1e-5 * abs(loss_b.item())
    for k, p in model.named_parameters():
        if k.endswith("temporalConv.bias"):  # identically 0 (BN2 follows the conv)
            assert ga[k].abs().max().item() < 1e-6 and p.grad.abs().max().item() < 1e-6
            continue
        tight = k.startswith("fc_layer") or k.startswith("conv.9.")
        assert rel_to_max(ga[k].cpu().numpy(), p.grad.cpu().numpy()) < (1e-4 if tight else 2e-2), k


@pytest.mark.parametrize("wd", [0.0, 0.01])
def test_fused_adam_matches_torch_adam(pkg, wd):
    g = torch.Generator().manual_seed(3)
    shapes = [(64, 3, 1, 1), (64,), (1, 18, 18), (64, 64, 9, 1), (400, 256), (5000,)]
    p0 = [torch.randn(s, generator=g) for s in shapes]
    grads = [[torch.randn(s, generator=g) for s in shapes] for _ in range(5)]
    ref = [p.clone().requires_grad_(True) for p in p0]
    opt_ref = torch.optim.Adam(ref, lr=1e-2, weight_decay=wd, foreach=False)
    dut = [p.clone().to(DEV).requires_grad_(True) for p in p0]
    opt = pkg.FusedAdam(dut, lr=1e-2, weight_decay=wd)
    for k in range(5):
        for p, gr in zip(ref, grads[k]):
            p.grad = gr.clone()
        for p, gr in zip(dut, grads[k]):
            p.grad = gr.to(DEV)      # fresh grad tensors every step: table rebuilt
        opt_ref.step()
        opt.step()
    torch.cuda.synchronize()
    for a, b in zip(dut, ref):
        d = (a.detach().cpu() - b.detach()).abs()
        assert (d <= 2e-6 * b.detach().abs() + 1e-7).all(), float(d.max())
    for a, b in zip(dut, ref):
        for key in ("exp_avg", "exp_avg_sq"):
            sa, sb = opt.state[a][key].cpu(), opt_ref.state[b][key]
            err = rel_to_max(sa.numpy(), sb.numpy())
            assert err < 1e-6, (key, err)
        assert opt.state[a]["step"].item() == opt_ref.state[b]["step"].item()


def test_fused_adam_state_dict_interchanges_with_torch_adam(pkg):
    g = torch.Generator().manual_seed(4)
    w = torch.randn(32, 16, generator=g)
    ref = [w.clone().requires_grad_(True)]
    opt_ref = torch.optim.Adam(ref, lr=1e-3, foreach=False)
    ref[0].grad = torch.randn(32, 16, generator=g)
    opt_ref.step()
    dut = [w.clone().to(DEV).requires_grad_(True)]
    opt = pkg.FusedAdam(dut, lr=1e-3)
    sd = opt_ref.state_dict()
    sd["state"] = {k: {kk: (vv.to(DEV) if kk != "step" else vv.clone()) for kk, vv in v.items()}
                   for k, v in sd["state"].items()}
    opt.load_state_dict(sd)
    with torch.no_grad():
        dut[0].copy_(ref[0].detach().to(DEV))
    gr = torch.randn(32, 16, generator=g)
    ref[0].grad, dut[0].grad = gr.clone(), gr.to(DEV)
    opt_ref.step()
    opt.step()
    torch.cuda.synchronize()
    assert np.allclose(dut[0].detach().cpu().numpy(), ref[0].detach().numpy(), rtol=2e-6,
                       atol=1e-8)


def test_fused_adam_param_groups_keep_their_tables(pkg):
    """Two parameter groups (different lr / weight decay) with gradients that
    stay in place across steps (as with dp.GradAllReduce bucket views): each
    group keeps its own device table, and the result matches torch's Adam."""
    g = torch.Generator().manual_seed(5)
    shapes = [(64, 3, 1, 1), (64,), (1, 18, 18), (400, 256)]
    p0 = [torch.randn(s, generator=g) for s in shapes]
    grads = [[torch.randn(s, generator=g) for s in shapes] for _ in range(4)]
    ref = [p.clone().requires_grad_(True) for p in p0]
    dut = [p.clone().to(DEV).requires_grad_(True) for p in p0]
    groups = lambda ps: [dict(params=ps[:2], lr=1e-2), dict(params=ps[2:], lr=3e-3,  # noqa
                                                                weight_decay=0.1)]
    opt_ref = torch.optim.Adam(groups(ref), foreach=False)
    opt = pkg.FusedAdam(groups(dut))
    for p in dut:
        p.grad = torch.zeros_like(p)
    for k in range(4):
        for p, gr in zip(ref, grads[k]):
            p.grad = gr.clone()
        for p, gr in zip(dut, grads[k]):
            p.grad.copy_(gr.to(DEV))     # same grad tensors every step
        opt_ref.step()
        opt.step()
        if k == 0:
            tables = {gi: t[1].data_ptr() for gi, t in opt._tables.items()}
    torch.cuda.synchronize()
    assert sorted(opt._tables) == [0, 1]
    assert {gi: t[1].data_ptr() for gi, t in opt._tables.items()} == tables  # not rebuilt
    for a, b in zip(dut, ref):
        d = (a.detach().cpu() - b.detach()).abs()
        assert (d <= 2e-6 * b.detach().abs() + 1e-7).all(), float(d.max())

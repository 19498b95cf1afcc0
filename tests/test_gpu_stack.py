"""GPU: the full ST-GCN stack (STGCNStack = L_STGCN's conv stack + head) on
the fused HIP blocks, against the reference's cfg1 golden run
(tests/golden/stack_cfg1.npz: N=4, C=3, T=50, V=18, 2 classes, seed 0).

The 10-block stack amplifies fp32 rounding (test_oracle_golden.py documents
up to a few % between the fp32 reference and exact arithmetic on some
BN-affine / dA grads), so each gradient is gated at max(1e-4, 3x the fp32
reference's own distance from the fp64 oracle), measured per tensor.
"""
import io
import contextlib

import numpy as np
import pytest
import torch

from conftest import load_npz, rel_to_max
from oracle import ref_cpu

pytestmark = pytest.mark.gpu


def _oracle_grads(dtype, ref, A):
    p, b = ref_cpu.init_stack_params(3, 2, A, seed=0)
    p = {k: v.clone().to(dtype).requires_grad_(True) for k, v in p.items()}
    b = {k: (v.clone().to(dtype) if v.is_floating_point() else v.clone()) for k, v in b.items()}
    st = ref_cpu.Stack(p, b)
    logits = st.forward(torch.from_numpy(ref["x"]), dtype=dtype)
    loss = torch.nn.functional.cross_entropy(logits, torch.from_numpy(ref["labels"]))
    loss.backward()
    return logits.detach(), loss.detach(), {k: v.grad for k, v in p.items()}, b


STACK_TIE = 1e-4  # relative to max|pre-ReLU| of the block (10 blocks of fp32 rounding)


def capture_relu_masks(model):
    """Forward hooks collecting each block's ReLU mask (y > 0) of the next
    forward pass; returns (masks list, remove function)."""
    masks = []
    hs = [blk.register_forward_hook(lambda m, i, y: masks.append((y > 0).detach().cpu()))
          for blk in model.conv]
    return masks, lambda: [h.remove() for h in hs]


def oracle_through_masks(p0, b0, x_ntvc, labels, masks, dtype):
    """The oracle stack differentiated through the HIP run's ReLU masks (as the
    block tests do): (logits, loss, grads, pre-ReLU values per block)."""
    p = {k: v.clone().to(dtype).requires_grad_(True) for k, v in p0.items()}
    b = {k: (v.clone().to(dtype) if v.is_floating_point() else v.clone()) for k, v in b0.items()}
    st = ref_cpu.Stack(p, b)
    lg = st.forward(x_ntvc, dtype=dtype, relu_masks=masks)
    ls = torch.nn.functional.cross_entropy(lg, labels)
    ls.backward()
    return lg.detach(), ls.detach(), {k: v.grad for k, v in p.items()}, st.pre


def check_relu_ties(pre64, masks):
    """The HIP ReLU masks may differ from exact arithmetic only at ties."""
    for i, (pr, m) in enumerate(zip(pre64, masks)):
        flips = m != (pr > 0)
        if flips.any():
            band = STACK_TIE * pr.abs().max().item()
            assert pr[flips].abs().max().item() < band, \
                f"block {i}: ReLU mask differs away from a tie ({int(flips.sum())} flips)"


def gate_stack_grads(model, g64, g32, skip=("temporalConv.bias",)):
    bad = []
    for k, v in model.named_parameters():
        if k.startswith("Masks.") or any(k.endswith(s) for s in skip):
            continue
        want = g64[k].detach().double().numpy()
        floor = rel_to_max(g32[k].detach().double().numpy(), want)
        err = rel_to_max(v.grad.detach().cpu().double().numpy(), want)
        if err > max(1e-4, 3 * floor):
            bad.append(f"{k}: {err:.2e} (ref32 {floor:.2e})")
    assert not bad, "; ".join(bad)


def snapshot_stack(model):
    """(params, buffers) of a stack in state_dict naming, on the CPU: the
    oracle's starting point for a run of ``model``."""
    p0 = {k: v.detach().cpu().clone() for k, v in model.named_parameters()}
    b0 = {k: v.detach().cpu().clone() for k, v in model.named_buffers()}
    return p0, b0


def gate_chained_vs_oracle(model, p0, b0, x_nctv, lab, masks, gemm, residual=False):
    """The deferred-dx chain changes the arithmetic of the BN2 backward sums
    (formed from the spatial backward's mask sums instead of summing a
    materialised dx), so a chained run is no longer bit-close to the unchained
    one on the BN-affine / A gradients, which the 10-block stack conditions
    badly (the fp32 reference's own error reaches several %).
    Both are held to the fp64 oracle instead, through the chained run's ReLU
    masks: fp32 modes at max(1e-4, 3x the fp32 oracle's error) per tensor,
    bf16 at max(2e-2, 5x the bf16-operand oracle's error). (bf16: the first
    block's BN1 bias, the end of the deepest backward path, sits at 3.99x with
    the unfused V = 50 spatial backward and 4.47x with the fused k_sp50_dx/_dA
    pair on this seed, 2.4-3.1x on seeds 6 and 7, while the two kernels' block
    errors vs fp64 agree to 3 digits: profiles/r3_diag_bf16_v50.txt. The ratio
    of two independent bf16 rounding samples through a 10-block chain spreads
    that wide; 4x sat on the edge of it.)"""
    x_ntvc = x_nctv.detach().cpu().permute(0, 2, 3, 1).contiguous()
    lab = lab.cpu()

    def run(dtype, bf16):
        p = {k: v.clone().to(dtype).requires_grad_(True) for k, v in p0.items()}
        b = {k: (v.clone().to(dtype) if v.is_floating_point() else v.clone())
             for k, v in b0.items()}
        st = ref_cpu.Stack(p, b, residual=residual)
        lg = st.forward(x_ntvc, dtype=dtype, gemm_bf16=bf16,
                        relu_masks=[m.to(dtype) for m in masks])
        torch.nn.functional.cross_entropy(lg, lab).backward()
        return {k: v.grad for k, v in p.items()}

    g64 = run(torch.float64, False)
    gref = run(torch.float32, gemm == "bf16")
    lim, fac = (2e-2, 5.0) if gemm == "bf16" else (1e-4, 3.0)
    bad = []
    for k, v in model.named_parameters():
        if k.startswith("Masks.") or k.endswith("temporalConv.bias"):
            continue
        want = g64[k].detach().double().numpy()
        floor = rel_to_max(gref[k].detach().double().numpy(), want)
        err = rel_to_max(v.grad.detach().cpu().double().numpy(), want)
        if err > max(lim, fac * floor):
            bad.append(f"{k}: {err:.2e} (ref {floor:.2e})")
    assert not bad, "; ".join(bad)


def test_stack_cfg1_matches_reference(pkg):
    ref = load_npz("stack_cfg1.npz")
    A = torch.from_numpy(load_npz("adjacency.npz")["V18_s0_d1"])
    torch.manual_seed(0)
    with contextlib.redirect_stdout(io.StringIO()):
        model = pkg.STGCNStack(3, 2, A)
    # same init as the reference (same module construction order)
    for k, v in model.named_parameters():
        flat = v.detach().reshape(-1)
        np.testing.assert_array_equal(flat[torch.as_tensor(ref["pidx." + k])].numpy(),
                                      ref["pval." + k])
    model = model.cuda().train()
    x = torch.from_numpy(ref["x"]).cuda()
    y = torch.from_numpy(ref["labels"]).cuda()
    logits = model(x)
    loss = torch.nn.functional.cross_entropy(logits, y)
    loss.backward()
    torch.cuda.synchronize()

    l64, loss64, g64, b64 = _oracle_grads(torch.float64, ref, A)
    l32, loss32, g32, _ = _oracle_grads(torch.float32, ref, A)
    assert rel_to_max(logits.detach().cpu().numpy(), ref["logits"]) < 1e-4
    assert abs(loss.item() - float(ref["loss"])) < 1e-5
    bad = []
    for k, v in model.named_parameters():
        got = v.grad.detach().cpu().double()
        if k.endswith("temporalConv.bias"):
            assert got.abs().max().item() < 1e-5, k
            continue
        want = g64[k].detach().double()
        floor = rel_to_max(g32[k].detach().double().numpy(), want.numpy())
        err = rel_to_max(got.numpy(), want.numpy())
        if err > max(1e-4, 3 * floor):
            bad.append(f"{k}: {err:.2e} (ref32 {floor:.2e})")
    assert not bad, "; ".join(bad)
    # running statistics after one training step
    for k, v in model.state_dict().items():
        if "running" in k:
            assert rel_to_max(v.cpu().numpy(), ref["after." + k]) < 1e-4, k


@pytest.mark.parametrize("residual,gemm", [(False, "fp32"), (True, "fp32"), (False, "bf16"),
                                            (False, "x3"), (True, "x3"), (False, "f16")])
def test_stack_chain_small_bn2_gamma(pkg, residual, gemm):
    """The chain link with BN2 gammas at 0 and 1e-4 on some channels of every
    block: rebuilding uhat = (y - b2) / g2 from the block
    output is ill-conditioned there, so the link must read U for those channels.
    Chained and unchained runs agree at the same gates as above. ADVICE round
    2: also on the benched stacks -- bf16 (V = 25, K = 3: U from the fused
    epilogues, dx from k_sp_bwd_fused; bf16 gate) and bf16x3 (fp32 gates)."""
    gr = pkg.graph
    if gemm == "bf16":
        V = 25
        A = gr.get_normalized_adjacency_matrices(2, 1, distances=gr.synthetic_distances(V),
                                                 graph=gr.graph_for(V))
    else:
        V = 18
        A = gr.get_normalized_adjacency_matrices(0, 1, graph=gr.graph_for(V))
    kw = dict(residual=residual,
              gemm_dtype=torch.bfloat16 if gemm == "bf16" else torch.float32,
              f32_gemm={"x3": "bf16x3", "f16": "f16x2"}.get(gemm, "mfma"))
    torch.manual_seed(11)
    with contextlib.redirect_stdout(io.StringIO()):
        m1 = pkg.STGCNStack(3, 10, A, **kw).cuda().train()
        m2 = pkg.STGCNStack(3, 10, A, **kw).cuda().train()
    with torch.no_grad():
        for blk in m1.conv:
            g = blk.batch_n_2.weight
            g[0:2] = 0.0
            g[2:4] = 1e-4
            g[4:6] = -1e-4
            blk.batch_n_2.bias[0:6] = torch.linspace(-0.5, 0.5, 6)
    m2.load_state_dict(m1.state_dict())
    p0, b0 = snapshot_stack(m1)
    x = torch.randn(6, 3, 40, V, generator=torch.Generator().manual_seed(12)).cuda()
    lab = torch.randint(0, 10, (6,), generator=torch.Generator().manual_seed(13)).cuda()
    masks, unhook = capture_relu_masks(m1)
    out1 = m1.forward_nctv(x)                      # chained
    unhook()
    h = x
    for blk in m2.conv:                            # unchained
        h = blk(h)
    out2 = m2.fc_layer(h.flatten(2).mean(dim=2))
    torch.nn.functional.cross_entropy(out1, lab).backward()
    torch.nn.functional.cross_entropy(out2, lab).backward()
    torch.cuda.synchronize()
    assert rel_to_max(out1.detach().cpu().numpy(), out2.detach().cpu().numpy()) < \
        (1e-3 if gemm == "bf16" else 1e-5)
    for k, a in m1.named_parameters():
        assert torch.isfinite(a.grad).all(), k
    if not residual:  # deferred dx: both runs against the fp64 oracle
        gate_chained_vs_oracle(m1, p0, b0, x, lab, masks, gemm)
        return
    bad = []
    for (k, a), (_, b) in zip(m1.named_parameters(), m2.named_parameters()):
        ga, gb = a.grad.detach().cpu().double().numpy(), b.grad.detach().cpu().double().numpy()
        if np.abs(gb).max() == 0:
            continue
        tol = 2e-3 if k.endswith("spatialConv.A") else 1e-4
        err = rel_to_max(ga, gb)
        if err > tol:
            bad.append(f"{k}: {err:.2e} > {tol:.0e}")
    assert not bad, "; ".join(bad)


@pytest.mark.parametrize("residual,drop", [(False, 0), (True, 0), (False, 0.5), (True, 0.3)])
def test_stack_chain_matches_unchained(pkg, residual, drop):
    """Cross-block fusion (network.StackChain: BN1 stats from the previous
    block's output pass, the previous block's ReLU+BN2 reduction from the next
    block's dx pass) gives the same results as running the blocks one by one,
    with and without the fused dropout (same per-block seeds in both runs)."""
    gr = pkg.graph
    A = gr.get_normalized_adjacency_matrices(0, 1, graph=gr.graph_for(18))
    torch.manual_seed(3)
    with contextlib.redirect_stdout(io.StringIO()):
        m1 = pkg.STGCNStack(3, 10, A, dropout_rate=drop, residual=residual).cuda().train()
        m2 = pkg.STGCNStack(3, 10, A, dropout_rate=drop, residual=residual).cuda().train()
    m2.load_state_dict(m1.state_dict())
    p0, b0 = snapshot_stack(m1)
    x = torch.randn(6, 3, 40, 18, generator=torch.Generator().manual_seed(4)).cuda()
    lab = torch.randint(0, 10, (6,), generator=torch.Generator().manual_seed(5)).cuda()
    masks, unhook = capture_relu_masks(m1)
    torch.manual_seed(9)
    out1 = m1.forward_nctv(x)                      # chained
    unhook()
    torch.manual_seed(9)
    h = x
    for blk in m2.conv:                            # unchained
        h = blk(h)
    out2 = m2.fc_layer(h.flatten(2).mean(dim=2))
    torch.nn.functional.cross_entropy(out1, lab).backward()
    torch.nn.functional.cross_entropy(out2, lab).backward()
    torch.cuda.synchronize()
    assert rel_to_max(out1.detach().cpu().numpy(), out2.detach().cpu().numpy()) < 1e-5
    for (k, a), (_, b) in zip(m1.named_buffers(), m2.named_buffers()):
        if a.is_floating_point():
            assert rel_to_max(a.cpu().numpy(), b.cpu().numpy()) < 1e-5, k
    if not residual and drop == 0:  # deferred dx: both runs against the fp64 oracle
        gate_chained_vs_oracle(m1, p0, b0, x, lab, masks, "fp32")
        return
    # dA of the deep blocks is a small difference of large terms (BN makes the
    # loss invariant to A's scale: |dA| ~ 1e-11 here) -- gated looser
    bad = []
    for (k, a), (_, b) in zip(m1.named_parameters(), m2.named_parameters()):
        ga, gb = a.grad.detach().cpu().double().numpy(), b.grad.detach().cpu().double().numpy()
        if np.abs(gb).max() == 0:
            continue
        if k.endswith("temporalConv.bias") and not residual:  # analytically 0: rounding noise
            assert np.abs(ga).max() < 1e-4, (k, np.abs(ga).max())
            continue
        tol = 2e-3 if k.endswith("spatialConv.A") else 1e-4
        err = rel_to_max(ga, gb)
        if err > tol:
            bad.append(f"{k}: {err:.2e} > {tol:.0e}")
    assert not bad, "; ".join(bad)
    for (k, a), (_, b) in zip(m1.named_buffers(), m2.named_buffers()):
        if a.is_floating_point():
            assert rel_to_max(a.cpu().numpy(), b.cpu().numpy()) < 1e-5, k


@pytest.mark.parametrize("V,K,gemm,T", [(18, 1, "fp32", 40), (18, 1, "x3", 300),
                                         (18, 1, "f16", 300),
                                         # the reference's default graph: V = 25,
                                         # unilabeling (K = 1), folded, unfused
                                         # SpatialConv backward
                                         (25, 1, "f16", 60), (25, 1, "x3", 40),
                                         (25, 3, "bf16", 40), (50, 3, "bf16", 24),
                                         (25, 3, "fp32", 40)])
def test_stack_deferred_dx_matches_unchained(pkg, monkeypatch, V, K, gemm, T):
    """ABI 5 deferred dx: inside the chained stack every block's BN1 backward
    apply is folded into the previous block's ReLU+BN2 backward pass (dx keeps
    dxhat; the spatial backward reads the previous block's U: k_spatial_bwd5 at
    V = 18 / 25 fp32, k_sp_bwd_fused at V = 25 bf16, k_spatial_bwd6 at V = 50).
    The chained stack must equal the blocks run one by one, and the deferral
    must have run on every link."""
    gr = pkg.graph
    if K == 1:
        A = gr.get_normalized_adjacency_matrices(0, 1, graph=gr.graph_for(V))
    else:
        A = gr.get_normalized_adjacency_matrices(2, 1, distances=gr.synthetic_distances(V),
                                                 graph=gr.graph_for(V))
    kw = dict(gemm_dtype=torch.bfloat16 if gemm == "bf16" else torch.float32,
              f32_gemm={"x3": "bf16x3", "f16": "f16x2"}.get(gemm, "mfma"))
    deferred = []
    orig = pkg.fused._chain_publish

    def spy(cc, prev_sums, dx, dx_coef=None):
        if prev_sums is not None:
            deferred.append(dx_coef is not None)
        return orig(cc, prev_sums, dx, dx_coef)

    monkeypatch.setattr(pkg.fused, "_chain_publish", spy)
    torch.manual_seed(5)
    with contextlib.redirect_stdout(io.StringIO()):
        m1 = pkg.STGCNStack(3, 10, A, **kw).cuda().train()
        m2 = pkg.STGCNStack(3, 10, A, **kw).cuda().train()
    m2.load_state_dict(m1.state_dict())
    p0, b0 = snapshot_stack(m1)
    N = 4
    x = torch.randn(N, 3, T, V, generator=torch.Generator().manual_seed(6)).cuda()
    lab = torch.randint(0, 10, (N,), generator=torch.Generator().manual_seed(7)).cuda()
    masks, unhook = capture_relu_masks(m1)
    out1 = m1.forward_nctv(x)                      # chained (deferred dx)
    unhook()
    h = x
    for blk in m2.conv:                            # unchained
        h = blk(h)
    out2 = m2.fc_layer(h.flatten(2).mean(dim=2))
    torch.nn.functional.cross_entropy(out1, lab).backward()
    torch.nn.functional.cross_entropy(out2, lab).backward()
    torch.cuda.synchronize()
    assert deferred == [True] * 9, deferred        # blocks 9..1 each deferred their dx
    assert rel_to_max(out1.detach().cpu().numpy(), out2.detach().cpu().numpy()) < \
        (1e-3 if gemm == "bf16" else 1e-5)
    for k, a in m1.named_parameters():
        assert torch.isfinite(a.grad).all(), k
        if k.endswith("temporalConv.bias"):  # analytically 0: rounding noise
            assert a.grad.abs().max().item() < (1e-3 if gemm == "bf16" else 1e-4), k
    gate_chained_vs_oracle(m1, p0, b0, x, lab, masks, gemm)


@pytest.mark.parametrize("observe", ["hook", "retain_grad", "replace"])
def test_stack_observed_intermediate_gradient(pkg, monkeypatch, observe):
    """A hook or retain_grad() on a block output between two chained blocks
    turns the deferred dx off for that link: the observer sees the true
    gradient of that output (equal to an unchained run's), a hook that
    replaces the tensor is honoured, and the other eight links still defer."""
    gr = pkg.graph
    A = gr.get_normalized_adjacency_matrices(0, 1, graph=gr.graph_for(18))
    deferred = []
    orig = pkg.fused._chain_publish

    def spy(cc, prev_sums, dx, dx_coef=None):
        if prev_sums is not None:
            deferred.append(dx_coef is not None)
        return orig(cc, prev_sums, dx, dx_coef)

    monkeypatch.setattr(pkg.fused, "_chain_publish", spy)
    torch.manual_seed(5)
    with contextlib.redirect_stdout(io.StringIO()):
        m1 = pkg.STGCNStack(3, 10, A).cuda().train()
        m2 = pkg.STGCNStack(3, 10, A).cuda().train()
    m2.load_state_dict(m1.state_dict())
    x = torch.randn(2, 3, 20, 18, generator=torch.Generator().manual_seed(6)).cuda()
    seen = []

    def run(m, chained):
        chain = pkg.network.StackChain() if chained else None
        h, mid = x, None
        for i, blk in enumerate(m.conv):
            h = blk(h, chain=chain) if chained else blk(h)
            if i == 4:
                mid = h
                if observe == "retain_grad":
                    h.retain_grad()
                elif observe == "hook":
                    h.register_hook(lambda g: seen.append(g.detach().clone()))
                else:
                    h.register_hook(lambda g: g * 2.0)  # a new tensor replaces the gradient
        h.sum().backward()
        torch.cuda.synchronize()
        return mid

    mid1 = run(m1, True)
    n_chained = len(deferred)
    mid2 = run(m2, False)
    assert deferred[:n_chained].count(False) == 1 and deferred[:n_chained].count(True) == 8
    if observe == "retain_grad":
        assert rel_to_max(mid1.grad.cpu().numpy(), mid2.grad.cpu().numpy()) < 1e-4
    elif observe == "hook":
        assert len(seen) == 2
        assert rel_to_max(seen[0].cpu().numpy(), seen[1].cpu().numpy()) < 1e-4
    for (k, a), b in zip(m1.named_parameters(), m2.parameters()):
        if a.grad is None:  # (parameters the loss does not reach)
            assert b.grad is None, k
            continue
        ga, gb = a.grad.cpu().numpy(), b.grad.cpu().numpy()
        if k.endswith("temporalConv.bias"):  # (analytically zero: rounding noise on both sides)
            assert np.abs(ga - gb).max() < 1e-6, k
            continue
        assert rel_to_max(ga, gb) < 2e-2, k


def test_stack_bf16_cfg3_shape(pkg):
    """cfg3 (NTU V=25, K=3 spatial partitioning, 60 classes) stack with bf16
    channel GEMMs at N=4, T=40, one training step: logits and loss against the
    fp64 oracle gated at max(2e-2, 3x the reference's own error when its convs
    run with bf16 operands (ref_cpu gemm_bf16)); every parameter gradient at
    max(2e-2, 4x that floor). The stack's ReLUs flip at bf16 ties in every
    bf16 implementation and the two implementations round at different points
    (the fused block rounds the joint-averaged G, the reference BN1(x)), so
    their errors are independent samples; the worst case measured is the
    first block's BN1 weight gradient (the end of the deepest backward path):
    20.7% here vs the bf16 reference's own 6.5% (3.2x), every other tensor
    within 3x."""
    gr = pkg.graph
    V, classes = 25, 60
    A = gr.get_normalized_adjacency_matrices(2, 1, distances=gr.synthetic_distances(V),
                                             graph=gr.graph_for(V))
    torch.manual_seed(0)
    with contextlib.redirect_stdout(io.StringIO()):
        model = pkg.STGCNStack(3, classes, A, gemm_dtype=torch.bfloat16)
    x = torch.randn(4, 40, V, 3, generator=torch.Generator().manual_seed(1))
    lab = torch.randint(0, classes, (4,), generator=torch.Generator().manual_seed(2))
    params0 = {k: v.detach().clone() for k, v in model.named_parameters()}
    model = model.cuda().train()
    logits = model(x.cuda())
    loss = torch.nn.functional.cross_entropy(logits, lab.cuda())
    loss.backward()
    torch.cuda.synchronize()

    def oracle(dtype, bf16):
        p = {k: v.clone().to(dtype).requires_grad_(True) for k, v in params0.items()}
        _, b = ref_cpu.init_stack_params(3, classes, A, seed=0)
        b = {k: (v.clone().to(dtype) if v.is_floating_point() else v.clone())
             for k, v in b.items()}
        lg = ref_cpu.Stack(p, b).forward(x, dtype=dtype, gemm_bf16=bf16)
        ls = torch.nn.functional.cross_entropy(lg, lab)
        ls.backward()
        return lg.detach(), ls.detach(), {k: v.grad for k, v in p.items()}

    l64, loss64, g64 = oracle(torch.float64, False)
    l16, loss16, g16 = oracle(torch.float32, True)
    lerr = rel_to_max(logits.detach().cpu().numpy(), l64.numpy())
    lfloor = rel_to_max(l16.numpy(), l64.numpy())
    assert lerr < max(2e-2, 3 * lfloor), (lerr, lfloor)
    assert abs(loss.item() - loss64.item()) < max(2e-2, 3 * abs(loss16.item() - loss64.item()))
    bad, worst = [], 0.0
    for k, v in model.named_parameters():
        got = v.grad.detach().cpu().double()
        if k.endswith("temporalConv.bias"):
            assert got.abs().max().item() < 1e-3, k
            continue
        want = g64[k].detach().double()
        floor = rel_to_max(g16[k].detach().double().numpy(), want.numpy())
        err = rel_to_max(got.numpy(), want.numpy())
        worst = max(worst, err)
        if err > max(2e-2, 4 * floor):
            bad.append(f"{k}: {err:.2e} (ref bf16 {floor:.2e})")
    print("logits", lerr, "worst grad", worst)
    assert not bad, "; ".join(bad)


# --- the exact benched configuration (round 2) --------------------------------

@pytest.mark.parametrize("f32_gemm", ["bf16x3", "f16x2", "f16x2-nog"])
def test_stack_cfg1_benched_path_matches_reference(pkg, f32_gemm):
    """bench.py's step on the cfg1 golden case: STGCNStack(f32_gemm="bf16x3")
    (temporal GEMMs as exact bf16 splits) or "f16x2" (the folded blocks' GEMMs
    as scaled 2-way fp16 splits), StackChain cross-block fusion and the
    fused HIP head (forward_loss: avg-pool + Linear + cross entropy). Logits and
    loss against the reference's fixture; gradients against the fp64 oracle
    differentiated through the HIP run's ReLU masks (which may differ from
    exact arithmetic only at ties), per tensor at max(1e-4, 3x the fp32
    oracle's own error through the same masks)."""
    ref = load_npz("stack_cfg1.npz")
    A = torch.from_numpy(load_npz("adjacency.npz")["V18_s0_d1"])
    torch.manual_seed(0)
    with contextlib.redirect_stdout(io.StringIO()):
        model = pkg.STGCNStack(3, 2, A, f32_gemm=f32_gemm)
    model = model.cuda().train()
    masks, unhook = capture_relu_masks(model)
    x = torch.from_numpy(ref["x"]).cuda().permute(0, 3, 1, 2).contiguous()
    y = torch.from_numpy(ref["labels"]).cuda()
    loss, logits = model.forward_loss(x, y)
    loss.backward()
    torch.cuda.synchronize()
    unhook()
    assert rel_to_max(logits.detach().cpu().numpy(), ref["logits"]) < 1e-4
    assert abs(loss.item() - float(ref["loss"])) < 1e-5
    p0, b0 = ref_cpu.init_stack_params(3, 2, A, seed=0)
    xr, lab = torch.from_numpy(ref["x"]), torch.from_numpy(ref["labels"])
    _, _, g64, pre64 = oracle_through_masks(p0, b0, xr, lab, masks, torch.float64)
    _, _, g32, _ = oracle_through_masks(p0, b0, xr, lab, masks, torch.float32)
    check_relu_ties(pre64, masks)
    for k, v in model.named_parameters():
        if k.endswith("temporalConv.bias"):
            assert v.grad.abs().max().item() < 1e-5, k
    gate_stack_grads(model, g64, g32)
    for k, v in model.state_dict().items():
        if "running" in k:
            assert rel_to_max(v.cpu().numpy(), ref["after." + k]) < 1e-4, k


@pytest.mark.parametrize("residual,f32_gemm", [(False, "bf16x3"), (True, "bf16x3"),
                                               (False, "f16x2"), (False, "f16x2-nog")])
def test_stack_chain_matches_unchained_bf16x3(pkg, residual, f32_gemm):
    """StackChain in the benched bf16x3 mode (at the bench's T = 300) gives the
    same results as the blocks run one by one, through the fused head."""
    gr = pkg.graph
    A = gr.get_normalized_adjacency_matrices(0, 1, graph=gr.graph_for(18))
    torch.manual_seed(3)
    with contextlib.redirect_stdout(io.StringIO()):
        m1 = pkg.STGCNStack(3, 400, A, residual=residual, f32_gemm=f32_gemm).cuda().train()
        m2 = pkg.STGCNStack(3, 400, A, residual=residual, f32_gemm=f32_gemm).cuda().train()
    m2.load_state_dict(m1.state_dict())
    x = torch.randn(4, 3, 300, 18, generator=torch.Generator().manual_seed(4)).cuda()
    lab = torch.randint(0, 400, (4,), generator=torch.Generator().manual_seed(5)).cuda()
    loss1, out1 = m1.forward_loss(x, lab)                 # chained + fused head
    h = x
    for blk in m2.conv:                                  # unchained + torch head
        h = blk(h)
    out2 = m2.fc_layer(h.flatten(2).mean(dim=2))
    loss2 = torch.nn.functional.cross_entropy(out2, lab)
    loss1.backward()
    loss2.backward()
    torch.cuda.synchronize()
    assert rel_to_max(out1.detach().cpu().numpy(), out2.detach().cpu().numpy()) < 1e-5
    assert abs(loss1.item() - loss2.item()) < 1e-5
    # (the fused head's dy differs from torch's head in the last bits; BN2's
    # weight gradient of a block followed by another block's BatchNorm is
    # analytically 0 with the default affine (sum dx * y, dx orthogonal to the
    # normalised y), so its rounding noise is measured against the scale of
    # the same block's BN2 bias gradient)
    ga_all = {k: a.grad.detach().cpu().double().numpy() for k, a in m1.named_parameters()}
    gb_all = {k: b.grad.detach().cpu().double().numpy() for k, b in m2.named_parameters()}
    bad = []
    for k, gb in gb_all.items():
        ga = ga_all[k]
        if np.abs(gb).max() == 0 or k.endswith("temporalConv.bias"):  # (analytically 0)
            continue
        tol = 2e-3 if k.endswith("spatialConv.A") else 1e-4
        if k.endswith("batch_n_2.weight"):
            scale = max(np.abs(gb).max(), np.abs(gb_all[k[:-len("weight")] + "bias"]).max())
            err = np.abs(ga - gb).max() / scale
        elif residual and k.endswith("spatialConv.W.bias"):
            # residual block: BN2 normalises the spatial output, so the W bias
            # gradient is analytically 0 as well (scale: the W weight gradient)
            scale = max(np.abs(gb).max(), np.abs(gb_all[k[:-len("bias")] + "weight"]).max())
            err = np.abs(ga - gb).max() / scale
        else:
            err = rel_to_max(ga, gb)
        if err > tol:
            bad.append(f"{k}: {err:.2e} > {tol:.0e}")
    assert not bad, "; ".join(bad)


def _bf16_stack_errors(pkg, V, seed, N, T, classes=60):
    """One bf16 stack training step (K = 3 spatial partitioning) vs the fp64
    oracle, and the reference's own bf16-operand error (ref_cpu gemm_bf16) on
    the same inputs: ({tensor: err}, {tensor: floor})."""
    gr = pkg.graph
    A = gr.get_normalized_adjacency_matrices(2, 1, distances=gr.synthetic_distances(V),
                                             graph=gr.graph_for(V))
    torch.manual_seed(seed)
    with contextlib.redirect_stdout(io.StringIO()):
        model = pkg.STGCNStack(3, classes, A, gemm_dtype=torch.bfloat16)
    x = torch.randn(N, T, V, 3, generator=torch.Generator().manual_seed(seed + 1))
    lab = torch.randint(0, classes, (N,), generator=torch.Generator().manual_seed(seed + 2))
    params0 = {k: v.detach().clone() for k, v in model.named_parameters()}
    model = model.cuda().train()
    loss, logits = model.forward_loss(x.cuda().permute(0, 3, 1, 2).contiguous(), lab.cuda())
    loss.backward()
    torch.cuda.synchronize()

    def oracle(dtype, bf16):
        p = {k: v.clone().to(dtype).requires_grad_(True) for k, v in params0.items()}
        _, b = ref_cpu.init_stack_params(3, classes, A, seed=seed)
        b = {k: (v.clone().to(dtype) if v.is_floating_point() else v.clone())
             for k, v in b.items()}
        lg = ref_cpu.Stack(p, b).forward(x, dtype=dtype, gemm_bf16=bf16)
        ls = torch.nn.functional.cross_entropy(lg, lab)
        ls.backward()
        return lg.detach(), ls.detach(), {k: v.grad for k, v in p.items()}

    l64, loss64, g64 = oracle(torch.float64, False)
    l16, loss16, g16 = oracle(torch.float32, True)
    errs = {"logits": rel_to_max(logits.detach().cpu().numpy(), l64.numpy()),
            "loss": abs(loss.item() - loss64.item())}
    floor = {"logits": rel_to_max(l16.numpy(), l64.numpy()),
             "loss": abs(loss16.item() - loss64.item())}
    for k, v in model.named_parameters():
        if k.endswith("temporalConv.bias"):
            assert v.grad.abs().max().item() < 1e-3, k
            continue
        want = g64[k].detach().double().numpy()
        errs[k] = rel_to_max(v.grad.detach().cpu().double().numpy(), want)
        floor[k] = rel_to_max(g16[k].detach().double().numpy(), want)
    return errs, floor


@pytest.mark.parametrize("V", [25, 50])
def test_stack_bf16_multi_seed(pkg, V):
    """cfg3 (V = 25) / cfg5 (V = 50) stacks with bf16 channel GEMMs through the
    benched path (StackChain + fused head), over three seeds at N = 8, T = 40.
    A single seed is a poor gate: the stack's ReLUs flip at bf16 ties and the
    deepest backward paths (first blocks' BN1 affine / dA) resample with any
    change of rounding upstream. Gate per tensor: the HIP error averaged over
    the seeds within max(2e-2, 2.5x the averaged error of the reference run
    with bf16 conv operands), and no single seed beyond max(2e-2, 4x the
    worst reference seed)."""
    seeds = (0, 10, 20)
    runs = [_bf16_stack_errors(pkg, V, s, N=8, T=40) for s in seeds]
    bad, ratios = [], {}
    for k in runs[0][0]:
        e = np.array([r[0][k] for r in runs])
        f = np.array([r[1][k] for r in runs])
        ratios[k] = e.mean() / max(f.mean(), 1e-30)
        if e.mean() > max(2e-2, 2.5 * f.mean()) or e.max() > max(2e-2, 4 * f.max()):
            bad.append(f"{k}: mean {e.mean():.2e} max {e.max():.2e} "
                       f"(ref bf16 mean {f.mean():.2e} max {f.max():.2e})")
    worst = sorted(ratios.items(), key=lambda kv: -kv[1])[:5]
    print(f"V={V} worst mean err / ref-bf16 floor:", [(k, round(r, 2)) for k, r in worst])
    assert not bad, "; ".join(bad)


@pytest.mark.gpu
@pytest.mark.parametrize("f32_gemm", ["f16x2", "bf16x3"])
def test_stack_lazy_links_bit_identical(pkg, f32_gemm):
    """ABI 8 (STGCN_PLAN_X_FROM_U): inside the training stack a block output that
    only the next block reads is never written -- the block writes only y's
    statistics (k_bn_relu_stats) and the next block's gather forms
    ReLU(BN2(U)) from U as k_bn_relu_fwd would. The step must be bit-identical
    to the stack that writes every output (loss, logits, running stats and
    every gradient), and a forward hook on a block keeps that block's output
    (and its input) written and exact."""
    gr = pkg.graph
    A = gr.get_normalized_adjacency_matrices(0, 1, graph=gr.graph_for(18))
    torch.manual_seed(3)
    with contextlib.redirect_stdout(io.StringIO()):
        m1 = pkg.STGCNStack(3, 400, A, f32_gemm=f32_gemm).cuda().train()
        m2 = pkg.STGCNStack(3, 400, A, f32_gemm=f32_gemm).cuda().train()
    m2.load_state_dict(m1.state_dict())
    m2.lazy_links = False
    x = torch.randn(4, 3, 300, 18, generator=torch.Generator().manual_seed(4)).cuda()
    lab = torch.randint(0, 400, (4,), generator=torch.Generator().manual_seed(5)).cuda()
    flags = pkg.fused.lazy_links(list(m1.conv), tuple(x.shape))
    assert flags == [True] * 9 + [False], flags
    seen = {}
    hook = m1.conv[4].register_forward_hook(lambda m, i, o: seen.__setitem__("y4", o.clone()))
    flags_h = pkg.fused.lazy_links(list(m1.conv), tuple(x.shape))
    assert flags_h == [True] * 3 + [False, False] + [True] * 4 + [False], flags_h
    hook.remove()
    for step in range(2):
        hooks = []
        if step == 1:  # an observed output: written, and the same as the unlazy stack's
            for m, key in ((m1, "y4"), (m2, "y4_ref")):
                hooks.append(m.conv[4].register_forward_hook(
                    lambda mod, i, o, key=key: seen.__setitem__(key, o.detach().clone())))
        loss1, out1 = m1.forward_loss(x, lab)
        loss2, out2 = m2.forward_loss(x, lab)
        for h in hooks:
            h.remove()
        m1.zero_grad()
        m2.zero_grad()
        loss1.backward()
        loss2.backward()
        torch.cuda.synchronize()
        assert torch.equal(out1, out2) and torch.equal(loss1, loss2), step
        # every gradient bit-identical: dA is summed from per-workgroup partials
        # in a fixed order (launch_dA_reduce), not by fp32 atomics
        g2 = {k: b.grad for k, b in m2.named_parameters()}
        for k, a in m1.named_parameters():
            assert torch.equal(a.grad, g2[k]), (step, k)
        for (k, a), b in zip(m1.named_buffers(), m2.buffers()):
            assert torch.equal(a, b), (step, k)
        if step == 1:
            assert torch.equal(seen["y4"], seen["y4_ref"])


@pytest.mark.parametrize("f32_gemm", ["f16x2", "mfma"])
def test_stack_head_pools_from_u(pkg, f32_gemm):
    """ABI 9 (stgcn_head_fwd_u): in a training step the last block's output is
    read only by the fused head, so neither it nor its statistics are formed;
    the head pools ReLU(BN2(U)) from the last block's U. Loss and logits are
    bit-identical to the stack that writes every output; a forward hook on the
    last block brings the written output back (and the hook sees it)."""
    gr = pkg.graph
    A = gr.get_normalized_adjacency_matrices(0, 1, graph=gr.graph_for(18))
    torch.manual_seed(5)
    with contextlib.redirect_stdout(io.StringIO()):
        m1 = pkg.STGCNStack(3, 60, A, f32_gemm=f32_gemm).cuda().train()
        m2 = pkg.STGCNStack(3, 60, A, f32_gemm=f32_gemm).cuda().train()
    m2.load_state_dict(m1.state_dict())
    m2.lazy_links = False
    x = torch.randn(3, 3, 64, 18, generator=torch.Generator().manual_seed(6)).cuda()
    lab = torch.randint(0, 60, (3,), generator=torch.Generator().manual_seed(7)).cuda()
    lib = pkg.hip_lib.lib()
    orig = lib.stgcn_head_fwd_u
    calls = []

    def counted(*a):
        calls.append(1)
        return orig(*a)
    lib.stgcn_head_fwd_u = counted
    try:
        for step in range(3):
            seen = {}
            hooks = []
            if step == 2:  # observed last output: written, the ordinary head
                hooks = [m.conv[-1].register_forward_hook(
                    lambda mod, i, o, key=key: seen.__setitem__(key, o.detach().clone()))
                    for m, key in ((m1, "y"), (m2, "y_ref"))]
            n0 = len(calls)
            loss1, out1 = m1.forward_loss(x, lab)
            n1 = len(calls)
            loss2, out2 = m2.forward_loss(x, lab)
            assert len(calls) == n1, "the unlazy stack must use the ordinary head"
            assert n1 - n0 == (0 if step == 2 else 1), step
            for h in hooks:
                h.remove()
            m1.zero_grad()
            m2.zero_grad()
            loss1.backward()
            loss2.backward()
            torch.cuda.synchronize()
            assert torch.equal(out1, out2) and torch.equal(loss1, loss2), step
            g2 = {k: b.grad for k, b in m2.named_parameters()}
            for k, a in m1.named_parameters():  # (dA from ordered partials: exact)
                assert torch.equal(a.grad, g2[k]), (step, k)
            for (k, a), b in zip(m1.named_buffers(), m2.buffers()):
                assert torch.equal(a, b), (step, k)
            if step == 2:
                assert torch.equal(seen["y"], seen["y_ref"])
    finally:
        lib.stgcn_head_fwd_u = orig


@pytest.mark.gpu
def test_stack_frozen_first_blocks(pkg):
    """with blocks 0-1 frozen (fine-tuning the later ones) and an
    input that needs no gradient, block 1's output needs no gradient either, so
    block 2's backward cannot defer its dx into block 1: the chain must write
    that output instead of leaving it to be formed from U (ABI 8), and the
    backward must run. Same loss, logits and trainable gradients as the stack
    that writes every output; the frozen blocks get no gradient."""
    gr = pkg.graph
    A = gr.get_normalized_adjacency_matrices(0, 1, graph=gr.graph_for(18))
    torch.manual_seed(8)
    with contextlib.redirect_stdout(io.StringIO()):
        m1 = pkg.STGCNStack(3, 60, A, f32_gemm="f16x2").cuda().train()
        m2 = pkg.STGCNStack(3, 60, A, f32_gemm="f16x2").cuda().train()
    m2.load_state_dict(m1.state_dict())
    m2.lazy_links = False
    for m in (m1, m2):
        m.conv[0].requires_grad_(False)
        m.conv[1].requires_grad_(False)
    x = torch.randn(3, 3, 64, 18, generator=torch.Generator().manual_seed(9)).cuda()
    lab = torch.randint(0, 60, (3,), generator=torch.Generator().manual_seed(10)).cuda()
    for step in range(2):
        loss1, out1 = m1.forward_loss(x, lab)
        loss2, out2 = m2.forward_loss(x, lab)
        m1.zero_grad()
        m2.zero_grad()
        loss1.backward()
        loss2.backward()
        torch.cuda.synchronize()
        assert torch.equal(out1, out2) and torch.equal(loss1, loss2), step
        g2 = {k: b.grad for k, b in m2.named_parameters()}
        for k, a in m1.named_parameters():
            if not a.requires_grad:
                assert a.grad is None and g2[k] is None, k
                continue
            assert torch.equal(a.grad, g2[k]), (step, k)


@pytest.mark.gpu
@pytest.mark.parametrize("V", [25, 50])
def test_stack_lazy_links_bf16(pkg, V):
    """ABI 8 on the bf16 blocks (cfg3 / cfg5, verdict r5 item 4): every block
    output that only the next block reads stays unwritten -- the next block's
    fused spatial forward (k_sp_fwd_bf16 / k_sp_fwd_wide) forms
    ReLU(BN2_prev(U_prev)) on staging, and its spatial backward reads U_prev in
    prev mode -- and the last output is pooled from U by the fused head. Loss,
    logits and running stats are bit-identical to the stack that writes every
    output; gradients agree to the order of the atomic adds."""
    gr = pkg.graph
    A = gr.get_normalized_adjacency_matrices(2, 1, distances=gr.synthetic_distances(V),
                                             graph=gr.graph_for(V))
    torch.manual_seed(11)
    with contextlib.redirect_stdout(io.StringIO()):
        m1 = pkg.STGCNStack(3, 60, A, gemm_dtype=torch.bfloat16).cuda().train()
        m2 = pkg.STGCNStack(3, 60, A, gemm_dtype=torch.bfloat16).cuda().train()
    m2.load_state_dict(m1.state_dict())
    m2.lazy_links = False
    x = torch.randn(4, 3, 40, V, generator=torch.Generator().manual_seed(12)).cuda()
    lab = torch.randint(0, 60, (4,), generator=torch.Generator().manual_seed(13)).cuda()
    flags = pkg.fused.lazy_links(list(m1.conv), tuple(x.shape))
    assert flags == [True] * 9 + [False], flags
    for step in range(2):
        loss1, out1 = m1.forward_loss(x, lab)
        loss2, out2 = m2.forward_loss(x, lab)
        m1.zero_grad()
        m2.zero_grad()
        loss1.backward()
        loss2.backward()
        torch.cuda.synchronize()
        assert torch.equal(out1, out2) and torch.equal(loss1, loss2), step
        g2 = {k: b.grad for k, b in m2.named_parameters()}
        for k, a in m1.named_parameters():
            b = g2[k]
            if k.endswith("temporalConv.bias") or k.endswith("batch_n_2.weight"):
                scale = g2[k.rsplit(".", 1)[0] + ".bias"].abs().max().item() if \
                    k.endswith("weight") else 1.0
                assert (a.grad - b).abs().max().item() <= 1e-5 * scale, (step, k)
                continue
            tol = 2e-3 if k.endswith("spatialConv.A") else 1e-5
            assert rel_to_max(a.grad.cpu().numpy(), b.cpu().numpy()) < tol, (step, k)
        for (k, a), b in zip(m1.named_buffers(), m2.buffers()):
            assert torch.equal(a, b), (step, k)

"""GPU parity of the reference's other callers of the hot path and of the
module-API corners added in round 2, all through the C-ABI library:

* ``SpatialConv.forward`` called on its own (st_graphconv.py:139-152;
  stgcn_spatial_fwd / _bwd) against the reference's fixtures and the fp64
  oracle (fp32 gate 1e-5), and with bf16 channel GEMMs (2e-2 gate);
* the block's backward in eval mode (BatchNorm on running statistics as
  constants: fine-tuning with frozen statistics / saliency), default and
  residual block, against the fp64 oracle;
* ``L_STGCN --use_edge_importance`` (``STGCNStack(use_edge_importance=True)``)
  against the reference's cfg1 fixture;
* the legacy ``STGCN`` class (src/network/stgcn.py) in eval mode: class
  probabilities and every gradient against the reference's fixture;
* the stack chain (network.StackChain) with ill-conditioned BN2 affine
  parameters (gamma2 = 0 and 1e-4 on some channels) against the unchained
  blocks.
"""
import glob
import io
import contextlib
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, load_npz, rel_to_max
from oracle import ref_cpu
from test_gpu_block import DEV, TOL, _random_case
from test_gpu_stack import capture_relu_masks, check_relu_ties, gate_stack_grads, \
    oracle_through_masks
from test_oracle_extra import legacy_running_stats

pytestmark = pytest.mark.gpu


def _spatial_fixtures():
    return sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLDEN, "spatialconv_*.npz")))


def _spatial_run(pkg, arrays, bf16=False):
    C_in, C_out = int(arrays["meta"][0]), int(arrays["meta"][1])
    A = torch.from_numpy(arrays["param.A"])
    torch.manual_seed(0)
    sc = pkg.SpatialConv(C_in, C_out, A, gemm_dtype=torch.bfloat16 if bf16 else torch.float32)
    sc.load_state_dict({k[len("param."):]: torch.from_numpy(v) for k, v in arrays.items()
                        if k.startswith("param.")})
    sc = sc.to(DEV)
    x = torch.from_numpy(arrays["x"]).to(DEV).requires_grad_(True)
    y = sc(x)
    y.backward(torch.from_numpy(arrays["g"]).to(DEV))
    torch.cuda.synchronize()
    out = {"y": y.detach().cpu(), "grad.x": x.grad.cpu()}
    for k, p in sc.named_parameters():
        out["grad." + k] = p.grad.cpu()
    return out


def _spatial_oracle(arrays, dtype, gemm_bf16=False):
    p = {k[len("param."):]: torch.from_numpy(v).to(dtype).requires_grad_(True)
         for k, v in arrays.items() if k.startswith("param.")}
    x = torch.from_numpy(arrays["x"]).to(dtype).requires_grad_(True)
    y = ref_cpu.spatial_conv(x, p["A"], p["W.weight"], p["W.bias"], gemm_bf16=gemm_bf16)
    (y * torch.from_numpy(arrays["g"]).to(dtype)).sum().backward()
    out = {"y": y.detach(), "grad.x": x.grad}
    for k, v in p.items():
        out["grad." + k] = v.grad
    return out


@pytest.mark.parametrize("fixture", _spatial_fixtures())
def test_spatialconv_standalone_matches_reference(pkg, fixture):
    ref = load_npz(fixture)
    got = _spatial_run(pkg, ref)
    want = _spatial_oracle(ref, torch.float64)
    ref32 = _spatial_oracle(ref, torch.float32)
    for k, w in want.items():
        err = rel_to_max(got[k].double().numpy(), w.double().numpy())
        floor = rel_to_max(ref32[k].double().numpy(), w.double().numpy())
        assert err < max(TOL, 2 * floor), (k, err, floor)
        # and the reference's own fp32 outputs
        assert rel_to_max(got[k].double().numpy(), ref[k]) < 5e-5, k


def test_spatialconv_standalone_bf16(pkg):
    """bf16 channel GEMMs (SURVEY §8c gate 2e-2, or 3x the reference run with
    bf16 conv operands where that is further from exact)."""
    ref = load_npz("spatialconv_s64x64_v25k3.npz")
    got = _spatial_run(pkg, ref, bf16=True)
    want = _spatial_oracle(ref, torch.float64)
    ref16 = _spatial_oracle(ref, torch.float32, gemm_bf16=True)
    f32 = _spatial_run(pkg, ref)
    for k, w in want.items():
        err = rel_to_max(got[k].double().numpy(), w.double().numpy())
        floor = rel_to_max(ref16[k].double().numpy(), w.double().numpy())
        assert err < max(2e-2, 3 * floor), (k, err, floor)
    assert not torch.equal(got["y"], f32["y"]), "bf16 kernels did not run"


def test_spatialconv_input_without_grad(pkg):
    ref = load_npz("spatialconv_s3x64_v18.npz")
    A = torch.from_numpy(ref["param.A"])
    torch.manual_seed(0)
    sc = pkg.SpatialConv(3, 64, A)
    sc.load_state_dict({k[len("param."):]: torch.from_numpy(v) for k, v in ref.items()
                        if k.startswith("param.")})
    sc = sc.to(DEV)
    y = sc(torch.from_numpy(ref["x"]).to(DEV))
    y.backward(torch.from_numpy(ref["g"]).to(DEV))
    want = _spatial_oracle(ref, torch.float64)
    assert rel_to_max(sc.W.weight.grad.cpu().double().numpy(),
                      want["grad.W.weight"].numpy()) < TOL


# --- eval-mode backward ------------------------------------------------------

def _eval_case(pkg, case, residual, seed=0):
    arrays, x, g = _random_case(pkg, *case, seed=seed, residual=residual)
    gen = torch.Generator().manual_seed(21)
    for k in list(arrays):
        if k.endswith("running_mean"):
            arrays[k] = (0.1 * torch.randn(arrays[k].shape, generator=gen)).numpy()
        elif k.endswith("running_var"):
            arrays[k] = (0.5 + torch.rand(arrays[k].shape, generator=gen)).numpy()
    return arrays, x, g


@pytest.mark.parametrize("case,residual,gemm", [
    ((64, 64, 1, 18, 1, 3, 40), False, "fp32"),
    ((64, 128, 2, 25, 3, 2, 33), False, "fp32"),
    ((3, 64, 1, 50, 3, 2, 20), False, "fp32"),
    ((64, 64, 1, 18, 1, 3, 40), True, "fp32"),
    ((64, 128, 2, 18, 1, 2, 37), True, "fp32"),
    # eval mode on the fused bf16 spatial forward / backward
    # (V = 25, K = 3, C_in >= 32: k_sp_fwd_wide + k_sp_bwd_fused, bf16 Z / dU
    # storage at stride 1, the kept-bf16-G dW'), V = 50 (k_sp_fwd_wide +
    # k_spatial_bwd6), and on the fp32 split path (x3), residual with a
    # strided projection included (its dWr / dbr at the fp32 gate). The oracle
    # takes the HIP run's final ReLU mask (ties at the bf16 resolution).
    ((64, 64, 1, 25, 3, 2, 40), False, "bf16"),
    ((64, 128, 2, 25, 3, 2, 33), False, "bf16"),
    ((64, 64, 1, 50, 3, 2, 17), False, "bf16"),
    ((64, 64, 1, 18, 1, 3, 40), False, "x3"),
    ((64, 128, 2, 18, 1, 2, 37), True, "x3"),
    # the benched f16x2 folded block without G: in eval mode its forward takes
    # max |x| from its own pass (no BN1 statistics pass runs)
    ((64, 64, 1, 18, 1, 3, 40), False, "f16"),
    ((64, 128, 2, 18, 1, 2, 37), False, "f16n"),
])
def test_block_eval_mode_backward(pkg, case, residual, gemm):
    """Eval mode with gradients (frozen BatchNorm statistics): the backward
    treats the running statistics as constants, like nn.BatchNorm2d.eval()."""
    arrays, x, g = _eval_case(pkg, case, residual)
    p, b = ref_cpu.block_params_from_arrays(arrays, dtype=torch.float32, requires_grad=False)
    stride = case[2]
    C_in, C_out = case[0], case[1]
    torch.manual_seed(0)
    A = p["spatialConv.A"]
    with contextlib.redirect_stdout(io.StringIO()):
        blk = pkg.SpatialTemporalConv(
            C_in, C_out, A, 9, stride, 4, dropout_rate=0.5, residual=residual,
            gemm_dtype=torch.bfloat16 if gemm == "bf16" else torch.float32,
            f32_gemm={"x3": "bf16x3", "f16": "f16x2", "f16n": "f16x2-nog"}.get(gemm, "mfma"))
    sd = {k: v for k, v in p.items()}
    sd.update({k: v for k, v in b.items()})
    blk.load_state_dict(sd)
    blk = blk.to(DEV).eval()
    xd = x.to(DEV).requires_grad_(True)
    y = blk(xd)
    y.backward(g.to(DEV))
    torch.cuda.synchronize()

    def oracle(dtype, gemm_bf16=False):
        pp = {k: v.to(dtype).requires_grad_(True) for k, v in p.items()}
        bb = {k: (v.to(dtype) if v.is_floating_point() else v) for k, v in b.items()}
        xx = x.to(dtype).requires_grad_(True)
        yy = ref_cpu.block_forward(xx, pp, bb, stride, residual=residual, training=False,
                                   dtype=dtype, gemm_bf16=gemm_bf16,
                                   relu_mask=(y.detach().cpu() > 0).to(dtype))
        yy.backward(g.to(dtype))
        out = {"y": yy.detach(), "grad.x": xx.grad}
        out.update({"grad." + k: v.grad for k, v in pp.items()})
        return out

    want = oracle(torch.float64)
    got = {"y": y.detach().cpu(), "grad.x": xd.grad.cpu()}
    got.update({"grad." + k: v.grad.cpu() for k, v in blk.named_parameters()})
    if gemm == "bf16":  # SURVEY §8c bf16 gate, or 3x the reference's own bf16-operand error
        ref16 = oracle(torch.float32, gemm_bf16=True)
        gate = {k: max(2e-2, 3 * rel_to_max(ref16[k].double().numpy(), w.double().numpy()))
                for k, w in want.items()}
        blk.gemm_dtype = torch.float32
        with torch.no_grad():
            y32 = blk(x.to(DEV))
        assert not torch.equal(y32.cpu(), got["y"]), "bf16 kernels did not run"
    else:
        gate = {k: (TOL if k in ("y", "grad.x") else 2 * TOL) for k in want}
    bad = []
    for k, w in want.items():  # (eval mode: the temporal bias gradient is not 0)
        err = rel_to_max(got[k].double().numpy(), w.double().numpy())
        if not err < gate[k]:
            bad.append(f"{k}: {err:.2e} >= {gate[k]:.1e}")
    assert not bad, "; ".join(bad)
    for k, v in blk.named_buffers():  # eval mode leaves the running statistics alone
        if "running" in k:
            assert torch.equal(v.cpu(), b[k]), k


# --- edge importance (L_STGCN --use_edge_importance) --------------------------

def test_edge_importance_stack_matches_reference(pkg):
    """STGCNStack(use_edge_importance=True) on the benched path (StackChain +
    fused head): logits / loss against the reference's fixture, gradients
    against the fp64 oracle through the HIP run's ReLU masks (as in
    test_gpu_stack.py; the masked graph has ReLU ties at fp32 resolution in
    the deep blocks)."""
    ref = load_npz("stack_cfg1_edge.npz")
    A = torch.from_numpy(load_npz("adjacency.npz")["V18_s0_d1"])
    torch.manual_seed(0)
    with contextlib.redirect_stdout(io.StringIO()):
        model = pkg.STGCNStack(3, 2, A, use_edge_importance=True, max_mask_jitter=0.05)
    p0, b0 = ref_cpu.init_stack_params(3, 2, A, seed=0, masks="jitter", max_mask_jitter=0.05)
    model = model.cuda().train()
    masks, unhook = capture_relu_masks(model)
    x = torch.from_numpy(ref["x"]).cuda()
    lab = torch.from_numpy(ref["labels"]).cuda()
    loss, logits = model.forward_loss(x.permute(0, 3, 1, 2).contiguous(), lab)
    loss.backward()
    torch.cuda.synchronize()
    unhook()
    assert rel_to_max(logits.detach().cpu().numpy(), ref["logits"]) < 1e-4
    assert abs(loss.item() - float(ref["loss"])) < 1e-5
    for k, v in model.named_parameters():
        if k.startswith("Masks."):
            assert v.grad is None, k  # dead in the reference as well
    xr, lr = torch.from_numpy(ref["x"]), torch.from_numpy(ref["labels"])
    _, _, g64, pre64 = oracle_through_masks(p0, b0, xr, lr, masks, torch.float64)
    _, _, g32, _ = oracle_through_masks(p0, b0, xr, lr, masks, torch.float32)
    check_relu_ties(pre64, masks)
    gate_stack_grads(model, g64, g32)


# --- the legacy STGCN class (src/network/stgcn.py) ----------------------------

def test_legacy_stgcn_eval_matches_reference(pkg):
    ref = load_npz("legacy_stgcn.npz")
    torch.manual_seed(0)
    with contextlib.redirect_stdout(io.StringIO()):
        model = pkg.STGCN(3, 9, 5)
    sd = model.state_dict()
    for k, v in legacy_running_stats(ref).items():
        sd[k].copy_(v)
    model = model.cuda().eval()
    x = torch.from_numpy(ref["x"]).cuda().requires_grad_(True)
    probs = model(x)
    probs.backward(torch.from_numpy(ref["g"]).cuda())
    torch.cuda.synchronize()
    assert rel_to_max(probs.detach().cpu().numpy(), ref["probs"]) < 1e-5
    assert rel_to_max(x.grad.cpu().numpy(), ref["grad.x"]) < 1e-4
    # every gradient against the fp64 oracle (eval mode: no ReLU-mask
    # dependence on batch statistics), at max(1e-4, 3x the fp32 oracle's own
    # error); the reference's sampled gradients at the same gate, except the
    # dA of the deep blocks (small differences of large terms: 1e-3)
    from test_oracle_extra import _legacy_oracle
    p64, _, _, _ = _legacy_oracle(ref, torch.float64)
    p32, _, _, _ = _legacy_oracle(ref, torch.float32)
    gate_stack_grads(model, {k: v.grad for k, v in p64.items()},
                     {k: v.grad for k, v in p32.items()}, skip=())
    bad = []
    for k, v in model.named_parameters():
        if k.startswith("Masks."):
            assert v.grad is None
            continue
        idx = torch.as_tensor(ref["pidx." + k])
        got = v.grad.detach().cpu().reshape(-1)[idx].numpy()
        err = rel_to_max(got, ref["gval." + k])
        if err > (1e-3 if k.endswith("spatialConv.A") else 1e-4):
            bad.append(f"{k}: sampled {err:.2e}")
    assert not bad, "; ".join(bad)


# --- stack chain with ill-conditioned BN2 affine parameters -------------------

@pytest.mark.parametrize("gval", [0.0, 1e-4])
def test_chain_with_tiny_bn2_gamma(pkg, gval):
    """The chained backward reconstructs the previous block's normalised BN2
    input from its output, uhat = (y - beta2) / gamma2; with gamma2 = 0 (or
    |beta2| >> |gamma2|) it reads the saved pre-BN2 tensor instead. Chained
    and unchained stacks must agree (no NaN)."""
    gr = pkg.graph
    A = gr.get_normalized_adjacency_matrices(0, 1, graph=gr.graph_for(18))
    torch.manual_seed(3)
    with contextlib.redirect_stdout(io.StringIO()):
        m1 = pkg.STGCNStack(3, 10, A).cuda().train()
        m2 = pkg.STGCNStack(3, 10, A).cuda().train()
    with torch.no_grad():
        for blk in m1.conv:
            c = blk.batch_n_2.weight.numel()
            blk.batch_n_2.weight[: c // 4] = gval
            blk.batch_n_2.bias.copy_(0.3 * torch.randn(c, generator=torch.Generator().manual_seed(c)))
    m2.load_state_dict(m1.state_dict())
    x = torch.randn(6, 3, 40, 18, generator=torch.Generator().manual_seed(4)).cuda()
    lab = torch.randint(0, 10, (6,), generator=torch.Generator().manual_seed(5)).cuda()
    out1 = m1.forward_nctv(x)
    h = x
    for blk in m2.conv:
        h = blk(h)
    out2 = m2.fc_layer(h.flatten(2).mean(dim=2))
    torch.nn.functional.cross_entropy(out1, lab).backward()
    torch.nn.functional.cross_entropy(out2, lab).backward()
    torch.cuda.synchronize()
    bad = []
    for (k, a), (_, b) in zip(m1.named_parameters(), m2.named_parameters()):
        ga, gb = a.grad.detach().cpu().double().numpy(), b.grad.detach().cpu().double().numpy()
        assert np.isfinite(ga).all(), k
        if np.abs(gb).max() == 0 or k.endswith("temporalConv.bias"):  # (analytically 0)
            continue
        # dA: small differences of large terms; BN affine: bias-type sums over
        # the whole batch (the chain sums them in a different kernel and order)
        tol = 2e-3 if k.endswith("spatialConv.A") else 5e-4 if ".batch_n" in k else 1e-4
        err = rel_to_max(ga, gb)
        if err > tol:
            bad.append(f"{k}: {err:.2e} > {tol:.0e}")
    assert not bad, "; ".join(bad)

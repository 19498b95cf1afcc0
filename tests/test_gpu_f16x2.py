"""GPU parity of the fp32 block with STGCN_F_F16X2 (``gemm="f16x2"``): the
folded block's temporal conv forward, data-grad and weight-grad GEMMs
(st-gcn_amd/csrc/kernels_x3.hip NPL = 2) as 2-way fp16 splits of operands
scaled by powers of two from their max |x| (x s = h + l, 22 significant bits;
three partial products hh, hl, lh; fp32 accumulate). BN1's sum of dxhat, which
nearly cancels, comes from the fp64 dU sums (kernels_fold.hip k_fold_sd), not
from the 22-bit data gradient.

The mode claims fp32-GEMM accuracy, so it is held to the SAME gate as the fp32
MFMA path and the bf16x3 path (test_gpu_block.py): rel-to-max
error vs the fp64 oracle below 1e-5 per output and gradient (or below twice
the fp32 reference's own error where that is larger), ReLU ties as there.
Each folded case also checks that the plan selected the fp16 splits and that
their results differ from the bf16x3 path's (the kernels ran). The scale
cases multiply the input by 1e-6 and 1e5: a fixed scale would underflow or
overflow fp16 there, the max-derived power-of-two scales must not.
"""
import pytest
import torch

from test_gpu_block import _compare, _oracle, _random_case, _run_hip

pytestmark = pytest.mark.gpu


# "f16x2_nog": the same GEMMs with G never formed (STGCN_F_NO_G; kernels_x3.hip
# bna_contract, k_wgrad_x3 QBN), held to the same gate
MODES = ["f16x2", "f16x2_nog"]


def _check(pkg, arrays, x, g, need_dx=True, gemm="f16x2"):
    got = _run_hip(pkg, arrays, x, g, need_dx=need_dx, gemm=gemm)
    want, floor = _oracle(arrays, got)
    if not need_dx:
        want.pop("grad.x")
    _compare(got, want, floor=floor)
    return got


def _plan(pkg, x, C_out, stride, K=1, gemm="f16x2"):
    return pkg.hip_lib.block_plan(pkg.fused.make_desc(
        tuple(x.shape), C_out, K, stride, 4, 1e-5, 0.1, True, **pkg.fused._gemm_flags(gemm)))


@pytest.mark.parametrize("case", [
    # C_in, C_out, stride, V, K, N, T
    (64, 64, 1, 18, 1, 4, 64),      # cfg2 L1-L3 shape (64-row tiles)
    (64, 128, 2, 18, 1, 3, 37),     # stride 2: the strided forward / weight-grad, odd T
    (128, 128, 1, 18, 1, 2, 40),    # 128-row tiles (MR = 2)
    (128, 256, 2, 18, 1, 2, 30),    # 128-row tiles, stride-2 forward, 8 chunks
    (256, 256, 1, 18, 1, 2, 19),    # 16 chunks, ragged T
    (24, 40, 1, 18, 1, 2, 23),      # partial channel chunk (24 = 16 + 8), partial rows
    (16, 16, 1, 18, 1, 2, 9),       # smallest folded block
])
@pytest.mark.parametrize("gemm", MODES)
def test_f16x2_block_random(pkg, case, gemm):
    arrays, x, g = _random_case(pkg, *case)
    got = _check(pkg, arrays, x, g, gemm=gemm)
    C_in, C_out, stride = case[:3]
    plan = _plan(pkg, x, C_out, stride, gemm=gemm)
    hl = pkg.hip_lib
    assert plan & hl.PLAN_FOLD and plan & hl.PLAN_F16X2, plan
    # (no G: the joint contraction inside the GEMMs)
    assert bool(plan & hl.PLAN_FOLD_NO_G) == (gemm == "f16x2_nog"), plan
    ref = _run_hip(pkg, arrays, x, g, gemm="f32x3")
    assert not torch.equal(got["y"], ref["y"]), "fp16-split forward did not run"
    assert not torch.equal(got["grad.temporalConv.weight"], ref["grad.temporalConv.weight"])


@pytest.mark.parametrize("gemm", MODES)
@pytest.mark.parametrize("xs,gs", [(1e-6, 1e-4), (1e5, 1e2)])
def test_f16x2_operand_scales(pkg, xs, gs, gemm):
    """Input (hence G: BN1 of a near-constant input is eps-dominated at 1e-6)
    and output gradient (hence dU) far from O(1): the power-of-two operand
    scales keep every GEMM at the fp32 gate. (The analytically-zero temporal
    bias gradient is gated absolutely at 1e-5, so the gradient scale stays
    within 1e2.)"""
    arrays, x, g = _random_case(pkg, 64, 128, 1, 18, 1, 2, 33, seed=3)
    x = x * xs
    arrays["x"] = x.numpy()
    g = g * gs
    arrays["g"] = g.numpy()
    _check(pkg, arrays, x, g, gemm=gemm)


@pytest.mark.parametrize("gemm", MODES)
def test_f16x2_full_size_block(pkg, gemm):
    """cfg2 L1-type shape at N = 32, T = 300 (the bench layer) at the fp32 gate."""
    arrays, x, g = _random_case(pkg, 64, 64, 1, 18, 1, 32, 300, seed=7)
    got = _check(pkg, arrays, x, g, gemm=gemm)
    for k, v in got.items():
        assert torch.isfinite(v).all(), k


def test_f16x2_backward_without_kept_bound(pkg, monkeypatch):
    """A caller that keeps nothing between forward and backward (stgcn_fwd_args_t
    .G null): the backward forms max |x| itself (one pass over x) for the
    weight gradient's operand scale; same fp32 gate."""
    monkeypatch.setattr(pkg.fused, "_keep_g", lambda ctx, x, desc: None)
    arrays, x, g = _random_case(pkg, 64, 128, 2, 18, 1, 2, 29, seed=6)
    _check(pkg, arrays, x, g, gemm="f16x2_nog")
    # (the unfolded first block: max |Z| by a pass over Z in the backward)
    arrays, x, g = _random_case(pkg, 3, 64, 1, 18, 1, 2, 30, seed=7)
    _check(pkg, arrays, x, g, need_dx=False)


@pytest.mark.parametrize("gemm", MODES)
def test_f16x2_l8_shape_block(pkg, gemm):
    """The dominant kernel's shape (cfg2 L8 / L9: 256 -> 256, T = 75) at
    N = 16: 16 channel chunks per tile (the longest reductions), 128-row tiles,
    at the fp32 gate."""
    arrays, x, g = _random_case(pkg, 256, 256, 1, 18, 1, 16, 75, seed=11)
    _check(pkg, arrays, x, g, gemm=gemm)
    assert _plan(pkg, x, 256, 1, gemm=gemm) & pkg.hip_lib.PLAN_F16X2


def _per_channel_err(got, want, axis):
    """max over channels c of max|got[c] - want[c]| / max|want[c]| (channel = axis)"""
    g = got.double().movedim(axis, 0).reshape(got.shape[axis], -1)
    w = want.detach().double().movedim(axis, 0).reshape(want.shape[axis], -1)
    return ((g - w).abs().amax(1) / w.abs().amax(1).clamp_min(1e-300))


@pytest.mark.parametrize("gemm", MODES)
def test_f16x2_mixed_scale_per_channel(pkg, gemm):
    """One input channel and one output channel's weights (its temporal conv
    row and its SpatialConv row) at 1e-4 of the rest: a single power-of-two
    scale per operand tensor must not cost the small channels their precision.
    Gated PER CHANNEL (not rel-to-max over the tensor, which cannot see a small
    channel): every channel of y, dx, dWt and dW' within max(1e-5, 2x the fp32
    reference's own error for that channel) of the fp64 oracle."""
    from oracle import ref_cpu
    arrays, x, g = _random_case(pkg, 64, 128, 1, 18, 1, 2, 33, seed=4)
    ci, co = 5, 17
    x = x.clone()
    x[:, ci] *= 1e-4
    arrays["x"] = x.numpy()
    for k in ("param.temporalConv.weight", "param.spatialConv.W.weight"):
        w = arrays[k].copy()
        w[co] *= 1e-4
        arrays[k] = w
    got = _run_hip(pkg, arrays, x, g, gemm=gemm)
    want, _ = _oracle(arrays, got)
    ref32 = ref_cpu.block_step(arrays, dtype=torch.float32, relu_mask=got["y"] > 0)
    bad = []
    for k, axis in (("y", 1), ("grad.x", 1), ("grad.temporalConv.weight", 0),
                    ("grad.spatialConv.W.weight", 0)):
        e = _per_channel_err(got[k], want[k], axis)
        f = _per_channel_err(ref32[k].detach(), want[k], axis)
        lim = torch.clamp(2.0 * f, min=1e-5)
        if (e > lim).any():
            c = int(torch.argmax(e / lim))
            bad.append(f"{k}[{c}]: {e[c]:.2e} > {lim[c]:.1e}")
    assert not bad, "; ".join(bad)


@pytest.mark.parametrize("gemm", ["f32x3", "f16x2"])
@pytest.mark.parametrize("case", [
    # C_in, C_out, stride, V, K, N, T: >= 16 input channels, < 16 output channels
    (16, 8, 1, 18, 1, 2, 9),
    (32, 8, 2, 18, 1, 2, 21),
])
def test_narrow_output_blocks_not_folded(pkg, case, gemm):
    """a block with C_out < 16 has a data gradient that reduces
    over fewer than 16 channels, which the split kernel (and its fused
    SpatialConv backward epilogue) does not run; such a block must not fold, and
    runs the unfolded kernels at the fp32 gate."""
    arrays, x, g = _random_case(pkg, *case)
    hl = pkg.hip_lib
    d = pkg.fused.make_desc(tuple(x.shape), case[1], 1, case[2], 4, 1e-5, 0.1, True,
                            **pkg.fused._gemm_flags(gemm))
    assert not hl.block_plan(d) & hl.PLAN_FOLD
    got = _run_hip(pkg, arrays, x, g, gemm=gemm)
    want, floor = _oracle(arrays, got)
    _compare(got, want, floor=floor)


def test_f16x2_residual_block_keeps_bf16x3(pkg):
    """Where the block neither folds nor is the unfolded K = 1 first block (the
    residual block) the flag changes nothing: no F16X2 bit, results bit-identical
    to the bf16x3 path (the adjacency gradient up to the order of its fp32 atomic
    partial sums, which differs from run to run)."""
    hl = pkg.hip_lib
    case = (64, 64, 1, 18, 1, 2, 30)
    arrays, x, g = _random_case(pkg, *case, residual=True)
    d = pkg.fused.make_desc(tuple(x.shape), case[1], 1, case[2], 4, 1e-5, 0.1, True,
                            residual=True, f16x2=True)
    assert not hl.block_plan(d) & hl.PLAN_F16X2
    a = _run_hip(pkg, arrays, x, g, gemm="f16x2")
    b = _run_hip(pkg, arrays, x, g, gemm="f32x3")
    for k in a:
        if k == "grad.spatialConv.A":
            torch.testing.assert_close(a[k], b[k], rtol=1e-5, atol=1e-6 * b[k].abs().max())
        else:
            assert torch.equal(a[k], b[k]), k


@pytest.mark.parametrize("case", [
    # C_in, C_out, stride, V, K, N, T: the first block (C_in = 3, not folded)
    (3, 64, 1, 18, 1, 2, 30),
    (3, 64, 1, 18, 1, 4, 300),      # cfg2 L0 at T = 300
    (3, 32, 2, 18, 1, 2, 23),       # stride 2, odd T
])
@pytest.mark.parametrize("need_dx", [False, True])
def test_f16x2_first_block(pkg, case, need_dx):
    """The unfolded K = 1 first block under STGCN_F_F16X2: the temporal conv
    forward and weight gradient on fp16 splits (max |Z| by a pass over Z,
    carried to the backward after the kept G), the data gradient on the 3-way
    splits; held to the fp32 gate."""
    arrays, x, g = _random_case(pkg, *case)
    got = _check(pkg, arrays, x, g, need_dx=need_dx)
    plan = _plan(pkg, x, case[1], case[2])
    hl = pkg.hip_lib
    assert plan & hl.PLAN_F16X2 and not plan & hl.PLAN_FOLD, plan
    ref = _run_hip(pkg, arrays, x, g, need_dx=need_dx, gemm="f32x3")
    assert not torch.equal(got["y"], ref["y"]), "fp16-split forward did not run"
    assert not torch.equal(got["grad.temporalConv.weight"], ref["grad.temporalConv.weight"])


@pytest.mark.parametrize("gemm", ["f32x3", "f16x2", "f16x2_nog"])
@pytest.mark.parametrize("case", [
    (64, 64, 1, 18, 1, 2, 40),      # stride 1: one data-gradient launch
    (64, 128, 2, 18, 1, 3, 37),     # stride 2: two data-gradient phases, odd T
    (128, 256, 1, 18, 1, 2, 19),    # 128-row tiles
])
def test_fold_prep_matches_own_operands(pkg, case, gemm):
    """ABI 7 stgcn_fold_prep (the stack's per-step weight operands in batched
    launches) runs exactly the kernels and arithmetic the block runs on its own:
    every output and gradient bit-identical (the adjacency gradient up to the
    order of its fp32 atomic partial sums), and at the fp32 gate."""
    arrays, x, g = _random_case(pkg, *case)
    a = _run_hip(pkg, arrays, x, g, gemm=gemm)
    b = _run_hip(pkg, arrays, x, g, gemm=gemm, prep=True)
    for k in a:
        if k == "grad.spatialConv.A":
            torch.testing.assert_close(b[k], a[k], rtol=1e-5, atol=1e-6 * a[k].abs().max())
        else:
            assert torch.equal(a[k], b[k]), k
    want, floor = _oracle(arrays, b)
    _compare(b, want, floor=floor)



@pytest.mark.parametrize("case", [
    # C_in, C_out, stride, V, K, N, T: the reference's default L_STGCN graph
    # (lightning_model.py:271: NTU joints, partitioning 0 = unilabeling, K = 1)
    (64, 64, 1, 25, 1, 3, 40),
    (64, 128, 2, 25, 1, 2, 31),     # stride 2, odd T
    (128, 128, 1, 25, 1, 2, 30),    # 128-row tiles
    (24, 40, 1, 25, 1, 2, 23),      # partial chunk / rows
])
@pytest.mark.parametrize("gemm", ["f16x2", "f32x3"])
def test_fold_default_graph_v25(pkg, case, gemm):
    """V = 25, K = 1 folds (STGCN_PLAN_FOLD): forward and weight gradient on the
    fp16 splits (f16x2), the data gradient on the 3-way bf16 splits with H
    stored and the unfused SpatialConv backward (the fused epilogue and the
    analytic BN1 sum are V = 18 only), all at the fp32 gate."""
    arrays, x, g = _random_case(pkg, *case)
    got = _check(pkg, arrays, x, g, gemm=gemm)
    plan = _plan(pkg, x, case[1], case[2], gemm=gemm)
    hl = pkg.hip_lib
    assert plan & hl.PLAN_FOLD and not plan & hl.PLAN_SP_BWD_FUSED, plan
    assert bool(plan & hl.PLAN_F16X2) == (gemm == "f16x2"), plan
    if gemm == "f16x2":
        ref = _run_hip(pkg, arrays, x, g, gemm="f32x3")
        assert not torch.equal(got["y"], ref["y"]), "fp16-split forward did not run"

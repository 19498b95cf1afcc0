"""GPU parity of the fp32 block with STGCN_F_F32X3: the temporal conv forward /
data-grad GEMMs (k_conv_x3), the stride-1 V=18 weight gradient (k_wgrad_x3)
and the spatial 1x1 weight gradient dW' (k_wgrad_sp<.., X3>) as exact 3-way bf16 operand splits with six partial products on the bf16
matrix cores (st-gcn_amd/csrc/kernels_x3.hip).

The mode claims fp32-GEMM accuracy, so it is held to the SAME gate as the fp32
MFMA path (test_gpu_block.py): rel-to-max error vs the fp64
oracle below 1e-5 per output and gradient (or below twice the fp32 reference's
own error where that is larger), ReLU ties as there. Each case also checks the
split kernels ran: the output is not bit-identical to the fp32 MFMA path's.
"""
import pytest
import torch

from conftest import block_fixtures, load_npz
from test_gpu_block import _compare, _oracle, _random_case, _run_hip

pytestmark = pytest.mark.gpu


def _check(pkg, arrays, x, g, residual=False, need_dx=True):
    got = _run_hip(pkg, arrays, x, g, need_dx=need_dx, gemm="f32x3")
    want, floor = _oracle(arrays, got)
    if not need_dx:
        want.pop("grad.x")
    _compare(got, want, residual=residual, floor=floor)
    return got


def _assert_fold_ran(pkg, arrays, x):
    """The folded forward writes the composite weights Wc[o][i][q] = sum_c
    Wt[o][c][q] W'[c][i] into the Z buffer it saves for the backward (capi.hip
    fold_wc_in_z): the first C_out * C_in * 9 floats of the saved Z must be
    Wc (fp64 GEMM rounded once to fp32)."""
    from oracle import ref_cpu
    p, b = ref_cpu.block_params_from_arrays(arrays, dtype=torch.float32, requires_grad=False)
    stride = int(arrays["meta"][2])
    dev = "cuda:0"
    cu = {k: v.to(dev).contiguous() for k, v in p.items()}
    bu = {k: v.to(dev).clone() for k, v in b.items() if "num_batches" not in k}
    xd = x.to(dev).float().contiguous().requires_grad_(True)
    Wt = cu["temporalConv.weight"].requires_grad_(True)
    y = pkg.fused.StgcnBlockFn.apply(
        xd, cu["spatialConv.A"], cu["spatialConv.W.weight"], cu["spatialConv.W.bias"], Wt,
        cu["temporalConv.bias"], cu["batch_n.weight"], cu["batch_n.bias"],
        cu["batch_n_2.weight"], cu["batch_n_2.bias"], bu["batch_n.running_mean"],
        bu["batch_n.running_var"], bu["batch_n_2.running_mean"], bu["batch_n_2.running_var"],
        stride, 4, 1e-5, 0.1, True, None, 0.0, "f32x3")
    Z = y.grad_fn.saved_tensors[1]
    C_out, C_in = Wt.shape[0], xd.shape[1]
    if Z.numel() < C_out * C_in * 9:
        return  # (Wc does not fit there: the library keeps it in its workspace)
    wc = torch.einsum("ocq,ci->oiq", p["temporalConv.weight"].double().reshape(C_out, C_out, 9),
                      p["spatialConv.W.weight"].double().reshape(C_out, C_in))
    got = Z.reshape(-1)[:C_out * C_in * 9].double().cpu().reshape(C_out, C_in, 9)
    assert (got - wc).abs().max().item() <= 1e-6 * wc.abs().max().item(), \
        "the folded forward did not run (Z does not hold Wc)"


@pytest.mark.parametrize("fixture", [f for f in block_fixtures()])
def test_f32x3_block_fixture(pkg, fixture):
    ref = load_npz(fixture)
    _check(pkg, ref, torch.from_numpy(ref["x"]), torch.from_numpy(ref["g"]),
           residual=bool(ref["meta"][7]))


@pytest.mark.parametrize("case", [
    # C_in, C_out, stride, V, K, N, T, residual
    (64, 64, 1, 18, 1, 4, 64, False),     # cfg2 L1 shape: fwd + dgrad on k_conv_x3<9,18>
    (64, 128, 2, 18, 1, 3, 37, False),    # stride 2: dgrad phases k_conv_x3<5|4,18>
    (128, 256, 2, 18, 1, 2, 30, False),   # 4 row tiles, 8 channel chunks
    (256, 256, 1, 18, 1, 2, 19, False),   # 16 chunks, ragged T
    (3, 64, 1, 18, 1, 3, 45, False),      # C_in = 3: spatial GEMM stays fp32 MFMA
    (24, 40, 1, 18, 1, 2, 23, False),     # partial channel chunk (24 = 16 + 8), partial rows
    (64, 64, 1, 25, 3, 2, 40, False),     # V = 25 (k_conv_x3<9,25>), K = 3
    (64, 128, 2, 25, 3, 2, 33, False),
    (64, 64, 1, 50, 3, 2, 17, False),     # V = 50: not covered -> fp32 MFMA kernels
    (64, 64, 2, 18, 1, 1, 1, False),      # T = 1
    (64, 64, 1, 18, 1, 3, 40, True),      # residual, identity
    (64, 128, 2, 18, 1, 2, 37, True),     # residual, projection
])
def test_f32x3_block_random(pkg, case):
    *shape, residual = case
    arrays, x, g = _random_case(pkg, *shape, residual=residual)
    got = _check(pkg, arrays, x, g, residual=residual)
    C_in, C_out, stride, V = shape[:4]
    if V in (18, 25) and C_out >= 16 and shape[6] > 1:
        # stride 1: the forward runs k_conv_x3; stride 2: the data-grad phases
        key = "y" if stride == 1 else "grad.x"
        ref = _run_hip(pkg, arrays, x, g, gemm="fp32")
        assert not torch.equal(got[key], ref[key]), "split kernels did not run"
        if V == 18:  # k_wgrad_x3 (temporal weight gradient, stride 1 and 2)
            k = "grad.temporalConv.weight"
            assert not torch.equal(got[k], ref[k]), "k_wgrad_x3 did not run"
        plan = pkg.hip_lib.block_plan(pkg.fused.make_desc(
            tuple(x.shape), C_out, shape[4], stride, 4, 1e-5, 0.1, True,
            residual=residual, f32x3=True))
        if V == 18 and shape[4] == 1 and not residual and C_in >= 16:
            # the folded block (W' inside the temporal conv's weights): the plan
            # says so, and the forward left Wc = Wt W' in the (opaque) Z buffer
            assert plan & pkg.hip_lib.PLAN_FOLD, plan
            # ... and its SpatialConv backward runs inside the data gradient
            # (H never in HBM): dA / dx / BN1 gradients are gated above
            assert plan & pkg.hip_lib.PLAN_SP_BWD_FUSED, plan
            _assert_fold_ran(pkg, arrays, x)
        else:
            # spatial dW' = dZ G^T on the split products (k_wgrad_sp<.., X3>)
            assert not plan & pkg.hip_lib.PLAN_FOLD and plan & pkg.hip_lib.PLAN_WSP_SPLIT, plan
            k = "grad.spatialConv.W.weight"
            assert not torch.equal(got[k], ref[k]), "k_wgrad_sp X3 did not run"
    if residual and (C_in != C_out or stride != 1):
        # the strided projection's dWr / dbr: present in both
        # runs, so _check held them to the fp32 gate above
        assert "grad.apply_residual.weight" in got and "grad.apply_residual.bias" in got


def test_f32x3_full_size_block(pkg):
    """cfg2 L1 shape at N=32, T=300 (the bench layer) at the fp32 gate."""
    arrays, x, g = _random_case(pkg, 64, 64, 1, 18, 1, 32, 300, seed=7)
    got = _check(pkg, arrays, x, g)
    for k, v in got.items():
        assert torch.isfinite(v).all(), k


def test_f32x3_without_dx(pkg):
    arrays, x, g = _random_case(pkg, 3, 64, 1, 18, 1, 2, 30)
    _check(pkg, arrays, x, g, need_dx=False)

"""GPU parity of the bf16 GEMM path (STGCN_F_BF16, BASELINE cfg3 / cfg5) against
the fp64 oracle.

The bf16 block rounds the operands of its channel GEMMs (spatial W, temporal
conv forward / data-grad / weight-grad, residual projection) to bf16 on the
bf16 matrix cores and accumulates in fp32; tensors, A, BatchNorm and the joint
contractions stay fp32. Tolerance: rel-to-max error
max|diff| / max|ref| below 2e-2 for the output and every gradient, against
the fp64 oracle (oracle/ref_cpu.py, the reference's op order) -- or, where the
reference itself run with bf16 GEMM operands (ref_cpu ``gemm_bf16``: its convs
with bf16-rounded inputs, weights and output gradients, fp32 accumulate) is
further than that from exact arithmetic, below FLOOR_FACTOR (3) times the
reference's own bf16 error (this happens for bias-type gradients that are sums
of many cancelling terms, e.g. the BN1 bias gradient of a 3-channel first
block; the rounding points differ between the reference's op order and the
fused block's, so both errors are independent samples of the same size and a
single sample of each needs the margin). ReLU ties are
handled as in test_gpu_block.py, with the tie band widened to bf16 rounding:
the HIP ReLU mask must agree with the exact one wherever the pre-ReLU value is
further than TIE_BF16 * max|pre-ReLU| from 0, and the oracle is then
differentiated through the HIP mask.

A second, tighter check pins the k-ordering of every bf16 GEMM: the same block
run with the fp32 path on the same inputs, and the bf16 result must sit within
the bf16 error band of it (and NOT equal it: the bf16 kernels ran).
"""
import numpy as np
import pytest
import torch

from conftest import rel_to_max
from oracle import ref_cpu
from test_gpu_block import DEV, _random_case

pytestmark = pytest.mark.gpu

TOL_BF16 = 2e-2
TIE_BF16 = 2e-2
FLOOR_FACTOR = 3.0


def _run(pkg, arrays, x, g, bf16, need_dx=True):
    p, b = ref_cpu.block_params_from_arrays(arrays, dtype=torch.float32, requires_grad=False)
    stride, residual = int(arrays["meta"][2]), bool(arrays["meta"][7])
    cu = {k: v.to(DEV).contiguous().requires_grad_(True) for k, v in p.items()}
    bu = {k: v.to(DEV).clone() for k, v in b.items() if "num_batches" not in k}
    xd = x.to(DEV).float().contiguous().requires_grad_(need_dx)
    common = (xd, cu["spatialConv.A"], cu["spatialConv.W.weight"], cu["spatialConv.W.bias"],
              cu["temporalConv.weight"], cu["temporalConv.bias"], cu["batch_n.weight"],
              cu["batch_n.bias"], cu["batch_n_2.weight"], cu["batch_n_2.bias"])
    running = (bu["batch_n.running_mean"], bu["batch_n.running_var"],
               bu["batch_n_2.running_mean"], bu["batch_n_2.running_var"])
    if residual:
        y = pkg.fused.StgcnResBlockFn.apply(
            *common, cu.get("apply_residual.weight"), cu.get("apply_residual.bias"), *running,
            stride, 4, 1e-5, 0.1, True, None, 0.0, "bf16" if bf16 else "fp32")
    else:
        y = pkg.fused.StgcnBlockFn.apply(*common, *running, stride, 4, 1e-5, 0.1, True, None,
                                         0.0, "bf16" if bf16 else "fp32")
    # residual block: the inner ReLU's mask (Za = ReLU(BN2(Z)) > 0, saved by the
    # Function) so the oracle can take the same subgradient choices there too
    inner = (y.grad_fn.saved_tensors[2] > 0).cpu() if residual else None
    y.backward(g.to(DEV).float())
    torch.cuda.synchronize()
    out = {"y": y.detach().cpu(), "inner_mask": inner}
    if need_dx:
        out["grad.x"] = xd.grad.cpu()
    for k, t in cu.items():
        out["grad." + k] = t.grad.cpu()
    for k, t in bu.items():
        out["after." + k] = t.cpu()
    return out


def _errors(got, want, residual):
    errs = {}
    for k, w in want.items():
        if k not in got or k.endswith("num_batches_tracked") or k == "inner_mask":
            continue
        if k == "grad.temporalConv.bias" and not residual:
            continue  # identically 0 (BN2 follows the conv): checked in absolute terms below
        errs[k] = rel_to_max(got[k].double().numpy(), w.detach().double().numpy())
    return errs


def _pre_inner(arrays):
    """BN2 output of a residual block (the inner ReLU's input), fp64."""
    p, b = ref_cpu.block_params_from_arrays(arrays, dtype=torch.float64, requires_grad=False)
    with torch.no_grad():
        x = torch.as_tensor(arrays["x"]).double()
        f = ref_cpu._bn(x, p, b, "batch_n", True, 0.1, 1e-5).clamp_min(0)
        f = ref_cpu.spatial_conv(f, p["spatialConv.A"], p["spatialConv.W.weight"],
                                 p["spatialConv.W.bias"])
        return ref_cpu._bn(f, p, b, "batch_n_2", True, 0.1, 1e-5)


def _check_bf16(pkg, case, residual=False, need_dx=True, seed=0):
    C_in, C_out, stride, V, K, N, T = case
    arrays, x, g = _random_case(pkg, C_in, C_out, stride, V, K, N, T, seed=seed,
                                residual=residual)
    got = _run(pkg, arrays, x, g, bf16=True, need_dx=need_dx)
    mask, inner = got["y"] > 0, got["inner_mask"]
    pre = ref_cpu.block_pre_relu(arrays)
    flips = mask != (pre > 0)
    if flips.any():
        band = TIE_BF16 * pre.abs().max().item()
        assert pre[flips].abs().max().item() < band, "ReLU mask differs away from a tie"
    if inner is not None:  # the inner ReLU mask may differ only at ties as well
        pin = _pre_inner(arrays)
        iflips = inner != (pin > 0)
        if iflips.any():
            band = TIE_BF16 * pin.abs().max().item()
            assert pin[iflips].abs().max().item() < band, \
                f"inner ReLU mask differs away from a tie ({int(iflips.sum())} flips)"
    want = ref_cpu.block_step(arrays, dtype=torch.float64, relu_mask=mask, inner_mask=inner)
    ref16 = ref_cpu.block_step(arrays, dtype=torch.float32, relu_mask=mask.float(),
                               gemm_bf16=True, inner_mask=inner)
    if not need_dx:
        want.pop("grad.x")
    errs = _errors(got, want, residual)
    floor = _errors(ref16, want, residual)
    bad = {k: (e, floor[k]) for k, e in errs.items() if not e < max(TOL_BF16, FLOOR_FACTOR * floor[k])}
    assert not bad, f"bf16 block vs fp64 oracle: {bad} (all: {errs})"
    if not residual:
        assert got["grad.temporalConv.bias"].abs().max().item() < 1e-3
    # the bf16 kernels ran (results differ from the fp32 path) and sit in the bf16 band of it
    f32 = _run(pkg, arrays, x, g, bf16=False, need_dx=need_dx)
    d = rel_to_max(got["y"].numpy(), f32["y"].numpy())
    assert 0 < d < TOL_BF16, f"bf16 vs fp32 path output difference {d}"
    return errs


@pytest.mark.parametrize("case", [
    # C_in, C_out, stride, V, K, N, T
    (3, 64, 1, 18, 1, 3, 45),       # first block, ragged T
    (64, 64, 1, 18, 1, 4, 64),      # cfg2 L1 shape
    (64, 128, 2, 18, 1, 3, 37),     # stride 2, odd T (stride-2 dgrad phases)
    (128, 256, 2, 18, 1, 2, 30),    # 4 row tiles
    (256, 256, 1, 18, 1, 2, 19),
    (3, 64, 1, 25, 3, 2, 40),       # cfg3 (NTU, spatial partitioning K=3)
    (64, 64, 1, 25, 3, 2, 40),
    (64, 128, 2, 25, 3, 2, 33),
    (128, 256, 2, 25, 3, 2, 21),
    (3, 64, 1, 50, 3, 2, 20),       # cfg5 (two-person V=50)
    (64, 64, 1, 50, 3, 2, 17),
    (64, 128, 2, 50, 3, 2, 23),     # k_sp_fwd_wide, 128 rows
    (128, 256, 2, 50, 3, 2, 13),    # k_sp_fwd_wide, 256 rows (per-wave epilogue)
    (256, 256, 1, 50, 3, 2, 7),     # 16 channel chunks, ragged last frame tile
    (24, 40, 1, 50, 3, 2, 11),      # partial chunk (24 = 16 + 8) and rows (40 of 64)
    (5, 21, 1, 18, 1, 2, 9),        # odd channel counts: partial tiles and chunks (5: fp32 W)
    (64, 64, 2, 25, 3, 8, 1),       # T = 1 (single frame: all taps but one in the halo)
    # k_wgrad_bf16_raw (V = 25, stride 1, bf16 Z / dU, even T): ragged last
    # item (42 = 10 * 4 + 2 frames), partial channel tiles (96 = 64 + 32 rows /
    # channels), two row tiles, and T = 2 (every tap but one in the halo)
    (32, 96, 1, 25, 3, 2, 42),
    (128, 128, 1, 25, 3, 3, 10),
    (64, 64, 1, 25, 3, 4, 2),
])
def test_bf16_block_matches_oracle(pkg, case):
    errs = _check_bf16(pkg, case)
    print(case, {k: float(np.format_float_scientific(v, 2)) for k, v in errs.items()})


@pytest.mark.parametrize("case", [
    (64, 64, 1, 18, 1, 3, 40),      # identity residual
    (64, 128, 2, 18, 1, 2, 37),     # projection, stride 2 (bf16 projection GEMMs)
    (64, 128, 2, 25, 3, 2, 33),
    (3, 64, 1, 50, 3, 2, 20),       # projection, stride 1
    (64, 64, 1, 50, 3, 2, 16),      # identity: k_sp_fwd_wide with ReLU input + BN2 statistics
    (64, 128, 2, 50, 3, 2, 19),     # projection: 128-row k_sp_fwd_wide
])
def test_bf16_residual_block_matches_oracle(pkg, case):
    errs = _check_bf16(pkg, case, residual=True)
    print(case, {k: float(np.format_float_scientific(v, 2)) for k, v in errs.items()})


def test_bf16_first_block_without_dx(pkg):
    _check_bf16(pkg, (3, 64, 1, 25, 3, 2, 30), need_dx=False)


def test_bf16_fused_spatial_backward_without_dx(pkg):
    """k_sp_bwd_fused (V = 25, K = 3, C_in % 32 == 0) with write_dx = 0: dA and
    the BN1 sums only, odd T * V (per-row DMA shifts) and a ragged frame tile."""
    _check_bf16(pkg, (64, 64, 1, 25, 3, 2, 29), need_dx=False)


def test_bf16_full_size_block(pkg):
    """cfg3 layer-1 shape (V=25, K=3, T=300) at N=16."""
    errs = _check_bf16(pkg, (64, 64, 1, 25, 3, 16, 300), seed=7)
    print({k: float(np.format_float_scientific(v, 2)) for k, v in errs.items()})


def test_bf16_cfg5_full_size_block(pkg):
    """cfg5 layer shape (V = 50 two-person graph, K = 3) at the full T = 300,
    N = 8: k_spatial_bwd6's persistent grid and its resident dA accumulators at
    a realistic grid size."""
    errs = _check_bf16(pkg, (64, 64, 1, 50, 3, 8, 300), seed=11)
    print({k: float(np.format_float_scientific(v, 2)) for k, v in errs.items()})


def test_bf16_v50_three_channel_blocks(pkg):
    """V = 50 fused spatial backward (k_sp50_dx / _dA) at C_in = 96: three
    32-channel blocks, more items than the 256-workgroup grid, so each
    workgroup's strided items must stay in one channel block (the grid is a
    multiple of 3 there)."""
    errs = _check_bf16(pkg, (96, 96, 1, 50, 3, 4, 300), seed=17)
    print({k: float(np.format_float_scientific(v, 2)) for k, v in errs.items()})


def test_bf16_cfg5_stride2_full_size_block(pkg):
    """cfg5 L4 shape (V = 50, K = 3, 64 -> 128 channels, stride 2) at T = 300,
    N = 4: bf16 Z / dU storage on a stride-2 block, read by the strided
    forward, the two data-gradient phases and the LDS-DMA weight gradient
    (k_wgrad_bf16<9,50,2,4,32,true>)."""
    errs = _check_bf16(pkg, (64, 128, 2, 50, 3, 4, 300), seed=13)
    print({k: float(np.format_float_scientific(v, 2)) for k, v in errs.items()})

"""GPU parity of the fused HIP block (through the C-ABI) against the oracle.

Tolerance: fp32 HIP vs the fp64 oracle, rel-to-max error
max|diff| / max|ref| below 1e-5 for outputs and gradients -- or, where the
reference's own fp32 arithmetic (the oracle run in fp32, same ops as the
reference) is further than that from exact arithmetic, below twice the
reference's own error for that tensor ("no worse than the reference"). The
latter happens for BN-heavy small batches (T=1) and for large-N bias-type
gradients (sums of ~1e5 cancelling terms). The temporal-conv bias gradient is
analytically zero (BN2 follows the conv) and is checked with an absolute
tolerance instead (non-residual block only: in the residual block it is a real
gradient). Residual blocks (full pre-activation, st_graphconv.py:60-82) use
the same gates.
"""
import numpy as np
import pytest
import torch

from conftest import block_fixtures, load_npz, rel_to_max
from oracle import ref_cpu

pytestmark = pytest.mark.gpu

TOL = 1e-5
ATOL_ZERO = 1e-5   # temporalConv.bias grad (identically 0 in exact arithmetic)
TOL_RUNNING = 1e-5

DEV = "cuda:0"


def _fold_prep(pkg, cu, xshape, C_out, K, stride, gemm):
    """ABI 7 stgcn_fold_prep of one folded block (as STGCNStack does per step)"""
    import ctypes
    hl = pkg.hip_lib
    lib = hl.lib()
    d = pkg.fused.make_desc(tuple(xshape), C_out, K, stride, 4, 1e-5, 0.1, True,
                            **pkg.fused._gemm_flags(gemm))
    nbytes = lib.stgcn_fold_prep_bytes(ctypes.byref(d))
    assert nbytes > 0, "the block does not fold"
    buf = torch.empty(nbytes, device=DEV, dtype=torch.uint8)
    w = hl.FoldWeights(*[hl.ptr(cu[k]) for k in (
        "spatialConv.A", "spatialConv.W.weight", "spatialConv.W.bias", "temporalConv.weight",
        "temporalConv.bias")])
    hl.check(lib.stgcn_fold_prep(1, (hl.Desc * 1)(d), (hl.FoldWeights * 1)(w),
                                 (ctypes.c_void_p * 1)(hl.ptr(buf)), hl.stream_handle(DEV)))
    return buf


def _run_hip(pkg, arrays, x, g, need_dx=True, gemm="fp32", prep=False):
    """Fused block fwd+bwd on the GPU; returns the oracle-style result dict.
    gemm: channel-GEMM arithmetic ("fp32", "f32x3", "bf16"; fused._gemm_flags).
    prep: the folded block's weight operands from stgcn_fold_prep (ABI 7)."""
    p, b = ref_cpu.block_params_from_arrays(arrays, dtype=torch.float32, requires_grad=False)
    stride, residual = int(arrays["meta"][2]), bool(arrays["meta"][7])
    cu = {k: v.to(DEV).contiguous().requires_grad_(True) for k, v in p.items()}
    cc = None
    if prep:
        with torch.no_grad():
            buf = _fold_prep(pkg, cu, x.shape, cu["temporalConv.weight"].shape[0],
                             cu["spatialConv.A"].shape[0], stride, gemm)
        cc = pkg.fused.ChainCtx(prep=buf)
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
            stride, 4, 1e-5, 0.1, True, None, 0.0, gemm)
    else:
        y = pkg.fused.StgcnBlockFn.apply(*common, *running, stride, 4, 1e-5, 0.1, True,
                                         cc, 0.0, gemm)
    y.backward(g.to(DEV).float())
    torch.cuda.synchronize()
    out = {"y": y.detach().cpu()}
    if need_dx:
        out["grad.x"] = xd.grad.cpu()
    for k, t in cu.items():
        out["grad." + k] = t.grad.cpu()
    for k, t in bu.items():
        out["after." + k] = t.cpu()
    return out


def _compare(got, want, residual=False, tol=TOL, floor=None):
    """floor: optional {key: rel error of the fp32 reference vs fp64}."""
    bad = []
    for k, w in want.items():
        if k not in got or k.endswith("num_batches_tracked"):
            continue
        gv = got[k].double().numpy()
        wv = w.detach().double().numpy() if torch.is_tensor(w) else np.asarray(w, np.float64)
        if k == "grad.temporalConv.bias" and not residual:
            err = float(np.abs(gv - wv).max())
            lim = max(ATOL_ZERO, 2.0 * floor.get("abs:" + k, 0.0)) if floor else ATOL_ZERO
            if err > lim:
                bad.append((k, err, lim))
            continue
        err = rel_to_max(gv, wv)
        lim = max(tol, 2.0 * floor.get(k, 0.0)) if floor else tol
        if err > lim:
            bad.append((k, err, lim))
    assert not bad, "; ".join(f"{k}: {e:.2e} > {l:.1e}" for k, e, l in bad)


@pytest.mark.parametrize("gemm", ["fp32", "f32x3", "f16x2"])
@pytest.mark.parametrize("fixture", block_fixtures())
def test_block_matches_reference_fixture(pkg, fixture, gemm):
    """The reference's own block fixtures through every fp32 GEMM mode: exact
    fp32 MFMA, the 3-way bf16 splits and the benched 2-way fp16 splits (the
    latter two where the block's GEMMs take them; elsewhere the same kernels as
    fp32), each at the fp32 gate against the fp64 oracle and within 5e-5 of the
    reference's own fp32 outputs."""
    ref = load_npz(fixture)
    residual = bool(ref["meta"][7])
    x = torch.from_numpy(ref["x"])
    g = torch.from_numpy(ref["g"])
    got = _run_hip(pkg, ref, x, g, gemm=gemm)
    want64, floor = _oracle(ref, got)
    _compare(got, want64, residual=residual, floor=floor)
    # and against the reference's own fp32 outputs (its rounding included)
    _compare(got, {k: torch.from_numpy(v) for k, v in ref.items()
                   if k == "y" or k.startswith("grad.")}, residual=residual, tol=5e-5)


# ReLU ties: a pre-ReLU value within fp32 rounding of 0 can land on either
# side in any fp32 implementation (the reference's included), and flipping one
# element changes every gradient by that element's contribution (~1e-3 of a
# BN2 bias grad at these sizes). The parity check therefore (1) requires the
# HIP ReLU mask to agree with the fp64 oracle's everywhere except at such ties
# (|pre-ReLU| < TIE), and (2) differentiates the oracle through the HIP mask.
TIE = 1e-5


def _oracle(arrays, got):
    mask = (got["y"] > 0)
    pre = ref_cpu.block_pre_relu(arrays)
    flips = (mask != (pre > 0))
    if flips.any():
        assert pre[flips].abs().max().item() < TIE, "ReLU mask differs away from a tie"
    want = ref_cpu.block_step(arrays, dtype=torch.float64, relu_mask=mask)
    ref32 = ref_cpu.block_step(arrays, dtype=torch.float32, relu_mask=mask)
    floor = {k: rel_to_max(ref32[k].detach().double().numpy(), v.detach().double().numpy())
             for k, v in want.items() if k in ref32 and "num_batches" not in k}
    k = "grad.temporalConv.bias"  # (analytically zero: its floor is the fp32 absolute error)
    if k in ref32 and k in want:
        floor["abs:" + k] = float((ref32[k].detach().double() - want[k].detach().double()).abs().max())
    return want, floor


def _random_case(pkg, C_in, C_out, stride, V, K, N, T, seed=0, residual=False, A=None):
    return _random_case_once(pkg, C_in, C_out, stride, V, K, N, T, seed, residual, A)


def _random_case_once(pkg, C_in, C_out, stride, V, K, N, T, seed=0, residual=False, A=None):
    gr = pkg.graph
    strat = 0 if K == 1 else 2
    if A is None:
        A = gr.get_normalized_adjacency_matrices(strat, 1, distances=gr.synthetic_distances(V),
                                                 graph=gr.graph_for(V))
    torch.manual_seed(seed)
    blk = pkg.SpatialTemporalConv(C_in, C_out, A, 9, stride, 4, dropout_rate=0,
                                  residual=residual)
    gen = torch.Generator().manual_seed(seed + 3)
    with torch.no_grad():
        for bn in (blk.batch_n, blk.batch_n_2):
            bn.weight.copy_(1.0 + 0.1 * torch.randn(bn.weight.shape, generator=gen))
            bn.bias.copy_(0.1 * torch.randn(bn.bias.shape, generator=gen))
    arrays = {"param." + k: v.detach().numpy() for k, v in blk.state_dict().items()}
    arrays["meta"] = np.array([C_in, C_out, stride, V, strat, N, T, int(residual)])
    x = torch.randn(N, C_in, T, V, generator=torch.Generator().manual_seed(seed + 1))
    T_out = (T - 1) // stride + 1
    g = torch.randn(N, C_out, T_out, V, generator=torch.Generator().manual_seed(seed + 2))
    arrays["x"] = x.numpy()
    arrays["g"] = g.numpy()
    return arrays, x, g


@pytest.mark.parametrize("case", [
    # C_in, C_out, stride, V, K, N, T
    (3, 64, 1, 18, 1, 3, 45),       # first block (C_in=3), ragged T
    (64, 64, 1, 18, 1, 4, 64),      # cfg2 L1 shape, small N
    (64, 128, 2, 18, 1, 3, 37),     # stride 2, odd T
    (128, 256, 2, 18, 1, 2, 30),    # L7 shape (R=256 -> 4 row tiles)
    (256, 256, 1, 18, 1, 2, 19),    # L8 shape
    (64, 64, 1, 25, 3, 2, 40),      # NTU: spatial partitioning K=3
    (64, 128, 2, 25, 3, 2, 33),
    (3, 64, 1, 50, 3, 2, 20),       # two-person V=50
    (64, 64, 1, 50, 3, 2, 17),
    (5, 7, 1, 18, 1, 2, 9),         # odd channel counts (partial tiles everywhere)
    (64, 64, 2, 18, 1, 1, 1),       # T=1 (single frame)
])
def test_block_matches_oracle_random(pkg, case):
    C_in, C_out, stride, V, K, N, T = case
    arrays, x, g = _random_case(pkg, C_in, C_out, stride, V, K, N, T)
    got = _run_hip(pkg, arrays, x, g)
    want, floor = _oracle(arrays, got)
    _compare(got, want, floor=floor)


@pytest.mark.parametrize("V", [50, 57])
def test_block_k1_many_joints(pkg, V):
    """One adjacency partition over more joints than the reference's graphs (a
    random sparse A; V = 57 is the largest joint count whose tiles fit LDS at
    these channel counts): the backward's per-tap dU sums (k_fold_tq) and the
    spatial kernels at V > 32. V = 70 is refused up front (STGCN_E_UNSUPPORTED,
    tile geometry), not run."""
    rng = np.random.default_rng(5)  # (a sparse random A: a dense positive one averages the
    # joints into near-constant channels whose BN2 statistics are ill-conditioned)
    A = 0.5 * np.eye(V) + rng.uniform(0.0, 1.0, (V, V)) * (rng.random((V, V)) < 0.15) / np.sqrt(V)
    A = torch.from_numpy(A[None]).float()
    arrays, x, g = _random_case(pkg, 16, 32, 1, V, 1, 2, 11, A=A)
    got = _run_hip(pkg, arrays, x, g)
    want, floor = _oracle(arrays, got)
    _compare(got, want, floor=floor)
    with pytest.raises(RuntimeError, match=r"failed \(-2\)"):  # STGCN_E_UNSUPPORTED
        pkg.hip_lib.block_plan(pkg.fused.make_desc((2, 16, 11, 70), 32, 1, 1, 4, 1e-5, 0.1, True))


def test_first_block_without_dx(pkg):
    """need_dx = 0 path (input does not require grad): params grads unchanged."""
    arrays, x, g = _random_case(pkg, 3, 64, 1, 18, 1, 2, 30)
    got = _run_hip(pkg, arrays, x, g, need_dx=False)
    want, floor = _oracle(arrays, got)
    want.pop("grad.x")
    _compare(got, want, floor=floor)


def test_full_size_block_properties(pkg):
    """cfg2 layer-1 shape at N=32 (oracle too slow at N=128): parity with the
    fp64 oracle on a slice of outputs plus size-independent properties."""
    arrays, x, g = _random_case(pkg, 64, 64, 1, 18, 1, 32, 300, seed=7)
    got = _run_hip(pkg, arrays, x, g)
    # BN2 followed by ReLU: per-channel pre-ReLU mean equals beta2 -> check the
    # batch statistics went through: y >= 0, and grads finite.
    assert (got["y"] >= 0).all()
    for k, v in got.items():
        assert torch.isfinite(v).all(), k
    want, floor = _oracle(arrays, got)
    _compare(got, want, floor=floor)


def test_eval_mode_uses_running_stats(pkg):
    arrays, x, _ = _random_case(pkg, 64, 128, 2, 18, 1, 2, 21)
    p, b = ref_cpu.block_params_from_arrays(arrays, dtype=torch.float32, requires_grad=False)
    # non-trivial running stats
    gen = torch.Generator().manual_seed(11)
    for k in b:
        if "running_mean" in k:
            b[k] = 0.1 * torch.randn(b[k].shape, generator=gen)
        elif "running_var" in k:
            b[k] = 0.5 + torch.rand(b[k].shape, generator=gen)
    cu = {k: v.to(DEV) for k, v in p.items()}
    bu = {k: v.to(DEV).clone() for k, v in b.items() if "num_batches" not in k}
    with torch.no_grad():
        y = pkg.fused.StgcnBlockFn.apply(
            x.to(DEV), cu["spatialConv.A"], cu["spatialConv.W.weight"], cu["spatialConv.W.bias"],
            cu["temporalConv.weight"], cu["temporalConv.bias"], cu["batch_n.weight"],
            cu["batch_n.bias"], cu["batch_n_2.weight"], cu["batch_n_2.bias"],
            bu["batch_n.running_mean"], bu["batch_n.running_var"],
            bu["batch_n_2.running_mean"], bu["batch_n_2.running_var"], 2, 4, 1e-5, 0.1, False)
    p64 = {k: v.double() for k, v in p.items()}
    b64 = {k: (v.double() if v.is_floating_point() else v) for k, v in b.items()}
    want = ref_cpu.block_forward(x.double(), p64, b64, 2, training=False, dtype=torch.float64)
    assert rel_to_max(y.cpu().numpy(), want.numpy()) < TOL
    for k in bu:  # eval mode leaves running stats untouched
        assert torch.equal(bu[k].cpu(), b[k])


@pytest.mark.parametrize("case", [
    # C_in, C_out, stride, V, K, N, T   (residual block, st_graphconv.py:60-82)
    (64, 64, 1, 18, 1, 3, 40),      # identity residual
    (64, 128, 2, 18, 1, 2, 37),     # projection, stride 2, odd T
    (3, 64, 1, 18, 1, 3, 45),       # projection, stride 1 (channels differ)
    (128, 128, 1, 25, 3, 2, 30),    # identity, K=3
    (64, 128, 2, 25, 3, 2, 33),     # projection, K=3
    (64, 64, 1, 50, 3, 2, 17),      # identity, V=50
    (5, 7, 2, 18, 1, 2, 9),         # odd channel counts, projection stride 2
])
def test_residual_block_matches_oracle_random(pkg, case):
    C_in, C_out, stride, V, K, N, T = case
    arrays, x, g = _random_case(pkg, C_in, C_out, stride, V, K, N, T, residual=True)
    got = _run_hip(pkg, arrays, x, g)
    want, floor = _oracle(arrays, got)
    _compare(got, want, residual=True, floor=floor)


def test_residual_block_without_dx(pkg):
    arrays, x, g = _random_case(pkg, 3, 64, 2, 18, 1, 2, 30, residual=True)
    got = _run_hip(pkg, arrays, x, g, need_dx=False)
    want, floor = _oracle(arrays, got)
    want.pop("grad.x")
    _compare(got, want, residual=True, floor=floor)


def test_residual_full_size_block(pkg):
    """cfg2 L4 shape (64 -> 128, stride 2, projection) at N=16, T=300."""
    arrays, x, g = _random_case(pkg, 64, 128, 2, 18, 1, 16, 300, seed=5, residual=True)
    got = _run_hip(pkg, arrays, x, g)
    for k, v in got.items():
        assert torch.isfinite(v).all(), k
    want, floor = _oracle(arrays, got)
    _compare(got, want, residual=True, floor=floor)


def test_residual_eval_mode(pkg):
    arrays, x, _ = _random_case(pkg, 64, 128, 2, 18, 1, 2, 21, residual=True)
    p, b = ref_cpu.block_params_from_arrays(arrays, dtype=torch.float32, requires_grad=False)
    gen = torch.Generator().manual_seed(12)
    for k in b:
        if "running_mean" in k:
            b[k] = 0.1 * torch.randn(b[k].shape, generator=gen)
        elif "running_var" in k:
            b[k] = 0.5 + torch.rand(b[k].shape, generator=gen)
    cu = {k: v.to(DEV) for k, v in p.items()}
    bu = {k: v.to(DEV).clone() for k, v in b.items() if "num_batches" not in k}
    with torch.no_grad():
        y = pkg.fused.StgcnResBlockFn.apply(
            x.to(DEV), cu["spatialConv.A"], cu["spatialConv.W.weight"], cu["spatialConv.W.bias"],
            cu["temporalConv.weight"], cu["temporalConv.bias"], cu["batch_n.weight"],
            cu["batch_n.bias"], cu["batch_n_2.weight"], cu["batch_n_2.bias"],
            cu["apply_residual.weight"], cu["apply_residual.bias"],
            bu["batch_n.running_mean"], bu["batch_n.running_var"],
            bu["batch_n_2.running_mean"], bu["batch_n_2.running_var"], 2, 4, 1e-5, 0.1, False)
    p64 = {k: v.double() for k, v in p.items()}
    b64 = {k: (v.double() if v.is_floating_point() else v) for k, v in b.items()}
    want = ref_cpu.block_forward(x.double(), p64, b64, 2, residual=True, training=False,
                                 dtype=torch.float64)
    assert rel_to_max(y.cpu().numpy(), want.numpy()) < TOL
    for k in bu:
        assert torch.equal(bu[k].cpu(), b[k])


# --- fused dropout (st_graphconv.py:50-54, :107-108) -----------------------
# The HIP block draws its keep mask from a counter-based hash of the flat NCTV
# output index (splitmix64, internal.h dropout_keep); torch's Philox stream is
# not reproducible outside torch, and any two dropout implementations differ
# in their random stream. Parity: the oracle differentiated through the SAME
# mask (relu mask x keep / (1-p)) -- everything else must match exactly as in
# the dropout-free tests -- and the mask is checked for its distribution.


def _keep_mask(seed, shape, p):
    e = np.arange(int(np.prod(shape)), dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + e * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z ^= z >> np.uint64(31)
    thresh = min(int(p * 2.0 ** 32), 2 ** 32 - 1)
    return torch.from_numpy(((z >> np.uint64(32)) >= np.uint64(thresh)).reshape(shape))


def _run_hip_dropout(pkg, arrays, x, g, drop):
    torch.manual_seed(1234)
    seed = int(torch.randint(0, 2 ** 62, (1,)).item())   # fused._dropout_seed's draw
    torch.manual_seed(1234)
    p, b = ref_cpu.block_params_from_arrays(arrays, dtype=torch.float32, requires_grad=False)
    stride, residual = int(arrays["meta"][2]), bool(arrays["meta"][7])
    cu = {k: v.to(DEV).contiguous().requires_grad_(True) for k, v in p.items()}
    bu = {k: v.to(DEV).clone() for k, v in b.items() if "num_batches" not in k}
    xd = x.to(DEV).float().contiguous().requires_grad_(True)
    common = (xd, cu["spatialConv.A"], cu["spatialConv.W.weight"], cu["spatialConv.W.bias"],
              cu["temporalConv.weight"], cu["temporalConv.bias"], cu["batch_n.weight"],
              cu["batch_n.bias"], cu["batch_n_2.weight"], cu["batch_n_2.bias"])
    running = (bu["batch_n.running_mean"], bu["batch_n.running_var"],
               bu["batch_n_2.running_mean"], bu["batch_n_2.running_var"])
    if residual:
        y = pkg.fused.StgcnResBlockFn.apply(
            *common, cu.get("apply_residual.weight"), cu.get("apply_residual.bias"), *running,
            stride, 4, 1e-5, 0.1, True, None, drop)
    else:
        y = pkg.fused.StgcnBlockFn.apply(*common, *running, stride, 4, 1e-5, 0.1, True,
                                         None, drop)
    y.backward(g.to(DEV).float())
    torch.cuda.synchronize()
    out = {"y": y.detach().cpu(), "grad.x": xd.grad.cpu()}
    for k, t in cu.items():
        out["grad." + k] = t.grad.cpu()
    for k, t in bu.items():
        out["after." + k] = t.cpu()
    return out, seed


@pytest.mark.parametrize("case", [
    # C_in, C_out, stride, V, K, N, T, residual, p
    (64, 64, 1, 18, 1, 3, 40, False, 0.5),     # specialised conv + bn_relu_fwd dropout
    (64, 128, 2, 18, 1, 2, 37, False, 0.2),
    (5, 7, 1, 18, 1, 2, 9, False, 0.5),        # generic conv, partial tiles
    (64, 64, 1, 18, 1, 3, 40, True, 0.5),      # dropout in the tconv epilogue
    (64, 128, 2, 25, 3, 2, 33, True, 0.3),     # projection residual, NTU graph
    (3, 64, 1, 50, 3, 2, 20, False, 0.9),
])
def test_block_dropout_matches_oracle(pkg, case):
    *shape, residual, drop = case
    C_in, C_out, stride, V, K, N, T = shape
    arrays, x, g = _random_case(pkg, C_in, C_out, stride, V, K, N, T, seed=5,
                                residual=residual)
    got, seed = _run_hip_dropout(pkg, arrays, x, g, drop)
    keep = _keep_mask(seed, tuple(got["y"].shape), drop)
    # mask statistics: the fraction kept is 1-p (binomial, 6 sigma)
    n = keep.numel()
    assert abs(keep.double().mean().item() - (1 - drop)) < 6 * (drop * (1 - drop) / n) ** 0.5
    y = got["y"]
    assert (y[~keep] == 0).all(), "dropped elements must be 0"
    pre = ref_cpu.block_pre_relu(arrays)
    relu = y > 0
    kflips = keep & (relu != (pre > 0))
    if kflips.any():
        assert pre[kflips].abs().max().item() < TIE, "ReLU mask differs away from a tie"
    mask = (keep & relu).double() / (1 - drop)
    want = ref_cpu.block_step(arrays, dtype=torch.float64, relu_mask=mask)
    ref32 = ref_cpu.block_step(arrays, dtype=torch.float32, relu_mask=mask.float())
    floor = {k: rel_to_max(ref32[k].detach().double().numpy(), v.detach().double().numpy())
             for k, v in want.items() if k in ref32 and "num_batches" not in k}
    _compare(got, want, residual=residual, floor=floor)


def test_block_dropout_seed_reproducible(pkg):
    """Same torch seed -> same mask; different seed -> different mask."""
    arrays, x, g = _random_case(pkg, 64, 64, 1, 18, 1, 2, 30, seed=2)
    a, sa = _run_hip_dropout(pkg, arrays, x, g, 0.5)
    b, sb = _run_hip_dropout(pkg, arrays, x, g, 0.5)
    assert sa == sb and torch.equal(a["y"], b["y"])
    assert not torch.equal(_keep_mask(sa, (2, 64, 30, 18), 0.5),
                           _keep_mask(sa + 1, (2, 64, 30, 18), 0.5))


@pytest.mark.parametrize("gemm", ["fp32", "f32x3", "f16x2"])
def test_bench_size_block(pkg, gemm):
    """The cfg2 layer-1 block at the bench's exact per-GPU size (N = 128,
    T = 300, V = 18), fp32 MFMA and the benched bf16x3 split path, against the
    fp64 oracle at the fp32 gate (bias-type gradients: 2x the fp32
    reference's own error, as everywhere)."""
    arrays, x, g = _random_case(pkg, 64, 64, 1, 18, 1, 128, 300, seed=9)
    got = _run_hip(pkg, arrays, x, g, gemm=gemm)
    for k, v in got.items():
        assert torch.isfinite(v).all(), k
    want, floor = _oracle(arrays, got)
    _compare(got, want, floor=floor)

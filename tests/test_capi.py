"""The C-ABI library builds, loads and exports every symbol include/stgcn_hip.h
declares; descriptor validation and workspace sizing work without a GPU."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "stgcn_hip.h")


def _header_functions():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|size_t|const char\s*\*)\s*\*?\s*(stgcn_\w+)\s*\(",
                                 text, flags=re.M)))


@pytest.fixture(scope="module")
def lib(pkg):
    return pkg.hip_lib.load_library()


def test_header_declares_entry_points(pkg):
    assert _header_functions() == sorted(pkg.hip_lib.EXPORTED)


def test_library_exports_every_header_symbol(pkg, lib):
    for name in _header_functions():
        assert hasattr(lib, name), name
    assert lib.stgcn_abi_version() == pkg.hip_lib.ABI_VERSION == 11


def _desc(pkg, **kw):
    base = dict(N=128, C_in=64, C_out=64, T=300, T_out=300, V=18, K=1, gamma=9, stride=1,
                pad=4, eps=1e-5, momentum=0.1, training=1, need_dx=1, flags=0)
    base.update(kw)
    return pkg.hip_lib.Desc(**base)


def test_check_desc_accepts_north_star_shapes(pkg, lib):
    for kw in (dict(), dict(C_in=3), dict(C_in=64, C_out=128, stride=2, T_out=150),
               dict(V=25, K=3), dict(V=50, K=3, C_in=256, C_out=256, T=75, T_out=75),
               dict(flags=1), dict(flags=1, C_in=64, C_out=128, stride=2, T_out=150),
               dict(flags=1, V=25, K=3, C_in=3),
               # STGCN_F_BF16 (cfg3 / cfg5 shapes, residual + bf16)
               dict(flags=2, V=25, K=3), dict(flags=2, V=50, K=3, C_in=128, C_out=256, stride=2,
                                               T_out=150), dict(flags=3, V=18),
               # STGCN_F_F32X3 (fp32 via bf16 splits), plain and residual; + STGCN_F_F16X2
               dict(flags=4), dict(flags=5, V=25, K=3), dict(flags=12),
               # + STGCN_F_NO_G (ABI 7)
               dict(flags=28)):
        d = _desc(pkg, **kw)
        assert lib.stgcn_check_desc(ctypes.byref(d)) == 0, kw
        assert lib.stgcn_fwd_workspace_bytes(ctypes.byref(d)) > 0
        assert lib.stgcn_bwd_workspace_bytes(ctypes.byref(d)) > 0


@pytest.mark.parametrize("kw,code", [
    (dict(flags=32), -2), (dict(flags=16), -1), (dict(flags=20), -1), (dict(flags=8), -1), (dict(flags=10), -1), (dict(flags=6), -1), (dict(gamma=7, pad=3, T_out=300), -2), (dict(stride=3, T_out=100), -2),
    (dict(T_out=299), -1), (dict(N=0), -1), (dict(V=300), -2)])
def test_check_desc_rejects(pkg, lib, kw, code):
    d = _desc(pkg, **kw)
    assert lib.stgcn_check_desc(ctypes.byref(d)) == code
    assert lib.stgcn_last_error()
    assert lib.stgcn_fwd_workspace_bytes(ctypes.byref(d)) == 0


def test_null_arguments_fail_without_touching_gpu(pkg, lib):
    d = _desc(pkg)
    args = pkg.hip_lib.FwdArgs()
    assert lib.stgcn_block_fwd(ctypes.byref(d), ctypes.byref(args), None, 0, None) == -1
    assert b"null" in lib.stgcn_last_error()


def test_residual_null_projection_fails(pkg, lib):
    """A projection residual block (C_in != C_out) needs Wr / br / Za."""
    d = _desc(pkg, flags=1, C_in=32)
    args = pkg.hip_lib.FwdArgs(*([ctypes.c_void_p(256)] * 18))  # dummy non-null core args
    assert lib.stgcn_block_fwd(ctypes.byref(d), ctypes.byref(args), None, 0, None) == -1
    assert b"residual" in lib.stgcn_last_error()


def test_cpu_tensors_fail_loudly(pkg):
    """No CPU fallback on the product path."""
    import torch
    A = torch.ones(1, 18, 18)
    blk = pkg.SpatialTemporalConv(3, 64, A, 9, 1, 4, dropout_rate=0)
    with pytest.raises(RuntimeError):
        blk(torch.randn(2, 3, 20, 18))


def test_spatial_desc_workspace_and_rejects(pkg, lib):
    """ABI 4 SpatialConv entry points: workspace queries for the reference's
    graphs; unknown flags / bad shapes rejected without touching the GPU."""
    SD = pkg.hip_lib.SpatialDesc
    for kw in (dict(V=18, K=1, C_in=3), dict(V=25, K=3), dict(V=50, K=3, flags=2)):
        base = dict(N=8, C_in=64, C_out=64, T=300, V=18, K=1, flags=0)
        base.update(kw)
        d = SD(**base)
        assert lib.stgcn_spatial_workspace_bytes(ctypes.byref(d), 0) > 0, kw
        assert lib.stgcn_spatial_workspace_bytes(ctypes.byref(d), 1) > 0, kw
    for kw in (dict(flags=1), dict(flags=4), dict(N=0), dict(V=300)):
        base = dict(N=8, C_in=64, C_out=64, T=300, V=18, K=1, flags=0)
        base.update(kw)
        d = SD(**base)
        assert lib.stgcn_spatial_workspace_bytes(ctypes.byref(d), 0) == 0, kw
    d = SD(N=8, C_in=64, C_out=64, T=30, V=18, K=1, flags=0)
    assert lib.stgcn_spatial_fwd(ctypes.byref(d), None, None, None, None, None, None, 0,
                                 None) == -1
    assert b"null" in lib.stgcn_last_error()


def test_block_plan_pins_the_paths(pkg, lib):
    """ABI 6 stgcn_block_plan (host logic, no GPU): the fp32 split path folds W'
    into the temporal conv on the cfg2 non-residual blocks with C_in >= 16
    (STGCN_PLAN_FOLD) and keeps the unfolded spatial dW' on split products where
    it does not fold (residual blocks); the bf16 path fuses both SpatialConv
    halves at V = 25, K = 3; the exact fp32-MFMA path selects none of these."""
    hl = pkg.hip_lib
    plan = lambda **kw: hl.block_plan(_desc(pkg, **kw))  # noqa: E731
    p = plan(flags=4)  # cfg2 L1-type block (64 -> 64)
    assert p & hl.PLAN_FOLD and p & hl.PLAN_TCONV_SPLIT and p & hl.PLAN_TWGRAD_SPLIT, p
    assert p & hl.PLAN_SP_BWD_FUSED, p  # the SpatialConv backward in the data gradient
    assert plan(flags=4, C_in=128, C_out=256, stride=2, T=150, T_out=75) & hl.PLAN_FOLD
    assert not plan(flags=4, C_in=3) & hl.PLAN_FOLD          # C_in < 16
    p = plan(flags=5)                                        # residual: never folded
    assert not p & hl.PLAN_FOLD and p & hl.PLAN_WSP_SPLIT, p
    assert not plan(flags=4, V=25, K=3) & hl.PLAN_FOLD       # K = 3
    # the reference's default graph (V = 25, unilabeling K = 1) folds too, with the
    # unfused SpatialConv backward (the fused epilogue is V = 18 only)
    p = plan(flags=12, V=25, K=1)
    assert p & hl.PLAN_FOLD and p & hl.PLAN_F16X2 and not p & hl.PLAN_SP_BWD_FUSED, p
    assert not p & hl.PLAN_X_FROM_U, p
    assert not plan(flags=12, V=50, K=1) & hl.PLAN_FOLD      # (no V = 50 split instances)
    p = plan(flags=2, V=25, K=3)
    assert p & hl.PLAN_SP_FWD_FUSED and p & hl.PLAN_SP_BWD_FUSED and not p & hl.PLAN_FOLD, p
    assert plan() == 0
    # STGCN_F_F16X2 (with F32X3): the folded GEMMs on fp16 splits; unfolded blocks unchanged
    p = plan(flags=12)
    assert p & hl.PLAN_FOLD and p & hl.PLAN_F16X2, p
    # the unfolded first block (C_in = 3): forward and weight gradient on fp16 splits
    p = plan(flags=12, C_in=3)
    assert p & hl.PLAN_F16X2 and not p & hl.PLAN_FOLD, p
    assert not plan(flags=13) & hl.PLAN_F16X2
    d = _desc(pkg, N=0)
    out = ctypes.c_uint32(7)
    assert lib.stgcn_block_plan(ctypes.byref(d), ctypes.byref(out)) == -1


def test_fold_prep_sizes(pkg, lib):
    """ABI 7 stgcn_fold_prep_bytes: a buffer for the folded split-path blocks
    (K = 1, V = 18, fp32 via splits), none for blocks that do not fold (first
    block C_in = 3, K = 3, residual, bf16, exact fp32 MFMA)."""
    fl = pkg.hip_lib
    folded = [dict(C_in=64, flags=12), dict(C_in=64, C_out=128, stride=2, T_out=150, flags=12),
              dict(C_in=64, flags=4), dict(C_in=64, flags=28), dict(C_in=64, V=25, flags=12)]
    for kw in folded:
        assert lib.stgcn_fold_prep_bytes(ctypes.byref(_desc(pkg, **kw))) > 0, kw
    for kw in (dict(C_in=3, flags=12), dict(V=25, K=3, flags=4), dict(C_in=64, flags=13),
               dict(C_in=64, flags=2), dict(C_in=64, flags=0)):
        assert lib.stgcn_fold_prep_bytes(ctypes.byref(_desc(pkg, **kw))) == 0, kw
    # no blocks: nothing to do, no GPU touched
    assert lib.stgcn_fold_prep(0, None, None, None, None) == 0



def test_x_from_u_plan_and_argument_checks(pkg, lib):
    """ABI 8 (host logic, no GPU): STGCN_PLAN_X_FROM_U on the folded training
    blocks that form G (cfg2 f16x2 / split paths) and, round 6, on the bf16
    blocks whose fused spatial forward stages x (cfg3 / cfg5: V = 25, 50 with
    K = 3); not in eval, not without G (STGCN_F_NO_G), not on residual blocks,
    not where the block neither folds nor runs the bf16 fused forward. A forward
    with prev_U on a block without the plan, and a backward with x null outside
    it, fail before any launch."""
    hl = pkg.hip_lib
    plan = lambda **kw: hl.block_plan(_desc(pkg, **kw))  # noqa: E731
    for kw in (dict(flags=12), dict(flags=4), dict(flags=12, C_in=128, C_out=256, stride=2,
                                                  T=150, T_out=75),
               dict(flags=2, V=25, K=3), dict(flags=2, V=50, K=3)):
        assert plan(**kw) & hl.PLAN_X_FROM_U, kw
    for kw in (dict(flags=12, training=0), dict(flags=28), dict(flags=12, C_in=3),
               dict(flags=13), dict(flags=3, V=25, K=3), dict(flags=2, V=25, K=3, training=0),
               dict(flags=0)):
        assert not plan(**kw) & hl.PLAN_X_FROM_U, kw
    one = ctypes.c_void_p(256)
    d = _desc(pkg, flags=0)  # exact fp32 MFMA: no X_FROM_U
    a = hl.FwdArgs(*([one] * 18))
    a.prev_U = a.prev_stats = a.prev_g2 = a.prev_b2 = one
    a.x_stats = one
    assert lib.stgcn_block_fwd(ctypes.byref(d), ctypes.byref(a), None, 0, None) == -1
    assert b"prev_U" in lib.stgcn_last_error()
    b = hl.BwdArgs(*([one] * 23))
    b.x = None
    b.G = one
    assert lib.stgcn_block_bwd(ctypes.byref(d), ctypes.byref(b), None, 0, None) == -1
    assert b"x null" in lib.stgcn_last_error()


def test_head_link_decision(pkg):
    """ABI 9: the last block's output is left to the fused head only for a
    non-residual block without dropout and without forward hooks."""
    import contextlib
    import io
    gr = pkg.graph
    A = gr.get_normalized_adjacency_matrices(0, 1, graph=gr.graph_for(18))
    with contextlib.redirect_stdout(io.StringIO()):
        m = pkg.STGCNStack(3, 10, A)
        mr = pkg.STGCNStack(3, 10, A, residual=True)
        md = pkg.STGCNStack(3, 10, A, dropout_rate=0.5)
    assert pkg.fused.head_link_ok(m.conv[-1])
    assert not pkg.fused.head_link_ok(mr.conv[-1])
    assert not pkg.fused.head_link_ok(md.conv[-1])
    h = m.conv[-1].register_forward_hook(lambda *a: None)
    assert not pkg.fused.head_link_ok(m.conv[-1])
    h.remove()
    assert pkg.fused.head_link_ok(m.conv[-1])

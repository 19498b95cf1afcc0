"""``StgcnBlockFn`` / ``StgcnResBlockFn`` — the fused ST-GCN block as
torch.autograd.Functions.

Forward and backward are single calls into libstgcn_hip.so
(``stgcn_block_fwd`` / ``stgcn_block_bwd``) on the current HIP stream. The
math is that of ``SpatialTemporalConv.forward`` (src/network/st_graphconv.py:
97-109 for the default block, the residual block :60-82 with apply_residual
:24-28; SpatialConv :139-152; no dropout) and of its autograd backward
(driven by lightning_model.py:199-205).
"""
import ctypes
import weakref

import torch

from . import hip_lib


def _f32c(t, name):
    if t.dtype != torch.float32 or not t.is_contiguous() or not t.is_cuda:
        raise RuntimeError(f"{name}: expected a contiguous float32 GPU tensor")
    return t


def make_desc(x_shape, C_out, K, stride, pad, eps, momentum, training, need_dx=1, gamma=9,
              residual=False, bf16=False, f32x3=False, f16x2=False, no_g=False):
    N, C_in, T, V = x_shape
    T_out = (T + 2 * pad - gamma) // stride + 1
    flags = ((hip_lib.F_RESIDUAL if residual else 0) | (hip_lib.F_BF16 if bf16 else 0)
             | (hip_lib.F_F32X3 if f32x3 or f16x2 or no_g else 0)
             | (hip_lib.F_F16X2 if f16x2 or no_g else 0) | (hip_lib.F_NO_G if no_g else 0))
    return hip_lib.Desc(N, C_in, C_out, T, T_out, V, K, gamma, stride, pad, eps, momentum,
                        int(training), int(need_dx), flags)


def _gemm_flags(gemm):
    """Channel-GEMM arithmetic of a block: "fp32" (fp32 MFMA), "f32x3" (fp32 via
    exact 3-way bf16 operand splits, STGCN_F_F32X3), "f16x2_nog" (f16x2 without G,
    STGCN_F_NO_G: the memory-lean folded block), "f16x2" (STGCN_F_F32X3 with
    the folded GEMMs as 2-way fp16 splits of power-of-two-scaled operands,
    STGCN_F_F16X2), "bf16" (STGCN_F_BF16)."""
    if gemm not in ("fp32", "f32x3", "f16x2", "f16x2_nog", "bf16"):
        raise ValueError(f"unknown gemm mode {gemm!r}")
    return {"bf16": gemm == "bf16", "f32x3": gemm == "f32x3", "f16x2": gemm == "f16x2",
            "no_g": gemm == "f16x2_nog"}


class Link:
    """Hand-over between two chained blocks in backward: the later block
    computes the earlier block's ReLU+BN2 backward sums while writing its dx
    (``sums``); the earlier block uses them only if the gradient it receives is
    that very dx tensor, unmodified (``dx_ref`` / ``dx_version``).

    Deferred dx (ABI 5, ``coef`` set): the later block left dxhat in that
    tensor (its BN1 backward apply is folded into the earlier block's ReLU+BN2
    backward pass, which takes ``coef``). Within ``model.STGCNStack`` the tensor
    goes straight from one block's backward to the other's; if anything
    replaced or modified it in between, the true gradient was never formed and
    the earlier block raises instead of using it."""

    def __init__(self):
        self.sums = None
        self.dx_ref = None
        self.dx_version = None
        self.coef = None

    def valid_for(self, dy):
        return (self.sums is not None and self.dx_ref is not None and self.dx_ref() is dy
                and dy._version == self.dx_version)


class ChainCtx:
    """Per-block chaining arguments (see network.StackChain): x_stats / y_stats
    (fp64 [sum, sumsq] per channel of the block input / output), the Link to
    the previous block (``in_link``, with its BN2 affine ``prev_g2/prev_b2``)
    and to the next one (``out_link``)."""

    def __init__(self, x_stats=None, y_stats=None, in_link=None, out_link=None, prev_g2=None,
                 prev_b2=None, prev_U=None, prev_stats=None, prep=None):
        self.x_stats, self.y_stats = x_stats, y_stats
        # ABI 7: this block's stgcn_fold_prep buffer of the step (or None)
        self.prep = prep
        self.in_link, self.out_link = in_link, out_link
        self.prev_g2, self.prev_b2 = prev_g2, prev_b2
        # the previous block's pre-BN2 tensor and [mean2 | invstd2] (ABI 4): read
        # by the link for channels where uhat = (x - b2) / g2 is ill-conditioned
        self.prev_U, self.prev_stats = prev_U, prev_stats
        # this block's (U, [mean2 | invstd2]) for the next block's link
        self.U, self.stats2 = None, None
        # ABI 8: this block's y is not written (the next block forms it from U);
        # this block's input is the previous block's ReLU(BN2(prev_U)) (x unwritten)
        self.y_lazy, self.x_from_u = False, False
        # ABI 9: the last block's y is read by the head only, which pools it from
        # U (stgcn_head_fwd_u): neither y nor its statistics are formed
        self.y_head = False


def stack_descs(blocks, x_shape, training=True):
    """The training descriptors of a block stack's blocks (network.SpatialTemporalConv,
    in order) for a stack input of shape x_shape (N, C, T, V)."""
    N, C, T, V = x_shape
    out = []
    for blk in blocks:
        sc, tc = blk.spatialConv, blk.temporalConv
        desc = make_desc((N, C, T, V), tc.out_channels, sc.A.shape[0], blk.stride, blk.pad,
                         blk.batch_n.eps, blk.batch_n.momentum, training,
                         residual=blk.residual, **_gemm_flags(blk.gemm_mode()))
        out.append(desc)
        C, T = tc.out_channels, desc.T_out
    return out


def _hooked(m):
    """Forward hooks that could see a block's output or input (module-level or global)."""
    from torch.nn.modules import module as _mod
    return bool(m._forward_hooks or m._forward_pre_hooks
                or getattr(_mod, "_global_forward_hooks", None)
                or getattr(_mod, "_global_forward_pre_hooks", None))


def head_link_ok(blk):
    """True when the last block's output can stay unwritten because only the
    fused head reads it (ABI 9, stgcn_head_fwd_u): non-residual, no dropout,
    no forward hooks that could observe it."""
    drop = blk.dropout.p if blk.dropout is not None else 0.0
    return not blk.residual and drop == 0 and not _hooked(blk)


def lazy_links(blocks, x_shape):
    """Per block of a training stack: True when its output y can stay unwritten --
    the next block reads the block's U and forms ReLU(BN2(U)) on load (ABI 8,
    STGCN_PLAN_X_FROM_U). Needs a non-residual block without dropout feeding a
    block with that plan, and no forward hooks that could observe y."""
    descs = stack_descs(blocks, x_shape)
    out = []
    for i, blk in enumerate(blocks):
        ok = False
        if i + 1 < len(blocks):
            nxt = blocks[i + 1]
            drop = blk.dropout.p if blk.dropout is not None else 0.0
            ok = (not blk.residual and drop == 0 and not _hooked(blk) and not _hooked(nxt)
                  and bool(hip_lib.block_plan(descs[i + 1]) & hip_lib.PLAN_X_FROM_U))
        out.append(ok)
    return out


class FoldPrep:
    """The per-step weight preparation of a block stack's folded blocks (ABI 7
    stgcn_fold_prep: every folded block's Wc, bias table, max |Wc|, packed
    forward / data-gradient weights and backward re-layouts in about a dozen
    launches for the whole stack, instead of ~11 small launches per block).
    One buffer per block, reused every step while (C, T, V) and the GEMM mode
    stay the same; a step's forward and backward use the same weights, so they
    read the same buffers."""

    def __init__(self):
        self._bufs = {}

    def run(self, blocks, x_shape, dev):
        """blocks: the stack's SpatialTemporalConv modules in order; x_shape the
        stack input (N, C, T, V). Returns one prep tensor (or None) per block."""
        lib = hip_lib.lib()
        descs, weights, ptrs, out = [], [], [], []
        for i, (blk, desc) in enumerate(zip(blocks, stack_descs(blocks, x_shape))):
            sc, tc = blk.spatialConv, blk.temporalConv
            gemm = blk.gemm_mode()
            nbytes = lib.stgcn_fold_prep_bytes(ctypes.byref(desc))
            buf = None
            if nbytes:
                # (the contents depend on the weights and (C, T, V) only: keyed
                # without the batch, one buffer per block, replaced when the
                # shape changes -- a ragged last batch reuses it)
                key = (tuple(x_shape[1:]), gemm, nbytes, dev)
                held = self._bufs.get(i)
                buf = held[1] if held is not None and held[0] == key else None
                if buf is None:
                    buf = torch.empty(nbytes, device=dev, dtype=torch.uint8)
                    self._bufs[i] = (key, buf)
                descs.append(desc)
                weights.append(hip_lib.FoldWeights(*[hip_lib.ptr(t) for t in (
                    sc.A, sc.W.weight, sc.W.bias, tc.weight, tc.bias)]))
                ptrs.append(hip_lib.ptr(buf))
            out.append(buf)
        if descs:
            n = len(descs)
            hip_lib.check(lib.stgcn_fold_prep(
                n, (hip_lib.Desc * n)(*descs), (hip_lib.FoldWeights * n)(*weights),
                (ctypes.c_void_p * n)(*ptrs), hip_lib.stream_handle(dev)))
        return out


def _observed(xref):
    """True when the block input's gradient is observed by the caller: a tensor
    hook or ``retain_grad()`` on it. Deferred dx would hand such an observer the
    BN1-side dxhat instead of dL/dx, so those blocks form dx in full."""
    x = xref() if xref is not None else None
    return x is not None and (x.retains_grad or bool(getattr(x, "_backward_hooks", None)))


def _chain_bwd_args(cc, dy, need_dx, C_in, dev, xref=None):
    """(dy_sums, dy_coef, prev_g2, prev_b2, prev_sums, prev_U, prev_stats, x_stats,
    dx_coef) for stgcn_block_bwd. xref: weak reference to the block input; no
    deferred dx (dx_coef None) when its gradient is observed (``_observed``)."""
    none = (None,) * 9
    if cc is None:
        return none
    dy_sums = dy_coef = None
    link = cc.out_link
    if link is not None and link.sums is not None:
        if link.valid_for(dy):
            dy_sums, dy_coef = link.sums, link.coef
        elif link.coef is not None:
            raise RuntimeError(
                "STGCNStack chain: the gradient between two chained blocks was replaced or "
                "modified in backward (a hook?); the deferred-dx chain cannot form it")
    if cc.in_link is not None and need_dx:
        prev_sums = torch.empty(2 * C_in, device=dev, dtype=torch.float64)
        dx_coef = (None if _observed(xref)
                   else torch.empty(5 * C_in, device=dev, dtype=torch.float32))
        return (dy_sums, dy_coef, cc.prev_g2, cc.prev_b2, prev_sums, cc.prev_U, cc.prev_stats,
                cc.x_stats, dx_coef)
    return (dy_sums, dy_coef) + (None,) * 7


def _chain_publish(cc, prev_sums, dx, dx_coef=None):
    if prev_sums is not None:
        cc.in_link.sums = prev_sums
        cc.in_link.coef = dx_coef
        cc.in_link.dx_ref = weakref.ref(dx)
        cc.in_link.dx_version = dx._version


def _dropout_seed(drop, training):
    """Seed of this call's fused dropout, drawn from torch's default generator
    (so torch.manual_seed reproduces it); 0 when inactive."""
    if not (training and drop > 0):
        return 0
    return int(torch.randint(0, 2 ** 62, (1,)).item())


def _per_row(dy):
    """The (N, C) base of a gradient expanded over its last two axes (strides
    (C, 1, 0, 0) over a contiguous (N, C) tensor), else None (ABI 10 dy_nc)."""
    if dy.dim() != 4 or dy.stride(2) != 0 or dy.stride(3) != 0:
        return None
    N, C = dy.shape[0], dy.shape[1]
    if dy.stride(1) != 1 or (N > 1 and dy.stride(0) != C) or dy.dtype != torch.float32:
        return None
    return dy


def _args(cls, ptrs, drop, seed, **extra):
    a = cls(*ptrs)
    a.dropout_p = float(drop)
    a.seed = seed
    for k, v in extra.items():
        setattr(a, k, v)
    return a


def _keep_g(ctx, x, desc):
    """Buffer for the joint contraction G when a backward will run (the
    forward writes it once; the backward then skips recomputing it), else None
    (eval / no-grad: the library uses its workspace). Size and format from
    stgcn_keep_g_bytes: fp32 (N, K*C_in, T, V), or bf16 frame tiles where the
    bf16 path's fused spatial kernel runs."""
    if not (torch.is_grad_enabled() or any(ctx.needs_input_grad)):
        return None
    nbytes = hip_lib.lib().stgcn_keep_g_bytes(ctypes.byref(desc))
    return torch.empty(nbytes, device=x.device, dtype=torch.uint8)


class StgcnBlockFn(torch.autograd.Function):
    """forward(x, A, W, bW, Wt, bWt, g1, b1, g2, b2, rm1, rv1, rm2, rv2,
               stride, pad, eps, momentum, training) -> y

    Running stats (rm*, rv*) are updated in place when ``training``.
    Backward returns dx, dA, dW, dbW, dWt, dbWt, dg1, db1, dg2, db2.
    """

    @staticmethod
    def forward(ctx, x, A, W, bW, Wt, bWt, g1, b1, g2, b2, rm1, rv1, rm2, rv2,
                stride, pad, eps, momentum, training, cc=None, drop=0.0, gemm="fp32"):
        lib = hip_lib.lib()
        # (the caller's input tensor: a hook / retain_grad() on it turns deferred dx off)
        ctx.xref = weakref.ref(x) if cc is not None else None
        # ABI 8: x never written (the previous block's ReLU(BN2(U)) formed on load:
        # x is that block's placeholder, shape only); y not written (the next
        # block does the same, or the fused head pools from U): a one-element
        # placeholder of y's shape, so no dead activation is allocated or saved
        xu = cc is not None and cc.x_from_u
        y_lazy = cc is not None and cc.y_lazy
        if not xu:
            x = x.contiguous()
        names = ("x", "A", "W", "bW", "Wt", "bWt", "g1", "b1", "g2", "b2",
                 "rm1", "rv1", "rm2", "rv2")
        tensors = (x, A, W, bW, Wt, bWt, g1, b1, g2, b2, rm1, rv1, rm2, rv2)
        seed = _dropout_seed(drop, training)
        for t, n in zip(tensors, names):
            if not (xu and n == "x"):
                _f32c(t, n)
        N, C_in, T, V = x.shape
        K = A.shape[0]
        C_out = Wt.shape[0]
        desc = make_desc(x.shape, C_out, K, stride, pad, eps, momentum, training,
                         **_gemm_flags(gemm))
        hip_lib.check(lib.stgcn_check_desc(ctypes.byref(desc)))
        dev = x.device
        y_shape = (N, C_out, desc.T_out, V)
        y = (torch.empty(1, device=dev, dtype=torch.float32).expand(y_shape) if y_lazy
             else torch.empty(y_shape, device=dev, dtype=torch.float32))
        Z = torch.empty((N, C_out, T, V), device=dev, dtype=torch.float32)
        U = torch.empty(y_shape, device=dev, dtype=torch.float32)
        stats = torch.empty(2 * C_in + 2 * C_out, device=dev, dtype=torch.float32)
        G = _keep_g(ctx, x, desc)
        nbytes = lib.stgcn_fwd_workspace_bytes(ctypes.byref(desc))
        ws = torch.empty(nbytes, device=dev, dtype=torch.uint8)
        prep = cc.prep if cc is not None else None
        args = _args(hip_lib.FwdArgs, [hip_lib.ptr(t) for t in (
            None if xu else x, A, W, bW, Wt, bWt, g1, b1, g2, b2, rm1, rv1, rm2, rv2,
            None if y_lazy else y, Z, U, stats,
            None, None, None, G, cc and cc.x_stats, cc and cc.y_stats)], drop, seed,
            prep=hip_lib.ptr(prep))
        if xu:
            args.prev_U, args.prev_stats = hip_lib.ptr(cc.prev_U), hip_lib.ptr(cc.prev_stats)
            args.prev_g2, args.prev_b2 = hip_lib.ptr(cc.prev_g2), hip_lib.ptr(cc.prev_b2)
        ctx.x_lazy = xu
        hip_lib.check(lib.stgcn_block_fwd(ctypes.byref(desc), ctypes.byref(args),
                                          hip_lib.ptr(ws), nbytes, hip_lib.stream_handle(dev)))
        ctx.save_for_backward(x, Z, U, stats, A, W, bW, Wt, g1, b1, g2, b2, G)
        ctx.prep = prep
        if cc is not None:
            cc.U, cc.stats2 = U, stats[2 * C_in:]
        ctx.cfg = (stride, pad, eps, momentum, training)
        ctx.gemm = gemm
        ctx.cc = cc
        ctx.drop = (drop, seed)
        return y

    @staticmethod
    def backward(ctx, dy):
        lib = hip_lib.lib()
        x, Z, U, stats, A, W, bW, Wt, g1, b1, g2, b2, G = ctx.saved_tensors
        stride, pad, eps, momentum, training = ctx.cfg
        need_dx = bool(ctx.needs_input_grad[0])
        C_out = Wt.shape[0]
        # ABI 10: a gradient constant over (T, V) (the pooling head's, expanded
        # from (N, C_out)) goes in as dy_nc; anything else as a contiguous dy
        dy_nc = _per_row(dy)
        dy_full = dy
        dy = None if dy_nc is not None else dy.contiguous()
        desc = make_desc(x.shape, C_out, A.shape[0], stride, pad, eps, momentum, training,
                         need_dx=need_dx, **_gemm_flags(ctx.gemm))
        dy_sums, dy_coef, pg2, pb2, psums, pU, pst, xst, dx_coef = _chain_bwd_args(
            ctx.cc, dy_full, need_dx, x.shape[1], x.device, ctx.xref)
        deferred = ctypes.c_int32(0)
        dx = torch.empty_like(x) if need_dx else None
        grads = [torch.empty_like(t) for t in (A, W, bW, Wt)]
        dbWt = torch.empty(C_out, device=x.device, dtype=torch.float32)
        dg1, db1, dg2, db2 = (torch.empty_like(t) for t in (g1, b1, g2, b2))
        nbytes = lib.stgcn_bwd_workspace_bytes(ctypes.byref(desc))
        ws = torch.empty(nbytes, device=x.device, dtype=torch.uint8)
        args = _args(hip_lib.BwdArgs, [hip_lib.ptr(t) for t in (
            dy, None if ctx.x_lazy else x, Z, U, stats, A, W, bW, Wt, g1, b1, g2, b2, dx,
            grads[0], grads[1], grads[2], grads[3], dbWt, dg1, db1, dg2, db2,
            None, None, None, None, None, G, dy_sums, pg2, pb2, psums)], *ctx.drop,
            prev_U=hip_lib.ptr(pU), prev_stats=hip_lib.ptr(pst), x_stats=hip_lib.ptr(xst),
            dx_coef=hip_lib.ptr(dx_coef),
            dx_deferred=ctypes.addressof(deferred) if dx_coef is not None else None,
            dy_coef=hip_lib.ptr(dy_coef), prep=hip_lib.ptr(ctx.prep), dy_nc=hip_lib.ptr(dy_nc))
        rc = lib.stgcn_block_bwd(ctypes.byref(desc), ctypes.byref(args), hip_lib.ptr(ws), nbytes,
                                 hip_lib.stream_handle(x.device))
        if rc == hip_lib.E_UNSUPPORTED and dy_nc is not None:  # (needs the full dy)
            dy = dy_full.contiguous()
            args.dy, args.dy_nc = hip_lib.ptr(dy), None
            rc = lib.stgcn_block_bwd(ctypes.byref(desc), ctypes.byref(args), hip_lib.ptr(ws),
                                     nbytes, hip_lib.stream_handle(x.device))
        hip_lib.check(rc)
        _chain_publish(ctx.cc, psums, dx, dx_coef if deferred.value else None)
        dA, dW, dbW, dWt = grads
        return (dx, dA, dW, dbW, dWt, dbWt, dg1, db1, dg2, db2,
                None, None, None, None, None, None, None, None, None, None, None, None)


class StgcnResBlockFn(torch.autograd.Function):
    """The full pre-activation residual block (st_graphconv.py:60-82, then the
    ReLU of :105):  y = ReLU(Conv9x1(ReLU(BN2(SpatialConv(ReLU(BN1(x)))))) + R(x)).

    forward(x, A, W, bW, Wt, bWt, g1, b1, g2, b2, Wr, br, rm1, rv1, rm2, rv2,
            stride, pad, eps, momentum, training) -> y
    R = identity when Wr is None (C_in == C_out, stride 1), else the 1x1
    projection Conv2d (Wr, br) with temporal stride. Backward returns the
    gradients of x, A, W, bW, Wt, bWt, g1, b1, g2, b2, Wr, br.
    """

    @staticmethod
    def forward(ctx, x, A, W, bW, Wt, bWt, g1, b1, g2, b2, Wr, br, rm1, rv1, rm2, rv2,
                stride, pad, eps, momentum, training, cc=None, drop=0.0, gemm="fp32"):
        lib = hip_lib.lib()
        x = x.contiguous()
        seed = _dropout_seed(drop, training)
        names = ("x", "A", "W", "bW", "Wt", "bWt", "g1", "b1", "g2", "b2",
                 "rm1", "rv1", "rm2", "rv2")
        for t, n in zip((x, A, W, bW, Wt, bWt, g1, b1, g2, b2, rm1, rv1, rm2, rv2), names):
            _f32c(t, n)
        if Wr is not None:
            _f32c(Wr, "Wr")
            _f32c(br, "br")
        N, C_in, T, V = x.shape
        K = A.shape[0]
        C_out = Wt.shape[0]
        desc = make_desc(x.shape, C_out, K, stride, pad, eps, momentum, training, residual=True,
                         **_gemm_flags(gemm))
        hip_lib.check(lib.stgcn_check_desc(ctypes.byref(desc)))
        if (Wr is None) != (C_in == C_out and stride == 1):
            raise RuntimeError("residual projection weights must be given iff shapes differ")
        dev = x.device
        y = torch.empty((N, C_out, desc.T_out, V), device=dev, dtype=torch.float32)
        Z = torch.empty((N, C_out, T, V), device=dev, dtype=torch.float32)
        Za = torch.empty_like(Z)
        stats = torch.empty(2 * C_in + 2 * C_out, device=dev, dtype=torch.float32)
        G = _keep_g(ctx, x, desc)
        nbytes = lib.stgcn_fwd_workspace_bytes(ctypes.byref(desc))
        ws = torch.empty(nbytes, device=dev, dtype=torch.uint8)
        args = _args(hip_lib.FwdArgs, [hip_lib.ptr(t) for t in (
            x, A, W, bW, Wt, bWt, g1, b1, g2, b2, rm1, rv1, rm2, rv2, y, Z, None, stats,
            Wr, br, Za, G, cc and cc.x_stats, cc and cc.y_stats)], drop, seed)
        hip_lib.check(lib.stgcn_block_fwd(ctypes.byref(desc), ctypes.byref(args),
                                          hip_lib.ptr(ws), nbytes, hip_lib.stream_handle(dev)))
        ctx.save_for_backward(x, Z, Za, y, stats, A, W, bW, Wt, g1, b1, g2, b2, Wr, G)
        ctx.cfg = (stride, pad, eps, momentum, training)
        ctx.gemm = gemm
        ctx.cc = cc
        ctx.drop = (drop, seed)
        return y

    @staticmethod
    def backward(ctx, dy):
        lib = hip_lib.lib()
        x, Z, Za, y, stats, A, W, bW, Wt, g1, b1, g2, b2, Wr, G = ctx.saved_tensors
        stride, pad, eps, momentum, training = ctx.cfg
        need_dx = bool(ctx.needs_input_grad[0])
        dy = dy.contiguous()
        C_out = Wt.shape[0]
        desc = make_desc(x.shape, C_out, A.shape[0], stride, pad, eps, momentum, training,
                         need_dx=need_dx, residual=True,
                         **_gemm_flags(ctx.gemm))
        dev = x.device
        dx = torch.empty_like(x) if need_dx else None
        dA, dW, dbW, dWt = (torch.empty_like(t) for t in (A, W, bW, Wt))
        dbWt = torch.empty(C_out, device=dev, dtype=torch.float32)
        dg1, db1, dg2, db2 = (torch.empty_like(t) for t in (g1, b1, g2, b2))
        dWr = torch.empty_like(Wr) if Wr is not None else None
        dbr = torch.empty(C_out, device=dev, dtype=torch.float32) if Wr is not None else None
        _, _, pg2, pb2, psums, pU, pst, _, _ = _chain_bwd_args(ctx.cc, dy, need_dx,
                                                               x.shape[1], dev)
        nbytes = lib.stgcn_bwd_workspace_bytes(ctypes.byref(desc))
        ws = torch.empty(nbytes, device=dev, dtype=torch.uint8)
        args = _args(hip_lib.BwdArgs, [hip_lib.ptr(t) for t in (
            dy, x, Z, None, stats, A, W, bW, Wt, g1, b1, g2, b2, dx,
            dA, dW, dbW, dWt, dbWt, dg1, db1, dg2, db2,
            Wr, Za, y, dWr, dbr, G, None, pg2, pb2, psums)], *ctx.drop,
            prev_U=hip_lib.ptr(pU), prev_stats=hip_lib.ptr(pst))
        hip_lib.check(lib.stgcn_block_bwd(ctypes.byref(desc), ctypes.byref(args),
                                          hip_lib.ptr(ws), nbytes, hip_lib.stream_handle(dev)))
        _chain_publish(ctx.cc, psums, dx)
        return (dx, dA, dW, dbW, dWt, dbWt, dg1, db1, dg2, db2, dWr, dbr,
                None, None, None, None, None, None, None, None, None, None, None, None)


class SpatialConvFn(torch.autograd.Function):
    """``SpatialConv.forward`` on its own (st_graphconv.py:139-152) through
    stgcn_spatial_fwd / stgcn_spatial_bwd (ABI 4):
    forward(x, A, W, bW, bf16) -> out (N, C_out, T, V); backward returns
    dx, dA, dW, dbW (W is the (K*C_out, C_in, 1, 1) Conv2d weight)."""

    @staticmethod
    def forward(ctx, x, A, W, bW, bf16=False):
        lib = hip_lib.lib()
        x = x.contiguous()
        for t, n in ((x, "x"), (A, "A"), (W, "W"), (bW, "bW")):
            _f32c(t, n)
        N, C_in, T, V = x.shape
        K = A.shape[0]
        C_out = W.shape[0] // K
        desc = hip_lib.SpatialDesc(N, C_in, C_out, T, V, K, hip_lib.F_BF16 if bf16 else 0)
        nbytes = lib.stgcn_spatial_workspace_bytes(ctypes.byref(desc), 0)
        if nbytes == 0:
            hip_lib.check(-2)
        out = torch.empty((N, C_out, T, V), device=x.device, dtype=torch.float32)
        ws = torch.empty(nbytes, device=x.device, dtype=torch.uint8)
        hip_lib.check(lib.stgcn_spatial_fwd(ctypes.byref(desc), *[hip_lib.ptr(t) for t in (
            x, A, W, bW, out, ws)], nbytes, hip_lib.stream_handle(x.device)))
        ctx.save_for_backward(x, A, W, bW)
        ctx.desc = desc
        return out

    @staticmethod
    def backward(ctx, dout):
        lib = hip_lib.lib()
        x, A, W, bW = ctx.saved_tensors
        dout = dout.contiguous()
        desc = ctx.desc
        dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        dA, dW, dbW = (torch.empty_like(t) for t in (A, W, bW))
        nbytes = lib.stgcn_spatial_workspace_bytes(ctypes.byref(desc), 1)
        ws = torch.empty(nbytes, device=x.device, dtype=torch.uint8)
        hip_lib.check(lib.stgcn_spatial_bwd(ctypes.byref(desc), *[hip_lib.ptr(t) for t in (
            dout, x, A, W, bW, dx, dA, dW, dbW, ws)], nbytes, hip_lib.stream_handle(x.device)))
        return dx, dA, dW, dbW, None

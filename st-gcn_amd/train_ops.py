"""The training-step ops around the block stack on the HIP library (SURVEY.md
§8(f) row 1): the classification head (global average pool over (T, V) +
Linear + cross entropy; lightning_model.py:105-107 and the loss of
training_step :202) as one autograd Function, and ``FusedAdam``, a drop-in for
``torch.optim.Adam`` (lightning_model.py:196-197) whose step is ONE kernel
launch over every parameter (same hyper-parameters, same per-parameter state
names ``step`` / ``exp_avg`` / ``exp_avg_sq``, so state_dicts interchange).
No CPU fallback: both raise without the HIP library / a GPU.
"""
import ctypes

import torch

from . import hip_lib


def _check_f32(t, name):
    if t.dtype != torch.float32 or not t.is_contiguous() or not t.is_cuda:
        raise RuntimeError(f"{name}: expected a contiguous float32 GPU tensor")


class StgcnHeadFn(torch.autograd.Function):
    """forward(y (N,C,T,V), W (classes,C), b (classes), labels int64 (N)) ->
    (loss (scalar, mean cross entropy), logits (N, classes), non-differentiable).
    Same arithmetic as ``F.cross_entropy(fc_layer(avg_pool2d(y, (T,V)).view(N,C)), labels)``.
    from_u = (U, stats2, g2, b2) (ABI 9, model.STGCNStack.forward_loss): y is the
    last block's UNWRITTEN output; the pool forms y = ReLU(BN2(U)) on load
    (stgcn_head_fwd_u, bit-identical); y still receives the gradient."""

    @staticmethod
    def forward(ctx, y, W, b, labels, from_u=None):
        lib = hip_lib.lib()
        if from_u is None:
            y = y.contiguous()
            _check_f32(y, "y")
        # (from_u: y is the block's unwritten output, a shape-only placeholder)
        for t, n in ((W, "W"), (b, "b")):
            _check_f32(t, n)
        if labels.dtype != torch.int64 or not labels.is_cuda:
            raise RuntimeError("labels: expected an int64 GPU tensor")
        labels = labels.contiguous()
        N, C = y.shape[0], y.shape[1]
        L = y[0, 0].numel()
        classes = W.shape[0]
        if W.shape[1] != C or b.shape[0] != classes or labels.shape[0] != N:
            raise RuntimeError("head: shape mismatch between y, W, b and labels")
        d = hip_lib.HeadDesc(N, C, L, classes)
        dev = y.device
        pooled = torch.empty((N, C), device=dev, dtype=torch.float32)
        logits = torch.empty((N, classes), device=dev, dtype=torch.float32)
        lossv = torch.empty(N, device=dev, dtype=torch.float32)
        loss = torch.empty((), device=dev, dtype=torch.float32)
        if from_u is not None:
            U, stats2, g2, b2 = from_u
            for t, n in ((U, "U"), (stats2, "stats2"), (g2, "g2"), (b2, "b2")):
                _check_f32(t, n)
            if U.shape != y.shape or stats2.numel() < 2 * C or g2.numel() != C or b2.numel() != C:
                raise RuntimeError("head: U / BN2 parameters do not match y")
            hip_lib.check(lib.stgcn_head_fwd_u(ctypes.byref(d), *[hip_lib.ptr(t) for t in (
                U, stats2, g2, b2, W, b, labels, pooled, logits, lossv, loss)],
                hip_lib.stream_handle(dev)))
        else:
            hip_lib.check(lib.stgcn_head_fwd(ctypes.byref(d), *[hip_lib.ptr(t) for t in (
                y, W, b, labels, pooled, logits, lossv, loss)], hip_lib.stream_handle(dev)))
        ctx.save_for_backward(pooled, logits, W, labels)
        ctx.shape = y.shape
        ctx.mark_non_differentiable(logits)
        return loss, logits

    @staticmethod
    def backward(ctx, dloss, _dlogits):
        lib = hip_lib.lib()
        pooled, logits, W, labels = ctx.saved_tensors
        N, C = pooled.shape
        classes = W.shape[0]
        dev = pooled.device
        L = 1
        for s in ctx.shape[2:]:
            L *= s
        d = hip_lib.HeadDesc(N, C, L, classes)
        dloss = dloss.reshape(1).float().contiguous()
        dlogits = torch.empty((N, classes), device=dev, dtype=torch.float32)
        dpooled = torch.empty((N, C), device=dev, dtype=torch.float32)
        dW = torch.empty_like(W)
        db = torch.empty(classes, device=dev, dtype=torch.float32)
        # ABI 10: the pool's gradient is constant over (T, V): only its value per
        # (n, c) is formed, returned as that (N, C) tensor expanded (stride 0) to
        # y's shape. A HIP block takes it as stgcn_bwd_args_t.dy_nc (no dy tensor
        # written or read); any other consumer materialises it (.contiguous()).
        dy_nc = torch.empty((N, C), device=dev, dtype=torch.float32)
        hip_lib.check(lib.stgcn_head_bwd_nc(ctypes.byref(d), *[hip_lib.ptr(t) for t in (
            pooled, logits, W, labels, dloss, dlogits, dpooled, dy_nc, dW, db)],
            hip_lib.stream_handle(dev)))
        dy = dy_nc.view(N, C, *([1] * (len(ctx.shape) - 2))).expand(ctx.shape)
        return dy, dW, db, None, None


class FusedAdam(torch.optim.Optimizer):
    """torch.optim.Adam (amsgrad=False, maximize=False, fp32 parameters on one
    device) with the update as one libstgcn_hip launch per step. The tensor
    table (pointers of param / grad / exp_avg / exp_avg_sq) is rebuilt on the
    host only when a pointer changed (e.g. grads re-allocated after
    zero_grad(set_to_none=True)) and copied to the device asynchronously from
    pinned memory; one table per parameter group (keyed by the group's index).

    capturable=True (as torch.optim.Adam(capturable=True)): the step count lives
    on the device (one float tensor per group, shared by the group's parameters'
    ``state["step"]``) and is advanced by the library (stgcn_adam_step_dev, ABI
    11), so ``step()`` reads nothing from the device and can be captured in a HIP
    graph (``GraphedStep``). A table built during a capture (the captured
    backward allocates new gradients) is written into a pinned buffer set aside
    by the last eager build and kept alive with the table: every replay's copy
    re-reads it."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0,
                 amsgrad=False, capturable=False):
        if amsgrad:
            raise NotImplementedError("FusedAdam: amsgrad")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self.capturable = capturable
        self._tables = {}  # group index -> (key, device table, chunks, ntensors, host table)
        self._spare = {}   # group index -> unused pinned table buffer (capturable)
        self._captured = []  # pinned tables a captured step's copies read

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        lib = hip_lib.lib()
        for gi, group in enumerate(self.param_groups):
            plist = [p for p in group["params"] if p.grad is not None]
            if not plist:
                continue
            for p in plist:
                _check_f32(p, "param")
                _check_f32(p.grad, "grad")
            if self.capturable:
                dstep = self._device_step(plist)
            else:
                for p in plist:
                    st = self.state[p]
                    if not st:
                        st["step"] = torch.tensor(0.0)
                        st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                        st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["step"] = st["step"] + 1  # (not in place: loaded state may share it)
                steps = {int(self.state[p]["step"].item()) for p in plist}
                if len(steps) != 1:
                    raise RuntimeError("FusedAdam: parameters of a group at different steps")
                step = steps.pop()
            tabs = [hip_lib.AdamTensor(p.data_ptr(), p.grad.data_ptr(),
                                       self.state[p]["exp_avg"].data_ptr(),
                                       self.state[p]["exp_avg_sq"].data_ptr(), p.numel())
                    for p in plist]
            key = tuple((t.param, t.grad, t.exp_avg, t.exp_avg_sq, t.numel) for t in tabs)
            dev = plist[0].device
            cached = self._tables.get(gi)
            if cached is None or cached[0] != key:
                n = len(tabs)
                nbytes = lib.stgcn_adam_table_bytes(n)
                if torch.cuda.is_current_stream_capturing():
                    # (no pinned allocation inside a capture: the spare buffer
                    # the last eager build left, never yet read by a copy)
                    host = self._spare.pop(gi, None)
                    if host is None or host.numel() < nbytes:
                        raise RuntimeError("FusedAdam: capture a step only after an eager "
                                           "step of the same parameters (GraphedStep warm-up)")
                    self._captured.append(host)  # (read by every replay: never freed)
                else:
                    host = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
                    if self.capturable:
                        self._spare[gi] = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
                chunks = ctypes.c_int64(0)
                arr = (hip_lib.AdamTensor * n)(*tabs)
                hip_lib.check(lib.stgcn_adam_build_table(arr, n, ctypes.c_void_p(host.data_ptr()),
                                                         nbytes, ctypes.byref(chunks)))
                dev_table = torch.empty(nbytes, dtype=torch.uint8, device=dev)
                dev_table.copy_(host, non_blocking=True)
                cached = (key, dev_table, chunks.value, n, host)
                self._tables[gi] = cached
            _, dev_table, nchunks, n, _ = cached
            b1, b2 = group["betas"]
            if self.capturable:
                hip_lib.check(lib.stgcn_adam_step_dev(
                    hip_lib.ptr(dev_table), n, nchunks, group["lr"], b1, b2,
                    group["eps"], group["weight_decay"], hip_lib.ptr(dstep),
                    hip_lib.stream_handle(dev)))
            else:
                hip_lib.check(lib.stgcn_adam_step(
                    hip_lib.ptr(dev_table), n, nchunks, group["lr"], b1, b2,
                    group["eps"], group["weight_decay"], step, hip_lib.stream_handle(dev)))
        return loss

    def _device_step(self, plist):
        """The group's device step count (float32, shape ()): created with the
        state (0), or taken over from loaded state once (one host read, outside
        any capture), then shared by every parameter of the group."""
        dev = plist[0].device
        shared = None
        for p in plist:
            st = self.state[p].get("step")
            if torch.is_tensor(st) and st.is_cuda and st.dtype == torch.float32 and st.dim() == 0:
                shared = st if shared is None else shared
        if shared is None or any(self.state[p].get("step") is not shared for p in plist):
            vals = {float(self.state[p]["step"]) for p in plist if "step" in self.state[p]}
            if len(vals) > 1:
                raise RuntimeError("FusedAdam: parameters of a group at different steps")
            shared = torch.full((), vals.pop() if vals else 0.0, device=dev, dtype=torch.float32)
            for p in plist:
                st = self.state[p]
                if "exp_avg" not in st:
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] = shared
        return shared


class GraphedStep:
    """One training step captured in a HIP graph and replayed (torch.cuda.graph
    over the caller's stream work: every libstgcn_hip launch goes to the capture
    stream, allocations come from the graph's private pool, so replays reuse the
    same buffers). ``step_fn()`` must be replay-safe: static inputs (copy new
    data into them before ``__call__``), no host reads of device values, no
    dropout (its seed is drawn on the host), optimizer ``FusedAdam(capturable=
    True)``. ``warmup`` eager calls run first on a side stream (the torch
    recipe: lazy allocations and table builds happen outside the capture).
    ``__call__`` replays and returns the tensors the captured call returned
    (their storage is rewritten by every replay)."""

    def __init__(self, step_fn, warmup=3):
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(warmup):
                step_fn()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()  # (the warm-up's host-to-device table copies have run)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.out = step_fn()

    def __call__(self):
        self.graph.replay()
        return self.out


class GraphedDPStep:
    """The multi-rank training step in two HIP graphs around an eager gradient
    all-reduce: graph A = ``dp.zero_grad()`` + ``fwd_bwd()`` under
    ``dp.no_sync()`` (the gradients accumulate into the bucket views,
    dp.GradAllReduce, and no collective is issued inside the capture), then
    ``dp.synchronize()`` eagerly (one all-reduce per bucket + the division by
    the world size), then graph B = ``opt_step()`` (FusedAdam(capturable=True)).
    The collectives stay outside the graphs, so the path is the same for RCCL and
    gloo; what is given up against the eager step is the overlap of the bucket
    all-reduces with backward (~11 MB per step: a small fraction of the step on
    xGMI), what is gained is the per-launch host work of ~220 launches. The
    result equals the eager DP step's: the same gradients reach the same
    all-reduce of each bucket (tests/dp_graph_worker.py). ``warmup`` full eager
    steps run first on a side stream (lazy allocations, Adam state, tables)."""

    def __init__(self, fwd_bwd, dp, opt_step, warmup=2):
        self.dp = dp

        def a():
            dp.zero_grad()
            with dp.no_sync():
                return fwd_bwd()

        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(warmup):
                a()
                dp.synchronize()
                opt_step()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self.graph_a = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph_a):
            self.out = a()
        self.graph_b = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph_b):
            opt_step()

    def __call__(self):
        self.graph_a.replay()
        self.dp.synchronize()
        self.graph_b.replay()
        return self.out

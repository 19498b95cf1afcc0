"""Data-parallel gradient all-reduce, bucketed and overlapped with backward.

One process per GPU (torch.distributed, backend "nccl" = RCCL on ROCm, over
xGMI). Each rank runs the full stack on its own N/world clips; BatchNorm stays
per replica (DDP semantics). Parameters are grouped into
buckets in reverse registration order (= the order backward produces them,
last block first). Every bucket owns one flat gradient buffer and each
parameter's ``.grad`` is a view into it ("gradient as bucket view"): autograd
accumulates straight into the bucket, so launching a bucket's all-reduce is
one asynchronous collective on the flat buffer, with no gather copy before it
and no scatter copy after it. When every gradient of a bucket has been
accumulated (``register_post_accumulate_grad_hook``) its all-reduce(SUM) is
issued, so the reduction of the late blocks' gradients overlaps the backward
of the earlier blocks; ``synchronize()`` waits and divides each flat buffer
by the world size in place.

Use ``zero_grad()`` (zeroes the flat buffers, keeps the views) instead of
``optimizer.zero_grad(set_to_none=True)``. If a gradient arrives that is not
the bucket view (the caller set ``.grad`` to None or replaced it), the hook
copies it into the view and re-installs the view.

Exactly one backward per ``synchronize()`` reduces. Gradient accumulation over
several backward passes runs the earlier ones under ``with dp.no_sync():``
(they only accumulate into the buckets, as DDP's no_sync); a second backward
outside it, before ``synchronize()``, would add into a buffer whose
all-reduce is in flight, so it raises before accumulating.

The reference has no distributed code of its own (only
PyTorch-Lightning's inherited Trainer flags could enable DDP); this is the
MI355X-native counterpart of that DDP path. With ~2.7 M fp32 parameters
(10.8 MB) per step the default 4 MB buckets give 3-4 collectives per step.
"""
import contextlib

import torch
import torch.distributed as dist


class GradAllReduce:
    TRACE_MAX = 1 << 16

    def __init__(self, model, world_size=None, bucket_bytes=4 << 20, group=None, trace=False):
        self.group = group
        self.world = world_size or dist.get_world_size(group)
        params = [p for p in model.parameters() if p.requires_grad]
        self.buckets = []
        cur, size = [], 0
        for p in reversed(params):
            if cur and (p.dtype != cur[0].dtype or p.device != cur[0].device):
                self.buckets.append(cur)
                cur, size = [], 0
            cur.append(p)
            size += p.numel() * p.element_size()
            if size >= bucket_bytes:
                self.buckets.append(cur)
                cur, size = [], 0
        if cur:
            self.buckets.append(cur)
        self._bucket_of, self._view = {}, {}
        self._flat = []
        for bi, ps in enumerate(self.buckets):
            flat = torch.zeros(sum(p.numel() for p in ps), dtype=ps[0].dtype,
                               device=ps[0].device)
            off = 0
            for p in ps:
                self._bucket_of[p] = bi
                self._view[p] = flat[off:off + p.numel()].view_as(p)
                off += p.numel()
            self._flat.append(flat)
        self._install_views()
        self._sync = True
        # observable overlap (trace=True, a diagnostic: off in training): (kind,
        # index) in arrival order -- ("grad", i) when parameter i's gradient has
        # been accumulated (i in model.parameters() order), ("launch", b) when
        # bucket b's all-reduce is issued; reset by synchronize(), kept in
        # ``last_trace``, at most TRACE_MAX entries (no_sync steps accumulate)
        self._index = {p: i for i, p in enumerate(params)}
        self._trace_on = trace
        self.trace, self.last_trace = [], []
        self._handles = [p.register_post_accumulate_grad_hook(self._hook) for p in params]
        self._handles += [p.register_hook(self._guard(p)) for p in params]
        self._reset()

    def _guard(self, p):
        bi = self._bucket_of[p]

        def check(grad):
            # runs before autograd accumulates into p.grad (the bucket view); a
            # second arrival of p's gradient before synchronize() -- also in a
            # bucket whose all-reduce never launched because one of its
            # parameters is unused -- would add into a buffer that is (or will
            # be) reduced for the first backward only
            # (in flight: always, no_sync or not -- the buffer is being reduced;
            # a repeated arrival counts only for a backward that reduces)
            if self._work[bi] is not None or (self._sync and p in self._seen):
                raise RuntimeError(
                    "GradAllReduce: a second backward before synchronize() would accumulate "
                    "into a bucket whose all-reduce is in flight; run the earlier "
                    "micro-batches under `with dp.no_sync():`")
            return grad
        return check

    @contextlib.contextmanager
    def no_sync(self):
        """Backward passes inside only accumulate into the bucket views; the
        next backward outside launches the all-reduce of the accumulated sum."""
        prev, self._sync = self._sync, False
        try:
            yield
        finally:
            self._sync = prev

    def _install_views(self):
        for p, v in self._view.items():
            if p.grad is not v:
                if p.grad is not None:
                    v.copy_(p.grad)
                p.grad = v

    def _reset(self):
        self._pending = [len(ps) for ps in self.buckets]
        self._work = [None] * len(self.buckets)
        self._seen = set()  # parameters whose gradient arrived since synchronize()

    def zero_grad(self):
        """Zero every bucket (one fill per flat buffer) and keep the views."""
        for flat in self._flat:
            flat.zero_()
        self._install_views()

    def _hook(self, p):
        v = self._view[p]
        if p.grad is not v:  # not accumulated into the bucket: move it there
            v.copy_(p.grad)
            p.grad = v
        if self._trace_on and len(self.trace) < self.TRACE_MAX:
            self.trace.append(("grad", self._index[p]))
        if not self._sync:
            return
        self._seen.add(p)
        bi = self._bucket_of[p]
        self._pending[bi] -= 1
        if self._pending[bi] == 0:
            self._launch(bi)

    def _launch(self, bi):
        if self._trace_on and len(self.trace) < self.TRACE_MAX:
            self.trace.append(("launch", bi))
        self._work[bi] = dist.all_reduce(self._flat[bi], op=dist.ReduceOp.SUM,
                                         group=self.group, async_op=True)

    def synchronize(self):
        """Wait for every bucket's all-reduce; the grads (bucket views) then
        hold the average over ranks."""
        for bi in range(len(self.buckets)):
            if self._work[bi] is None:  # some grads never arrived (unused params)
                self._install_views()
                self._launch(bi)
            self._work[bi].wait()
            self._flat[bi].div_(self.world)
        self._install_views()
        self.last_trace, self.trace = self.trace, []
        self._reset()

    def remove(self):
        for h in self._handles:
            h.remove()

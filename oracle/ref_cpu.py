"""ORACLE — CPU restatement of the reference's ST-GCN block / stack (TEST INFRASTRUCTURE).

This module is test infrastructure only. It may be imported by ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg, and there
only as the checker or the timed CPU baseline. The product path
(``st-gcn_amd/``) never imports it.

It restates, op for op and in the same order, the arithmetic of:
  * ``SpatialConv.forward``            src/network/st_graphconv.py:139-152
      Y = Conv1x1(x) + b  (:148);  view (N,K,C_out,T,V) (:149);
      out = einsum('kvw,nkctw->nctv', A, Y)  (:150)
  * ``SpatialTemporalConv.forward``     src/network/st_graphconv.py:85-109
      non-residual: BN1(x.float()) -> spatial -> Conv(9x1, stride (s,1),
      pad (4,0), bias) -> BN2 -> ReLU(clone) -> [Dropout]       (:97-109)
      residual:     clone -> BN1 -> ReLU -> spatial -> BN2 -> ReLU ->
      temporal conv -> += residual(identity | 1x1 stride conv)   (:60-82)
  * ``L_STGCN.forward``                 src/lightning_model.py:91-112
      permute NTVC->NCTV, 10 blocks, avg_pool2d over (T,V), Linear
  * training loss                        src/lightning_model.py:199-205
BatchNorm in training mode uses batch statistics (biased variance for
normalisation, unbiased for the running_var update, eps 1e-5, momentum 0.1)
exactly as ``nn.BatchNorm2d`` (st_graphconv.py:34,46).

Backward is the autograd derivative of these same ops, which is what the
reference's training step computes (lightning_model.py:199-205 -> autograd).

Pinning: checked against the golden vectors in ``tests/golden`` that were
produced by running the reference itself (``tests/golden/make_golden.py``);
see ``tests/test_oracle_golden.py``.

All functions take an explicit ``dtype`` so the same restatement runs in
float32 (the reference's arithmetic) or float64 (a tighter yardstick).
"""
import torch
import torch.nn.functional as F

# Reference layer table (src/lightning_model.py:65-86): (C_out, stride).
LAYERS = [(64, 1), (64, 1), (64, 1), (64, 1), (128, 2), (128, 1), (128, 1),
          (256, 2), (256, 1), (256, 1)]

BLOCK_PARAM_NAMES = [
    "batch_n.weight", "batch_n.bias", "spatialConv.A", "spatialConv.W.weight",
    "spatialConv.W.bias", "temporalConv.weight", "temporalConv.bias",
    "batch_n_2.weight", "batch_n_2.bias",
]
BLOCK_BUFFER_NAMES = [
    "batch_n.running_mean", "batch_n.running_var", "batch_n.num_batches_tracked",
    "batch_n_2.running_mean", "batch_n_2.running_var", "batch_n_2.num_batches_tracked",
]


def _bn(x, p, b, prefix, training, momentum, eps):
    rm, rv = b.get(prefix + ".running_mean"), b.get(prefix + ".running_var")
    y = F.batch_norm(x, rm, rv, p[prefix + ".weight"], p[prefix + ".bias"],
                     training=training, momentum=momentum, eps=eps)
    nbt = prefix + ".num_batches_tracked"
    if training and nbt in b:
        b[nbt] += 1
    return y


def _bf16(t):
    """Round to bf16 (nearest even) and back to t's dtype."""
    return t.to(torch.bfloat16).to(t.dtype)


class _Bf16Conv(torch.autograd.Function):
    """Conv2d whose GEMM operands are rounded to bf16 in forward (input,
    weight) and backward (grad_output and the saved rounded operands), with
    the accumulation in the tensors' own dtype: the reference's conv as it
    runs with bf16 channel GEMMs (BASELINE cfg3 / cfg5). Used only to measure
    the reference's own error in that precision (the parity tests' floor)."""

    @staticmethod
    def forward(ctx, x, w, b, stride, pad):
        xr, wr = _bf16(x), _bf16(w)
        ctx.save_for_backward(xr, wr)
        ctx.cfg = (stride, pad, b is not None)
        return F.conv2d(xr, wr, b, stride=stride, padding=pad)

    @staticmethod
    def backward(ctx, gy):
        xr, wr = ctx.saved_tensors
        stride, pad, has_b = ctx.cfg
        gr = _bf16(gy)
        dx = torch.nn.grad.conv2d_input(xr.shape, wr, gr, stride=stride, padding=pad)
        dw = torch.nn.grad.conv2d_weight(xr, wr.shape, gr, stride=stride, padding=pad)
        db = gy.sum(dim=(0, 2, 3)) if has_b else None
        return dx, dw, db, None, None


def _conv(x, w, b, stride=(1, 1), padding=(0, 0), gemm_bf16=False):
    if gemm_bf16:
        return _Bf16Conv.apply(x, w, b, stride, padding)
    return F.conv2d(x, w, b, stride=stride, padding=padding)


def spatial_conv(x, A, W, bW, gemm_bf16=False):
    """st_graphconv.py:139-152."""
    N, _, T, V = x.shape
    K = A.shape[0]
    C_out = W.shape[0] // K
    y = _conv(x, W, bW, gemm_bf16=gemm_bf16)
    y = y.view(N, K, C_out, T, V)
    return torch.einsum("kvw,nkctw->nctv", A, y)


def block_forward(x, p, b, stride, pad=4, residual=False, training=True,
                  momentum=0.1, eps=1e-5, dtype=torch.float32, relu_mask=None,
                  return_pre_relu=False, gemm_bf16=False, inner_mask=None):
    """One SpatialTemporalConv step. ``p``: parameter tensors keyed by the
    reference's state_dict names (BLOCK_PARAM_NAMES [+ apply_residual.*]);
    ``b``: running buffers (updated in place when ``training``).

    ``relu_mask`` (optional, 0/1 tensor shaped like the output): use this
    mask for the final ReLU instead of ``f > 0`` — used by the parity tests to
    differentiate through the SAME subgradient choice as the implementation
    under test at ReLU ties (|pre-ReLU| below fp32 resolution).

    ``gemm_bf16``: run the convolutions with bf16-rounded operands
    (``_Bf16Conv``), everything else unchanged. ``inner_mask`` (residual
    block): the same as ``relu_mask`` for the inner ReLU after BN2 (:77)."""
    x = x.to(dtype)
    A = p["spatialConv.A"]
    if residual:
        res = x.clone()
        f = _bn(x, p, b, "batch_n", training, momentum, eps)
        f = F.relu(f.clone(), inplace=True)
        f = spatial_conv(f, A, p["spatialConv.W.weight"], p["spatialConv.W.bias"], gemm_bf16)
        f = _bn(f, p, b, "batch_n_2", training, momentum, eps)
        f = F.relu(f.clone(), inplace=True) if inner_mask is None else f * inner_mask.to(f.dtype)
        f = _conv(f, p["temporalConv.weight"], p["temporalConv.bias"],
                  stride=(stride, 1), padding=(pad, 0), gemm_bf16=gemm_bf16)
        if "apply_residual.weight" in p:
            f = f + _conv(res, p["apply_residual.weight"], p["apply_residual.bias"],
                          stride=(stride, 1), gemm_bf16=gemm_bf16)
        else:
            f = f + res
    else:
        f = _bn(x, p, b, "batch_n", training, momentum, eps)
        f = spatial_conv(f, A, p["spatialConv.W.weight"], p["spatialConv.W.bias"], gemm_bf16)
        f = _conv(f, p["temporalConv.weight"], p["temporalConv.bias"],
                  stride=(stride, 1), padding=(pad, 0), gemm_bf16=gemm_bf16)
        f = _bn(f, p, b, "batch_n_2", training, momentum, eps)
    if return_pre_relu:
        return f
    if relu_mask is not None:
        return f * relu_mask.to(f.dtype)
    return F.relu(f.clone(), inplace=True)  # nn.ReLU(inplace=True) on a clone (:49, :105)


def block_params_from_arrays(arrays, prefix="param.", dtype=torch.float32, requires_grad=True):
    """Split a fixture dict into (params, buffers) tensors."""
    p, b = {}, {}
    for k, v in arrays.items():
        if not k.startswith(prefix):
            continue
        name = k[len(prefix):]
        t = torch.as_tensor(v)
        if "running" in name or "num_batches" in name:
            b[name] = t.clone().to(dtype if t.is_floating_point() else t.dtype)
        else:
            p[name] = t.clone().to(dtype).requires_grad_(requires_grad)
    return p, b


def block_step(arrays, dtype=torch.float64, relu_mask=None, gemm_bf16=False, inner_mask=None):
    """Run fwd+bwd of one block fixture on the oracle; returns a dict with
    the same keys the fixture stores (y, grad.*, after.*)."""
    meta = arrays["meta"]
    stride, residual = int(meta[2]), bool(meta[7])
    p, b = block_params_from_arrays(arrays, dtype=dtype)
    x = torch.as_tensor(arrays["x"]).to(dtype).requires_grad_(True)
    g = torch.as_tensor(arrays["g"]).to(dtype)
    y = block_forward(x, p, b, stride, residual=residual, dtype=dtype, relu_mask=relu_mask,
                      gemm_bf16=gemm_bf16, inner_mask=inner_mask)
    (y * g).sum().backward()
    out = {"y": y.detach(), "grad.x": x.grad}
    for k, t in p.items():
        out["grad." + k] = t.grad
    for k, t in b.items():
        out["after." + k] = t
    return out


def block_pre_relu(arrays, dtype=torch.float64):
    """Pre-ReLU output (BN2 output) of a block fixture, no grad."""
    meta = arrays["meta"]
    p, b = block_params_from_arrays(arrays, dtype=dtype, requires_grad=False)
    with torch.no_grad():
        return block_forward(torch.as_tensor(arrays["x"]), p, b, int(meta[2]),
                             residual=bool(meta[7]), dtype=dtype, return_pre_relu=True)


class Stack:
    """Functional restatement of ``L_STGCN`` (lightning_model.py:35-112) for a
    given parameter dict (state_dict naming: ``conv.{i}.*``, ``fc_layer.*``)."""

    def __init__(self, params, buffers, residual=False):
        self.p, self.b, self.residual = params, buffers, residual

    def forward(self, x_ntvc, training=True, dtype=torch.float32, gemm_bf16=False,
                relu_masks=None):
        """relu_masks (optional, one 0/1 tensor per block): each block's final
        ReLU uses that mask (block_forward's relu_mask: the parity tests
        differentiate through the implementation's own subgradient choices at
        ReLU ties); the blocks' pre-ReLU values are then kept in ``self.pre``."""
        x = x_ntvc.to(dtype).permute(0, 3, 1, 2)
        self.pre = []
        for i, (_, s) in enumerate(LAYERS):
            pre = f"conv.{i}."
            p = {k[len(pre):]: v for k, v in self.p.items() if k.startswith(pre)}
            b = {k[len(pre):]: v for k, v in self.b.items() if k.startswith(pre)}
            if relu_masks is None:
                x = block_forward(x, p, b, s, residual=self.residual, training=training,
                                  dtype=dtype, gemm_bf16=gemm_bf16)
            else:
                f = block_forward(x, p, b, s, residual=self.residual, training=training,
                                  dtype=dtype, gemm_bf16=gemm_bf16, return_pre_relu=True)
                self.pre.append(f.detach())
                x = f * relu_masks[i].to(f.dtype)
            for k, v in b.items():
                self.b[pre + k] = v
        V = x.shape[3]
        x = F.avg_pool2d(x, (x.shape[2], V))
        x = x.view(x.shape[0], x.shape[1])
        return F.linear(x, self.p["fc_layer.weight"], self.p["fc_layer.bias"])


def init_stack_params(C_in, nr_classes, A, seed=0, residual=False, masks=None,
                      max_mask_jitter=0.001):
    """Parameters with the reference's module init order under
    ``torch.manual_seed(seed)`` (lightning_model.py:65-88): for every block
    BN1, W, temporal conv, BN2 (st_graphconv.py:28-46), then the FC layer.
    Returns (params, buffers) dicts in state_dict naming.

    masks: None (no edge importance), "jitter" (L_STGCN --use_edge_importance,
    lightning_model.py:53-57: ten masks 1 + 2(randn_like(A) - 0.5)*jitter drawn
    before the blocks) or "ones" (legacy STGCN, stgcn.py:33-35); the masks are
    returned in params as ``Masks.{i}`` and block i starts from A * Masks[i]."""
    import torch.nn as nn
    torch.manual_seed(seed)
    p, b = {}, {}
    mk = [None] * len(LAYERS)
    if masks == "jitter":
        jit = [2 * (torch.randn_like(A) - 0.5) * max_mask_jitter for _ in LAYERS]
        mk = [jit[i] + torch.ones(A.shape) for i in range(len(LAYERS))]
    elif masks == "ones":
        mk = [torch.ones(A.shape) for _ in LAYERS]
    for i, m in enumerate(mk):
        if m is not None:
            p[f"Masks.{i}"] = m
    c = C_in
    for i, (co, s) in enumerate(LAYERS):
        pre = f"conv.{i}."
        if residual and not (c == co and s == 1):
            r = nn.Conv2d(c, co, kernel_size=1, stride=(s, 1))
            p[pre + "apply_residual.weight"] = r.weight.detach()
            p[pre + "apply_residual.bias"] = r.bias.detach()
        bn1 = nn.BatchNorm2d(c)
        K = A.shape[0]
        w = nn.Conv2d(c, K * co, (1, 1))
        t = nn.Conv2d(co, co, kernel_size=(9, 1), stride=(s, 1), padding=(4, 0))
        bn2 = nn.BatchNorm2d(co)
        for name, m in (("batch_n", bn1), ("batch_n_2", bn2)):
            p[pre + name + ".weight"] = m.weight.detach()
            p[pre + name + ".bias"] = m.bias.detach()
            b[pre + name + ".running_mean"] = m.running_mean.clone()
            b[pre + name + ".running_var"] = m.running_var.clone()
            b[pre + name + ".num_batches_tracked"] = m.num_batches_tracked.clone()
        p[pre + "spatialConv.A"] = (A if mk[i] is None else A * mk[i]).float().clone()
        p[pre + "spatialConv.W.weight"] = w.weight.detach()
        p[pre + "spatialConv.W.bias"] = w.bias.detach()
        p[pre + "temporalConv.weight"] = t.weight.detach()
        p[pre + "temporalConv.bias"] = t.bias.detach()
        c = co
    fc = nn.Linear(256, nr_classes)
    p["fc_layer.weight"] = fc.weight.detach()
    p["fc_layer.bias"] = fc.bias.detach()
    return p, b

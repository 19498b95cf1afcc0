"""Drop-in module API of the reference's ``src/network/st_graphconv.py``.

``SpatialTemporalConv`` and ``SpatialConv`` keep the reference's constructor
signatures, child-module names and state_dict keys (st_graphconv.py:9-58,
:116-136), so ``L_STGCN`` (lightning_model.py:65-86) / ``STGCN``
(stgcn.py:40-51) build unchanged against them and checkpoints interchange.
``forward`` runs the fused MI355X HIP block (``fused.StgcnBlockFn``).

There is no CPU fallback: on a CPU tensor or without the HIP library the
forward raises.
"""
import torch
import torch.nn as nn

from . import hip_lib
from .fused import ChainCtx, Link, SpatialConvFn, StgcnBlockFn, StgcnResBlockFn


class StackChain:
    """Cross-block fusion state for one forward pass of a block stack
    (``model.STGCNStack`` passes one; a drop-in user of single blocks does not
    need it). When block i+1's input is exactly block i's output (same tensor,
    unmodified), block i+1 takes its BN1 batch statistics from block i's output
    pass instead of re-reading x, and in backward computes block i's ReLU+BN2
    reduction while writing its dx. Any other input (dropout in between, user
    code, eval mode) breaks the chain and both blocks fall back to their own
    passes: results are the same either way."""

    def __init__(self, defer_counts=False):
        """defer_counts: the caller (model.STGCNStack) applies the blocks'
        num_batches_tracked increments itself with ``flush_counts``."""
        self.defer_counts = defer_counts
        self.counters = []
        self.reset()

    def reset(self):
        self.y, self.y_version, self.y_stats, self.link, self.g2b2 = None, None, None, None, None
        self.u_stats = None
        self.y_lazy = False  # self.y was not written (ABI 8): the next block reads U

    def set_lazy(self, flags):
        """Per block: its output goes to the next block as ReLU(BN2(U)) formed on
        load, and is never written (ABI 8, STGCN_PLAN_X_FROM_U; model.STGCNStack
        decides, knowing the next block)."""
        self.lazy = list(flags)

    def head_ready(self, y):
        """The stack's last output y was left unwritten for the fused head (ABI 9):
        the head pools ReLU(BN2(U)) from the last block's U."""
        return (self.y_lazy and self.y is y and y._version == self.y_version
                and self.u_stats is not None and self.g2b2 is not None)

    def next_lazy(self):
        lazy = getattr(self, "lazy", None)
        return lazy.pop(0) if lazy else False

    def set_prep(self, preps):
        """The stack's per-block stgcn_fold_prep buffers of this step (fused.FoldPrep),
        handed to the blocks in order."""
        self.preps = list(preps)

    def next_prep(self):
        preps = getattr(self, "preps", None)
        return preps.pop(0) if preps else None

    def count_batch(self, *counters):
        """BatchNorm num_batches_tracked increments of the chained blocks, applied
        by ``flush_counts`` in one multi-tensor launch instead of two per block."""
        self.counters.extend(counters)

    def flush_counts(self):
        if self.counters:
            torch._foreach_add_(self.counters, 1)
            self.counters = []


class SpatialConv(nn.Module):
    """Reference: st_graphconv.py:111-152. Holds the trainable adjacency A
    (K, V, V) and the 1x1 conv W (C_in -> K*C_out). Inside
    ``SpatialTemporalConv`` the layer's arithmetic runs in the fused block;
    called on its own, ``forward`` runs the HIP spatial kernels
    (``fused.SpatialConvFn``: stgcn_spatial_fwd / _bwd) with the reference's
    semantics: out[n,c,t,v] = sum_k sum_w A[k,v,w] (W x + b)[n,k,c,t,w]."""

    def __init__(self, C_in, C_out, A, gemm_dtype=torch.float32):
        super().__init__()
        self.C_in = C_in
        self.C_out = C_out
        self.A = nn.Parameter(A.float())
        self.K = self.A.shape[0]
        self.V = self.A.shape[1]
        self.W = nn.Conv2d(C_in, self.K * C_out, (1, 1))
        # (not in the reference) bf16 channel GEMMs for the standalone call
        self.gemm_dtype = gemm_dtype

    def forward(self, f_in):
        """f_in (N, C_in, T, V) -> (N, C_out, T, V) (st_graphconv.py:139-152)."""
        return SpatialConvFn.apply(f_in.float(), self.A, self.W.weight, self.W.bias,
                                   self.gemm_dtype == torch.bfloat16)


class SpatialTemporalConv(nn.Module):
    """Reference: st_graphconv.py:4-109 (same arguments, children, state_dict).

    Accelerated: the default and the residual block (full pre-activation,
    st_graphconv.py:60-82), training and eval mode, with dropout (p > 0,
    training) fused into the block's output pass (counter-based mask,
    regenerated in backward; a different random stream from torch's).
    """

    def __init__(self, C_in, C_out, A, gamma, temporal_stride, temporal_padding,
                 dropout_rate=0.5, residual=False, gemm_dtype=torch.float32,
                 f32_gemm="mfma"):
        super().__init__()
        if gemm_dtype not in (torch.float32, torch.bfloat16):
            raise ValueError("gemm_dtype must be torch.float32 or torch.bfloat16")
        if f32_gemm not in ("mfma", "bf16x3", "f16x2", "f16x2-nog"):
            raise ValueError("f32_gemm must be 'mfma', 'bf16x3', 'f16x2' or 'f16x2-nog'")
        # (not in the reference) how fp32 channel GEMMs run: "mfma" on the fp32
        # matrix cores, "bf16x3" as exact 3-way bf16 operand splits with six
        # partial products on the bf16 matrix cores (fp32-GEMM accuracy,
        # STGCN_F_F32X3; the stride-1 temporal conv forward and data-grad),
        # "f16x2" the same with the folded block's temporal GEMMs as 2-way fp16
        # splits of power-of-two-scaled operands (three products, STGCN_F_F16X2),
        # "f16x2-nog" that without the joint contraction G ever formed or kept
        # (STGCN_F_NO_G: less activation memory, slower)
        self.f32_gemm = f32_gemm
        # (not in the reference) arithmetic of the channel GEMMs: bf16 rounds the
        # GEMM operands to bf16 on the bf16 matrix cores (fp32 accumulate; tensors,
        # parameters, A and BatchNorm stay fp32) — BASELINE cfg3 / cfg5
        self.gemm_dtype = gemm_dtype
        if residual:
            if C_in == C_out and temporal_stride == 1:
                self.apply_residual = lambda x: x
            else:
                self.apply_residual = nn.Conv2d(C_in, C_out, kernel_size=1,
                                                stride=(temporal_stride, 1))
        self.residual = residual
        self.batch_n = nn.BatchNorm2d(C_in)
        self.spatialConv = SpatialConv(C_in, C_out, A)
        self.temporalConv = nn.Conv2d(C_out, C_out, kernel_size=(gamma, 1),
                                      stride=(temporal_stride, 1),
                                      padding=(temporal_padding, 0))
        self.batch_n_2 = nn.BatchNorm2d(C_out)
        self.relu = nn.ReLU(inplace=True)
        if dropout_rate != 0:
            print('Using dropout')
            self.dropout = nn.Dropout(dropout_rate, inplace=True)
        else:
            print('Not using dropout')
            self.dropout = None
        self.gamma = gamma
        self.stride = temporal_stride
        self.pad = temporal_padding

    def gemm_mode(self):
        """The channel-GEMM arithmetic of this block (fused._gemm_flags mode)."""
        if getattr(self, "gemm_dtype", torch.float32) == torch.bfloat16:
            return "bf16"
        return {"bf16x3": "f32x3", "f16x2": "f16x2", "f16x2-nog": "f16x2_nog"}.get(
            getattr(self, "f32_gemm", "mfma"), "fp32")

    def forward(self, f_in, chain=None):
        """``chain``: optional ``StackChain`` (not part of the reference API)."""
        bn1, bn2 = self.batch_n, self.batch_n_2
        if bn1.momentum is None or bn2.momentum is None:
            raise NotImplementedError("BatchNorm momentum=None (cumulative average)")
        training = self.training
        if training and chain is not None and chain.defer_counts:  # (chain.flush_counts)
            chain.count_batch(bn1.num_batches_tracked, bn2.num_batches_tracked)
        elif training:
            bn1.num_batches_tracked.add_(1)
            bn2.num_batches_tracked.add_(1)
        sc = self.spatialConv
        x = f_in.float()
        drop = self.dropout.p if (self.dropout is not None and training) else 0.0
        gemm = self.gemm_mode()
        cc = None
        lazy = chain.next_lazy() if chain is not None else False
        if chain is not None and chain.y_lazy and not (
                training and x is chain.y and x._version == chain.y_version
                and chain.link is not None):
            raise RuntimeError("STGCNStack chain: a block output that was never written "
                               "(formed by the next block from U) reached other code")
        if chain is not None and training:
            # (the backward link derives this block's ReLU mask from its output:
            # not with dropout on that output, nor for the residual block)
            # (y_stats: [sum | sumsq | cnt | su | xu] per output channel, ABI 5, then
            # the max |y| words, ABI 7)
            cc = ChainCtx(y_stats=torch.empty(
                              hip_lib.y_stats_doubles(self.temporalConv.out_channels),
                              device=x.device, dtype=torch.float64),
                          prep=chain.next_prep(),
                          out_link=None if (self.residual or drop > 0) else Link())
            # (an unwritten y is read back only by the next block's backward, which
            # rebuilds it from U while deferring dx into this block; it can defer
            # only if y needs a gradient -- not when this block and its input are
            # frozen, e.g. fine-tuning the later blocks: then y is written)
            y_grad = (not torch.is_grad_enabled() or x.requires_grad
                      or any(p.requires_grad for p in self.parameters()))
            cc.y_lazy = bool(lazy) and cc.out_link is not None and y_grad
            if cc.y_lazy and lazy == "head":  # (ABI 9: the fused head pools it from U)
                cc.y_head, cc.y_stats = True, None
            if chain.y is not None and x is chain.y and x._version == chain.y_version:
                cc.x_stats = chain.y_stats
                if chain.link is not None:
                    cc.in_link = chain.link
                    cc.prev_g2, cc.prev_b2 = chain.g2b2
                    cc.prev_U, cc.prev_stats = chain.u_stats
                    cc.x_from_u = chain.y_lazy
        if self.residual:
            proj = self.apply_residual if isinstance(self.apply_residual, nn.Conv2d) else None
            y = StgcnResBlockFn.apply(
                x, sc.A, sc.W.weight, sc.W.bias, self.temporalConv.weight,
                self.temporalConv.bias, bn1.weight, bn1.bias, bn2.weight, bn2.bias,
                proj.weight if proj is not None else None,
                proj.bias if proj is not None else None,
                bn1.running_mean, bn1.running_var, bn2.running_mean, bn2.running_var,
                self.stride, self.pad, bn1.eps, bn1.momentum, training, cc, drop, gemm)
        else:
            y = StgcnBlockFn.apply(
                x, sc.A, sc.W.weight, sc.W.bias, self.temporalConv.weight,
                self.temporalConv.bias, bn1.weight, bn1.bias, bn2.weight, bn2.bias,
                bn1.running_mean, bn1.running_var, bn2.running_mean, bn2.running_var,
                self.stride, self.pad, bn1.eps, bn1.momentum, training, cc, drop, gemm)
        if chain is not None:
            if cc is None:
                chain.reset()
            else:
                chain.y, chain.y_version, chain.y_stats = y, y._version, cc.y_stats
                chain.y_lazy = cc.y_lazy
                chain.link = cc.out_link
                chain.g2b2 = None if self.residual else (bn2.weight, bn2.bias)
                chain.u_stats = None if self.residual else (cc.U, cc.stats2)
        return y  # dropout (p > 0, training) is fused into the block's output pass

"""The ST-GCN stack as built by ``L_STGCN`` (src/lightning_model.py:35-112),
on the drop-in blocks. Same child names and state_dict keys
(``conv.{i}.*``, ``fc_layer.*``), same module construction order (so the same
``torch.manual_seed`` yields the same initial parameters), same forward:
NTVC -> permute -> 10 blocks -> avg_pool2d over (T, V) -> Linear.
"""
import torch
import torch.nn as nn

from .graph import Strategy, get_normalized_adjacency_matrices
from .fused import FoldPrep, head_link_ok, lazy_links
from .network import SpatialTemporalConv, StackChain
from .train_ops import StgcnHeadFn

# (C_out, temporal stride) per block, lightning_model.py:65-86.
LAYERS = [(64, 1), (64, 1), (64, 1), (64, 1), (128, 2), (128, 1), (128, 1),
          (256, 2), (256, 1), (256, 1)]


class STGCNStack(nn.Module):
    """use_edge_importance / max_mask_jitter: the reference's edge-importance
    masks (lightning_model.py:53-59): ten masks 1 + 2(randn - 0.5)*jitter drawn
    before the blocks (same RNG consumption), registered as ``Masks.{i}``
    (state_dict interchange), each block built on A * Masks[i]. As in the
    reference the masks only scale the blocks' initial A (each block's
    ``spatialConv.A`` is its own leaf parameter), so they receive no gradient.

    Intermediate block outputs: in training the chained backward (deferred dx,
    fused.Link) hands block i the BN1-side gradient of block i+1 and forms the
    true gradient of block i's output inside block i's kernels, so that gradient
    is never materialised. A tensor hook or ``retain_grad()`` on a block output
    turns the deferral off for that link (the true gradient is formed and seen);
    ``torch.autograd.grad(loss, block_output)`` cannot be detected from inside
    the block and is not supported in a chained training step (run the blocks
    unchained, e.g. one by one, for that)."""

    def __init__(self, C_in, nr_classes, A, gamma=9, dropout_rate=0, residual=False,
                 gemm_dtype=torch.float32, f32_gemm="mfma", use_edge_importance=False,
                 max_mask_jitter=0.001):
        super().__init__()
        pad = (gamma - 1) // 2
        self.K, self.V = A.shape[0], A.shape[1]
        self.nr_classes = nr_classes
        n_layers = len(LAYERS)
        if use_edge_importance:
            jitters = [2 * (torch.randn_like(A) - 0.5) * max_mask_jitter for _ in range(n_layers)]
            self.Masks = nn.ParameterList([nn.Parameter(jitters[i] + torch.ones(A.shape))
                                           for i in range(n_layers)])
        else:
            self.Masks = [torch.ones(A.shape) for _ in range(n_layers)]  # not trainable
        blocks, c = [], C_in
        for i, (co, s) in enumerate(LAYERS):
            blocks.append(SpatialTemporalConv(c, co, A * self.Masks[i], gamma, s, pad,
                                              dropout_rate=dropout_rate, residual=residual,
                                              gemm_dtype=gemm_dtype, f32_gemm=f32_gemm))
            c = co
        self.conv = nn.Sequential(*blocks).float()
        self.fc_layer = nn.Linear(256, nr_classes).float()

    def _chain(self, x, head=False):
        """The StackChain of a training forward, with the stack's folded blocks'
        weight-only operands formed for this step (fused.FoldPrep, ABI 7).
        head: the fused head follows (forward_loss), so the last block's output
        can stay unwritten too (ABI 9)."""
        if not self.training:
            return None
        chain = StackChain(defer_counts=True)
        if x.is_cuda:
            if getattr(self, "_fold_prep", None) is None:
                self._fold_prep = FoldPrep()
            chain.set_prep(self._fold_prep.run(list(self.conv), tuple(x.shape), x.device))
            # (ABI 8: block outputs that only the next block reads stay unwritten;
            # self.lazy_links = False writes every one)
            if getattr(self, "lazy_links", True):
                flags = lazy_links(list(self.conv), tuple(x.shape))
                if head and head_link_ok(self.conv[-1]):
                    flags[-1] = "head"
                chain.set_lazy(flags)
        return chain

    def forward_nctv(self, x):
        # same as self.conv(x), with cross-block fusion (network.StackChain)
        chain = self._chain(x)
        for blk in self.conv:
            x = blk(x, chain=chain)
        if chain is not None:
            chain.flush_counts()
        # global average pool over (T, V) (lightning_model.py:105): a mean over
        # the contiguous T*V axis; ROCm's avg_pool2d with a (T, V) window is a
        # slow generic kernel (1.7 ms at N=128), the reduction is ~20 us.
        x = x.flatten(2).mean(dim=2)
        return self.fc_layer(x)

    def forward(self, x):
        """x: (N, T, V, C_in) as in L_STGCN.forward (lightning_model.py:101)."""
        return self.forward_nctv(x.permute(0, 3, 1, 2))

    def forward_loss(self, x, labels):
        """Training step's forward with the fused HIP head: x (N, C_in, T, V)
        NCTV, labels int64 (N) -> (mean cross-entropy loss, logits); the same
        arithmetic as F.cross_entropy(self.forward_nctv(x), labels)
        (lightning_model.py:105-107, :202)."""
        chain = self._chain(x, head=True)
        for blk in self.conv:
            x = blk(x, chain=chain)
        if chain is not None:
            chain.flush_counts()
            if chain.head_ready(x):  # (ABI 9: x was never written; pooled from U)
                U, stats2 = chain.u_stats
                return StgcnHeadFn.apply(x, self.fc_layer.weight, self.fc_layer.bias, labels,
                                         (U, stats2) + tuple(chain.g2b2))
        return StgcnHeadFn.apply(x, self.fc_layer.weight, self.fc_layer.bias, labels)


class STGCN(nn.Module):
    """The legacy network class of the reference (src/network/stgcn.py:8-80),
    on the drop-in blocks: same constructor (C_in, gamma, nr_classes, strat, d,
    edge_importance), same child names / state_dict keys (``Masks.{i}`` when
    edge_importance, ``conv.{i}.*``, ``fc_layer.*``), the blocks' default
    dropout 0.5 (stgcn.py:40-51), and a softmax over the classes at the end of
    forward (stgcn.py:77). ``graph`` (not in the reference) selects the
    skeleton; the reference builds on its default body25 graph (V = 25)."""

    def __init__(self, C_in, gamma, nr_classes, strat=Strategy.UNI_LABELING, d=1,
                 edge_importance=True, graph=None, gemm_dtype=torch.float32, f32_gemm="mfma"):
        super().__init__()
        self.nr_classes = nr_classes
        temporal_padding = (gamma - 1) // 2
        A = get_normalized_adjacency_matrices(strat, d, graph=graph)
        self.K = A.shape[0]
        self.V = A.shape[1]
        self.C_in = C_in
        self.C_out = 256
        if edge_importance:
            self.Masks = nn.ParameterList([nn.Parameter(torch.ones(A.shape)) for _ in range(10)])
        else:
            self.Masks = [torch.ones(A.shape) for _ in range(10)]  # not trainable
        blocks, c = [], C_in
        for i, (co, s) in enumerate(LAYERS):
            blocks.append(SpatialTemporalConv(c, co, A * self.Masks[i], gamma, s,
                                              temporal_padding, gemm_dtype=gemm_dtype,
                                              f32_gemm=f32_gemm))
            c = co
        self.conv = nn.Sequential(*blocks).float()
        self.fc_layer = nn.Linear(256, self.nr_classes).float()
        self.softmax = nn.Softmax(dim=1)

    def forward(self, x):
        """x: (N, T, V, C_in) -> class probabilities (N, nr_classes)."""
        x = x.permute(0, 3, 1, 2)
        x = self.conv(x)
        x = x.flatten(2).mean(dim=2)  # avg_pool2d over (T, V) (stgcn.py:72-73)
        return self.softmax(self.fc_layer(x))


def flops_per_clip(C_in, T, V, K, nr_classes, gamma=9):
    """Algorithmic fwd+bwd FLOPs per clip:
    per layer fwd = 2*C_in*K*C_out*T*V + 2*K*C_out*T*V^2 + 2*gamma*C_out^2*T_out*V;
    bwd = dgrad (same three terms, minus the W term for layer 0) + wgrad (same
    three terms); plus the head 3 * 2*256*classes."""
    total, c, t = 0, C_in, T
    for i, (co, s) in enumerate(LAYERS):
        to = (t + 2 * ((gamma - 1) // 2) - gamma) // s + 1
        w = 2 * c * K * co * t * V
        a = 2 * K * co * t * V * V
        tc = 2 * gamma * co * co * to * V
        total += (w + a + tc) + ((0 if i == 0 else w) + a + tc) + (w + a + tc)
        c, t = co, to
    return total + 3 * 2 * 256 * nr_classes

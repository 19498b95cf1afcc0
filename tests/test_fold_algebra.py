"""CPU check (fp64) of the folded block's algebra (st-gcn_amd/csrc/kernels_fold.hip,
capi.hip fold_w): with one adjacency partition the SpatialConv channel GEMM
Z = W' G + bZ (st_graphconv.py:139-152, G = BN1(x) A^T) folds into the temporal
conv (st_graphconv.py:41-43, :99):

    U[o,t]  = sum_q Wc_q G[s t + q - 4] + BT[o,t],   Wc_q = Wt_q W'
    dWt_q   = dWc_q W'^T + sum_v Tq[o,v] bZ[c,v],     dWc_q = sum dU G[s t + q - 4]^T
    dW'     = sum_q Wt_q^T dWc_q,    H = W'^T dZ = conv^T(dU; Wc),
    sum_{n,t} dZ[c,v] = sum_q sum_o Wt[o,c,q] Tq[o,v],
    sum_{n,t} H[c,v]  = sum_q sum_o Wc[o,c,q] Tq[o,v]   (BN1's sum of dxhat, k_fold_sd)

Tq is built exactly as the kernels build it (k_fold_tq: the per-clip-summed
dU with the boundary frames of fold_slots subtracted), BT as k_fold_bias.
Checked against torch autograd of the unfolded block on random data, stride 1
and 2, odd and even T, T shorter than the kernel.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F


def fold_slots(T, To, st):
    nb0 = min(To, (4 + st - 1) // st)
    tb1 = max(nb0, min(To, (T - 4 + st - 1) // st))
    return nb0, tb1


def fold_bt(Wt, bt, bZ, T, To, st):
    R = Wt.shape[0]
    V = bZ.shape[1]
    bq = np.einsum("ocq,cv->qov", Wt, bZ)
    BT = np.zeros((R, To, V))
    for t in range(To):
        t0 = st * t - 4
        BT[:, t, :] = bt[:, None]
        for q in range(9):
            if 0 <= t0 + q < T:
                BT[:, t, :] += bq[q]
    return BT


def fold_tq(dU, T, st):
    N, R, To, V = dU.shape
    cs = dU.sum(axis=0)  # k_fold_colsum: [R][To][V]
    nb0, tb1 = fold_slots(T, To, st)
    frames = list(range(nb0)) + list(range(tb1, To))
    assert len(frames) <= 8
    tot = cs.sum(axis=1)
    Tq = np.zeros((9, R, V))
    for q in range(9):
        a = tot.copy()
        for t in frames:
            if not (0 <= st * t + q - 4 < T):
                a -= cs[:, t, :]
        Tq[q] = a
    return Tq


@pytest.mark.parametrize("N,C,R,T,V,st", [(2, 5, 7, 12, 3, 1), (2, 5, 7, 13, 3, 2),
                                          (1, 4, 6, 3, 2, 1), (3, 4, 4, 9, 4, 2),
                                          (2, 3, 8, 20, 5, 2)])
def test_fold_matches_unfolded_block(N, C, R, T, V, st):
    g = torch.Generator().manual_seed(N * 100 + T)
    d = torch.float64
    G = torch.randn(N, C, T, V, generator=g, dtype=d, requires_grad=True)
    W = torch.randn(R, C, generator=g, dtype=d, requires_grad=True)
    b = torch.randn(R, generator=g, dtype=d)
    rs = torch.rand(V, generator=g, dtype=d) + 0.5  # rowsum(A)
    bZ = (b[:, None] * rs[None, :])
    Wt = torch.randn(R, R, 9, generator=g, dtype=d, requires_grad=True)
    bt = torch.randn(R, generator=g, dtype=d)
    # the unfolded block (reference op order)
    Z = torch.einsum("ri,nitv->nrtv", W, G) + bZ[None, :, None, :]
    Z.retain_grad()
    U = F.conv2d(Z, Wt[..., None], bt, stride=(st, 1), padding=(4, 0))
    To = U.shape[2]
    dU = torch.randn(U.shape, generator=g, dtype=d)
    U.backward(dU)

    Gn, Wn, Wtn = G.detach().numpy(), W.detach().numpy(), Wt.detach().numpy()
    # forward: composite weights + per-frame bias table
    Wc = np.einsum("ocq,ci->oiq", Wtn, Wn)
    BT = fold_bt(Wtn, bt.numpy(), bZ.numpy(), T, To, st)
    Uf = F.conv2d(torch.from_numpy(Gn), torch.from_numpy(Wc)[..., None], None, stride=(st, 1),
                  padding=(4, 0)).numpy() + BT[None]
    np.testing.assert_allclose(Uf, U.detach().numpy(), rtol=1e-10, atol=1e-10)

    # backward
    dUn = dU.numpy()
    Gt = torch.from_numpy(Gn)
    dWc = torch.nn.grad.conv2d_weight(Gt, (R, C, 9, 1), dU, stride=(st, 1),
                                      padding=(4, 0))[..., 0].numpy()
    Tq = fold_tq(dUn, T, st)
    dWt = np.einsum("oiq,ci->ocq", dWc, Wn) + np.einsum("qov,cv->ocq", Tq, bZ.numpy())
    np.testing.assert_allclose(dWt, Wt.grad.numpy(), rtol=1e-10, atol=1e-9)
    dWp = np.einsum("ocq,oiq->ci", Wtn, dWc)
    np.testing.assert_allclose(dWp, W.grad.numpy(), rtol=1e-10, atol=1e-9)
    # H = W'^T dZ = the data gradient of the conv with Wc (G's gradient)
    H = torch.nn.grad.conv2d_input(Gt.shape, torch.from_numpy(Wc)[..., None], dU,
                                   stride=(st, 1), padding=(4, 0)).numpy()
    np.testing.assert_allclose(H, G.grad.numpy(), rtol=1e-10, atol=1e-9)
    SdZ = np.einsum("ocq,qov->cv", Wtn, Tq)
    np.testing.assert_allclose(SdZ, Z.grad.sum(dim=(0, 2)).numpy(), rtol=1e-10, atol=1e-9)
    # the analytic BN1 sum of the folded backward (k_fold_red64 + k_fold_sd):
    # sum_{n,t} H[c,v] = sum_q sum_o Wc[o,c,q] Tq[q,o,v], and with
    # dxhat[c,t,w] = sum_v A[v,w] H[c,t,v]: sum_{n,t,w} dxhat = sum_v SdH rowsum(A)
    SdH = np.einsum("ocq,qov->cv", Wc, Tq)
    np.testing.assert_allclose(SdH, H.sum(axis=(0, 2)), rtol=1e-10, atol=1e-9)
    A = np.random.default_rng(N + T).uniform(0.0, 1.0, (V, V))
    dxhat = np.einsum("vw,nctv->nctw", A, H)
    np.testing.assert_allclose(SdH @ A.sum(axis=1), dxhat.sum(axis=(0, 2, 3)), rtol=1e-10,
                               atol=1e-9)

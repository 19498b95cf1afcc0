"""CPU check of the deferred-dx chain's algebra (ABI 5; capi.hip, k_chain_coef
in kernels.hip): block i's BN1 backward apply folded into block i-1's
ReLU+BN2 backward needs block i-1's sums  sum m*dx  and  sum m*dx*uhat  BEFORE
dx exists. The kernel forms them from the prev-mode sums of the spatial
backward (s1 = sum m*dxhat, s2 = sum m*dxhat*uhat) and block i-1's forward
sums (sum x, cnt = sum m, su = sum m*uhat, xu = sum x*uhat). This restates
k_chain_coef's formula in fp64 and compares it with the direct sums over the
materialised dx (the unchained path, k_bn1_bwd_apply), for random tensors
including channels with gamma2 = 0 and |beta2| >> |gamma2|."""
import torch


def _case(seed):
    g = torch.Generator().manual_seed(seed)
    N, C, T, V = 3, 6, 11, 5
    U = torch.randn(N, C, T, V, generator=g, dtype=torch.float64) * 2 + 0.3
    mean2 = U.mean((0, 2, 3))
    invstd2 = 1 / (U.var((0, 2, 3), unbiased=False) + 1e-5).sqrt()
    g2 = torch.randn(C, generator=g, dtype=torch.float64)
    b2 = torch.randn(C, generator=g, dtype=torch.float64)
    g2[0], b2[0] = 0.0, 0.7          # gamma2 = 0: x constant on the mask
    g2[1], b2[1] = 1e-4, -0.5        # |beta2| >> |gamma2|
    c = lambda v: v.view(1, C, 1, 1)
    uhat = (U - c(mean2)) * c(invstd2)
    t = uhat * c(g2) + c(b2)
    m = (t > 0).double()
    x = t.clamp_min(0)                # the previous block's output = this block's input
    M = N * T * V
    mu1 = x.mean((0, 2, 3))
    is1 = 1 / (x.var((0, 2, 3), unbiased=False) + 1e-5).sqrt()
    g1 = torch.randn(C, generator=g, dtype=torch.float64)
    dxhat = torch.randn(N, C, T, V, generator=g, dtype=torch.float64)
    return dict(C=C, M=M, c=c, uhat=uhat, m=m, x=x, mu1=mu1, is1=is1, g1=g1, dxhat=dxhat)


def test_chain_coef_formula_matches_direct_sums():
    for seed in range(5):
        d = _case(seed)
        c, M = d["c"], d["M"]
        xn = (d["x"] - c(d["mu1"])) * c(d["is1"])
        sd = d["dxhat"].sum((0, 2, 3))
        sdn = (d["dxhat"] * xn).sum((0, 2, 3))
        a = d["is1"] * d["g1"]
        md, mdn = sd / M, sdn / M
        dx = c(a) * (d["dxhat"] - c(md) - xn * c(mdn))        # k_bn1_bwd_apply
        want1 = (dx * d["m"]).sum((0, 2, 3))
        want2 = (dx * d["m"] * d["uhat"]).sum((0, 2, 3))
        # k_chain_coef
        s1 = (d["m"] * d["dxhat"]).sum((0, 2, 3))
        s2 = (d["m"] * d["dxhat"] * d["uhat"]).sum((0, 2, 3))
        sx = d["x"].sum((0, 2, 3))
        cnt = d["m"].sum((0, 2, 3))
        su = (d["m"] * d["uhat"]).sum((0, 2, 3))
        xu = (d["x"] * d["uhat"]).sum((0, 2, 3))
        p1 = a * (s1 - md * cnt - mdn * d["is1"] * (sx - d["mu1"] * cnt))
        p2 = a * (s2 - md * su - mdn * d["is1"] * (xu - d["mu1"] * su))
        scale = dx.abs().sum((0, 2, 3)) + 1e-300
        assert ((p1 - want1).abs() / scale).max() < 1e-12, seed
        assert ((p2 - want2).abs() / (scale * d["uhat"].abs().max())).max() < 1e-12, seed
        # the coefficients reproduce dx itself (dy_coef in k_bn_relu_bwd_apply)
        dy = c(a) * (d["dxhat"] - c(md) - (d["x"] - c(d["mu1"])) * c(d["is1"]) * c(mdn))
        assert torch.allclose(dy, dx, rtol=0, atol=1e-12)

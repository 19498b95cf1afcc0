"""The training step captured in a HIP graph (train_ops.GraphedStep, the
bench's N=1 step mode) and the device-step Adam it needs (ABI 11,
stgcn_adam_step_dev; torch.optim.Adam(capturable=True) semantics for
lightning_model.py:196-197). Gates:
- FusedAdam(capturable=True) against FusedAdam with the host step count:
  identical parameters and moments over 6 steps (the same fp32 element
  arithmetic; the bias corrections formed in double on the device instead of
  the host -- a 1-ulp difference in double that changed a float would fail
  this, so it is allowed only as 1 ulp of fp32 per element);
- a graphed STGCNStack step (f16x2 folded blocks, the benched mode; and the
  bf16 K = 3 path) against the same step run eagerly from the same init:
  loss, logits and every parameter equal after warm-up + replays (every kernel
  of the step is deterministic: no order-dependent atomics in the benched path).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _ulp_close(a, b, ulps=1):
    """|a - b| <= ulps * ulp(max(|a|, |b|)) per element (fp32)."""
    a, b = a.float(), b.float()
    m = torch.maximum(a.abs(), b.abs())
    ulp = torch.nextafter(m, torch.full_like(m, float("inf"))) - m
    return bool(((a - b).abs() <= ulps * ulp).all())


@pytest.mark.parametrize("wd", [0.0, 0.01])
def test_fused_adam_capturable_matches_host_step(pkg, wd):
    g = torch.Generator().manual_seed(7)
    shapes = [(64, 3, 9), (256,), (400, 256), (18, 18)]
    p0 = [torch.randn(s, generator=g) for s in shapes]
    grads = [[torch.randn(s, generator=g) for s in shapes] for _ in range(6)]
    pa = [t.to(DEV).requires_grad_(True) for t in p0]
    pb = [t.to(DEV).requires_grad_(True) for t in p0]
    oa = pkg.FusedAdam(pa, lr=1e-3, weight_decay=wd)
    ob = pkg.FusedAdam(pb, lr=1e-3, weight_decay=wd, capturable=True)
    for gs in grads:
        for p, gg in zip(pa, gs):
            p.grad = gg.to(DEV)
        for p, gg in zip(pb, gs):
            p.grad = gg.to(DEV)
        oa.step()
        ob.step()
    torch.cuda.synchronize()
    step_b = ob.state[pb[0]]["step"]
    assert step_b.is_cuda and float(step_b) == 6.0
    assert all(ob.state[p]["step"] is step_b for p in pb)  # one counter per group
    for a, b in zip(pa, pb):
        assert _ulp_close(a.detach(), b.detach())
        for k in ("exp_avg", "exp_avg_sq"):
            assert _ulp_close(oa.state[a][k], ob.state[b][k])


def _stack(pkg, V, K, bf16):
    gr = pkg.graph
    if K == 1:
        A = gr.get_normalized_adjacency_matrices(0, 1, graph=gr.graph_for(V))
    else:
        A = gr.get_normalized_adjacency_matrices(2, 1, distances=gr.synthetic_distances(V),
                                                 graph=gr.graph_for(V))
    torch.manual_seed(0)
    m = pkg.STGCNStack(3, 10, A, gemm_dtype=torch.bfloat16 if bf16 else torch.float32,
                       f32_gemm="f16x2")
    return m.to(DEV)


@pytest.mark.parametrize("V,K,bf16", [(18, 1, False), (25, 3, True)])
def test_graphed_step_matches_eager(pkg, V, K, bf16):
    N, T = 4, 32
    g = torch.Generator().manual_seed(3)
    x = torch.randn(N, 3, T, V, generator=g).to(DEV)
    labels = torch.randint(0, 10, (N,), generator=g).to(DEV)

    def make():
        m = _stack(pkg, V, K, bf16)
        opt = pkg.FusedAdam(list(m.parameters()), lr=1e-3, capturable=True)

        def step():
            opt.zero_grad(set_to_none=True)
            loss, logits = m.forward_loss(x, labels)
            loss.backward()
            opt.step()
            return loss, logits
        return m, step

    ma, step_a = make()
    mb, step_b = make()
    for _ in range(5):  # eager: 5 steps
        la, ga = step_a()
    graphed = pkg.GraphedStep(step_b, warmup=2)  # 2 eager steps, capture
    for _ in range(3):  # + 3 replays
        lb, gb = graphed()
    torch.cuda.synchronize()
    assert torch.equal(la, lb) and torch.equal(ga, gb)
    for (ka, a), (kb, b) in zip(ma.state_dict().items(), mb.state_dict().items()):
        assert ka == kb
        assert torch.equal(a, b), ka

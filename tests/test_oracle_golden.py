"""Pin the oracle (oracle/ref_cpu.py) and the graph module against golden
vectors produced by the reference itself (tests/golden/make_golden.py)."""
import numpy as np
import pytest
import torch

from conftest import block_fixtures, load_npz, rel_to_max
from oracle import ref_cpu

# fp32 oracle vs fp32 reference: same ops, same library -> tiny differences
# only from thread scheduling; fp64 oracle vs fp32 reference: the fp32 noise
# floor measured in SURVEY §8c (<= 5e-6 rel-to-max).
TOL_FP32 = 1e-5
# The fp32 reference itself is off exact arithmetic by up to ~4e-5 on the
# W-bias grad of the residual variant (BN2 right after the spatial conv makes
# that grad a small difference of large terms), so the fp64 yardstick gets 5e-5.
TOL_FP64 = 5e-5
ATOL_ZERO_GRAD = 1e-6  # temporalConv.bias grad is analytically 0


@pytest.mark.parametrize("fixture", block_fixtures())
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_block_oracle_matches_reference(fixture, dtype):
    ref = load_npz(fixture)
    out = ref_cpu.block_step(ref, dtype=dtype)
    residual = bool(ref["meta"][7])
    for k, v in out.items():
        want = ref[k]
        got = v.detach().double().numpy()
        if k == "grad.temporalConv.bias" and not residual:
            assert np.abs(got - want).max() < ATOL_ZERO_GRAD * max(1.0, np.abs(ref["g"]).max()), k
            continue
        if k.endswith("num_batches_tracked"):
            assert int(got) == int(want)
            continue
        tol = TOL_FP32 if dtype == torch.float32 else TOL_FP64
        assert rel_to_max(got, want) < tol, (fixture, k, rel_to_max(got, want))


def test_stack_init_matches_reference_init():
    ref = load_npz("stack_cfg1.npz")
    A = torch.from_numpy(load_npz("adjacency.npz")["V18_s0_d1"])
    p, _ = ref_cpu.init_stack_params(3, 2, A, seed=0)
    for k, v in p.items():
        flat = v.reshape(-1)
        np.testing.assert_array_equal(flat[torch.as_tensor(ref["pidx." + k])].numpy(), ref["pval." + k])
        assert abs(flat.double().sum().item() - float(ref["psum." + k])) <= 1e-9 * max(1, abs(float(ref["psum." + k])))


def _stack_step(dtype):
    ref = load_npz("stack_cfg1.npz")
    A = torch.from_numpy(load_npz("adjacency.npz")["V18_s0_d1"])
    p, b = ref_cpu.init_stack_params(3, 2, A, seed=0)
    p = {k: v.clone().to(dtype).requires_grad_(True) for k, v in p.items()}
    b = {k: (v.clone().to(dtype) if v.is_floating_point() else v.clone()) for k, v in b.items()}
    st = ref_cpu.Stack(p, b)
    logits = st.forward(torch.from_numpy(ref["x"]), dtype=dtype)
    loss = torch.nn.functional.cross_entropy(logits, torch.from_numpy(ref["labels"]))
    loss.backward()
    worst = 0.0
    for k, v in p.items():
        got = v.grad.reshape(-1)
        if k.endswith("temporalConv.bias"):
            assert got.abs().max().item() < 1e-6
            continue
        gn = float(ref["gnorm." + k])
        sampled = got[torch.as_tensor(ref["pidx." + k])].numpy()
        worst = max(worst, abs(got.norm().item() - gn) / gn,
                    rel_to_max(sampled, ref["gval." + k]))
    return ref, logits, loss, worst


def test_stack_forward_backward_matches_reference():
    """fp32 oracle vs the fp32 reference: same ops in the same order."""
    ref, logits, loss, worst = _stack_step(torch.float32)
    assert rel_to_max(logits.detach().numpy(), ref["logits"]) < 1e-5
    assert abs(loss.item() - float(ref["loss"])) < 1e-6
    assert worst < 1e-4, worst


def test_stack_fp32_conditioning_is_documented():
    """The 10-block stack amplifies fp32 rounding: the fp32 reference's grads
    sit up to a few % away from exact (fp64) arithmetic on some params (the
    dA / BN-affine grads are small differences of large terms because BN makes
    the loss invariant to the scale of A). This bounds what any fp32
    implementation (including the HIP one) can match at stack level; block-level
    parity is where the tight 1e-5 gate applies (Parity)."""
    ref, logits, loss, worst = _stack_step(torch.float64)
    assert rel_to_max(logits.detach().numpy(), ref["logits"]) < 1e-4
    assert abs(loss.item() - float(ref["loss"])) < 1e-5
    assert 1e-4 < worst < 0.1, worst


def test_adjacency_matches_reference(pkg):
    gr = pkg.graph
    ref = load_npz("adjacency.npz")
    for key, want in ref.items():
        V, s, d = key.split("_")
        V, s, d = int(V[1:]), int(s[1:]), int(d[1:])
        A = gr.get_normalized_adjacency_matrices(s, d, distances=gr.synthetic_distances(V),
                                                 graph=gr.graph_for(V))
        np.testing.assert_array_equal(A.numpy(), want, err_msg=key)


def test_adjacency_dense_and_large(pkg):
    """the bug-compatible normalisation makes A dense with
    entries ~1e4-1e5."""
    A = pkg.graph.get_normalized_adjacency_matrices(0, 1, graph=pkg.graph.graph_for(18))
    assert (A > 1e4).all()

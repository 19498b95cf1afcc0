"""Round-2 pins of the oracle and the host-side mirrors against fixtures the
reference itself produced (tests/golden/make_golden.py --only extra):

* SpatialConv used on its own (src/network/st_graphconv.py:139-152);
* L_STGCN with --use_edge_importance (lightning_model.py:53-57: jittered
  masks drawn before the blocks, ``Masks.{i}`` in the state_dict);
* the legacy network class STGCN (src/network/stgcn.py:8-80) in eval mode
  (masks of ones, dropout 0.5 blocks, softmax output) -- forward and backward
  through BatchNorm on running statistics.

The host-side module mirrors (``STGCNStack(use_edge_importance=True)``,
``STGCN``) are checked here for init equality and state_dict keys (CPU); their
GPU forward/backward is in tests/test_gpu_callers.py.
"""
import glob
import io
import contextlib
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, load_npz, rel_to_max
from oracle import ref_cpu


def _spatial_fixtures():
    return sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLDEN, "spatialconv_*.npz")))


@pytest.mark.parametrize("fixture", _spatial_fixtures())
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_spatialconv_oracle_matches_reference(fixture, dtype):
    ref = load_npz(fixture)
    p = {k[len("param."):]: torch.from_numpy(v).to(dtype).requires_grad_(True)
         for k, v in ref.items() if k.startswith("param.")}
    x = torch.from_numpy(ref["x"]).to(dtype).requires_grad_(True)
    y = ref_cpu.spatial_conv(x, p["A"], p["W.weight"], p["W.bias"])
    (y * torch.from_numpy(ref["g"]).to(dtype)).sum().backward()
    tol = 1e-5 if dtype == torch.float32 else 5e-5
    assert rel_to_max(y.detach().double().numpy(), ref["y"]) < tol
    assert rel_to_max(x.grad.double().numpy(), ref["grad.x"]) < tol
    for k, v in p.items():
        assert rel_to_max(v.grad.double().numpy(), ref["grad." + k]) < tol, k


def _check_init(p, ref):
    for k, v in p.items():
        flat = v.detach().reshape(-1)
        np.testing.assert_array_equal(flat[torch.as_tensor(ref["pidx." + k])].numpy(),
                                      ref["pval." + k], err_msg=k)


def test_edge_importance_oracle_matches_reference():
    ref = load_npz("stack_cfg1_edge.npz")
    A = torch.from_numpy(load_npz("adjacency.npz")["V18_s0_d1"])
    p, b = ref_cpu.init_stack_params(3, 2, A, seed=0, masks="jitter", max_mask_jitter=0.05)
    _check_init(p, ref)
    assert sorted(k for k in p if k.startswith("Masks.")) == sorted(
        k for k in ref["state_keys"] if k.startswith("Masks."))
    p = {k: v.clone().requires_grad_(True) for k, v in p.items()}
    logits = ref_cpu.Stack(p, b).forward(torch.from_numpy(ref["x"]))
    loss = torch.nn.functional.cross_entropy(logits, torch.from_numpy(ref["labels"]))
    loss.backward()
    assert rel_to_max(logits.detach().numpy(), ref["logits"]) < 1e-5
    assert abs(loss.item() - float(ref["loss"])) < 1e-6
    for k, v in p.items():
        if k.startswith("Masks."):  # dead in the reference too (no gradient)
            assert v.grad is None and ("gval." + k) not in ref
            continue
        if k.endswith("temporalConv.bias"):
            continue
        got = v.grad.reshape(-1)[torch.as_tensor(ref["pidx." + k])].numpy()
        assert rel_to_max(got, ref["gval." + k]) < 1e-4, k


def test_edge_importance_stack_init_and_keys(pkg):
    ref = load_npz("stack_cfg1_edge.npz")
    A = torch.from_numpy(load_npz("adjacency.npz")["V18_s0_d1"])
    torch.manual_seed(0)
    with contextlib.redirect_stdout(io.StringIO()):
        model = pkg.STGCNStack(3, 2, A, use_edge_importance=True, max_mask_jitter=0.05)
    assert list(model.state_dict().keys()) == list(ref["state_keys"])
    _check_init(dict(model.named_parameters()), ref)


def legacy_running_stats(ref):
    """The fixture's calibrated running statistics (state_dict naming)."""
    return {k[len("run."):]: torch.from_numpy(v) for k, v in ref.items() if k.startswith("run.")}


def _legacy_oracle(ref, dtype):
    A = torch.from_numpy(load_npz("adjacency.npz")["V25_s0_d1"])
    p, b = ref_cpu.init_stack_params(3, 5, A, seed=0, masks="ones")
    _check_init(p, ref)
    b.update(legacy_running_stats(ref))
    p = {k: v.clone().to(dtype).requires_grad_(True) for k, v in p.items()}
    b = {k: (v.clone().to(dtype) if v.is_floating_point() else v) for k, v in b.items()}
    x = torch.from_numpy(ref["x"]).to(dtype).requires_grad_(True)
    probs = torch.softmax(ref_cpu.Stack(p, b).forward(x, training=False, dtype=dtype), dim=1)
    (probs * torch.from_numpy(ref["g"]).to(dtype)).sum().backward()
    return p, b, x, probs


def test_legacy_stgcn_oracle_matches_reference():
    ref = load_npz("legacy_stgcn.npz")
    p, b, x, probs = _legacy_oracle(ref, torch.float32)
    assert rel_to_max(probs.detach().numpy(), ref["probs"]) < 1e-5
    assert rel_to_max(x.grad.numpy(), ref["grad.x"]) < 1e-4
    for k, v in p.items():
        if k.startswith("Masks."):
            continue
        got = v.grad.reshape(-1)[torch.as_tensor(ref["pidx." + k])].numpy()
        assert rel_to_max(got, ref["gval." + k]) < 1e-4, k


def test_legacy_stgcn_init_and_keys(pkg):
    ref = load_npz("legacy_stgcn.npz")
    torch.manual_seed(0)
    with contextlib.redirect_stdout(io.StringIO()):
        model = pkg.STGCN(3, 9, 5)
    assert list(model.state_dict().keys()) == list(ref["state_keys"])
    _check_init(dict(model.named_parameters()), ref)
    assert all(blk.dropout is not None and blk.dropout.p == 0.5 for blk in model.conv)

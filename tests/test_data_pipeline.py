"""Host input pipeline vs fixtures produced by the
reference itself (tests/golden/make_golden.py --only data): loop-padding
collate (src/data/util.py:12-47), augmentation under fixed np.random seeds
(src/data/augmentation.py:8-69), joint distances to the centre of gravity
(src/data/calculate_distances.py:7-48). All bit-exact (float64 numpy)."""
import os
import tempfile

import numpy as np
import pytest
import torch

from conftest import load_npz


@pytest.fixture(scope="module")
def gold():
    return load_npz("data_pipeline.npz")


def test_loopy_pad_collate_matches_reference(pkg, gold):
    batch = [(gold[f"collate_in_{i}"], np.array([i % 6])) for i in range(5)]
    xx, labels = pkg.data.loopy_pad_collate_fn(batch)
    assert xx.dtype == torch.float64 and tuple(xx.shape) == gold["collate_out_x"].shape
    assert np.array_equal(xx.numpy(), gold["collate_out_x"])
    assert np.array_equal(labels.numpy(), gold["collate_out_labels"])


def test_pad_array_with_loops_edge_cases(pkg):
    x = np.arange(2 * 3 * 2 * 1, dtype=np.float64).reshape(2, 3, 2, 1)
    assert pkg.data.pad_array_with_loops(x, 3) is x          # already long enough
    assert pkg.data.pad_array_with_loops(x, 2) is x          # longer: untouched (no cut)
    y = pkg.data.pad_array_with_loops(x, 7)
    assert np.array_equal(y[:, 3:6], x) and np.array_equal(y[:, 6], x[:, 0])


@pytest.mark.parametrize("seed", range(6))
def test_augment_data_matches_reference(pkg, gold, seed):
    np.random.seed(seed)
    out = pkg.data.augment_data(gold["augment_in"])
    assert np.array_equal(out, gold[f"augment_out_seed{seed}"])


def test_augment_data_keeps_input(pkg, gold):
    seqs = gold["augment_in"].copy()
    np.random.seed(1)
    pkg.data.augment_data(seqs)
    assert np.array_equal(seqs, gold["augment_in"])


def test_joint_distances_match_reference(pkg, gold):
    clips = [gold[f"dist_clip{i}"] for i in gold["dist_listdir_order"]]
    d = pkg.data.joint_distances(clips, V=25)
    assert np.array_equal(d, gold["dist_out"])


def test_calculate_distances_file_level(pkg, gold):
    with tempfile.TemporaryDirectory() as tmp:
        os.makedirs(os.path.join(tmp, "data"))
        for i in range(3):
            np.save(os.path.join(tmp, "data", f"clip{i}.npy"), gold[f"dist_clip{i}"])
        out = os.path.join(tmp, "distances.npy")
        d = pkg.data.calculate_distances(V=25, dataset_dir=os.path.join(tmp, "data"),
                                         output_file=out)
        assert np.allclose(np.load(out), gold["dist_out"], rtol=1e-14, atol=0)
        assert np.array_equal(np.load(out), d)


def test_distances_feed_spatial_partitioning(pkg, gold):
    """The measured distances drive strategy 2 (spatial configuration) like the
    synthetic ones: K = 3 partitions, finite normalized A."""
    gr = pkg.graph
    A = gr.get_normalized_adjacency_matrices(2, 1, distances=gold["dist_out"],
                                             graph=gr.graph_for(25))
    assert tuple(A.shape) == (3, 25, 25) and torch.isfinite(A).all()


def test_load_clip_drops_confidence(pkg):
    with tempfile.TemporaryDirectory() as tmp:
        clip = np.random.default_rng(0).standard_normal((6, 25, 3))
        np.save(os.path.join(tmp, "c.npy"), clip)
        assert np.array_equal(pkg.data.load_clip(os.path.join(tmp, "c.npy")), clip[:, :, :2])


@pytest.mark.gpu
def test_device_loader_feeds_the_stack(pkg, gold):
    """Ragged clips -> loop-pad collate -> augment -> DeviceLoader (pinned,
    async) -> NCTV fp32 on the GPU -> a training step of the fused stack."""
    rng = np.random.default_rng(3)
    batches = []
    for b in range(3):
        items = [(rng.standard_normal((1, t, 25, 2)) * 40 + 100, np.array([(b + i) % 6]))
                 for i, t in enumerate((9 + b, 5, 12))]
        x, y = pkg.data.loopy_pad_collate_fn(items)
        np.random.seed(b)
        x = torch.from_numpy(pkg.data.augment_data(x.numpy()))
        batches.append((x, y))
    gr = pkg.graph
    A = gr.get_normalized_adjacency_matrices(2, 1, distances=gold["dist_out"],
                                             graph=gr.graph_for(25))
    torch.manual_seed(0)
    model = pkg.STGCNStack(2, 6, A).to("cuda:0")
    opt = pkg.FusedAdam(model.parameters(), lr=1e-3)
    seen = 0
    for (xd, yd), (x, y) in zip(pkg.data.DeviceLoader(batches, "cuda:0"), batches):
        assert xd.is_contiguous() and xd.dtype == torch.float32
        assert torch.equal(xd.cpu(), x.float().permute(0, 3, 1, 2))
        assert torch.equal(yd.cpu(), y)
        opt.zero_grad(set_to_none=True)
        loss, _ = model.forward_loss(xd, yd)
        loss.backward()
        opt.step()
        assert torch.isfinite(loss).item()
        seen += 1
    assert seen == 3

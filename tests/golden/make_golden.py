"""Generate golden fixtures by running the REFERENCE itself (this container only).

Usage: python3 -B tests/golden/make_golden.py [/root/reference]

The reference (nagyrajmund/st-gcn, pure Python over PyTorch) is imported from
its read-only checkout; nothing of it is copied. Two third-party modules it
imports but that are absent here and off the arithmetic path are replaced by
in-process stubs: ``pytorch_lightning`` (``lightning_model.py:5-7,21``) and
``seaborn`` (pulled in by ``lightning_model.py:19``). Bytecode writing is
disabled so the read-only tree is untouched.

Outputs (small .npz files next to this script):
  adjacency.npz   normalized A for V=25 (strategies 0-3), V=18 / V=50 (0-2)
                  computed by src/data/adjacency.py with adj_list/nr_of_joints
                  patched for V != 25.
  block_*.npz     one SpatialTemporalConv (src/network/st_graphconv.py) in
                  training mode: params, x, upstream grad g, y, every grad,
                  running stats after the step.
  stack_cfg1.npz  full L_STGCN (src/lightning_model.py) cfg1 plumbing case:
                  logits, loss, param checksums and sampled grads.
  spatialconv_*.npz  SpatialConv on its own (st_graphconv.py:139-152).
  stack_cfg1_edge.npz  the cfg1 case with --use_edge_importance (masks).
  legacy_stgcn.npz  src/network/stgcn.py STGCN in eval mode (probs + grads).
  data_pipeline.npz  host input pipeline:
                  src/data/util.py loopy_pad_collate_fn on a ragged batch,
                  src/data/augmentation.py augment_data under fixed
                  np.random seeds, src/data/calculate_distances.py on
                  synthetic (T, 25, 3) .npy clips written to a temp dir.

  --only data     regenerate data_pipeline.npz only.
  --only extra    regenerate the round-2 fixtures only (spatialconv_*,
                  stack_cfg1_edge, legacy_stgcn).
"""
import argparse
import os
import sys
import tempfile
import types

sys.dont_write_bytecode = True

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))


def _install_stubs():
    pl = types.ModuleType("pytorch_lightning")
    core = types.ModuleType("pytorch_lightning.core")
    lightning = types.ModuleType("pytorch_lightning.core.lightning")
    callbacks = types.ModuleType("pytorch_lightning.callbacks")

    class LightningModule(nn.Module):
        pass

    class Trainer:
        @staticmethod
        def add_argparse_args(parser):
            return parser

    class EarlyStopping:
        def __init__(self, *a, **k):
            pass

    lightning.LightningModule = LightningModule
    core.lightning = lightning
    pl.core = core
    pl.Trainer = Trainer
    callbacks.EarlyStopping = EarlyStopping
    pl.callbacks = callbacks
    sys.modules.update({
        "pytorch_lightning": pl,
        "pytorch_lightning.core": core,
        "pytorch_lightning.core.lightning": lightning,
        "pytorch_lightning.callbacks": callbacks,
    })
    sns = types.ModuleType("seaborn")
    sns.set = lambda *a, **k: None
    sys.modules.setdefault("seaborn", sns)


COCO18_ADJ = None  # filled from the build's graph module (same edges)


def _graph_lists(V):
    """adj_list / opposite_joints dicts for V in {18, 50} from the build's
    graph definitions (the reference has V=25 only)."""
    sys.path.insert(0, os.path.join(HERE, "..", ".."))
    from stgcn_loader import load
    g = load().graph.graph_for(V)
    return g.adj_list, g.opposite_joints


def _patched_adjacency(adjacency, V):
    import contextlib

    @contextlib.contextmanager
    def ctx():
        saved = (adjacency.adj_list, adjacency.nr_of_joints, adjacency.opposite_joints)
        if V != 25:
            adj, opp = _graph_lists(V)
            adjacency.adj_list, adjacency.nr_of_joints, adjacency.opposite_joints = adj, V, opp
        try:
            yield
        finally:
            adjacency.adj_list, adjacency.nr_of_joints, adjacency.opposite_joints = saved
    return ctx()


def _distance_file(V, tmpdir):
    path = os.path.join(tmpdir, f"dist{V}.npy")
    np.save(path, np.linspace(1.0, 2.0, V))
    return path


def make_adjacency(adjacency, tmpdir):
    out = {}
    for V, strats in ((25, (0, 1, 2, 3)), (18, (0, 1, 2)), (50, (0, 1, 2))):
        for s in strats:
            for d in ((1, 2) if s in (0, 1) else (1,)):
                with _patched_adjacency(adjacency, V):
                    A = adjacency.get_normalized_adjacency_matrices(
                        s, d, distance_file=_distance_file(V, tmpdir))
                out[f"V{V}_s{s}_d{d}"] = A.numpy().astype(np.float32)
    np.savez_compressed(os.path.join(HERE, "adjacency.npz"), **out)
    return out


BLOCK_CASES = [
    # name, C_in, C_out, stride, V, strategy, N, T, residual
    ("b3x64_v18", 3, 64, 1, 18, 0, 2, 32, False),
    ("b64x64_v18", 64, 64, 1, 18, 0, 2, 24, False),
    ("b64x128s2_v18", 64, 128, 2, 18, 0, 2, 24, False),
    ("b128x256s2_v18", 128, 256, 2, 18, 0, 2, 8, False),
    ("b64x64_v25k3", 64, 64, 1, 25, 2, 2, 20, False),
    ("b64x128s2_v25k3", 64, 128, 2, 25, 2, 2, 16, False),
    ("b3x64_v50k3", 3, 64, 1, 50, 2, 2, 12, False),
    ("res64x64_v18", 64, 64, 1, 18, 0, 2, 20, True),
    ("res64x128s2_v18", 64, 128, 2, 18, 0, 2, 20, True),
]


def make_block(st_graphconv, adj_mats, name, C_in, C_out, stride, V, strat, N, T, residual):
    A = torch.from_numpy(adj_mats[f"V{V}_s{strat}_d1"])
    torch.manual_seed(0)
    blk = st_graphconv.SpatialTemporalConv(C_in, C_out, A, 9, stride, 4,
                                           dropout_rate=0, residual=residual)
    # BN affine params at init are 1/0; perturb them (seeded) so the affine
    # paths are exercised by the fixture.
    g0 = torch.Generator().manual_seed(3)
    with torch.no_grad():
        for bn in (blk.batch_n, blk.batch_n_2):
            bn.weight.copy_(1.0 + 0.1 * torch.randn(bn.weight.shape, generator=g0))
            bn.bias.copy_(0.1 * torch.randn(bn.bias.shape, generator=g0))
    blk.train()
    params0 = {k: v.detach().clone() for k, v in blk.state_dict().items()}
    x = torch.randn(N, C_in, T, V, generator=torch.Generator().manual_seed(1))
    x.requires_grad_(True)
    y = blk(x)
    g = torch.randn(y.shape, generator=torch.Generator().manual_seed(2))
    (y * g).sum().backward()
    rec = {"x": x.detach().numpy(), "g": g.numpy(), "y": y.detach().numpy(),
           "grad.x": x.grad.numpy()}
    for k, v in params0.items():
        rec["param." + k] = v.numpy()
    for k, p in blk.named_parameters():
        rec["grad." + k] = p.grad.numpy()
    for k, v in blk.state_dict().items():
        if "running" in k or "num_batches" in k:
            rec["after." + k] = v.numpy()
    meta = np.array([C_in, C_out, stride, V, strat, N, T, int(residual)], dtype=np.int64)
    rec["meta"] = meta
    np.savez_compressed(os.path.join(HERE, f"block_{name}.npz"), **rec)


def make_stack_cfg1(lightning_model, adjacency):
    parser = lightning_model.build_argument_parser()
    hp = parser.parse_args(["--C_in", "3", "--nr_classes", "2"])
    with _patched_adjacency(adjacency, 18):
        torch.manual_seed(0)
        model = lightning_model.L_STGCN(hp)
    model.train()
    N, T, V, C = 4, 50, 18, 3
    x = torch.randn(N, T, V, C, generator=torch.Generator().manual_seed(1))
    y = torch.randint(0, 2, (N,), generator=torch.Generator().manual_seed(2))
    logits = model(x)
    loss = torch.nn.functional.cross_entropy(logits, y)
    loss.backward()
    rec = {"x": x.numpy(), "labels": y.numpy(), "logits": logits.detach().numpy(),
           "loss": np.array(loss.item())}
    gen = torch.Generator().manual_seed(4)
    for k, p in model.named_parameters():
        flat_p = p.detach().reshape(-1)
        flat_g = p.grad.reshape(-1)
        idx = torch.randint(0, flat_p.numel(), (min(256, flat_p.numel()),), generator=gen)
        rec["pidx." + k] = idx.numpy()
        rec["pval." + k] = flat_p[idx].numpy()
        rec["psum." + k] = np.array(flat_p.double().sum().item())
        rec["gval." + k] = flat_g[idx].numpy()
        rec["gsum." + k] = np.array(flat_g.double().sum().item())
        rec["gnorm." + k] = np.array(flat_g.double().norm().item())
    for k, v in model.state_dict().items():
        if "running" in k:
            rec["after." + k] = v.numpy()
    np.savez_compressed(os.path.join(HERE, "stack_cfg1.npz"), **rec)


SPATIAL_CASES = [
    # name, C_in, C_out, V, strategy, N, T
    ("s3x64_v18", 3, 64, 18, 0, 2, 20),
    ("s64x64_v25k3", 64, 64, 25, 2, 2, 16),
    ("s64x128_v50k3", 64, 128, 50, 2, 2, 9),
]


def make_spatialconv(st_graphconv, adj_mats, name, C_in, C_out, V, strat, N, T):
    """SpatialConv used on its own (st_graphconv.py:139-152), fwd + bwd."""
    A = torch.from_numpy(adj_mats[f"V{V}_s{strat}_d1"])
    torch.manual_seed(0)
    sc = st_graphconv.SpatialConv(C_in, C_out, A)
    params0 = {k: v.detach().clone() for k, v in sc.state_dict().items()}
    x = torch.randn(N, C_in, T, V, generator=torch.Generator().manual_seed(1))
    x.requires_grad_(True)
    y = sc(x)
    g = torch.randn(y.shape, generator=torch.Generator().manual_seed(2))
    (y * g).sum().backward()
    rec = {"x": x.detach().numpy(), "g": g.numpy(), "y": y.detach().numpy(),
           "grad.x": x.grad.numpy(), "meta": np.array([C_in, C_out, V, strat, N, T])}
    for k, v in params0.items():
        rec["param." + k] = v.numpy()
    for k, p in sc.named_parameters():
        rec["grad." + k] = p.grad.numpy()
    np.savez_compressed(os.path.join(HERE, f"spatialconv_{name}.npz"), **rec)


def _sampled(model, rec, gen, grads=True):
    for k, p in model.named_parameters():
        flat_p = p.detach().reshape(-1)
        idx = torch.randint(0, flat_p.numel(), (min(256, flat_p.numel()),), generator=gen)
        rec["pidx." + k] = idx.numpy()
        rec["pval." + k] = flat_p[idx].numpy()
        rec["psum." + k] = np.array(flat_p.double().sum().item())
        if grads and p.grad is not None:
            flat_g = p.grad.reshape(-1)
            rec["gval." + k] = flat_g[idx].numpy()
            rec["gsum." + k] = np.array(flat_g.double().sum().item())
            rec["gnorm." + k] = np.array(flat_g.double().norm().item())
    rec["state_keys"] = np.array(list(model.state_dict().keys()))


def make_stack_cfg1_edge(lightning_model, adjacency):
    """L_STGCN --use_edge_importance (lightning_model.py:53-57), cfg1 shape."""
    parser = lightning_model.build_argument_parser()
    hp = parser.parse_args(["--C_in", "3", "--nr_classes", "2", "--use_edge_importance", "True",
                            "--max_mask_jitter", "0.05"])
    with _patched_adjacency(adjacency, 18):
        torch.manual_seed(0)
        model = lightning_model.L_STGCN(hp)
    model.train()
    N, T, V, C = 4, 50, 18, 3
    x = torch.randn(N, T, V, C, generator=torch.Generator().manual_seed(1))
    y = torch.randint(0, 2, (N,), generator=torch.Generator().manual_seed(2))
    logits = model(x)
    loss = torch.nn.functional.cross_entropy(logits, y)
    loss.backward()
    rec = {"x": x.numpy(), "labels": y.numpy(), "logits": logits.detach().numpy(),
           "loss": np.array(loss.item())}
    _sampled(model, rec, torch.Generator().manual_seed(4))
    np.savez_compressed(os.path.join(HERE, "stack_cfg1_edge.npz"), **rec)


def make_legacy_stgcn(stgcn):
    """The legacy STGCN class (src/network/stgcn.py:8-80: edge-importance masks
    of ones, blocks with the default dropout 0.5, softmax output) in eval mode
    (dropout off, BatchNorm on running statistics): probabilities and the
    gradients of sum(probs * g). The running statistics are calibrated first
    (one no-grad training-mode pass over the same clips with momentum 1 and
    the dropouts at p = 0, so they equal that batch's statistics): with the
    reference's un-normalised A (entries ~1e4) arbitrary running statistics
    overflow fp32 within a few blocks. They are stored in the fixture."""
    torch.manual_seed(0)
    model = stgcn.STGCN(3, 9, 5)
    N, T, V, C = 3, 30, 25, 3
    x = torch.randn(N, T, V, C, generator=torch.Generator().manual_seed(1))
    with torch.no_grad():
        for blk in model.conv:
            blk.batch_n.momentum = blk.batch_n_2.momentum = 1.0
            blk.dropout.p = 0.0
        model.train()
        model(x)
        for blk in model.conv:
            blk.batch_n.momentum = blk.batch_n_2.momentum = 0.1
            blk.dropout.p = 0.5
    model.eval()
    x.requires_grad_(True)
    probs = model(x)
    g = torch.randn(probs.shape, generator=torch.Generator().manual_seed(2))
    (probs * g).sum().backward()
    rec = {"x": x.detach().numpy(), "g": g.numpy(), "probs": probs.detach().numpy(),
           "grad.x": x.grad.numpy()}
    for name, buf in model.named_buffers():
        if "running" in name:
            rec["run." + name] = buf.numpy()
    _sampled(model, rec, torch.Generator().manual_seed(4))
    np.savez_compressed(os.path.join(HERE, "legacy_stgcn.npz"), **rec)


def make_data_pipeline(util, augmentation, calc):
    rec = {}
    rng = np.random.default_rng(7)
    # ragged batch of (1, T_i, 25, 2) clips with int labels (loopy_pad_collate_fn)
    lens = [5, 9, 3, 9, 1]
    batch = []
    for i, t in enumerate(lens):
        x = rng.standard_normal((1, t, 25, 2))
        rec[f"collate_in_{i}"] = x
        batch.append((x, np.array([i % 6])))
    xx, labels = util.loopy_pad_collate_fn(batch)
    rec["collate_out_x"] = xx.numpy()
    rec["collate_out_labels"] = labels.numpy()
    # augment_data under fixed global-RNG seeds (np.random, as the reference uses)
    seqs = rng.standard_normal((4, 20, 25, 2)) * 50 + 100
    rec["augment_in"] = seqs
    for seed in range(6):
        np.random.seed(seed)
        rec[f"augment_out_seed{seed}"] = augmentation.augment_data(seqs)
    # calculate_distances over synthetic clips (T, 25, 3): x, y, confidence
    with tempfile.TemporaryDirectory() as d:
        os.makedirs(os.path.join(d, "data"))
        names = []
        for i, t in enumerate((7, 12, 4)):
            clip = rng.standard_normal((t, 25, 3)) * 30 + 200
            np.save(os.path.join(d, "data", f"clip{i}.npy"), clip)
            rec[f"dist_clip{i}"] = clip
        names = os.listdir(os.path.join(d, "data"))
        out = os.path.join(d, "distances.npy")
        calc.calculate_distances(V=25, dataset_dir=os.path.join(d, "data"), output_file=out)
        rec["dist_out"] = np.load(out)
        rec["dist_listdir_order"] = np.array([int(n[4]) for n in names])
    np.savez_compressed(os.path.join(HERE, "data_pipeline.npz"), **rec)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("reference", nargs="?", default="/root/reference")
    ap.add_argument("--only", choices=["data", "extra"], default=None)
    args = ap.parse_args()
    _install_stubs()
    sys.path.insert(0, os.path.join(args.reference, "src"))
    import io
    import contextlib
    if args.only == "data":
        sys.path.insert(0, os.path.join(args.reference, "src", "data"))
        with contextlib.redirect_stdout(io.StringIO()):
            from data import util, augmentation, calculate_distances  # noqa: E402
        make_data_pipeline(util, augmentation, calculate_distances)
        print("wrote data_pipeline.npz to", HERE)
        return
    with contextlib.redirect_stdout(io.StringIO()):
        from data import adjacency  # noqa: E402
        from network import st_graphconv  # noqa: E402
        import lightning_model  # noqa: E402
        from network import stgcn  # noqa: E402
    torch.set_num_threads(8)
    if args.only == "extra":  # round-2 fixtures (round-1 files untouched)
        with np.load(os.path.join(HERE, "adjacency.npz")) as f:
            mats = {k: f[k] for k in f.files}
    else:
        with tempfile.TemporaryDirectory() as tmp:
            mats = make_adjacency(adjacency, tmp)
    with contextlib.redirect_stdout(io.StringIO()):
        if args.only != "extra":
            for case in BLOCK_CASES:
                make_block(st_graphconv, mats, *case)
            make_stack_cfg1(lightning_model, adjacency)
        for case in SPATIAL_CASES:
            make_spatialconv(st_graphconv, mats, *case)
        make_stack_cfg1_edge(lightning_model, adjacency)
        make_legacy_stgcn(stgcn)
    print("wrote fixtures to", HERE)


if __name__ == "__main__":
    main()

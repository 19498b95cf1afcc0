"""Host input pipeline for real skeleton data.

Mirrors of the reference's host-side data functions, bit-compatible with them
(checked against fixtures produced by the reference itself,
tests/golden/data_pipeline.npz):

  * ``pad_array_with_loops`` / ``loopy_pad_collate_fn``  src/data/util.py:12-47
  * ``augment_data``       src/data/augmentation.py:8-69 (same draws from
                           ``np.random``, in the same order)
  * ``load_clip``          the per-clip part of KTHDataset.__getitem__,
                           src/data/datasets.py:144-160 (.npy (T, 25, 3):
                           x, y, OpenPose confidence; the confidence dropped)
  * ``calculate_distances`` src/data/calculate_distances.py:7-48 (mean joint
                           distance to the per-frame centre of gravity: the
                           input of the spatial-configuration partitioning,
                           ``graph.get_normalized_adjacency_matrices(2, ...)``)

and what the reference leaves to Lightning: ``DeviceLoader`` turns collated
(N, T, V, C) float64 batches into the NCTV fp32 device layout the fused blocks
consume (the permute of lightning_model.py:101, done on the GPU), staging
through pinned host memory with the copy of batch i+1 in flight on a side
stream while batch i trains. Variable T is fine: the HIP blocks take any T.
"""
import os

import numpy as np
import torch


def pad_array_with_loops(x, target_len):
    """(N, T, V, C) -> (N, target_len, V, C) by repeating the clip from its
    start (np.pad 'wrap'); unchanged when already long enough
    (src/data/util.py:12-30)."""
    if x.shape[1] >= target_len:
        return x
    return np.pad(x, [(0, 0), (0, target_len - x.shape[1]), (0, 0), (0, 0)], mode="wrap")


def loopy_pad_collate_fn(batch):
    """[(x (1, T_i, V, C), label (1,)), ...] -> (xx (N, T*, V, C), labels (N,))
    with T* = max T_i, every clip loop-padded (src/data/util.py:33-47)."""
    max_len = max(x.shape[1] for x, _ in batch)
    xx = torch.cat([torch.from_numpy(pad_array_with_loops(x, max_len)) for x, _ in batch])
    labels = torch.cat([torch.from_numpy(np.asarray(y)) for _, y in batch])
    return xx, labels


_ROTATIONS = [15, -15, 5, -5, 10, -10]
_TRANSLATIONS = [[5, 5], [0, 5], [5, 0]]
_SCALES = [1.05, 1.1, 0.95]
_TRANSFORMS = ["rotation", "translation", "scaling", "flip"]


def augmentation_matrix(rng=np.random):
    """The random homogeneous 3x3 transform of augment_data
    (src/data/augmentation.py:15-45): two draws (with replacement) from
    {rotation, translation, scaling, flip}, then one parameter draw per chosen
    kind, composed in that fixed order. Consumes ``rng`` exactly as the
    reference consumes ``np.random``."""
    chosen = rng.choice(_TRANSFORMS, 2)
    T = np.eye(3)
    if "rotation" in chosen:
        theta = np.radians(rng.choice(_ROTATIONS))
        c, s = np.cos(theta), np.sin(theta)
        T = np.array([[c, s, 0], [-s, c, 0], [0, 0, 1]]).dot(T)
    if "translation" in chosen:
        tx, ty = _TRANSLATIONS[rng.choice(range(3))]
        T = np.array([[1, 0, tx], [0, 1, ty], [0, 0, 1]]).dot(T)
    if "scaling" in chosen:
        f = rng.choice(_SCALES)
        T = np.array([[f, 0, 0], [0, f, 0], [0, 0, 1]]).dot(T)
    if "flip" in chosen:
        T = np.array([[-1, 0, 0], [0, 1, 0], [0, 0, 1]]).dot(T)
    return T


def augment_data(sequences, rng=np.random):
    """Apply one random transform to every (T, 25, 2) sequence of
    ``sequences`` (src/data/augmentation.py:8-69): homogeneous coordinates
    [x, y, 0] (the reference fills the third coordinate with 0, not 1, so
    translations do not move the points — kept as is) times the matrix from
    the right."""
    T = augmentation_matrix(rng)
    out = []
    for seq in sequences:
        n, v, d = seq.shape
        if v != 25:
            raise ValueError("augment_data: the reference's transform is for 25 joints")
        h = np.zeros((n, v, d + 1))
        h[:, :, :2] = np.copy(seq)
        h = np.reshape(h, (n * v, d + 1)).dot(T)
        out.append(np.reshape(h, (n, v, d + 1))[:, :, :2])
    return np.asarray(out)


def load_clip(path):
    """One clip of the KTH numpy format: (T, 25, 3) [x, y, confidence] ->
    (T, 25, 2) joint coordinates (datasets.py:144-160 with
    use_confidence_scores=False, the only supported mode there)."""
    seq = np.load(path, allow_pickle=False)
    return seq[:, :, :-1]


def _joint_distances(clip, V, acc, cnt):
    for t in range(clip.shape[0]):
        x, y = clip[t, :, 0], clip[t, :, 1]
        gx, gy = np.average(x), np.average(y)
        acc += np.sqrt((gx - clip[t, :V, 0]) ** 2 + (gy - clip[t, :V, 1]) ** 2)
        cnt += 1


def joint_distances(clips, V=25):
    """Mean distance of every joint to the per-frame centre of gravity over
    all frames of ``clips`` (iterable of (T, V, >=2) arrays), accumulated in
    the reference's order (clip by clip, frame by frame)."""
    acc, cnt = np.zeros(V), np.zeros(V)
    for c in clips:
        _joint_distances(c, V, acc, cnt)
    return acc / cnt


def calculate_distances(V=25, dataset_dir="../datasets/KTH_Action_Dataset",
                        output_file="../datasets/KTH_Action_Dataset/dist/distances.npy"):
    """File-level mirror of src/data/calculate_distances.py:7-48: every .npy
    clip of ``dataset_dir`` (os.listdir order, as the reference) -> saved
    (V,) distances; also returned."""
    files = [f for f in os.listdir(dataset_dir) if f.endswith(".npy") and f != output_file]
    d = joint_distances((np.load(os.path.join(dataset_dir, f), allow_pickle=False)
                         for f in files), V)
    np.save(output_file, d)
    return d


class DeviceLoader:
    """Iterate (x_nctv fp32 on ``device``, labels int64 on ``device``) from an
    iterable of collated (x (N, T, V, C), labels (N,)) CPU batches. Each batch
    is converted to fp32 into pinned memory, copied with non_blocking=True on
    a side stream one batch ahead, and permuted NTVC -> NCTV on the device
    (lightning_model.py:101)."""

    def __init__(self, batches, device):
        self.batches = batches
        self.device = torch.device(device)
        self.stream = torch.cuda.Stream(self.device)

    def _stage(self, item):
        x, y = item
        xh = torch.as_tensor(x).to(torch.float32).pin_memory()
        yh = torch.as_tensor(y).to(torch.int64).pin_memory()
        with torch.cuda.stream(self.stream):
            xd = xh.to(self.device, non_blocking=True)
            yd = yh.to(self.device, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        return xd, yd, ev

    def __iter__(self):
        it = iter(self.batches)
        nxt = None
        try:
            nxt = self._stage(next(it))
        except StopIteration:
            return
        while nxt is not None:
            xd, yd, ev = nxt
            try:
                nxt = self._stage(next(it))
            except StopIteration:
                nxt = None
            cur = torch.cuda.current_stream(self.device)
            cur.wait_event(ev)
            xd.record_stream(cur)
            yd.record_stream(cur)
            yield xd.permute(0, 3, 1, 2).contiguous(), yd

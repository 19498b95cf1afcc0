"""Skeleton graphs and partitioned, normalized adjacency tensors.

Mirror of the reference's graph layer:
  * strategies / DFS neighbourhoods / partitioning follow
    ``src/data/adjacency.py:7-158`` (``Strategy``, ``increase_neighbourhood``,
    ``create_adjacency_matrices``);
  * ``normalize`` is bug-compatible with ``src/data/adjacency.py:161-183``:
    ``(diag(rowsum) + alpha) ** -1/2`` adds alpha to EVERY element before the
    power, so every off-diagonal entry of Lambda becomes alpha**-1/2 and the
    resulting A is dense;
  * the BODY_25 graph (V=25) is the reference's ``adj_list`` /
    ``opposite_joints`` (``src/data/util.py:131-180``).

The reference hard-codes V=25. The north-star configs also need V=18
(OpenPose-COCO / Kinetics-skeleton layout) and V=50 (two stacked BODY_25
persons, no edges between them); those are defined here, and the reference's
own functions were run on them (with its module globals patched) to produce
the golden fixtures under ``tests/golden``.

This is one-time CPU work (untimed), not part of the GPU hot path.
"""
from enum import IntEnum

import numpy as np
import torch


class Strategy(IntEnum):
    """Partitioning strategies (``src/data/adjacency.py:7-11``)."""
    UNI_LABELING = 0
    DISTANCE = 1
    SPATIAL_CONFIGURATION = 2
    SYMMETRICAL = 3


# BODY_25 adjacency list (src/data/util.py:156-180).
_BODY25_EDGES = [
    (0, 1), (0, 15), (0, 16), (1, 2), (1, 5), (1, 8), (2, 3), (3, 4), (5, 6),
    (6, 7), (8, 9), (8, 12), (9, 10), (10, 11), (11, 22), (11, 24), (12, 13),
    (13, 14), (14, 19), (14, 21), (15, 17), (16, 18), (19, 20), (22, 23),
]

# BODY_25 left/right pairs (src/data/util.py:131-152).
_BODY25_OPPOSITE = {2: 5, 3: 6, 4: 7, 5: 2, 6: 3, 7: 4, 9: 12, 10: 13,
                    11: 14, 12: 9, 13: 10, 14: 11, 15: 16, 16: 15, 17: 18,
                    18: 17, 19: 22, 20: 23, 21: 24, 22: 19, 23: 20, 24: 21}

# OpenPose COCO-18 (Kinetics-skeleton) bones, the layout ST-GCN uses for
# Kinetics. Not in the reference.
_COCO18_EDGES = [
    (4, 3), (3, 2), (7, 6), (6, 5), (13, 12), (12, 11), (10, 9), (9, 8),
    (11, 5), (8, 2), (5, 1), (2, 1), (0, 1), (15, 0), (14, 0), (17, 15),
    (16, 14),
]
_COCO18_OPPOSITE = {2: 5, 3: 6, 4: 7, 5: 2, 6: 3, 7: 4, 8: 11, 9: 12,
                    10: 13, 11: 8, 12: 9, 13: 10, 14: 15, 15: 14, 16: 17,
                    17: 16}


def _adj_from_edges(edges, num_joints):
    """Undirected adjacency list with the insertion order of ``edges``."""
    adj = {i: [] for i in range(num_joints)}
    for a, b in edges:
        adj[a].append(b)
        adj[b].append(a)
    return adj


class SkeletonGraph:
    """A joint graph: ``num_joints`` V, an adjacency list and left/right pairs."""

    def __init__(self, name, num_joints, adj_list, opposite_joints):
        self.name = name
        self.num_joints = num_joints
        self.adj_list = adj_list
        self.opposite_joints = opposite_joints


def body25():
    # Reference order of neighbours (util.py:156-180) is what the DFS sees;
    # a sorted list reproduces it exactly for BODY_25.
    adj = _adj_from_edges(_BODY25_EDGES, 25)
    adj = {k: sorted(v) for k, v in adj.items()}
    return SkeletonGraph("body25", 25, adj, dict(_BODY25_OPPOSITE))


def coco18():
    adj = _adj_from_edges(_COCO18_EDGES, 18)
    adj = {k: sorted(v) for k, v in adj.items()}
    return SkeletonGraph("coco18", 18, adj, dict(_COCO18_OPPOSITE))


def two_person_body25():
    """Two BODY_25 skeletons stacked as joints 0-24 and 25-49 (no cross edges)."""
    one = body25()
    adj = {}
    for k, v in one.adj_list.items():
        adj[k] = list(v)
        adj[k + 25] = [x + 25 for x in v]
    opp = dict(one.opposite_joints)
    opp.update({k + 25: v + 25 for k, v in one.opposite_joints.items()})
    return SkeletonGraph("body25x2", 50, adj, opp)


def graph_for(num_joints):
    """The graph this build uses for V in {18, 25, 50}."""
    if num_joints == 25:
        return body25()
    if num_joints == 18:
        return coco18()
    if num_joints == 50:
        return two_person_body25()
    raise ValueError(f"no skeleton graph defined for V={num_joints}")


def increase_neighbourhood(graph, neighbour_elements, open_elements):
    """One DFS expansion step (``src/data/adjacency.py:13-32``).

    Mutates ``neighbour_elements`` and consumes ``open_elements`` exactly as the
    reference does; returns the newly opened joints in discovery order.
    """
    new_open = []
    while open_elements:
        curr = open_elements.pop(0)
        fresh = [x for x in graph.adj_list[curr] if x not in neighbour_elements]
        neighbour_elements.extend(fresh)
        new_open.extend(fresh)
    return new_open


def create_adjacency_matrices(strat=Strategy.UNI_LABELING, d=1, distances=None,
                              graph=None):
    """Partition matrices (``src/data/adjacency.py:34-158``).

    ``distances`` replaces the reference's ``np.load(distance_file)``
    (``adjacency.py:101``) for the spatial-configuration strategy: a length-V
    array of mean distances to the centre of gravity.
    Returns a list of (V, V) float32 tensors.
    """
    graph = graph or body25()
    V = graph.num_joints
    strat = Strategy(int(strat))

    def neighbourhood(i, steps, on_step=None):
        neigh, opened = [i], [i]
        for dist in range(steps):
            opened = increase_neighbourhood(graph, neigh, opened)
            if on_step is not None:
                on_step(dist, opened)
        return neigh

    if strat == Strategy.UNI_LABELING:
        A = torch.zeros((V, V))
        for i in range(V):
            for nb in neighbourhood(i, d):
                A[i][nb] = 1
        return [A]

    if strat == Strategy.DISTANCE:
        mats = [torch.eye(V)] + [torch.zeros((V, V)) for _ in range(d)]
        for i in range(V):
            def mark(dist, opened, i=i):
                for nb in opened:
                    mats[dist + 1][i][nb] = 1
            neighbourhood(i, d, mark)
        return mats

    if strat == Strategy.SPATIAL_CONFIGURATION:
        if distances is None:
            raise ValueError("Distance file not provided")
        dist = np.asarray(distances)
        mats = [torch.zeros((V, V)) for _ in range(3)]
        for i in range(V):
            root = dist[i]
            for nb in neighbourhood(i, d):
                nd = dist[nb]
                label = 0 if nd == root else (1 if nd < root else 2)
                mats[label][i][nb] = 1
        return mats

    if strat == Strategy.SYMMETRICAL:
        opp = graph.opposite_joints
        mats = [torch.eye(V)] + [torch.zeros((V, V)) for _ in range(d)]
        for i in range(V):
            def mark(dist, opened, i=i):
                for nb in opened:
                    mats[dist + 1][i][nb] = 1
                    if nb in opp:
                        mats[dist + 1][i][opp[nb]] = 1
            neighbourhood(i, d, mark)
            # The reference uses the loop variable of the last DFS step here
            # (adjacency.py:155-156), i.e. always partition d.
            if i in opp:
                mats[d][i][opp[i]] = 1
        return mats

    raise ValueError(f"unknown strategy {strat}")


def normalize(matrices, expo=-1 / 2, alpha=0.001):
    """Bug-compatible normalisation (``src/data/adjacency.py:161-183``).

    ``Lambda = (diag(rowsum(A)) + alpha) ** expo`` with alpha added to every
    element (so off-diagonals become alpha**expo), then ``Lambda @ A @ Lambda``.
    Computed in float32 like the reference (``torch.Tensor`` default dtype).
    """
    K = len(matrices)
    V0, V1 = matrices[0].shape
    out = torch.empty(K, V0, V1, dtype=torch.float32)
    for i, A in enumerate(matrices):
        A = A.to(torch.float32)
        lam = (torch.diag(torch.sum(A, axis=1)) + alpha) ** expo
        out[i] = lam @ A @ lam
    return out


def get_normalized_adjacency_matrices(strat=Strategy.UNI_LABELING, d=1, alpha=0.001,
                                      distances=None, graph=None):
    """(K, V, V) float32 adjacency (``src/data/adjacency.py:186-200``)."""
    return normalize(create_adjacency_matrices(strat, d, distances=distances, graph=graph),
                     alpha=alpha)


def synthetic_distances(num_joints):
    """Distances used for the spatial strategy in the benchmark configs
    (``linspace(1, 2, V)``)."""
    return np.linspace(1.0, 2.0, num_joints)

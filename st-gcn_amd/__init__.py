"""stgcn_amd — MI355X-native ST-GCN block training path.

Drop-in for the reference's ``src/network`` module API
(``SpatialTemporalConv`` / ``SpatialConv``, st_graphconv.py:4-152) whose
forward/backward run on hand-written gfx950 HIP kernels behind a C-ABI
library (``include/stgcn_hip.h``). Import via ``stgcn_loader.load()``.
"""
from . import graph, hip_lib, fused, network, model, dp, train_ops, data  # noqa: F401
from .network import SpatialConv, SpatialTemporalConv  # noqa: F401
from .model import STGCN, STGCNStack, flops_per_clip  # noqa: F401
from .train_ops import FusedAdam, GraphedDPStep, GraphedStep, StgcnHeadFn  # noqa: F401

__all__ = ["graph", "hip_lib", "fused", "network", "model", "train_ops", "data", "SpatialConv",
           "SpatialTemporalConv", "STGCN", "STGCNStack", "flops_per_clip", "FusedAdam", "GraphedDPStep", "GraphedStep", "StgcnHeadFn"]

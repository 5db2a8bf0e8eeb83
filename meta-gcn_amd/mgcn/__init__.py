"""mgcn -- MI355X-native GCN message passing (the Â·X aggregation of
jzhou316/meta-gcn) behind the reference's own module surface.

    mgcn.models : gcn_meta surface (NodeModelAdditive, GCNMultiKernel,
                  GCNLayer, GCNModel, scatter_, activation)
    mgcn.pyg    : PyG-1.x surface used by kernel/ (GCNConv, GINConv, SAGEConv,
                  GraphConv, global_mean_pool, JumpingKnowledge)
    mgcn.ops    : fused aggregation autograd ops
    mgcn.graph  : device CSR plans + cache
    mgcn.dist   : destination-range sharding over torch.distributed (RCCL)

All compute goes through libmgcn.so (include/mgcn.h); there is no CPU path.
"""
import torch  # noqa: F401  -- must be imported before libmgcn binds libamdhip64

from . import _lib
from ._lib import MgcnError, check_device, load, set_option
from .graph import GraphPlan, build_plan, clear_cache, plan_for
from .ops import aggregate, scatter_, segment_mean

__version__ = "0.1.0"

__all__ = ["MgcnError", "check_device", "load", "set_option", "GraphPlan", "build_plan", "plan_for",
           "clear_cache", "aggregate", "scatter_", "segment_mean", "_lib"]

"""PyG-1.x conv surface used by the reference's kernel/ package, on mgcn.

kernel/gcn.py, gin.py, graph_sage.py, top_k*.py, sag_pool*.py, ... import
``GCNConv, GINConv, SAGEConv, GraphConv, global_mean_pool, JumpingKnowledge``
from ``torch_geometric.nn`` (kernel/gcn.py:4, gin.py:4, graph_sage.py:4,
top_k.py:4-5).  The same names, constructor arguments and forward signatures
live here; only the import line changes.

PyG is not vendored and its version is not pinned by the reference (SURVEY.md
§8(c)); the API evidence (``propagate('add', ...)``, 6-tuple TopKPooling,
``batch.__slices__``) places it at PyG 1.3.x with torch 1.2.  The semantics
below are PyG 1.3.x's, chosen and recorded in DESIGN.md:

* GCNConv   add_remaining_self_loops (fill 1, or 2 if improved); deg over
            edge_index[0]; norm = dinv[src] * w * dinv[dst]; sum; + bias.
            Identical to gcn_meta's NodeModelAdditive(deg_norm='sm') on a
            graph whose self-loops are already present (in-repo copy of this
            normalisation: src/gcn_meta/models/gcn.py:57-78).
* GINConv   remove_self_loops; nn((1 + eps) * x + sum_j x_j).
* SAGEConv  add_remaining_self_loops; mean_j (w_j x_j) then @ W, + bias,
            optional L2 normalise.
* GraphConv (sum|mean|max)_j (w_j * (x_j @ W)) + Linear(x); no self loops.
"""
from __future__ import annotations

import math
import weakref
from collections import OrderedDict

import torch
import torch.nn.functional as F
from torch import nn
from torch.nn import Parameter

from .graph import cache_key, plan_for
from .models import Linear, glorot, zeros
from .ops import aggregate_plan, gcn_layer, linear, scatter_


def uniform(size, tensor):
    """torch_geometric.nn.inits.uniform (PyG 1.3)."""
    bound = 1.0 / math.sqrt(size)
    if tensor is not None:
        tensor.data.uniform_(-bound, bound)


def reset(nn_module):
    """torch_geometric.nn.inits.reset (PyG 1.3)."""
    def _reset(item):
        if hasattr(item, 'reset_parameters'):
            item.reset_parameters()
    if nn_module is not None:
        if hasattr(nn_module, 'children') and len(list(nn_module.children())) > 0:
            for item in nn_module.children():
                _reset(item)
        else:
            _reset(nn_module)


# --------------------------------------------------- self-loop bookkeeping
_DERIVED: "OrderedDict[tuple, tuple]" = OrderedDict()


def _derived(kind: str, edge_index, edge_weight, num_nodes, fill, build):
    """Cache derived edge lists (loops added/removed) per source edge_index,
    so the graph plan cache sees the same derived tensor every call."""
    key = (kind, cache_key(edge_index, num_nodes), fill,
           None if edge_weight is None else (edge_weight.data_ptr(), edge_weight._version))
    hit = _DERIVED.get(key)
    if hit is not None:
        ref_ei, ref_ew, val = hit
        if ref_ei() is edge_index and (edge_weight is None or ref_ew() is edge_weight):
            _DERIVED.move_to_end(key)
            return val
    val = build()
    _DERIVED[key] = (weakref.ref(edge_index),
                     weakref.ref(edge_weight) if edge_weight is not None else None, val)
    while len(_DERIVED) > 16:
        _DERIVED.popitem(last=False)
    return val


def add_remaining_self_loops(edge_index, edge_weight=None, fill_value=1, num_nodes=None):
    """torch_geometric.utils.add_remaining_self_loops (PyG 1.3): drop existing
    loops, append one loop per node at the end, carrying over the weight of
    an existing loop (else ``fill_value``)."""
    N = int(num_nodes if num_nodes is not None else int(edge_index.max()) + 1)
    row, col = edge_index[0], edge_index[1]
    mask = row != col
    loop_index = torch.arange(0, N, dtype=row.dtype, device=row.device)
    loop_index = loop_index.unsqueeze(0).repeat(2, 1)
    if edge_weight is not None:
        assert edge_weight.numel() == edge_index.size(1)
        inv_mask = ~mask
        loop_weight = torch.full((N,), fill_value, dtype=edge_weight.dtype,
                                 device=edge_weight.device)
        remaining = edge_weight[inv_mask]
        if remaining.numel() > 0:
            # PyG's ``loop_weight[row[inv_mask]] = remaining`` on the CPU:
            # with several loops on one node the last one in COO order wins.
            # A device index_put picks an arbitrary one, so take the last
            # position per node explicitly.
            loops_at = row[inv_mask]
            pos = torch.arange(loops_at.numel(), device=row.device)
            last = torch.full((N,), -1, dtype=pos.dtype, device=row.device)
            last.scatter_reduce_(0, loops_at, pos, reduce='amax')
            has = last >= 0
            loop_weight[has] = remaining[last[has]]
        edge_weight = torch.cat([edge_weight[mask], loop_weight], dim=0)
    edge_index = torch.cat([edge_index[:, mask], loop_index], dim=1)
    return edge_index, edge_weight


def remove_self_loops(edge_index, edge_attr=None):
    """torch_geometric.utils.remove_self_loops (PyG 1.3)."""
    mask = edge_index[0] != edge_index[1]
    edge_index = edge_index[:, mask]
    return edge_index, (None if edge_attr is None else edge_attr[mask])


def _with_loops(edge_index, edge_weight, num_nodes, fill):
    if edge_weight is not None and edge_weight.requires_grad and torch.is_grad_enabled():
        # the weights carry this call's autograd graph: derive them afresh
        # (the loop-augmented edge list itself stays cached for the plan cache)
        ei = _derived("loops", edge_index, None, num_nodes, fill,
                      lambda: add_remaining_self_loops(edge_index, None, fill, num_nodes))[0]
        return ei, add_remaining_self_loops(edge_index, edge_weight, fill, num_nodes)[1]
    return _derived("loops", edge_index, edge_weight, num_nodes, fill,
                    lambda: add_remaining_self_loops(edge_index, edge_weight, fill, num_nodes))


def _without_loops(edge_index, num_nodes):
    return _derived("noloops", edge_index, None, num_nodes, 0,
                    lambda: remove_self_loops(edge_index)[0])


# ------------------------------------------------------------------ convs
class GCNConv(nn.Module):
    """PyG 1.3 GCNConv(in_channels, out_channels, improved=False, cached=False,
    bias=True); forward(x, edge_index, edge_weight=None)."""

    def __init__(self, in_channels, out_channels, improved=False, cached=False, bias=True,
                 **kwargs):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.improved = improved
        self.cached = cached
        self.weight = Parameter(torch.Tensor(in_channels, out_channels))
        if bias:
            self.bias = Parameter(torch.Tensor(out_channels))
        else:
            self.register_parameter('bias', None)
        self.reset_parameters()

    def reset_parameters(self):
        glorot(self.weight)
        zeros(self.bias)

    def forward(self, x, edge_index, edge_weight=None, relu=False):
        N = x.size(0)
        fill = 2 if self.improved else 1
        if edge_weight is None:
            # GCNConv.norm: unit weights first, then add_remaining_self_loops
            # (an existing loop keeps its weight 1; new loops get `fill`)
            edge_weight = _derived("ones", edge_index, None, N, 0, lambda: torch.ones(
                edge_index.size(1), dtype=x.dtype, device=edge_index.device))
        ei, ew = _with_loops(edge_index, edge_weight, N, fill)
        plan = plan_for(ei, N)
        norm = plan.norm('sm', edge_weight=ew)
        # x @ W, then propagate: one fused launch per direction where it applies
        return gcn_layer(x, self.weight, plan, norm, 'add', self.bias, relu)

    def __repr__(self):
        return '{}({}, {})'.format(self.__class__.__name__, self.in_channels, self.out_channels)


class GINConv(nn.Module):
    """PyG 1.3 GINConv(nn, eps=0, train_eps=False); forward(x, edge_index)."""

    def __init__(self, nn, eps=0, train_eps=False, **kwargs):
        super().__init__()
        self.nn = nn
        self.initial_eps = eps
        if train_eps:
            self.eps = torch.nn.Parameter(torch.Tensor([eps]))
        else:
            self.register_buffer('eps', torch.Tensor([eps]))
        self.reset_parameters()

    def reset_parameters(self):
        reset(self.nn)
        self.eps.data.fill_(self.initial_eps)

    def forward(self, x, edge_index):
        x = x.unsqueeze(-1) if x.dim() == 1 else x
        N = x.size(0)
        ei = _without_loops(edge_index, N)
        plan = plan_for(ei, N)
        agg = aggregate_plan(x, plan, plan.norm(None), 'add')
        return self.nn((1 + self.eps) * x + agg)

    def __repr__(self):
        return '{}(nn={})'.format(self.__class__.__name__, self.nn)


class SAGEConv(nn.Module):
    """PyG 1.3 SAGEConv(in_channels, out_channels, normalize=False,
    concat=False, bias=True); forward(x, edge_index, edge_weight=None)."""

    def __init__(self, in_channels, out_channels, normalize=False, concat=False, bias=True,
                 **kwargs):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.normalize = normalize
        self.concat = concat
        in_c = 2 * in_channels if concat else in_channels
        self.weight = Parameter(torch.Tensor(in_c, out_channels))
        if bias:
            self.bias = Parameter(torch.Tensor(out_channels))
        else:
            self.register_parameter('bias', None)
        self.reset_parameters()

    def reset_parameters(self):
        uniform(self.weight.size(0), self.weight)
        uniform(self.weight.size(0), self.bias)

    def forward(self, x, edge_index, edge_weight=None, size=None):
        x = x.unsqueeze(-1) if x.dim() == 1 else x
        N = x.size(0)
        ei, ew = _with_loops(edge_index, edge_weight, N, 1)
        plan = plan_for(ei, N)
        norm = plan.norm(None, edge_weight=ew)
        if self.concat:
            out = aggregate_plan(x, plan, norm, 'mean')
            out = torch.cat([x, out], dim=-1)
            out = linear(out, self.weight)
            if self.bias is not None:
                out = out + self.bias
        else:
            # mean of the neighbourhood, then @ W + b (PyG 1.3's order): one
            # fused launch where it applies, else the aggregation and the GEMM
            # in that order
            out = gcn_layer(x, self.weight, plan, norm, 'mean', self.bias, aggregate_first=True)
        if self.normalize:
            out = F.normalize(out, p=2, dim=-1)
        return out

    def __repr__(self):
        return '{}({}, {})'.format(self.__class__.__name__, self.in_channels, self.out_channels)


class GraphConv(nn.Module):
    """PyG 1.3 GraphConv(in_channels, out_channels, aggr='add', bias=True);
    forward(x, edge_index, edge_weight=None)."""

    def __init__(self, in_channels, out_channels, aggr='add', bias=True, **kwargs):
        super().__init__()
        assert aggr in ['add', 'mean', 'max']
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.aggr = aggr
        self.weight = Parameter(torch.Tensor(in_channels, out_channels))
        self.lin = Linear(in_channels, out_channels, bias=bias)  # libmgcn GEMMs, nn.Linear state_dict
        self.reset_parameters()

    def reset_parameters(self):
        uniform(self.in_channels, self.weight)
        self.lin.reset_parameters()

    def forward(self, x, edge_index, edge_weight=None, size=None):
        x = x.unsqueeze(-1) if x.dim() == 1 else x
        plan = plan_for(edge_index, x.size(0))
        norm = plan.norm(None, edge_weight=edge_weight)
        if self.aggr == 'max':
            # max does not commute with W: x @ W on the MFMA GEMM, then the max
            agg = aggregate_plan(linear(x, self.weight), plan, norm, 'max')
        else:
            agg = gcn_layer(x, self.weight, plan, norm, self.aggr)
        return agg + self.lin(x)

    def __repr__(self):
        return '{}({}, {})'.format(self.__class__.__name__, self.in_channels, self.out_channels)


# ------------------------------------------------------------------ readout
def global_add_pool(x, batch, size=None):
    size = int(batch.max().item() + 1) if size is None else size
    return scatter_('add', x, batch, dim_size=size)


def global_mean_pool(x, batch, size=None):
    """PyG global_mean_pool = scatter_mean(x, batch) (kernel/gcn.py:29)."""
    size = int(batch.max().item() + 1) if size is None else size
    return scatter_('mean', x, batch, dim_size=size)


def global_max_pool(x, batch, size=None):
    size = int(batch.max().item() + 1) if size is None else size
    return scatter_('max', x, batch, dim_size=size)


class JumpingKnowledge(torch.nn.Module):
    """PyG 1.3 JumpingKnowledge(mode, channels=None, num_layers=None)."""

    def __init__(self, mode, channels=None, num_layers=None):
        super().__init__()
        self.mode = mode.lower()
        assert self.mode in ['cat', 'max', 'lstm']
        if mode == 'lstm':
            assert channels is not None and num_layers is not None
            self.lstm = torch.nn.LSTM(channels, (num_layers * channels) // 2, bidirectional=True,
                                      batch_first=True)
            self.att = torch.nn.Linear(2 * ((num_layers * channels) // 2), 1)  # on 3-D LSTM output
        self.reset_parameters()

    def reset_parameters(self):
        if hasattr(self, 'lstm'):
            self.lstm.reset_parameters()
        if hasattr(self, 'att'):
            self.att.reset_parameters()

    def forward(self, xs):
        assert isinstance(xs, list) or isinstance(xs, tuple)
        if self.mode == 'cat':
            return torch.cat(xs, dim=-1)
        elif self.mode == 'max':
            return torch.stack(xs, dim=-1).max(dim=-1)[0]
        x = torch.stack(xs, dim=1)
        alpha, _ = self.lstm(x)
        alpha = self.att(alpha).squeeze(-1)
        alpha = torch.softmax(alpha, dim=-1)
        return (x * alpha.unsqueeze(-1)).sum(dim=1)

    def __repr__(self):
        return '{}({})'.format(self.__class__.__name__, self.mode)


__all__ = ["GCNConv", "GINConv", "SAGEConv", "GraphConv", "global_add_pool", "global_mean_pool",
           "global_max_pool", "JumpingKnowledge", "add_remaining_self_loops", "remove_self_loops"]

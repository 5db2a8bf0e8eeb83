"""Graph pooling operators of the reference's kernel/ nets, on mgcn.

The pooling nets (kernel/top_k*.py, sag_pool*.py, edge_pool.py, graclus.py,
diff_pool.py, set2set.py, sort_pool.py, global_attention.py, hard_pool.py)
import these from ``torch_geometric.nn`` (PyG 1.3.x, un-vendored; SURVEY.md
§8(f) rank 4) and HardPooling from the reference itself
(src/gcn_meta/models/hard_attention_pool.py:23-131).  Same names,
constructor arguments, forward signatures and return tuples as PyG 1.3.

Every per-node / per-edge segment reduction (softmax denominators, score
maxima, cluster pooling, attention read-outs) runs on libmgcn's segment SpMM
(:func:`mgcn.ops.scatter_`, the same kernels as the GCN aggregation), the
convolutions on mgcn's convs, the feature transforms on its GEMMs.  Index
bookkeeping (sorting scores, relabelling kept nodes, coalescing edge lists)
is torch on the same HIP device.  Two steps are sequential by definition
and run on the host as in PyG: EdgePooling's greedy edge contraction
(PyG 1.3 ``__merge_edges__`` is a Python loop over score-sorted edges) and
nothing else -- graclus's matching is a parallel handshake on the device.

Parity: HardPooling's eval-mode forward is pinned to the reference code
(tests/golden/hardpool_*.npz, made by tests/golden/make_golden.py); the PyG
operators follow PyG 1.3's published algorithms and are tested against
independent CPU restatements (parity unpinned beyond those: no fixtures of
PyG exist in the reference).
"""
from __future__ import annotations

from collections import namedtuple

import torch
import torch.nn.functional as F
from torch.nn import Parameter

from . import _lib as L
from .graph import build_view
from .models import activation, glorot, zeros
from .ops import bmm, scatter_, spmm_fwd
from .pyg import GraphConv, remove_self_loops, uniform

EPS = 1e-15


# ------------------------------------------------------------- utilities
def scatter_max_arg(src: torch.Tensor, index: torch.Tensor, dim_size: int,
                    fill_value: float | None = None):
    """torch_scatter 1.x ``scatter_max(src, index, 0, None, dim_size,
    fill_value)`` for [E] / [E, F] ``src``: (max, argmax) per row, argmax =
    the winning position in ``src`` (ties: the later one, torch_scatter's CPU
    scan), -1 and value 0 for empty rows.  With ``fill_value`` the scan starts
    from it (``src >= out``): an entry below it never wins, so a row whose
    maximum is below ``fill_value`` (or that is empty) gets argmax -1 and
    value ``fill_value`` (hard_attention_pool.py:76 passes -1e16).  No
    autograd (callers use the argmax)."""
    squeeze = src.dim() == 1
    x = (src.unsqueeze(1) if squeeze else src).detach().contiguous()
    E = x.size(0)
    ids = torch.arange(E, dtype=torch.int64, device=x.device)
    view = build_view(index, ids, int(dim_size), E)
    out, arg = spmm_fwd(view, None, x, L.REDUCE_MAX)
    arg = arg.to(torch.int64)
    if fill_value is not None:
        fill = torch.tensor(fill_value, dtype=out.dtype, device=out.device)
        lose = (arg < 0) | (out < fill)
        arg = arg.masked_fill(lose, -1)
        out = torch.where(lose, fill, out)
    return (out.squeeze(1), arg.squeeze(1)) if squeeze else (out, arg)


def softmax(src: torch.Tensor, index: torch.Tensor, num_nodes: int | None = None):
    """torch_geometric.utils.softmax (PyG 1.3; also common.py:68-90):
    exp(src - max_group) / (sum_group exp(.) + 1e-16), per group of ``index``."""
    if num_nodes is None:
        num_nodes = int(index.max().item()) + 1 if index.numel() else 0
    out = src - scatter_('max', src.detach(), index, dim_size=num_nodes)[index]
    out = out.exp()
    return out / (scatter_('add', out, index, dim_size=num_nodes)[index] + 1e-16)


def num_per_graph(batch: torch.Tensor, size: int | None = None) -> torch.Tensor:
    size = int(batch.max().item()) + 1 if size is None else size
    return torch.bincount(batch, minlength=size)


def to_dense_batch(x: torch.Tensor, batch: torch.Tensor | None = None, fill_value=0.0):
    """torch_geometric.utils.to_dense_batch (PyG 1.3): [B, N_max, *] + mask."""
    if batch is None:
        batch = x.new_zeros(x.size(0), dtype=torch.long)
    batch_size = int(batch[-1].item()) + 1 if batch.numel() else 0
    num_nodes = num_per_graph(batch, batch_size)
    cum = torch.cat([batch.new_zeros(1), num_nodes.cumsum(0)])
    max_n = int(num_nodes.max().item()) if batch_size else 0
    idx = torch.arange(batch.size(0), device=x.device)
    idx = (idx - cum[batch]) + batch * max_n
    out = x.new_full([batch_size * max_n] + list(x.size())[1:], fill_value)
    out[idx] = x
    mask = torch.zeros(batch_size * max_n, dtype=torch.bool, device=x.device)
    mask[idx] = True
    return out.view([batch_size, max_n] + list(x.size())[1:]), mask.view(batch_size, max_n)


def coalesce(edge_index: torch.Tensor, num_nodes: int) -> torch.Tensor:
    """torch_sparse.coalesce without values: sorted by (row, col), unique."""
    if edge_index.numel() == 0:
        return edge_index
    key = torch.unique(edge_index[0] * num_nodes + edge_index[1], sorted=True)
    return torch.stack([key // num_nodes, key % num_nodes], 0)


def filter_adj(edge_index, edge_attr, perm, num_nodes=None):
    """torch_geometric.nn.pool.topk_pool.filter_adj (PyG 1.3): keep edges
    whose endpoints are both in ``perm``, relabelled to positions in perm."""
    if num_nodes is None:
        num_nodes = int(edge_index.max().item()) + 1 if edge_index.numel() else 0
    mask = perm.new_full((num_nodes,), -1)
    mask[perm] = torch.arange(perm.size(0), dtype=torch.long, device=perm.device)
    row, col = mask[edge_index[0]], mask[edge_index[1]]
    keep = (row >= 0) & (col >= 0)
    row, col = row[keep], col[keep]
    if edge_attr is not None:
        edge_attr = edge_attr[keep]
    return torch.stack([row, col], dim=0), edge_attr


def topk(x: torch.Tensor, ratio: float, batch: torch.Tensor, min_score=None, tol=1e-7):
    """torch_geometric.nn.pool.topk_pool.topk (PyG 1.3): per graph, the
    ceil(ratio * n) highest scores (or those above min_score), in descending
    score order, graphs in order.  Ties keep node order (stable sort)."""
    if min_score is not None:
        scores_max = scatter_('max', x, batch)[batch] - tol
        scores_min = scores_max.clamp(max=min_score)
        return torch.nonzero(x > scores_min).view(-1)
    num_nodes = num_per_graph(batch)
    batch_size, max_n = num_nodes.size(0), int(num_nodes.max().item())
    cum = torch.cat([num_nodes.new_zeros(1), num_nodes.cumsum(0)[:-1]])
    index = torch.arange(batch.size(0), device=x.device)
    index = (index - cum[batch]) + batch * max_n
    dense = x.new_full((batch_size * max_n,), torch.finfo(x.dtype).min)
    dense[index] = x
    _, perm = dense.view(batch_size, max_n).sort(dim=-1, descending=True, stable=True)
    perm = (perm + cum.view(-1, 1)).view(-1)
    k = (ratio * num_nodes.to(torch.float)).ceil().to(torch.long)
    keep = torch.arange(max_n, device=x.device).view(1, -1) < k.view(-1, 1)
    return perm[keep.view(-1)]


# ---------------------------------------------------------- TopK / SAG
class TopKPooling(torch.nn.Module):
    """PyG 1.3 TopKPooling(in_channels, ratio=0.5, min_score=None,
    multiplier=1, nonlinearity=torch.tanh); forward returns
    (x, edge_index, edge_attr, batch, perm, score[perm])."""

    def __init__(self, in_channels, ratio=0.5, min_score=None, multiplier=1,
                 nonlinearity=torch.tanh):
        super().__init__()
        self.in_channels = in_channels
        self.ratio = ratio
        self.min_score = min_score
        self.multiplier = multiplier
        self.nonlinearity = nonlinearity
        self.weight = Parameter(torch.Tensor(1, in_channels))
        self.reset_parameters()

    def reset_parameters(self):
        uniform(self.in_channels, self.weight)

    def forward(self, x, edge_index, edge_attr=None, batch=None, attn=None):
        if batch is None:
            batch = edge_index.new_zeros(x.size(0))
        attn = x if attn is None else attn
        attn = attn.unsqueeze(-1) if attn.dim() == 1 else attn
        score = (attn * self.weight).sum(dim=-1)
        if self.min_score is None:
            score = self.nonlinearity(score / self.weight.norm(p=2, dim=-1))
        else:
            score = softmax(score, batch)
        return _select(x, edge_index, edge_attr, batch, score, self.ratio, self.min_score,
                       self.multiplier)

    def __repr__(self):
        return '{}({}, {}={}, multiplier={})'.format(
            self.__class__.__name__, self.in_channels,
            'ratio' if self.min_score is None else 'min_score',
            self.ratio if self.min_score is None else self.min_score, self.multiplier)


def _select(x, edge_index, edge_attr, batch, score, ratio, min_score, multiplier):
    perm = topk(score, ratio, batch, min_score)
    x = x[perm] * score[perm].view(-1, 1)
    x = multiplier * x if multiplier != 1 else x
    batch = batch[perm]
    edge_index, edge_attr = filter_adj(edge_index, edge_attr, perm, num_nodes=score.size(0))
    return x, edge_index, edge_attr, batch, perm, score[perm]


class SAGPooling(torch.nn.Module):
    """PyG 1.3 SAGPooling(in_channels, ratio=0.5, GNN=GraphConv,
    min_score=None, multiplier=1, nonlinearity=torch.tanh): the score is a
    one-channel GNN (on mgcn's SpMM) of the node features."""

    def __init__(self, in_channels, ratio=0.5, GNN=GraphConv, min_score=None, multiplier=1,
                 nonlinearity=torch.tanh, **kwargs):
        super().__init__()
        self.in_channels = in_channels
        self.ratio = ratio
        self.gnn = GNN(in_channels, 1, **kwargs)
        self.min_score = min_score
        self.multiplier = multiplier
        self.nonlinearity = nonlinearity
        self.reset_parameters()

    def reset_parameters(self):
        self.gnn.reset_parameters()

    def forward(self, x, edge_index, edge_attr=None, batch=None, attn=None):
        if batch is None:
            batch = edge_index.new_zeros(x.size(0))
        attn = x if attn is None else attn
        attn = attn.unsqueeze(-1) if attn.dim() == 1 else attn
        score = self.gnn(attn, edge_index).view(-1)
        if self.min_score is None:
            score = self.nonlinearity(score)
        else:
            score = softmax(score, batch)
        return _select(x, edge_index, edge_attr, batch, score, self.ratio, self.min_score,
                       self.multiplier)

    def __repr__(self):
        return '{}({}, {}, {}={}, multiplier={})'.format(
            self.__class__.__name__, self.gnn.__class__.__name__, self.in_channels,
            'ratio' if self.min_score is None else 'min_score',
            self.ratio if self.min_score is None else self.min_score, self.multiplier)


# ------------------------------------------------------------ EdgePooling
UnpoolDescription = namedtuple("UnpoolDescription",
                               ["edge_index", "cluster", "batch", "new_edge_score"])


def edge_merge_greedy(edge_index: torch.Tensor, order: torch.Tensor, num_nodes: int):
    """PyG 1.3 EdgePooling.__merge_edges__ matching on the device
    (``mgcn_edge_merge_greedy``): PyG walks the edges by descending score and
    contracts an edge when both endpoints are still free, the free nodes left
    over becoming singleton clusters in ascending node order; the same
    matching and numbering is built here as the locally-dominant matching in
    rounds.  Returns (cluster [N] int64, chosen edge ids int64, number of
    clusters); one host sync for the two counts."""
    lib = L.load()
    dev = L.require_device(edge_index, order)
    ei = edge_index.to(torch.int64).contiguous()
    order = order.to(torch.int64).contiguous()
    E = ei.size(1)
    N = int(num_nodes)
    if order.numel() != E:
        raise ValueError(f"edge_merge_greedy: order has {order.numel()} entries for {E} edges")
    cluster = torch.empty(N, dtype=torch.int64, device=dev)
    chosen = torch.empty(max(E, 1), dtype=torch.int64, device=dev)
    counts = torch.empty(2, dtype=torch.int64, device=dev)
    ws_bytes = int(lib.mgcn_edge_merge_workspace_bytes(N, E))
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    with L.device_guard(dev):
        rc = lib.mgcn_edge_merge_greedy(N, E, L.ptr(ei[0]), L.ptr(ei[1]), L.ptr(order),
                                        L.ptr(ws), ws_bytes, L.ptr(cluster), L.ptr(chosen),
                                        L.ptr(counts), L.stream_of(dev))
    L.check(rc, "mgcn_edge_merge_greedy")
    n_chosen, C = (int(v) for v in counts.tolist())
    if n_chosen < 0:
        raise IndexError(f"edge_merge_greedy: edge_index outside [0, {N}) or order not a "
                         f"permutation of [0, {E})")
    return cluster, chosen[:n_chosen], C


class EdgePooling(torch.nn.Module):
    """PyG 1.3 EdgePooling(in_channels, edge_score_method=None, dropout=0,
    add_to_edge_score=0.5); forward(x, edge_index, batch) returns
    (x, edge_index, batch, unpool_info) -- FOUR values (kernel/edge_pool.py:40
    unpacks six, which fails against PyG; the net here unpacks four)."""

    def __init__(self, in_channels, edge_score_method=None, dropout=0, add_to_edge_score=0.5):
        super().__init__()
        self.in_channels = in_channels
        if edge_score_method is None:
            edge_score_method = self.compute_edge_score_softmax
        self.compute_edge_score = edge_score_method
        self.add_to_edge_score = add_to_edge_score
        self.dropout = dropout
        from .models import Linear
        self.lin = Linear(2 * in_channels, 1)
        self.reset_parameters()

    def reset_parameters(self):
        self.lin.reset_parameters()

    @staticmethod
    def compute_edge_score_softmax(raw_edge_score, edge_index, num_nodes):
        return softmax(raw_edge_score, edge_index[1], num_nodes)

    @staticmethod
    def compute_edge_score_tanh(raw_edge_score, edge_index, num_nodes):
        return torch.tanh(raw_edge_score)

    @staticmethod
    def compute_edge_score_sigmoid(raw_edge_score, edge_index, num_nodes):
        return torch.sigmoid(raw_edge_score)

    def forward(self, x, edge_index, batch):
        e = torch.cat([x[edge_index[0]], x[edge_index[1]]], dim=-1)
        e = self.lin(e).view(-1)
        e = F.dropout(e, p=self.dropout, training=self.training)
        e = self.compute_edge_score(e, edge_index, x.size(0))
        e = e + self.add_to_edge_score
        return self.merge_edges(x, edge_index, batch, e)

    def merge_edges(self, x, edge_index, batch, edge_score):
        N = x.size(0)
        order = torch.argsort(edge_score.detach(), descending=True, stable=True)
        cluster, chosen, C = edge_merge_greedy(edge_index, order, N)
        new_x = scatter_('add', x, cluster, dim_size=C)
        new_edge_score = edge_score[chosen]
        if C > chosen.numel():
            new_edge_score = torch.cat([new_edge_score,
                                        x.new_ones(C - chosen.numel())])
        new_x = new_x * new_edge_score.view(-1, 1)
        new_edge_index = coalesce(cluster[edge_index], C)
        new_batch = x.new_empty(C, dtype=torch.long).scatter_(0, cluster, batch)
        info = UnpoolDescription(edge_index=edge_index, cluster=cluster, batch=batch,
                                 new_edge_score=new_edge_score)
        return new_x, new_edge_index, new_batch, info

    def unpool(self, x, unpool_info):
        new_x = x / unpool_info.new_edge_score.view(-1, 1)
        new_x = new_x[unpool_info.cluster]
        return new_x, unpool_info.edge_index, unpool_info.batch

    def __repr__(self):
        return '{}({})'.format(self.__class__.__name__, self.in_channels)


# ---------------------------------------------------------------- graclus
def graclus(edge_index, weight=None, num_nodes=None, max_rounds=64):
    """torch_cluster.graclus (PyG 1.3's ``graclus``): a greedy matching of
    each node with one unmatched neighbour, preferring heavier edges; cluster
    id = the smaller node id of the pair, unmatched nodes keep their own id.
    Run as a parallel handshake on the device: every free node proposes to
    its best free neighbour (edge weight, then a random per-round priority
    of the pair), mutual proposals are matched, until no free node has a
    free neighbour.  torch_cluster visits nodes in a random order too, so
    the matching is random either way (parity unpinned; tests check that
    it is a valid maximal matching)."""
    N = int(num_nodes if num_nodes is not None else int(edge_index.max()) + 1)
    dev = edge_index.device
    row, col = edge_index[0], edge_index[1]
    keep = row != col
    row, col = row[keep], col[keep]
    w = (weight[keep] if weight is not None else torch.ones(row.numel(), device=dev)).float()
    cluster = torch.full((N,), -1, dtype=torch.long, device=dev)
    for _ in range(max_rounds):
        free = cluster < 0
        ok = free[row] & free[col]
        if not bool(ok.any()):
            break
        r, c, ww = row[ok], col[ok], w[ok]
        prio = torch.rand(N, device=dev)
        key = ww * 4.0 + prio[r] + prio[c]  # symmetric: the global best edge is mutual
        order = torch.argsort(key, descending=True, stable=True)
        order = order[torch.argsort(r[order], stable=True)]  # by row, best first
        rs, cs = r[order], c[order]
        first = torch.ones_like(rs, dtype=torch.bool)
        first[1:] = rs[1:] != rs[:-1]
        prop = torch.full((N,), -1, dtype=torch.long, device=dev)
        prop[rs[first]] = cs[first]
        u = torch.nonzero(prop >= 0).view(-1)
        v = prop[u]
        mutual = prop[v] == u
        u, v = u[mutual], v[mutual]
        m = torch.minimum(u, v)
        cluster[u] = m
        cluster[v] = m
    free = cluster < 0
    cluster[free] = torch.arange(N, device=dev)[free]
    return cluster


def consecutive_cluster(src):
    """PyG 1.3 pool.consecutive.consecutive_cluster: relabel to 0..C-1 (in
    sorted id order) and, per cluster, one member (the last one)."""
    unique, inv = torch.unique(src, sorted=True, return_inverse=True)
    pos = torch.arange(inv.size(0), device=inv.device)
    perm = torch.full((unique.size(0),), -1, dtype=torch.long, device=inv.device)
    perm.scatter_reduce_(0, inv, pos, reduce="amax")  # deterministic "last member"
    return inv, perm


def pool_edge(cluster, edge_index, edge_attr=None):
    num_nodes = cluster.size(0)
    edge_index = cluster[edge_index.view(-1)].view(2, -1)
    edge_index, edge_attr = remove_self_loops(edge_index, edge_attr)
    if edge_index.numel() > 0:
        if edge_attr is not None:
            raise NotImplementedError("pool_edge with edge_attr (unused by the kernel/ nets)")
        edge_index = coalesce(edge_index, num_nodes)
    return edge_index, edge_attr


def max_pool_x(cluster, x, batch, size=None):
    """PyG 1.3 max_pool_x: cluster-wise max (empty -> 0) and the pooled batch."""
    cluster, perm = consecutive_cluster(cluster)
    x = scatter_('max', x, cluster, dim_size=int(perm.numel()))
    return x, batch[perm]


def max_pool(cluster, data, transform=None):
    """PyG 1.3 max_pool(cluster, data): pooled x (cluster-wise max), edges
    (relabelled, loops removed, coalesced) and batch, as a new Batch."""
    cluster, perm = consecutive_cluster(cluster)
    x = scatter_('max', data.x, cluster, dim_size=int(perm.numel()))
    index, attr = pool_edge(cluster, data.edge_index, getattr(data, "edge_attr", None))
    batch = None if data.batch is None else data.batch[perm]
    out = type(data)(x=x, edge_index=index, batch=batch)
    return transform(out) if transform is not None else out


# ------------------------------------------------------------- read-outs
def global_sort_pool(x, batch, k):
    """PyG 1.3 global_sort_pool: per graph, nodes sorted by their last
    feature (descending), the first k (padded), flattened to [B, k * D]."""
    fill_value = x.min().item() - 1
    batch_x, _ = to_dense_batch(x, batch, fill_value)
    B, N, D = batch_x.size()
    _, perm = batch_x[:, :, -1].sort(dim=-1, descending=True, stable=True)
    perm = perm + (torch.arange(B, device=perm.device) * N).view(-1, 1)
    batch_x = batch_x.view(B * N, D)[perm].view(B, N, D)
    if N >= k:
        batch_x = batch_x[:, :k].contiguous()
    else:
        batch_x = torch.cat([batch_x, batch_x.new_full((B, k - N, D), fill_value)], dim=1)
    batch_x = torch.where(batch_x == fill_value, torch.zeros_like(batch_x), batch_x)
    return batch_x.view(B, k * D)


class GlobalAttention(torch.nn.Module):
    """PyG 1.3 GlobalAttention(gate_nn, nn=None): softmax-gated sum per graph."""

    def __init__(self, gate_nn, nn=None):
        super().__init__()
        self.gate_nn = gate_nn
        self.nn = nn
        self.reset_parameters()

    def reset_parameters(self):
        from .pyg import reset
        reset(self.gate_nn)
        reset(self.nn)

    def forward(self, x, batch, size=None):
        x = x.unsqueeze(-1) if x.dim() == 1 else x
        size = int(batch[-1].item()) + 1 if size is None else size
        gate = self.gate_nn(x).view(-1, 1)
        x = self.nn(x) if self.nn is not None else x
        assert gate.dim() == x.dim() and gate.size(0) == x.size(0)
        gate = softmax(gate, batch, size)
        return scatter_('add', gate * x, batch, dim_size=size)

    def __repr__(self):
        return '{}(gate_nn={}, nn={})'.format(self.__class__.__name__, self.gate_nn, self.nn)


class Set2Set(torch.nn.Module):
    """PyG 1.3 Set2Set(in_channels, processing_steps, num_layers=1): LSTM
    query, softmax attention per graph, read-out [q, r] of width 2C."""

    def __init__(self, in_channels, processing_steps, num_layers=1):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = 2 * in_channels
        self.processing_steps = processing_steps
        self.num_layers = num_layers
        self.lstm = torch.nn.LSTM(self.out_channels, self.in_channels, num_layers)
        self.reset_parameters()

    def reset_parameters(self):
        self.lstm.reset_parameters()

    def forward(self, x, batch):
        batch_size = int(batch.max().item()) + 1
        h = (x.new_zeros((self.num_layers, batch_size, self.in_channels)),
             x.new_zeros((self.num_layers, batch_size, self.in_channels)))
        q_star = x.new_zeros(batch_size, self.out_channels)
        for _ in range(self.processing_steps):
            q, h = self.lstm(q_star.unsqueeze(0), h)
            q = q.view(batch_size, self.in_channels)
            e = (x * q[batch]).sum(dim=-1, keepdim=True)
            a = softmax(e, batch, num_nodes=batch_size)
            r = scatter_('add', a * x, batch, dim_size=batch_size)
            q_star = torch.cat([q, r], dim=-1)
        return q_star

    def __repr__(self):
        return '{}({}, {})'.format(self.__class__.__name__, self.in_channels, self.out_channels)


# ----------------------------------------------------------------- dense
class DenseSAGEConv(torch.nn.Module):
    """PyG 1.3 DenseSAGEConv(in_channels, out_channels, normalize=False,
    bias=True); forward(x [B,N,C], adj [B,N,N], mask=None, add_loop=True)."""

    def __init__(self, in_channels, out_channels, normalize=False, bias=True):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.normalize = normalize
        self.weight = Parameter(torch.Tensor(in_channels, out_channels))
        self.bias = Parameter(torch.Tensor(out_channels)) if bias else None
        if not bias:
            self.register_parameter('bias', None)
        self.reset_parameters()

    def reset_parameters(self):
        uniform(self.in_channels, self.weight)
        uniform(self.in_channels, self.bias)

    def forward(self, x, adj, mask=None, add_loop=True):
        x = x.unsqueeze(0) if x.dim() == 2 else x
        adj = adj.unsqueeze(0) if adj.dim() == 2 else adj
        B, N, _ = adj.size()
        if add_loop:
            adj = adj.clone()
            idx = torch.arange(N, dtype=torch.long, device=adj.device)
            adj[:, idx, idx] = 1
        out = bmm(adj, x)
        out = out / adj.sum(dim=-1, keepdim=True).clamp(min=1)
        out = bmm(out, self.weight)
        if self.bias is not None:
            out = out + self.bias
        if self.normalize:
            out = F.normalize(out, p=2, dim=-1)
        if mask is not None:
            out = out * mask.view(B, N, 1).to(x.dtype)
        return out

    def __repr__(self):
        return '{}({}, {})'.format(self.__class__.__name__, self.in_channels, self.out_channels)


def dense_diff_pool(x, adj, s, mask=None):
    """PyG 1.3 dense_diff_pool: (S^T X, S^T A S, link loss, entropy loss)
    with S = softmax(s) over clusters."""
    x = x.unsqueeze(0) if x.dim() == 2 else x
    adj = adj.unsqueeze(0) if adj.dim() == 2 else adj
    s = s.unsqueeze(0) if s.dim() == 2 else s
    batch_size, num_nodes, _ = x.size()
    s = torch.softmax(s, dim=-1)
    if mask is not None:
        mask = mask.view(batch_size, num_nodes, 1).to(x.dtype)
        x, s = x * mask, s * mask
    st = s.transpose(1, 2)  # (a strided view: the kernel reads it in place)
    out = bmm(st, x)
    out_adj = bmm(bmm(st, adj), s)
    link_loss = adj - bmm(s, st)
    link_loss = torch.norm(link_loss, p=2) / adj.numel()
    ent_loss = (-s * torch.log(s + EPS)).sum(dim=-1).mean()
    return out, out_adj, link_loss, ent_loss


# ------------------------------------------------------------ HardPooling
def gumbel_samples(base: torch.Tensor) -> torch.Tensor:
    """hard_attention_pool.py:12-20: iid Gumbel(0, 1) noise shaped like base."""
    noise = torch.rand(base.size(), device=base.device, dtype=base.dtype)
    eps = 1e-20
    return -torch.log(-torch.log(noise + eps) + eps)


class HardPooling(torch.nn.Module):
    """src/gcn_meta/models/hard_attention_pool.py:23-131 (the reference's own
    module; kernel/hard_pool.py uses it as SAGPooling).

    Edge attention a_e = act(<[x_src, x_dst], att_weight>).  Training: Gumbel
    noise, /temperature, softmax over each SOURCE node's out-edges, dropout;
    the graph is kept (perm = all nodes).  Eval: per source node the single
    best out-edge (argmax; +Gumbel noise when ``sample``) gets weight 1, the
    rest 0; messages x_src * a_e are aggregated at the targets; the nodes
    that received a selected edge are kept and the edge list filtered.
    Returns (x, edge_index, edge_attr, batch, perm, score) like TopKPooling.

    Mirrors one reference quirk: a node with no out-edge has argmax -1 in
    torch_scatter 1.x, and ``alpha_1hot[argmax + ...] = 1`` then marks the
    LAST edge (index -1) -- kept, so outputs match the reference."""

    def __init__(self, in_channels, att_act='none', att_dropout=0.0, aggr='add', bias=False,
                 temperature=0.1, sample=False, **kwargs):
        super().__init__()
        self.in_channels = in_channels
        self.aggr = aggr
        self.temperature = temperature
        self.sample = sample
        self.att_weight = Parameter(torch.Tensor(1, 2 * in_channels))
        self.att_act = activation(att_act)
        self.att_dropout = torch.nn.Dropout(p=att_dropout)
        if bias:
            self.bias = Parameter(torch.Tensor(in_channels))
        else:
            self.register_parameter('bias', None)
        self.reset_parameters()

    def reset_parameters(self):
        glorot(self.att_weight)
        zeros(self.bias)

    def forward(self, x, edge_index, batch, edge_attr=None, attn_store=None):
        N = x.size(0)
        x_j = x[edge_index[0]]
        x_i = x[edge_index[1]]
        alpha = self.att_act((torch.cat([x_j, x_i], dim=-1) * self.att_weight)
                             .sum(dim=-1, keepdim=True))
        if self.training:
            alpha = (alpha + gumbel_samples(alpha)) / self.temperature
            alpha = softmax(alpha, edge_index[0], num_nodes=N)
            alpha = self.att_dropout(alpha)
        else:
            if self.sample:
                alpha = alpha + gumbel_samples(alpha)
            # torch_scatter.scatter_max(..., fill_value=-1e16) (:76): a node
            # whose out-edge scores are all below -1e16 has no winner (-1)
            _, argmax = scatter_max_arg(alpha, edge_index[0], N, fill_value=-1e16)  # [N, 1]
            E = alpha.size(0)
            hot = torch.zeros(E, device=alpha.device, dtype=alpha.dtype)
            hot[argmax.view(-1) % max(E, 1)] = 1.0  # -1 (no out-edge) -> last edge
            alpha = hot.view(-1, 1)
        x_j = x_j * alpha.view(-1, 1)
        x = scatter_(self.aggr, x_j, edge_index[1], dim_size=N)
        if self.bias is not None:
            x = x + self.bias
        if attn_store is not None:
            attn_store.append(alpha)
        score = x.new_zeros(x.shape[0])
        if self.training:
            perm = torch.arange(x.size(0), device=x.device)
        else:
            edge_select = (alpha > 0).view(-1)
            perm = edge_index[1, edge_select].unique()
            x = x[perm]
            batch = batch[perm]
            edge_index, edge_attr = filter_adj(edge_index, edge_attr, perm,
                                               num_nodes=score.size(0))
        return x, edge_index, edge_attr, batch, perm, score


__all__ = ["TopKPooling", "SAGPooling", "EdgePooling", "HardPooling", "GlobalAttention",
           "Set2Set", "DenseSAGEConv", "dense_diff_pool", "global_sort_pool", "graclus",
           "max_pool", "max_pool_x", "softmax", "topk", "filter_adj", "to_dense_batch",
           "consecutive_cluster", "pool_edge", "scatter_max_arg", "coalesce",
           "edge_merge_greedy"]

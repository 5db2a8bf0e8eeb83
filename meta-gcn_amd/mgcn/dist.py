"""Destination-range sharding of the GCN aggregation over torch.distributed.

The reference is single-device; north_star asks for the
edge list to be sharded by destination-node range across the GPUs of a node
with an RCCL exchange of node embeddings over xGMI.  Design:

* nodes are split into P contiguous ranges balanced on (in-edges + rows);
  rank k owns rows [lo_k, hi_k) of X, of every layer's output and of dX;
* forward, per layer:  H_k = X_k W  ->  all_gather(H_k)  ->  local SpMM over
  the rank's destination rows (every in-edge of a destination is local, in COO
  order, so the forward stays bit-identical to one device);
* backward, per layer: dY_k (ReLU mask, bias partial) -> all_gather(dY_k) ->
  local adjoint SpMM over the rank's SOURCE rows (the src-grouped view restricted
  to [lo_k, hi_k), all of their out-edges, in COO order) -> dH_k, again
  bit-identical to one device.  Gathering dY (instead of reduce-scattering
  partial dH, the "all-reduce of partial embeddings" form) moves the same bytes
  and keeps the per-edge summation order;
* replicated parameters: one bucketed all_reduce of every weight/bias gradient
  per step (the DP part of the step).

All-gathers use a padded layout [P * max_rows, F]; CSR column indices are
remapped once to those padded positions so the SpMM reads the gathered buffer
in place (no unpack copy).  One all_gather of 4 N F (P-1)/P bytes per rank
per layer per direction; on MI355X's point-to-point xGMI each peer slice has
its own link (~153 GB/s), SURVEY.md §8(e) gives the arithmetic.

The local compute goes through a backend object (default :class:`HipBackend`,
i.e. libmgcn); tests substitute a CPU double to exercise the partitioning and
collective logic under the gloo backend.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.distributed as dist

from . import _lib as L
from .graph import CSRView


class HipBackend:
    """Local compute on libmgcn (the only production backend)."""

    def build_plan(self, edge_index, num_nodes):
        from .graph import build_plan
        return build_plan(edge_index, num_nodes)

    def norm(self, plan, method, deg=None, edge_weight=None):
        return plan.norm(method, deg=deg, edge_weight=edge_weight)

    def finalize_view(self, view):
        from .graph import schedule_rows
        return schedule_rows(view)

    def spmm_fwd(self, *a, **k):
        from .ops import spmm_fwd
        return spmm_fwd(*a, **k)

    def spmm_bwd(self, *a, **k):
        from .ops import spmm_bwd
        return spmm_bwd(*a, **k)

    def relu_bwd_colsum(self, *a, **k):
        from .ops import relu_bwd_colsum
        return relu_bwd_colsum(*a, **k)

    def linear(self, x, W):
        from .ops import linear
        return linear(x, W)


def partition_nodes(rowptr: torch.Tensor, parts: int) -> list[int]:
    """Contiguous node ranges with ~equal (in-edges + rows) per part."""
    rp = rowptr.to("cpu", torch.int64)
    n = rp.numel() - 1
    cost = rp + torch.arange(n + 1, dtype=torch.int64)  # cumulative cost up to row i
    total = int(cost[-1])
    bounds = [0]
    for k in range(1, parts):
        target = total * k // parts
        b = int(torch.searchsorted(cost, torch.tensor(target), right=False))
        bounds.append(max(bounds[-1], min(b, n)))
    bounds.append(n)
    return bounds


@dataclass
class Shard:
    rank: int
    world: int
    bounds: list
    lo: int
    hi: int
    max_rows: int
    fwd: CSRView        # rows = my destinations, col = padded source positions
    bwd: CSRView        # rows = my sources, col = padded destination positions
    w_fwd: torch.Tensor | None
    w_bwd: torch.Tensor | None
    row_scale: torch.Tensor | None
    cnt_pad: torch.Tensor  # max(in-degree, 1) at padded positions (MEAN adjoint)

    @property
    def rows(self) -> int:
        return self.hi - self.lo


def _remap(col: torch.Tensor, bounds: list, max_rows: int) -> torch.Tensor:
    """Global node id -> row of the padded all-gather buffer."""
    b = torch.tensor(bounds, dtype=torch.int64, device=col.device)
    c = col.to(torch.int64)
    owner = torch.bucketize(c, b[1:], right=True)
    return (c + owner * max_rows - b[owner]).to(torch.int32)


def _slice_view(view: CSRView, lo: int, hi: int, bounds, max_rows, world):
    rp = view.rowptr[lo:hi + 1]
    beg = int(rp[0]) if hi >= lo else 0
    end = int(rp[-1])
    return CSRView(rowptr=(rp - beg).contiguous(),
                   col=_remap(view.col[beg:end], bounds, max_rows).contiguous(),
                   eid=view.eid[beg:end].contiguous(), n_rows=hi - lo,
                   n_cols=world * max_rows), beg, end


def build_shard(edge_index: torch.Tensor, num_nodes: int, deg_norm="sm", deg=None,
                edge_weight=None, group=None, backend=None, device=None) -> Shard:
    """Every rank builds the global CSR views on its own device (one-time),
    then keeps its slice.  ``edge_index`` is the full graph on every rank."""
    backend = backend or HipBackend()
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    if device is not None:
        edge_index = edge_index.to(device)
    plan = backend.build_plan(edge_index, num_nodes)
    norm = backend.norm(plan, deg_norm, deg, edge_weight)
    bounds = partition_nodes(plan.fwd.rowptr, world)
    max_rows = max(bounds[k + 1] - bounds[k] for k in range(world)) if world else 0
    max_rows = max(max_rows, 1)
    lo, hi = bounds[rank], bounds[rank + 1]
    fwd, fb, fe = _slice_view(plan.fwd, lo, hi, bounds, max_rows, world)
    bwd, bb, be = _slice_view(plan.bwd, lo, hi, bounds, max_rows, world)
    fwd, bwd = backend.finalize_view(fwd), backend.finalize_view(bwd)
    w_fwd = None if norm.w_fwd is None else norm.w_fwd[fb:fe].contiguous()
    w_bwd = None if norm.w_bwd is None else norm.w_bwd[bb:be].contiguous()
    row_scale = None if norm.row_scale_bwd is None else norm.row_scale_bwd[lo:hi].contiguous()
    cnt_pad = torch.ones(world * max_rows, dtype=torch.float32, device=plan.in_cnt.device)
    for k in range(world):
        a, b = bounds[k], bounds[k + 1]
        cnt_pad[k * max_rows:k * max_rows + (b - a)] = plan.in_cnt[a:b]
    return Shard(rank, world, bounds, lo, hi, max_rows, fwd, bwd, w_fwd, w_bwd, row_scale,
                 cnt_pad)


def _all_gather_rows(local: torch.Tensor, shard: Shard, group=None) -> torch.Tensor:
    """[rows, F] per rank -> padded [world * max_rows, F] on every rank."""
    F = local.size(1)
    buf = torch.empty(shard.max_rows, F, dtype=local.dtype, device=local.device)
    buf[:local.size(0)].copy_(local)
    if shard.max_rows > local.size(0):
        buf[local.size(0):].zero_()
    out = torch.empty(shard.world * shard.max_rows, F, dtype=local.dtype, device=local.device)
    if shard.world == 1:
        out.copy_(buf)
    elif dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, buf, group=group)
    else:
        dist.all_gather(list(out.chunk(shard.world)), buf, group=group)
    return out


class _ShardedAggregate(torch.autograd.Function):
    @staticmethod
    def forward(ctx, H_local, bias, shard: Shard, reduce: int, relu: bool, backend, group):
        Hpad = _all_gather_rows(H_local.contiguous(), shard, group)
        Y, argmax = backend.spmm_fwd(shard.fwd, shard.w_fwd, Hpad, reduce, bias, relu)
        ctx.shard, ctx.reduce, ctx.relu, ctx.backend, ctx.group = shard, reduce, relu, backend, group
        ctx.has_bias = bias is not None
        ctx.save_for_backward(Y if relu else None, argmax)
        return Y

    @staticmethod
    def backward(ctx, dZ):
        Y, argmax = ctx.saved_tensors
        sh, be = ctx.shard, ctx.backend
        need_b = ctx.has_bias and ctx.needs_input_grad[1]
        dY, db = be.relu_bwd_colsum(dZ.contiguous(), Y, ctx.relu, need_b)
        dYpad = _all_gather_rows(dY, sh, ctx.group)
        argpad = None
        if ctx.reduce == L.REDUCE_MAX:
            argpad = _all_gather_rows(argmax, sh, ctx.group)
        dH = be.spmm_bwd(sh.bwd, sh.w_bwd, sh.row_scale, dYpad, ctx.reduce,
                         cnt=sh.cnt_pad if ctx.reduce == L.REDUCE_MEAN else None, argmax=argpad)
        return dH, db, None, None, None, None, None


def sharded_aggregate(H_local, shard: Shard, aggr="add", bias=None, relu=False, backend=None,
                      group=None):
    """Aggregation of the rank's destination rows; H_local = this rank's rows."""
    return _ShardedAggregate.apply(H_local, bias, shard, L.REDUCE_CODES[aggr], bool(relu),
                                   backend or HipBackend(), group)


def allreduce_grads(params, group=None) -> None:
    """One bucketed all_reduce (sum) of the replicated parameters' gradients."""
    grads = [p.grad for p in params if p.grad is not None]
    if not grads or not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    flat = torch.cat([g.reshape(-1) for g in grads])
    dist.all_reduce(flat, group=group)
    off = 0
    for g in grads:
        n = g.numel()
        g.copy_(flat[off:off + n].view_as(g))
        off += n


class ShardedGCN:
    """Stack of GCN layers (NodeModelAdditive 'sm'/'add' + bias, ReLU between
    layers) over a destination-range sharded graph; the bench's N > 1 model."""

    def __init__(self, edge_index, num_nodes, Ws, bs, device, deg_norm="sm", aggr="add",
                 group=None, backend=None):
        self.backend = backend or HipBackend()
        self.group = group
        self.device = device
        self.shard = build_shard(edge_index, num_nodes, deg_norm, group=group,
                                 backend=self.backend, device=device)
        self.aggr = aggr
        self.W = [w.to(device).clone().requires_grad_(True) for w in Ws]
        self.b = [b.to(device).clone().requires_grad_(True) for b in bs]

    def params(self):
        return self.W + self.b

    def local_rows(self, full: torch.Tensor) -> torch.Tensor:
        return full[self.shard.lo:self.shard.hi].to(self.device)

    def forward(self, X_local):
        h = X_local
        L_ = len(self.W)
        for i in range(L_):
            H = self.backend.linear(h, self.W[i])
            h = sharded_aggregate(H, self.shard, self.aggr, self.b[i], relu=i < L_ - 1,
                                  backend=self.backend, group=self.group)
        return h

    def step_fn(self, X, dY):
        Xl = self.local_rows(X)
        dYl = self.local_rows(dY)
        params = self.params()

        def step():
            for p in params:
                p.grad = None
            out = self.forward(Xl)
            out.backward(dYl)
            allreduce_grads(params, self.group)
        return step

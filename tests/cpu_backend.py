"""CPU test double of mgcn.dist.HipBackend (TEST CODE ONLY).

Lets the destination-range sharding, padded all-gathers and gradient
all-reduce of mgcn.dist run under the gloo backend on a machine without a
GPU.  The arithmetic follows the same contract as libmgcn (CSR rows in COO
order, sequential per-row sums via torch CPU index_add_, which accumulates
in index order), so sharded and single-process runs can be compared.
"""
from __future__ import annotations

import numpy as np
import torch

from mgcn import _lib as L
from mgcn.graph import CSRView, GraphPlan, NormPlan


def _view(key, other, n_key, n_other):
    order = torch.from_numpy(np.argsort(key.numpy(), kind="stable"))
    counts = torch.bincount(key, minlength=n_key)
    rowptr = torch.zeros(n_key + 1, dtype=torch.int64)
    rowptr[1:] = torch.cumsum(counts, 0)
    return CSRView(rowptr=rowptr, col=other[order].to(torch.int32), eid=order.to(torch.int32),
                   n_rows=n_key, n_cols=n_other)


class CpuBackend:
    def build_plan(self, edge_index, num_nodes):
        ei = edge_index.cpu()
        fwd = _view(ei[1], ei[0], num_nodes, num_nodes)
        bwd = _view(ei[0], ei[1], num_nodes, num_nodes)
        in_cnt = (fwd.rowptr[1:] - fwd.rowptr[:-1]).clamp(min=1).float()
        return GraphPlan(num_nodes, ei.size(1), torch.device("cpu"), fwd, bwd, in_cnt)

    def norm(self, plan, method, deg=None, edge_weight=None):
        assert edge_weight is None
        if method is None:
            return NormPlan(0, None, None, None, None, None)
        deg = (plan.bwd.rowptr[1:] - plan.bwd.rowptr[:-1]).float() if deg is None else deg
        dinv = 1.0 / torch.sqrt(deg) if method == "sm" else 1.0 / deg
        dinv[dinv == float("inf")] = 0
        n = plan.num_nodes

        def wts(view, rows_are_dst):
            r = torch.repeat_interleave(torch.arange(n), view.rowptr[1:] - view.rowptr[:-1])
            c = view.col.long()
            s, d = (c, r) if rows_are_dst else (r, c)
            return dinv[s] * dinv[d] if method == "sm" else dinv[s]

        if method == "rw":
            return NormPlan(2, wts(plan.fwd, True), None, dinv, deg, dinv)
        return NormPlan(1, wts(plan.fwd, True), wts(plan.bwd, False), None, deg, dinv)

    @staticmethod
    def _rows(view):
        return torch.repeat_interleave(torch.arange(view.n_rows),
                                       view.rowptr[1:] - view.rowptr[:-1])

    def finalize_view(self, view):
        return view

    def spmm_fwd(self, view, w, H, reduce, bias=None, relu=False):
        rows = self._rows(view)
        x = H[view.col.long()]
        if w is not None:
            x = x * w.view(-1, 1)
        F = H.size(1)
        argmax = None
        if reduce == L.REDUCE_MAX:
            y = torch.full((view.n_rows, F), L.MAX_FILL)
            argmax = torch.full((view.n_rows, F), -1, dtype=torch.int32)
            for k in range(x.size(0)):
                m = x[k] >= y[rows[k]]
                y[rows[k]][m] = x[k][m]
                argmax[rows[k]][m] = view.eid[k]
            fill = y == L.MAX_FILL
            y[fill] = 0
            argmax[fill] = -1
        else:
            y = torch.zeros(view.n_rows, F).index_add_(0, rows, x)
            if reduce == L.REDUCE_MEAN:
                cnt = (view.rowptr[1:] - view.rowptr[:-1]).clamp(min=1).float()
                y = y / cnt.view(-1, 1)
        if bias is not None:
            y = y + bias.detach()
        if relu:
            y = torch.where(y < 0, torch.zeros_like(y), y)
        return y, argmax

    def spmm_bwd(self, view, w, row_scale, dY, reduce, cnt=None, argmax=None):
        rows = self._rows(view)
        c = view.col.long()
        g = dY[c]
        if reduce == L.REDUCE_MEAN:
            g = g / cnt[c].view(-1, 1)
        if reduce == L.REDUCE_MAX:
            g = torch.where(argmax[c] == view.eid.view(-1, 1), g, torch.zeros_like(g))
        if w is not None:
            g = g * w.view(-1, 1)
        out = torch.zeros(view.n_rows, dY.size(1)).index_add_(0, rows, g)
        if row_scale is not None:
            out = out * row_scale.view(-1, 1)
        return out

    def relu_bwd_colsum(self, dZ, Z, relu, want_db):
        dY = torch.where(Z > 0, dZ, torch.zeros_like(dZ)) if relu else dZ
        return dY, (dY.sum(0) if want_db else None)

    def linear(self, x, W):
        return torch.matmul(x, W)

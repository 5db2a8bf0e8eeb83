"""CPU test double of mgcn.dist.HipBackend (TEST CODE ONLY).

Lets the destination-range sharding, chunked table all-gathers and gradient
all-reduce of mgcn.dist run under the gloo backend on a machine without a
GPU.  The arithmetic follows the same contract as libmgcn: CSR rows in COO
order (stable sort), sequential per-row sums (torch CPU index_add_
accumulates in index order), rowptr entries as absolute slot indices (row
ranges of a view share its col / eid arrays), and dense products whose
per-row result does not depend on how many rows are in the call (an
explicit k-ordered sum), so sharded and single-process runs compare bitwise
wherever the GPU path does.
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


def _mm(A, W):
    """A @ W as sum_k A[:, k] W[k, :] in k order: row-count independent."""
    out = torch.zeros(A.size(0), W.size(1), dtype=torch.float32)
    for k in range(A.size(1)):
        out = out + A[:, k:k + 1] * W[k]
    return out


def _slots(view):
    """(row of each slot, slot ids) of the view's rows (absolute rowptr)."""
    rp = view.rowptr
    a, b = int(rp[0]), int(rp[-1])
    rows = torch.repeat_interleave(torch.arange(view.n_rows), rp[1:] - rp[:-1])
    return rows, torch.arange(a, b)


class CpuBackend:
    # ------------------------------------------------------------ graph prep
    def build_plan(self, edge_index, num_nodes):
        ei = edge_index.cpu()
        fwd = _view(ei[1], ei[0], num_nodes, num_nodes)
        bwd = _view(ei[0], ei[1], num_nodes, num_nodes)
        in_cnt = (fwd.rowptr[1:] - fwd.rowptr[:-1]).clamp(min=1).float()
        return GraphPlan(num_nodes, ei.size(1), torch.device("cpu"), fwd, bwd, in_cnt)

    def build_view(self, key, other, n_key, n_other):
        return _view(key.cpu(), other.cpu(), n_key, n_other)

    def degree_norm(self, n, bwd, deg, ew, code):
        if deg is None:
            rows, slots = _slots(bwd)
            w = torch.ones(slots.numel()) if ew is None else ew[bwd.eid[slots].long()]
            deg = torch.zeros(n).index_add_(0, rows, w)
        deg = deg.float()
        dinv = 1.0 / torch.sqrt(deg) if code == L.NORM_SM else 1.0 / deg
        dinv[dinv == float("inf")] = 0
        return deg, dinv

    def edge_norm(self, view, rows_are_dst, dinv, ew, code):
        rows, slots = _slots(view)
        c = view.col[slots].long()
        s, d = (c, rows) if rows_are_dst else (rows, c)
        w = None if ew is None else ew[view.eid[slots].long()]
        if code == L.NORM_NONE:
            return w
        if code == L.NORM_RW:
            return dinv[s] if w is None else dinv[s] * w
        return dinv[s] * dinv[d] if w is None else dinv[s] * w * dinv[d]

    def norm(self, plan, method, deg=None, edge_weight=None):
        assert edge_weight is None
        if method is None:
            return NormPlan(0, None, None, None, None, None)
        code = L.NORM_CODES[method]
        deg, dinv = self.degree_norm(plan.num_nodes, plan.bwd, deg, None, code)
        if method == "rw":
            return NormPlan(2, self.edge_norm(plan.fwd, True, dinv, None, code), None, dinv, deg,
                            dinv)
        return NormPlan(1, self.edge_norm(plan.fwd, True, dinv, None, code),
                        self.edge_norm(plan.bwd, False, dinv, None, code), None, deg, dinv)

    def finalize_view(self, view):
        return view

    def fused_ok(self, shard, F_in, F_out, reduce):
        return reduce in (L.REDUCE_SUM, L.REDUCE_MEAN)

    # ------------------------------------------------------------ aggregation
    def _aggregate(self, view, w, H):
        rows, slots = _slots(view)
        x = H[view.col[slots].long()]
        if w is not None:
            x = x * w[slots].view(-1, 1)
        return rows, slots, x

    def spmm_fwd(self, view, w, H, reduce, bias=None, relu=False):
        rows, slots, x = self._aggregate(view, w, H)
        F = H.size(1)
        argmax = None
        if reduce == L.REDUCE_MAX:
            y = torch.full((view.n_rows, F), L.MAX_FILL)
            argmax = torch.full((view.n_rows, F), -1, dtype=torch.int32)
            for k in range(x.size(0)):
                m = x[k] >= y[rows[k]]
                y[rows[k]][m] = x[k][m]
                argmax[rows[k]][m] = view.eid[slots[k]]
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
        rows, slots = _slots(view)
        c = view.col[slots].long()
        g = dY[c]
        if reduce == L.REDUCE_MEAN:
            g = g / cnt[c].view(-1, 1)
        if reduce == L.REDUCE_MAX:
            g = torch.where(argmax[c] == view.eid[slots].view(-1, 1), g, torch.zeros_like(g))
        if w is not None:
            g = g * w[slots].view(-1, 1)
        out = torch.zeros(view.n_rows, dY.size(1)).index_add_(0, rows, g)
        if row_scale is not None:
            out = out * row_scale.view(-1, 1)
        return out

    # ------------------------------------------------ packed table exchange
    # (libmgcn mgcn_pack_rows_count / _values, mgcn_unpack_rows: the same
    # buffer layout [hdr: n x W pairs (mask_w, pos_w)][vals], bit-pattern test)
    @staticmethod
    def _bits_to_words(bits):
        n, F = bits.shape
        w = bits.view(n, F // 32, 32).to(torch.int64) << torch.arange(32, dtype=torch.int64)
        w = w.sum(-1)
        return torch.where(w >= 2 ** 31, w - 2 ** 32, w).to(torch.int32)

    @staticmethod
    def _words_to_bits(words, F):
        w = words.to(torch.int64) & 0xFFFFFFFF
        return ((w.unsqueeze(-1) >> torch.arange(32, dtype=torch.int64)) & 1).bool().view(-1, F)

    def pack_count(self, rows, hdr, counts):
        bits = rows.contiguous().view(torch.int32) != 0
        hdr[:, 0::2] = self._bits_to_words(bits)
        counts.copy_(bits.sum(1).to(torch.int32))

    def pack_values(self, rows, offs, hdr, vals):
        F = rows.size(1)
        v = rows.contiguous().view(torch.int32)
        bits = self._words_to_bits(hdr[:, 0::2].contiguous(), F)
        nz = v[bits]
        vals[:nz.numel()] = nz
        per_word = bits.view(-1, F // 32, 32).sum(-1).to(torch.int64)
        below = torch.cumsum(per_word, 1) - per_word
        hdr[:, 1::2] = (offs.to(torch.int64).view(-1, 1) + below).to(torch.int32)

    def pack_rows(self, rows, hdr, vals, total):
        counts = torch.empty(rows.size(0), dtype=torch.int32)
        self.pack_count(rows, hdr, counts)
        offs = torch.cumsum(counts, 0, dtype=torch.int32) - counts
        self.pack_values(rows, offs, hdr, vals)
        total[0] = int(counts.sum())

    def pack_rows_ok(self, F):
        return F in (32, 64, 128, 256)

    def unpack(self, buf, n_seg, n, seg_words, out):
        F = out.size(1)
        words = F // 32
        for p in range(n_seg):
            seg = buf[p * seg_words:(p + 1) * seg_words]
            out[p * n:(p + 1) * n] = self._unpack_seg(seg, n, F)

    def _unpack_seg(self, seg, n, F):
        words = F // 32
        hdr = seg[:2 * n * words].view(n, 2 * words)
        bits = self._words_to_bits(hdr[:, 0::2].contiguous(), F)
        o = torch.zeros(n, F, dtype=torch.int32)
        k = int(bits.sum())
        o[bits] = seg[2 * n * words:2 * n * words + k]
        return o.view(torch.float32)

    def packed_gather_ok(self, F):
        return True  # (the double takes packed tables at any width)

    def _dense_table(self, tab, view):
        """A PackedTable expanded (the double's stand-in for the in-place
        gather) and the view's packed columns mapped back to table rows."""
        rows = []
        for s_ in range(tab.n_seg):
            buf = tab.bufs[tab.seg_buf[s_]]
            rows.append(self._unpack_seg(buf[tab.seg_off[s_]:], tab.seg_rows, tab.F))
        dense = torch.cat(rows)
        c = view.col.to(torch.int64)
        t = (c >> tab.row_bits) * tab.seg_rows + (c & ((1 << tab.row_bits) - 1))
        v = CSRView(rowptr=view.rowptr, col=t.to(torch.int32), eid=view.eid, n_rows=view.n_rows,
                    n_cols=dense.size(0), n_edges=view.n_edges)
        return dense, v

    def relu_bwd_colsum(self, dZ, Z, relu, want_db, row_div=None):
        dY = torch.where(Z > 0, dZ, torch.zeros_like(dZ)) if relu else dZ
        db = dY.sum(0) if want_db else None
        if row_div is not None:
            dY = dY / row_div.view(-1, 1)
        return dY, db

    def linear(self, x, W):
        return torch.matmul(x, W)

    # ------------------------------------------------------------ fused layer
    def spmm_xw_fwd(self, view, w, X, W, reduce, bias=None, relu=False, relu_mask=None,
                    want_z=False, out=None, z_out=None):
        if not isinstance(X, torch.Tensor):  # a PackedTable
            X, view = self._dense_table(X, view)
        rows, _, x = self._aggregate(view, w, X)
        Z = torch.zeros(view.n_rows, X.size(1)).index_add_(0, rows, x)
        A = Z
        if reduce == L.REDUCE_MEAN:
            cnt = (view.rowptr[1:] - view.rowptr[:-1]).clamp(min=1).float()
            A = Z / cnt.view(-1, 1)
        y = _mm(A, W.detach())
        if bias is not None:
            y = y + bias.detach()
        if relu:
            y = torch.where(y < 0, torch.zeros_like(y), y)
        if relu_mask is not None:
            relu_mask.copy_((y > 0).to(torch.int32)[:, :relu_mask.size(1)])  # a token mask
            self._masks[relu_mask.data_ptr()] = (y > 0)
        if out is not None:
            out.copy_(y)
        if want_z and z_out is not None:
            z_out.copy_(Z)
        return (y, Z) if want_z else y

    def spmm_xw_bwd_dx(self, view_t, w_t, row_scale, dY, W, relu_mask=None, row_div=None,
                       out=None, colsum=None):
        if not isinstance(dY, torch.Tensor):  # a PackedTable
            dY, view_t = self._dense_table(dY, view_t)
        dH = self.spmm_bwd(view_t, w_t, row_scale, dY, L.REDUCE_SUM)
        dX = _mm(dH, W.detach().t())
        cs = None
        if relu_mask is not None:
            dX = torch.where(self._masks[relu_mask.data_ptr()], dX, torch.zeros_like(dX))
            cs = dX.sum(0)
            if row_div is not None:
                dX = dX / row_div.view(-1, 1)
        out.copy_(dX)
        if colsum is not None and cs is not None:
            colsum.add_(cs)
            return None
        return cs

    def gemm_bwd_dw(self, Z, dY, W, dh_colsum=False):
        return torch.matmul(Z.t(), dY), (dY.sum(0) if dh_colsum else None)

    def __init__(self):
        self._masks = {}

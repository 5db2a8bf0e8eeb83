"""Graph plans: the device-resident CSR views the aggregation kernels stream.

A :class:`GraphPlan` is built once per static ``edge_index`` (libmgcn
``mgcn_csr_build``) and holds

* ``fwd``  -- edges grouped by destination ``edge_index[1]`` (rows = dst,
  col = src): the forward SpMM walks one row per destination;
* ``bwd``  -- edges grouped by source ``edge_index[0]`` (rows = src, col =
  dst): the adjoint SpMM for ``dH = A^T dY`` and the out-degree of
  ``degnorm_const`` (gcn_base_models.py:124-126 sums over ``edge_index[0]``);
* ``in_cnt`` -- ``max(in-degree, 1)`` as float, torch_scatter 1.x's
  ``count.clamp(min=1)`` of ``scatter_mean``.

Within every row the edges keep their COO order, which is the order the
reference's CPU ``scatter_add``/``index_add_`` accumulate in, so sums match bit
for bit.  Normalisation weights (:class:`NormPlan`) hang off the plan, keyed by
method / ``deg`` / ``edge_weight``.

Plans are cached (``plan_for``), keyed by the identity of the ``edge_index``
tensor (a weak reference, its ``_version`` counter and ``num_nodes``): the
reference recomputes ``degnorm_const`` and re-scatters the COO list on every
forward (gcn_base_models.py:215); graphs are static across layers and epochs,
so this engine prepares them once.
"""
from __future__ import annotations

import weakref
from collections import OrderedDict
from dataclasses import dataclass, field

import torch

from . import _lib as L


# Rows with more edges than this are aggregated by a whole workgroup
# (libmgcn's heavy-row path); the lane-group kernel would otherwise
# serialise on them (degree-skewed graphs, config 3).
HEAVY_THRESHOLD = 128


@dataclass
class CSRView:
    """Edges grouped by one endpoint; ``col`` holds the other endpoint."""
    rowptr: torch.Tensor  # int64 [n_rows + 1]
    col: torch.Tensor     # int32 [nnz]
    eid: torch.Tensor     # int32 [nnz] original COO edge id of each slot
    n_rows: int
    n_cols: int
    # row schedule (mgcn_row_schedule): row ids by degree, heaviest first;
    # the first n_heavy (> heavy_thr edges) take the workgroup path, the
    # first n_giant of those the giant launch.  None: natural order.
    order: torch.Tensor | None = None
    n_heavy: int = 0
    n_giant: int = 0
    heavy_thr: int = HEAVY_THRESHOLD
    # edges of this view when it is a row range of a larger one (``col`` /
    # ``eid`` then hold the whole array, rowptr indexes into it): host-side
    # bookkeeping only (byte counts of a launch), None = all of ``col``
    n_edges: int | None = None

    @property
    def nnz(self) -> int:
        return int(self.col.numel())

    @property
    def edges(self) -> int:
        return self.nnz if self.n_edges is None else int(self.n_edges)

    def rows(self, a: int, b: int, n_edges: int | None = None) -> "CSRView":
        """Rows [a, b) as a view over the same col / eid arrays (the kernels
        take rowptr entries as absolute slot indices), in natural row order
        (no schedule: for the fused layer kernels, which never read one; a
        view with heavy rows cannot be split)."""
        if self.n_heavy:
            raise ValueError("CSRView.rows: a view with heavy rows cannot be split by rows")
        return CSRView(rowptr=self.rowptr[a:b + 1], col=self.col, eid=self.eid, n_rows=b - a,
                       n_cols=self.n_cols, n_edges=n_edges)

    @property
    def heavy(self) -> torch.Tensor | None:
        """int32 ids of the heavy rows, heaviest first."""
        return None if self.order is None or self.n_heavy == 0 else self.order[:self.n_heavy]


def schedule_rows(view: CSRView, thr: int | None = None) -> CSRView:
    """Fill ``view.order`` / ``n_heavy`` / ``n_giant`` (mgcn_row_schedule).

    The degree order pays on skewed graphs (waves of similar-degree rows,
    longest first); on near-uniform ones (Erdos-Renyi, config 2) it only
    scatters the row-pointer and edge-slot reads, so there the natural order
    is kept (``order`` None): no heavy rows and max degree <= 4x mean + 8."""
    import ctypes
    if thr is None:
        thr = HEAVY_THRESHOLD  # read at call time (a tuning run may set it)
    lib = L.load()
    dev = view.rowptr.device
    if view.n_rows == 0:
        return view
    order = torch.empty(view.n_rows, dtype=torch.int32, device=dev)
    ws = torch.empty(lib.mgcn_row_schedule_workspace_bytes(view.n_rows), dtype=torch.uint8,
                     device=dev)
    n_heavy = ctypes.c_int64(0)
    n_giant = ctypes.c_int64(0)
    with L.device_guard(dev):
        rc = lib.mgcn_row_schedule(view.n_rows, L.ptr(view.rowptr), int(thr), L.ptr(order),
                                   ctypes.byref(n_heavy), ctypes.byref(n_giant), L.ptr(ws),
                                   ws.numel(), L.stream_of(dev))
    L.check(rc, "mgcn_row_schedule")
    view.heavy_thr = int(thr)
    view.n_heavy = int(n_heavy.value)
    view.n_giant = int(n_giant.value)
    if view.n_heavy == 0:
        top = int(order[0])
        max_deg = int(view.rowptr[top + 1] - view.rowptr[top])
        if max_deg <= 4 * view.nnz / view.n_rows + 8:
            view.order, view.n_giant = None, 0
            return view
    view.order = order
    return view


find_heavy = schedule_rows  # earlier name


@dataclass
class NormPlan:
    """Per-slot weights of both views for one (method, deg, edge_weight)."""
    method: int
    w_fwd: torch.Tensor | None       # float [nnz] in fwd slot order (None: unweighted)
    w_bwd: torch.Tensor | None       # float [nnz] in bwd slot order
    row_scale_bwd: torch.Tensor | None  # RW without edge weights: dinv post-scale
    deg: torch.Tensor | None
    dinv: torch.Tensor | None
    # True: w_fwd (or, for 'rw' without edge weights, the per-slot dinv in
    # w_fwd) carries autograd history back to edge_weight / deg -- the
    # aggregation then takes the weights as an input (ops._AggregateW) and
    # returns their gradient (libmgcn mgcn_edge_weight_grad); never cached.
    grad: bool = False


@dataclass
class GraphPlan:
    num_nodes: int
    nnz: int
    device: torch.device
    fwd: CSRView
    bwd: CSRView
    in_cnt: torch.Tensor  # float [num_nodes] = max(in-degree, 1)
    norms: dict = field(default_factory=dict)
    _key_refs: list = field(default_factory=list)
    _slot_map: torch.Tensor | None = None
    _coo: tuple | None = None

    def slot_map(self) -> torch.Tensor:
        """int32 [nnz]: the fwd-view slot of every bwd-view slot (mgcn_slot_map),
        built on first use (max aggregation)."""
        if self._slot_map is None:
            lib = L.load()
            dev = self.device
            out = torch.empty(max(self.nnz, 1), dtype=torch.int32, device=dev)
            ws = torch.empty(int(lib.mgcn_slot_map_workspace_bytes(self.nnz)), dtype=torch.uint8,
                             device=dev)
            with L.device_guard(dev):
                rc = lib.mgcn_slot_map(self.nnz, L.ptr(self.fwd.eid), L.ptr(self.bwd.eid),
                                       L.ptr(out), L.ptr(ws), ws.numel(), L.stream_of(dev))
            L.check(rc, "mgcn_slot_map")
            self._slot_map = out
        return self._slot_map

    # ------------------------------------------------------------------ norms
    def coo(self) -> tuple[torch.Tensor, torch.Tensor]:
        """(src, dst) int64 [nnz] in COO (edge id) order, rebuilt from the fwd
        view on first use (the differentiable norm of :func:`_grad_norm`)."""
        if self._coo is None:
            eid = self.fwd.eid.long()
            src = torch.empty(self.nnz, dtype=torch.int64, device=self.device)
            dst = torch.empty(self.nnz, dtype=torch.int64, device=self.device)
            src[eid] = self.fwd.col.long()
            cnt = self.fwd.rowptr[1:] - self.fwd.rowptr[:-1]
            dst[eid] = torch.repeat_interleave(
                torch.arange(self.num_nodes, device=self.device), cnt, output_size=self.nnz)
            self._coo = (src, dst)
        return self._coo

    def norm(self, method: str | None, deg: torch.Tensor | None = None,
             edge_weight: torch.Tensor | None = None) -> NormPlan:
        """Normalisation weights, as NodeModelBase.degnorm_const computes them
        (gcn_base_models.py:65-146):

        * ``edge_weight`` given -> the degree is recomputed from it and
          ``deg`` is ignored (:102-110);
        * else ``deg`` given -> used as is (:119-121);
        * else ``deg`` = out-degree (edge count over ``edge_index[0]``, :117).
        ``method`` None means unnormalised (``edge_weight`` then acts as a
        plain message weight, PyG GraphConv/SAGEConv).
        """
        code = L.NORM_CODES[method]
        if edge_weight is not None or code == L.NORM_NONE:
            # unnormalised: degnorm_const never reads deg (gcn_base_models.py:209-211)
            deg = None
        if torch.is_grad_enabled() and any(t is not None and t.requires_grad
                                           for t in (edge_weight, deg)):
            # degnorm_const is differentiable in edge_weight / deg
            # (gcn_base_models.py:102-140): build the weights through autograd
            return _grad_norm(self, code, deg, edge_weight)
        key = (code, _tkey(deg), _tkey(edge_weight))
        hit = self.norms.get(key)
        if hit is not None and _alive(hit[1]):
            return hit[0]
        plan = _build_norm(self, code, deg, edge_weight)
        self.norms[key] = (plan, [weakref.ref(_owner(t)) for t in (deg, edge_weight)
                                  if t is not None])
        if len(self.norms) > 8:
            self.norms.pop(next(iter(self.norms)))
        return plan


def _tkey(t: torch.Tensor | None):
    # (storage, version counter, geometry): an in-place update through the
    # tensor bumps _version and misses the cache; writes through ``.data``
    # (which do not bump it) are invisible here -- call plan.norms.clear()
    # after such a write.
    if t is None:
        return None
    return (t.data_ptr(), t._version, tuple(t.shape), tuple(t.stride()), t.dtype)


def _owner(t: torch.Tensor) -> torch.Tensor:
    # a view such as batch.x[:, 1] is a new Python object per call; its base
    # outlives it, shares its version counter, and is what we keep a ref to
    return t._base if t._base is not None else t


def _alive(refs) -> bool:
    return all(r() is not None for r in refs)


def _f32(t: torch.Tensor | None, n: int, name: str, device) -> torch.Tensor | None:
    if t is None:
        return None
    t = t.reshape(-1)
    if t.numel() != n:
        raise ValueError(f"{name} has {t.numel()} entries, expected {n}")
    if t.device != device:
        raise L.MgcnError(f"{name} is on {t.device}, graph is on {device}")
    return t.to(torch.float32).contiguous()


def build_view(key: torch.Tensor, other: torch.Tensor, n_key: int, n_other: int,
               schedule: bool = True) -> CSRView:
    """CSR over ``key`` (libmgcn ``mgcn_csr_build``); stable in COO order;
    ``schedule`` fills the row schedule (:func:`schedule_rows`)."""
    lib = L.load()
    dev = L.require_device(key, other)
    key = key.to(torch.int64).contiguous()
    other = other.to(torch.int64).contiguous()
    nnz = int(key.numel())
    rowptr = torch.empty(n_key + 1, dtype=torch.int64, device=dev)
    col = torch.empty(max(nnz, 1), dtype=torch.int32, device=dev)[:nnz]
    eid = torch.empty(max(nnz, 1), dtype=torch.int32, device=dev)[:nnz]
    ws_bytes = int(lib.mgcn_csr_workspace_bytes(nnz, n_key))
    ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
    with L.device_guard(dev):
        rc = lib.mgcn_csr_build(L.ptr(key), L.ptr(other), nnz, n_key, n_other, L.ptr(rowptr),
                                L.ptr(col), L.ptr(eid), L.ptr(ws), ws_bytes, L.stream_of(dev))
    L.check(rc, "mgcn_csr_build")
    view = CSRView(rowptr=rowptr, col=col, eid=eid, n_rows=n_key, n_cols=n_other)
    return schedule_rows(view) if schedule else view


def build_plan(edge_index: torch.Tensor, num_nodes: int) -> GraphPlan:
    if edge_index.dim() != 2 or edge_index.size(0) != 2:
        raise ValueError(f"edge_index must be [2, E], got {tuple(edge_index.shape)}")
    dev = L.require_device(edge_index)
    src, dst = edge_index[0], edge_index[1]
    fwd = build_view(dst, src, num_nodes, num_nodes)
    bwd = build_view(src, dst, num_nodes, num_nodes)
    in_cnt = (fwd.rowptr[1:] - fwd.rowptr[:-1]).clamp_(min=1).to(torch.float32)
    return GraphPlan(num_nodes=num_nodes, nnz=int(edge_index.size(1)), device=dev, fwd=fwd,
                     bwd=bwd, in_cnt=in_cnt)


def _build_norm(g: GraphPlan, code: int, deg, edge_weight) -> NormPlan:
    lib = L.load()
    dev = g.device
    n = g.num_nodes
    ew = _f32(edge_weight, g.nnz, "edge_weight", dev)
    if code == L.NORM_NONE:
        if ew is None:
            return NormPlan(code, None, None, None, None, None)
        dinv = None
        dg = None
    else:
        deg_in = _f32(deg, n, "deg", dev)
        dg = torch.empty(n, dtype=torch.float32, device=dev)
        dinv = torch.empty(n, dtype=torch.float32, device=dev)
        with L.device_guard(dev):
            rc = lib.mgcn_degree_norm(n, L.ptr(g.bwd.rowptr), L.ptr(g.bwd.eid), L.ptr(deg_in),
                                      L.ptr(ew), code, L.ptr(dg), L.ptr(dinv), L.stream_of(dev))
        L.check(rc, "mgcn_degree_norm")
    if code == L.NORM_RW and ew is None:
        # x * dinv before the gather (gcn_base_models.py:217-220): the forward
        # products are H[src] * dinv[src]; the adjoint post-scales by dinv[src].
        w_fwd = _edge_norm(g.fwd, True, dinv, None, code)
        return NormPlan(code, w_fwd, None, dinv, dg, dinv)
    w_fwd = _edge_norm(g.fwd, True, dinv, ew, code)
    w_bwd = _edge_norm(g.bwd, False, dinv, ew, code)
    return NormPlan(code, w_fwd, w_bwd, None, dg, dinv)


class _DegNorm(torch.autograd.Function):
    """dinv = deg^-1/2 ('sm') or deg^-1 ('rw'), inf -> 0, with deg the given
    one or the weighted out-degree sum_{e: src_e = n} edge_weight_e
    (gcn_base_models.py:112-135; forward = libmgcn mgcn_degree_norm, bit for
    bit).  Backward = autograd of the reference's ops: pow's derivative,
    zeroed where the in-place ``deg_inv_sqrt[... == inf] = 0`` overwrote the
    entry (as there, 0 * the derivative's inf is NaN at deg = 0), then the
    degree sum's adjoint, a gather over the edges' sources."""

    @staticmethod
    def forward(ctx, ew, deg, g, code):
        dg, dinv = degree_norm(g.num_nodes, g.bwd, None if deg is None else deg.detach(),
                               None if ew is None else ew.detach(), code)
        ctx.g, ctx.code, ctx.has_ew = g, code, ew is not None
        ctx.save_for_backward(dg)
        return dinv

    @staticmethod
    def backward(ctx, grad):
        (dg,) = ctx.saved_tensors
        e, c = (-1.5, -0.5) if ctx.code == L.NORM_SM else (-2.0, -1.0)
        gdeg = grad.masked_fill(dg == 0, 0.0) * (c * dg.pow(e))
        if ctx.has_ew:
            src, _ = ctx.g.coo()
            return gdeg[src], None, None, None
        return None, gdeg, None, None


def _grad_norm(g: GraphPlan, code: int, deg, edge_weight) -> NormPlan:
    """:meth:`GraphPlan.norm` when edge_weight or deg requires grad: the same
    weights (bit for bit), formed by differentiable ops in COO order exactly
    as degnorm_const writes them (``deg_inv_sqrt[row] * edge_weight *
    deg_inv_sqrt[col]``, gcn_base_models.py:137-142), then gathered into the
    views' slot orders.  Only the fwd weights keep the history; the adjoint's
    copies are detached (their gradient comes through the fwd ones)."""
    dev = g.device
    ew = None
    if edge_weight is not None:
        ew = edge_weight.reshape(-1)
        if ew.numel() != g.nnz:
            raise ValueError(f"edge_weight has {ew.numel()} entries, expected {g.nnz}")
        if ew.device != dev:
            raise L.MgcnError(f"edge_weight is on {ew.device}, graph is on {dev}")
        ew = ew.to(torch.float32)
    if deg is not None:
        deg = deg.reshape(-1).to(torch.float32)
        if deg.numel() != g.num_nodes:
            raise ValueError(f"deg has {deg.numel()} entries, expected {g.num_nodes}")
    feid, beid = g.fwd.eid.long(), g.bwd.eid.long()
    if code == L.NORM_NONE:  # plain message weights (PyG GraphConv / SAGEConv)
        return NormPlan(code, ew[feid], ew.detach()[beid], None, None, None, grad=True)
    src, dst = g.coo()
    dinv = _DegNorm.apply(ew, deg, g, code)
    if code == L.NORM_RW and ew is None:
        # x * dinv before the gather (gcn_base_models.py:217-220): per fwd slot
        # dinv[src]; the adjoint post-scales by dinv
        return NormPlan(code, dinv[g.fwd.col.long()], None, dinv.detach(), None, dinv, grad=True)
    if code == L.NORM_SM:
        w = dinv[src] * ew * dinv[dst] if ew is not None else dinv[src] * dinv[dst]
    else:
        w = dinv[src] * ew
    return NormPlan(code, w[feid], w.detach()[beid], None, None, dinv.detach(), grad=True)


def degree_norm(n: int, bwd: CSRView | None, deg, ew, code: int):
    """(deg, dinv) of rows [0, n) (libmgcn ``mgcn_degree_norm``,
    gcn_base_models.py:112-135): ``deg`` given -> used as is; else the
    (weighted) out-degree summed over each row of the source-grouped ``bwd``
    view in COO order."""
    lib = L.load()
    dev = (deg if deg is not None else bwd.rowptr).device
    dg = torch.empty(n, dtype=torch.float32, device=dev)
    dinv = torch.empty(n, dtype=torch.float32, device=dev)
    with L.device_guard(dev):
        rc = lib.mgcn_degree_norm(n, None if bwd is None else L.ptr(bwd.rowptr),
                                  None if bwd is None else L.ptr(bwd.eid), L.ptr(deg), L.ptr(ew),
                                  code, L.ptr(dg), L.ptr(dinv), L.stream_of(dev))
    L.check(rc, "mgcn_degree_norm")
    return dg, dinv


def edge_norm(view: CSRView, rows_are_dst: bool, dinv, ew, code) -> torch.Tensor:
    """Per-slot weights of ``view`` (libmgcn ``mgcn_edge_norm``)."""
    return _edge_norm(view, rows_are_dst, dinv, ew, code)


def _edge_norm(view: CSRView, rows_are_dst: bool, dinv, ew, code) -> torch.Tensor:
    lib = L.load()
    dev = view.rowptr.device
    w = torch.empty(max(view.nnz, 1), dtype=torch.float32, device=dev)[:view.nnz]
    with L.device_guard(dev):
        rc = lib.mgcn_edge_norm(view.n_rows, view.nnz, L.ptr(view.rowptr), L.ptr(view.col),
                                L.ptr(view.eid), int(rows_are_dst), L.ptr(dinv), L.ptr(ew), code,
                                L.ptr(w), L.stream_of(dev))
    L.check(rc, "mgcn_edge_norm")
    return w


# ------------------------------------------------------------------- cache
_CACHE: "OrderedDict[tuple, tuple]" = OrderedDict()
_CACHE_SIZE = 16


def cache_key(edge_index: torch.Tensor, num_nodes: int) -> tuple:
    return (edge_index.data_ptr(), edge_index._version, tuple(edge_index.shape),
            edge_index.dtype, str(edge_index.device), int(num_nodes))


def plan_for(edge_index: torch.Tensor, num_nodes: int) -> GraphPlan:
    """Cached :func:`build_plan`.  An entry is valid only while the very
    ``edge_index`` tensor it was built from is alive and unmodified."""
    key = cache_key(edge_index, num_nodes)
    hit = _CACHE.get(key)
    if hit is not None:
        ref, plan = hit
        if ref() is edge_index:
            _CACHE.move_to_end(key)
            return plan
        del _CACHE[key]
    plan = build_plan(edge_index, num_nodes)
    _CACHE[key] = (weakref.ref(edge_index), plan)
    while len(_CACHE) > _CACHE_SIZE:
        _CACHE.popitem(last=False)
    return plan


def clear_cache() -> None:
    _CACHE.clear()

"""TEST INFRASTRUCTURE ONLY -- the CPU oracle for the GCN aggregation path.

Used solely as the checker by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py; the product (meta-gcn_amd/mgcn) never imports
it.  Two restatements of the reference's arithmetic live here:

* the C oracle (oracle/mgcn_oracle.c -> _build/liboracle.so), called through
  ctypes on numpy arrays: sequential, COO edge order, one rounding per op --
  the bit-exact definition used for parity;
* ``torch_layer_reference``: the reference's op sequence written with torch
  CPU ops (matmul -> index_select -> mul -> scatter_add_ -> + bias, autograd
  backward), i.e. gcn_base_models.py:199-243 with torch_scatter 1.x's
  scatter_add (= ``out.scatter_add_(0, index.expand_as(src), src)``).  This is
  the timed CPU baseline ("kind": "port").

Pinned by the fixtures in tests/golden/ (tests/test_oracle.py).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "liboracle.so")

NORM = {None: 0, "sm": 1, "rw": 2}
REDUCE = {"add": 0, "sum": 0, "mean": 1, "max": 2}

_lib = None


def build() -> str:
    subprocess.run(["make", "-C", HERE, "-s"], check=True)
    return LIB


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        vp, i64, i = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
        L.oracle_degnorm.argtypes = [i64, i64, vp, vp, vp, vp, i, vp, vp, vp]
        L.oracle_aggr_fwd.argtypes = [i64, i64, i64, vp, vp, vp, vp, i, vp, i, vp, vp]
        L.oracle_aggr_bwd.argtypes = [i64, i64, i64, i64, vp, vp, vp, vp, i, vp, vp, i, vp, vp, vp]
        L.oracle_segment_mean.argtypes = [i64, i64, vp, vp, vp]
        for f in (L.oracle_degnorm, L.oracle_aggr_fwd, L.oracle_aggr_bwd, L.oracle_segment_mean):
            f.restype = None
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _f32(a):
    return None if a is None else np.ascontiguousarray(a, dtype=np.float32)


def _i64(a):
    return np.ascontiguousarray(a, dtype=np.int64)


def degnorm(edge_index, num_nodes, deg=None, edge_weight=None, method="sm"):
    """(deg_used[N], dinv[N], norm_per_edge[E]) -- gcn_base_models.py:65-146."""
    ei = _i64(edge_index)
    src, dst = np.ascontiguousarray(ei[0]), np.ascontiguousarray(ei[1])
    E = src.size
    deg_out = np.empty(num_nodes, np.float32)
    dinv = np.empty(num_nodes, np.float32)
    norm = np.empty(max(E, 1), np.float32)
    lib().oracle_degnorm(num_nodes, E, _p(src), _p(dst), _p(_f32(deg)), _p(_f32(edge_weight)),
                         NORM[method], _p(deg_out), _p(dinv), _p(norm))
    return deg_out, dinv, norm[:E]


def edge_factors(edge_index, num_nodes, deg_norm, deg=None, edge_weight=None):
    """(w_fwd[E] or None, w_bwd[E] or None, row_scale[N] or None) of a layer."""
    if deg_norm is None:
        return None, None, None
    _, dinv, norm = degnorm(edge_index, num_nodes, deg, edge_weight, deg_norm)
    if deg_norm == "rw" and edge_weight is None:
        return norm, None, dinv
    return norm, norm, None


def aggr_fwd(edge_index, H, w=None, reduce="add", bias=None, relu=False, num_nodes=None):
    """(Y[N, F], argmax[N, F] int64 or None)."""
    ei = _i64(edge_index)
    src, dst = np.ascontiguousarray(ei[0]), np.ascontiguousarray(ei[1])
    H = _f32(H)
    N = H.shape[0] if num_nodes is None else num_nodes
    F = H.shape[1]
    Y = np.empty((N, F), np.float32)
    am = np.empty((N, F), np.int64) if REDUCE[reduce] == 2 else None
    lib().oracle_aggr_fwd(N, src.size, F, _p(src), _p(dst), _p(H), _p(_f32(w)), REDUCE[reduce],
                          _p(_f32(bias)), int(bool(relu)), _p(Y), _p(am))
    return Y, am


def aggr_bwd(edge_index, dZ, w=None, row_scale=None, reduce="add", Z=None, relu=False,
             argmax=None, want_db=False, num_src=None):
    """(dH[N_src, F], db[F] or None)."""
    ei = _i64(edge_index)
    src, dst = np.ascontiguousarray(ei[0]), np.ascontiguousarray(ei[1])
    dZ = _f32(dZ)
    N, F = dZ.shape
    Ns = N if num_src is None else num_src
    dH = np.empty((Ns, F), np.float32)
    db = np.empty(F, np.float32) if want_db else None
    am = None if argmax is None else _i64(argmax)
    lib().oracle_aggr_bwd(N, Ns, src.size, F, _p(src), _p(dst), _p(_f32(w)), _p(_f32(row_scale)),
                          REDUCE[reduce], _p(dZ), _p(_f32(Z) if relu else None), int(bool(relu)),
                          _p(am), _p(dH), _p(db))
    return dH, db


def segment_mean(x, ptr):
    x = _f32(x)
    ptr = _i64(ptr)
    out = np.empty((ptr.size - 1, x.shape[1]), np.float32)
    lib().oracle_segment_mean(ptr.size - 1, x.shape[1], _p(ptr), _p(x), _p(out))
    return out


def layer_fwd_bwd(x, edge_index, W, b, dZ, deg_norm="sm", aggr="add", relu=False, deg=None,
                  edge_weight=None):
    """NodeModelAdditive (+ optional fused ReLU) forward and backward on the CPU.

    The matmuls are float32 numpy (rounding differs from any BLAS, so compare
    layer outputs with a tolerance); the aggregation is the bit-exact oracle.
    Returns dict with Z, dx, dW, db.
    """
    N = x.shape[0]
    H = (x.astype(np.float32) @ W.astype(np.float32)).astype(np.float32)
    wf, wb, rs = edge_factors(edge_index, N, deg_norm, deg, edge_weight)
    Z, am = aggr_fwd(edge_index, H, wf, aggr, b, relu)
    dH, db = aggr_bwd(edge_index, dZ, wb, rs, aggr, Z, relu, am, want_db=b is not None)
    return {"H": H, "Z": Z, "dH": dH, "dx": dH @ W.T, "dW": x.T @ dH, "db": db, "argmax": am}


# ------------------------------------------------- PyG 1.3 conv restatements
def add_remaining_self_loops(edge_index, edge_weight=None, fill=1.0, num_nodes=None):
    """PyG 1.3 ``add_remaining_self_loops`` (not vendored in the reference;
    used by GCNConv / SAGEConv as kernel/gcn.py:10 and graph_sage.py:10 call
    them): existing self-loops are dropped, one loop per node is appended, a
    node that had a loop keeps that loop's weight (last in COO order), the
    others get ``fill``.  Returns (edge_index, edge_weight or None)."""
    ei = np.asarray(edge_index, np.int64)
    N = int(num_nodes if num_nodes is not None else ei.max() + 1)
    mask = ei[0] != ei[1]
    loops = np.arange(N, dtype=np.int64)
    ei2 = np.concatenate([ei[:, mask], np.stack([loops, loops])], 1)
    if edge_weight is None:
        return ei2, None
    ew = np.asarray(edge_weight, np.float32)
    lw = np.full(N, fill, np.float32)
    inv = ~mask
    lw[ei[0][inv]] = ew[inv]
    return ei2, np.concatenate([ew[mask], lw]).astype(np.float32)


def remove_self_loops(edge_index):
    """PyG 1.3 ``remove_self_loops`` (GINConv, kernel/gin.py:10)."""
    ei = np.asarray(edge_index, np.int64)
    return ei[:, ei[0] != ei[1]]


def gcnconv_fwd_bwd(x, edge_index, W, b, dZ, edge_weight=None, improved=False):
    """PyG 1.3 GCNConv forward + backward with the oracle aggregation:
    add_remaining_self_loops with unit (or given) weights, 'sm' norm over
    edge_index[0] with the weights, sum, + b.  The
    matmuls are fp32 numpy, so only W = I results are bit-comparable."""
    N = x.shape[0]
    ew = edge_weight
    if ew is None:
        ew = np.ones(np.asarray(edge_index).shape[1], np.float32)
    ei2, ew2 = add_remaining_self_loops(edge_index, ew, 2.0 if improved else 1.0, N)
    H = (x.astype(np.float32) @ W.astype(np.float32)).astype(np.float32)
    _, _, norm = degnorm(ei2, N, None, ew2, "sm")
    Y, _ = aggr_fwd(ei2, H, norm, "add", b)
    dH, db = aggr_bwd(ei2, dZ, norm, None, "add", want_db=b is not None)
    return {"y": Y, "dH": dH, "dx": dH @ W.T, "dW": x.T @ dH, "db": db, "edge_index": ei2,
            "norm": norm}


# ---------------------------------------------------------------- torch CPU
def torch_layer_reference(x, edge_index, W, b, deg_norm="sm", aggr="add", deg=None,
                          edge_weight=None):
    """The reference's op sequence (gcn_base_models.py:199-243, common.py:37-66)
    in torch CPU ops, autograd-capable; ``aggr`` 'add' only (the timed CPU
    baseline of bench.py).  ``edge_weight``: degnorm_const's weighted form
    (:102-142: degree = scatter_add of the weights over edge_index[0]; norm =
    dinv[row] * w * dinv[col] ('sm') or dinv[row] * w ('rw')), differentiable
    in the weights.  Returns the layer output tensor."""
    import torch
    src, dst = edge_index[0], edge_index[1]
    h = torch.matmul(x, W)
    if deg_norm is None:
        x_j = torch.index_select(h, 0, src)
    else:
        if edge_weight is not None:
            deg = torch.zeros(x.size(0), dtype=h.dtype).scatter_add(0, src, edge_weight)
        elif deg is None:
            deg = torch.zeros(x.size(0), dtype=h.dtype).scatter_add_(
                0, src, torch.ones(src.numel(), dtype=h.dtype))
        dinv = deg.pow(-0.5) if deg_norm == "sm" else deg.pow(-1)
        dinv = dinv.masked_fill(dinv == float("inf"), 0)
        if edge_weight is not None:
            norm = (dinv[src] * edge_weight * dinv[dst] if deg_norm == "sm"
                    else dinv[src] * edge_weight)
            x_j = torch.index_select(h, 0, src) * norm.view(-1, 1)
        elif deg_norm == "rw":
            x_j = torch.index_select(h * dinv.view(-1, 1), 0, src)
        else:
            norm = dinv[src] * dinv[dst]
            x_j = torch.index_select(h, 0, src) * norm.view(-1, 1)
    if aggr != "add":
        raise NotImplementedError("torch_layer_reference times the 'add' path only")
    out = torch.zeros(x.size(0), h.size(1), dtype=h.dtype)
    out = out.scatter_add(0, dst.view(-1, 1).expand_as(x_j), x_j)
    return out + b if b is not None else out

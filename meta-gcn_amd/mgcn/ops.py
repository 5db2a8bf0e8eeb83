"""Autograd-aware aggregation ops on top of libmgcn.

``aggregate`` is the fused replacement for the reference's message-passing
core (src/gcn_meta/models/gcn_base_models.py:209-241 + common.py:37-66):

    x_j = index_select(H, 0, src) * norm      # [E, F] materialised
    y   = torch_scatter.scatter_{add,mean,max}(x_j, dst, dim_size=N)
    y[y == -1e38] = 0                          # max only
    y   = y + bias ; y = relu(y)               # layer epilogue

Here it is one HIP kernel per direction (libmgcn ``mgcn_spmm_fwd`` /
``mgcn_spmm_bwd``); the [E, F] tensor never exists.  Gradients follow the
reference's autograd graph operation for operation (gather of dY, multiply by
norm, index_add over sources in edge order; mean divides dY by the count;
max routes through the saved argmax), so the adjoint is bit-identical too.
"""
from __future__ import annotations

import os
from collections import Counter
from dataclasses import dataclass

import torch

from . import _lib as L
from .graph import CSRView, GraphPlan, NormPlan, plan_for


# optional callable(name, start: bool, rows=None, edges=None) called right
# before / after each libmgcn launch on its stream (bench.py's HIP-event timer);
# the start call carries the launch's row and edge counts for byte accounting
_TIMER = None
# fused aggregate-then-transform forward for 128 -> 128 sum / mean layers
# (mgcn_spmm_xw_fwd); MGCN_FUSE_XW=0 selects the GEMM + SpMM launches
_FUSE_XW = os.environ.get("MGCN_FUSE_XW", "1") != "0"


# Middle layers of a stack (dX wanted, a ReLU mask below) keep the dW + dX
# gather kernel: Z write + dW pass + dX-only gather cost 1.18 ms there
# against 1.15 for the one kernel; the top layer (its bias gradient rides in
# the dW pass) and the bottom layer (no gather at all) take the Z form.
# MGCN_Z_MIDDLE=1 sends the middle layers through Z as well.
_Z_MIDDLE = os.environ.get("MGCN_Z_MIDDLE", "0") != "0"
# the top 128-wide layer of a stack (sum, no ReLU) takes the dW + dX adjoint
# (the DWS kernel) instead of keeping Z for the dense Z^T dY pass: env
# MGCN_TOP_FULL=0 turns it off.  Its bias gradient (dY's column sums) comes
# from a column-sum pass over dY (0.095 ms) -- config 2: 5.02 vs 5.04-5.07
# ms/step (A/B on one box) -- or, MGCN_TOP_HCS=1, from the adjoint launch
# itself (mgcn_spmm_xw_bwd_hcs: its dY row reads and their registers cost
# that launch ~0.25 ms, 5.16-5.19)
_TOP_FULL = os.environ.get("MGCN_TOP_FULL", "1") != "0"
_TOP_HCS = os.environ.get("MGCN_TOP_HCS", "0") != "0"
# (with _TOP_FULL: the top bias gradient from the bottom layer's dW pass, which
# streams dY beside its own operands -- mgcn_gemm_bwd_dw_cs; env
# MGCN_TOP_CS_DEFER=0: a column-sum pass of its own)
_TOP_CS_DEFER = os.environ.get("MGCN_TOP_CS_DEFER", "1") != "0"
# max layers with dX: the dW + dX adjoint with the winner-bit routing in one
# launch (mgcn_spmm_xw_bwd with win_mask: the warp-specialised kernel) instead
# of mgcn_spmm_bwd + mgcn_gemm_bwd: env MGCN_MAX_FULL=0 turns it off
_MAX_FULL = os.environ.get("MGCN_MAX_FULL", "1") != "0"


def set_fused_layers(enabled: bool) -> None:
    """Use (True, the default) or bypass the fused aggregate+transform layer
    kernels (mgcn_spmm_xw_fwd / _bwd) where they apply."""
    global _FUSE_XW
    _FUSE_XW = bool(enabled)


def set_z_middle(enabled: bool) -> None:
    """Send the middle layers of a fused stack through the Z^T dY + dX-only
    backward too (True; env MGCN_Z_MIDDLE=1) or keep them on the one dW + dX
    gather kernel (False, the default)."""
    global _Z_MIDDLE
    _Z_MIDDLE = bool(enabled)


def set_kernel_timer(timer) -> None:
    """Install (or clear with None) a hook called right before and after each
    libmgcn launch, on the launch stream -- used to time kernels with events."""
    global _TIMER
    _TIMER = timer


def _contig_f32(t: torch.Tensor, name: str) -> torch.Tensor:
    if t.dtype != torch.float32:
        raise TypeError(f"{name} must be float32 (the reference computes in fp32), got {t.dtype}")
    if t.dim() != 2:
        raise ValueError(f"{name} must be 2-D [N, F], got {tuple(t.shape)}")
    if t.stride(1) != 1 or t.stride(0) < t.size(1):
        t = t.contiguous()
    return t


def spmm_fwd(view: CSRView, w: torch.Tensor | None, H: torch.Tensor, reduce: int,
             bias: torch.Tensor | None = None, relu: bool = False,
             out: torch.Tensor | None = None, mask_plan: GraphPlan | None = None,
             relu_mask: torch.Tensor | None = None):
    """Y[view.n_rows, F] = epi(reduce_k H[col_k] * w_k); returns (Y, argmax).

    Max with ``mask_plan`` (the plan ``view`` belongs to): instead of argmax
    the kernel writes every edge's winner bits at its slot (int32
    [nnz, ceil(F/32)] bit patterns), returned in argmax's place.
    ``relu_mask`` (int32 [n_rows, 4], with relu and F <= 128) receives the
    Y > 0 bits the dX GEMM's fused ReLU backward reads (:func:`gemm_nn`)."""
    lib = L.load()
    H = _contig_f32(H, "H")
    dev = L.require_device(H, view.rowptr, w, bias)
    if H.size(0) != view.n_cols:
        raise ValueError(f"H has {H.size(0)} rows, graph has {view.n_cols} source nodes")
    F = H.size(1)
    Y = out if out is not None else torch.empty(view.n_rows, F, dtype=torch.float32, device=dev)
    argmax = mask = None
    if reduce == L.REDUCE_MAX:
        if mask_plan is not None:
            mask = torch.empty(max(mask_plan.nnz, 1), (F + 31) // 32, dtype=torch.int32,
                               device=dev)
        else:
            argmax = torch.empty(view.n_rows, F, dtype=torch.int32, device=dev)
    if bias is not None:
        bias = bias.detach().to(torch.float32).contiguous()
        if bias.numel() != F:
            raise ValueError(f"bias has {bias.numel()} entries, expected {F}")
    if _TIMER is not None:
        _TIMER("spmm_fwd", True, view.n_rows, view.edges)
    with L.device_guard(dev):
        rc = lib.mgcn_spmm_fwd(view.n_rows, F, L.ptr(view.rowptr), L.ptr(view.col),
                               L.ptr(view.eid), L.ptr(w), L.ptr(H), H.stride(0), L.ptr(Y),
                               Y.stride(0), reduce, L.ptr(bias), int(bool(relu)), L.ptr(argmax),
                               L.ptr(mask), L.ptr(relu_mask), L.ptr(view.order), view.n_heavy,
                               view.n_giant, L.stream_of(dev))
    if _TIMER is not None:
        _TIMER("spmm_fwd", False)
    L.check(rc, "mgcn_spmm_fwd")
    return Y, (mask if mask is not None else argmax)


# The fused kernels address the gathered table (X forward, dY backward) with
# 32-bit byte offsets: mgcn_spmm_xw_fwd / _bwd reject a table of more than
# 4 GiB - 16 bytes (fused.hip, the n_cols * ld * 4 checks), i.e. more than
# 8,388,607 rows at F = 128.  Larger graphs take the two-launch path, whose
# SpMM indexes with 64-bit offsets.
XW_MAX_TABLE_BYTES = 0xfffffff0


def spmm_xw_supported(view: CSRView, F_in: int, F_out: int, reduce: int,
                      ld: int | None = None) -> bool:
    """True when :func:`spmm_xw_fwd` (``view`` the fwd view, gathering [n_cols,
    F_in] rows of leading dimension ``ld``) or :func:`spmm_xw_bwd` (``view``
    the bwd view, gathering dY, F_in / F_out swapped) takes this layer:
    128 -> 128 or 256 -> 256, sum or mean, no heavy rows (skewed graphs keep
    the GEMM + heavy-row SpMM path); at 128 a gathered table within the
    kernels' 32-bit offsets (:data:`XW_MAX_TABLE_BYTES`; the 256-wide kernels
    give every gathered row a 64-bit base).  At 256 the backward is the
    dX-only form (:func:`xw_full_supported`)."""
    ld = int(F_in) if ld is None else max(int(ld), int(F_in))
    small = int(F_in) <= 128
    return (view.n_heavy == 0 and view.n_cols > 0 and
            (not small or view.n_cols * ld * 4 <= XW_MAX_TABLE_BYTES) and
            bool(L.load().mgcn_spmm_xw_supported(int(F_in), int(F_out), int(reduce))))


def xw_full_supported(F_in: int, F_out: int) -> bool:
    """mgcn_spmm_xw_bwd's dW-accumulating form (and its max adjoint): 128 x 128."""
    return bool(L.load().mgcn_spmm_xw_bwd_full_supported(int(F_in), int(F_out)))


def mask_words(F: int) -> int:
    """int32 ReLU mask words per row: 4 per 128 features (bit b of word
    4 (f >> 7) + v <-> feature f = 128 (f >> 7) + 4 b + v)."""
    return 4 * ((int(F) + 127) // 128)


def layer_fusable(plan: GraphPlan, x: torch.Tensor, W: torch.Tensor, reduce: int) -> bool:
    """Both directions of a layer on ``plan`` fit the fused kernels: the
    forward gathers x over the fwd view, the backward dY over the bwd view."""
    return (x.dim() == 2 and x.dtype == torch.float32 and W.dtype == torch.float32 and
            x.is_cuda and x.size(0) == plan.fwd.n_cols == plan.fwd.n_rows and
            spmm_xw_supported(plan.fwd, W.size(0), W.size(1), reduce, x.stride(0)) and
            spmm_xw_supported(plan.bwd, W.size(1), W.size(0), L.REDUCE_SUM))


def spmm_xw_fwd(view: CSRView, w: torch.Tensor | None, X: torch.Tensor, W: torch.Tensor,
                reduce: int, bias: torch.Tensor | None = None, relu: bool = False,
                relu_mask: torch.Tensor | None = None, want_z: bool = False,
                out: torch.Tensor | None = None, z_out: torch.Tensor | None = None):
    """Y = epi((reduce_k X[col_k] * w_k) @ W + bias) in one launch
    (``mgcn_spmm_xw_fwd``): the layer's GEMM fused behind its aggregation, so
    X @ W is never written.  Sum / mean only (they commute with W).  With
    ``want_z`` returns (Y, Z): Z = the aggregated rows before W (for mean
    before the division), from which the backward forms dW = Z^T dY.
    ``out`` / ``z_out``: [n_rows, F] row-major buffers (16-byte aligned rows)
    to write Y / Z into instead of new tensors.  ``X`` may be a
    :class:`PackedTable` (128- or 256-wide layers; the view's columns then
    are packed positions): the rows are gathered from the packed exchange buffers in
    place (``mgcn_spmm_xw_fwd_packed``), bit for bit the dense table's result."""
    lib = L.load()
    packed = isinstance(X, PackedTable)
    if not packed:
        X = _contig_f32(X, "X")
        if X.stride(0) % 4 or X.data_ptr() % 16:
            X = X.contiguous()
    W = W.detach()
    dev = L.require_device(X.words if packed else X, W, view.rowptr, w, bias, relu_mask)
    F_in, F_out = W.shape
    if packed:
        if X.F != F_in:
            raise ValueError(f"spmm_xw_fwd: packed table of F = {X.F}, W is [{F_in}, {F_out}]")
    elif X.size(0) != view.n_cols:
        raise ValueError(f"X has {X.size(0)} rows, graph has {view.n_cols} source nodes")
    elif X.size(1) != F_in:
        raise ValueError(f"spmm_xw_fwd: X is [{X.size(0)}, {X.size(1)}], W is [{F_in}, {F_out}]")
    if W.dtype != torch.float32 or W.stride(1) != 1:
        W = W.to(torch.float32).contiguous()
    if bias is not None:
        bias = bias.detach().to(torch.float32).contiguous()
        if bias.numel() != F_out:
            raise ValueError(f"bias has {bias.numel()} entries, expected {F_out}")
    if relu_mask is not None:
        # the kernel writes n_rows x 16 B of mask words through this pointer
        if not relu:
            raise ValueError("spmm_xw_fwd: relu_mask needs relu")
        mw = mask_words(F_out)
        if (relu_mask.shape != (view.n_rows, mw) or relu_mask.dtype != torch.int32 or
                not relu_mask.is_contiguous() or relu_mask.data_ptr() % 16):
            raise ValueError(f"spmm_xw_fwd: relu_mask must be a contiguous, 16-byte aligned "
                             f"int32 [{view.n_rows}, {mw}] tensor")
    Y = out if out is not None else torch.empty(view.n_rows, F_out, dtype=torch.float32,
                                                device=dev)
    Z = None
    if want_z:
        Z = z_out if z_out is not None else torch.empty(view.n_rows, F_in, dtype=torch.float32,
                                                        device=dev)
    for name, t, f in (("out", Y, F_out), ("z_out", Z, F_in)):
        if t is not None and (t.dtype != torch.float32 or t.dim() != 2 or t.size(0) != view.n_rows
                              or t.size(1) != f or t.stride(1) != 1 or t.stride(0) % 4
                              or t.data_ptr() % 16):
            raise ValueError(f"spmm_xw_fwd: {name} must be float32 [{view.n_rows}, {f}] with "
                             f"16-byte aligned rows")
    ws_bytes = int(lib.mgcn_spmm_xw_fwd_workspace_bytes(F_in, F_out))
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev) if ws_bytes else None
    tname = ("spmm_xw_fwd_z" if want_z else "spmm_xw_fwd") + ("_pk" if packed else "")
    if _TIMER is not None:
        _TIMER(tname, True, view.n_rows, view.edges)
    with L.device_guard(dev):
        if packed:
            pk = X.c_struct()
            rc = lib.mgcn_spmm_xw_fwd_packed(view.n_rows, F_in, F_out, L.ptr(view.rowptr),
                                             L.ptr(view.col), L.ptr(w), L.byref(pk), L.ptr(W),
                                             W.stride(0), L.ptr(bias), L.ptr(Y), Y.stride(0),
                                             reduce, int(bool(relu)), L.ptr(relu_mask), L.ptr(Z),
                                             Z.stride(0) if Z is not None else 0, L.ptr(ws),
                                             ws_bytes, L.stream_of(dev))
        else:
            rc = lib.mgcn_spmm_xw_fwd(view.n_rows, view.n_cols, F_in, F_out, L.ptr(view.rowptr),
                                      L.ptr(view.col), L.ptr(w), L.ptr(X), X.stride(0), L.ptr(W),
                                      W.stride(0), L.ptr(bias), L.ptr(Y), Y.stride(0), reduce,
                                      int(bool(relu)), L.ptr(relu_mask), L.ptr(Z),
                                      Z.stride(0) if Z is not None else 0, L.ptr(ws), ws_bytes,
                                      L.stream_of(dev))
    if _TIMER is not None:
        _TIMER(tname, False)
    L.check(rc, "mgcn_spmm_xw_fwd_packed" if packed else "mgcn_spmm_xw_fwd")
    return (Y, Z) if want_z else Y


def spmm_xw_bwd(view_t: CSRView, w_t: torch.Tensor | None, row_scale: torch.Tensor | None,
                dY: torch.Tensor, X: torch.Tensor, W: torch.Tensor, want_dx: bool = True,
                relu_mask: torch.Tensor | None = None, row_div: torch.Tensor | None = None,
                win_mask: torch.Tensor | None = None, slot_map: torch.Tensor | None = None,
                dx_out: torch.Tensor | None = None, colsum_acc: torch.Tensor | None = None,
                dy_colsum_out: torch.Tensor | None = None):
    """Both adjoints of a 128 -> 128 layer from one pass (``mgcn_spmm_xw_bwd``):
    dH = A^T dY [* row_scale] stays on chip, and dW = X^T dH, dX = dH W^T
    (with the lower layer's ReLU mask / row divisor / bias column sums, as
    :func:`gemm_bwd`) are formed from it.  Max: ``win_mask`` (the forward's
    winner bits, :func:`spmm_fwd` with ``mask_plan``) and the plan's
    ``slot_map`` route dY as :func:`spmm_bwd` does.  ``dy_colsum_out`` (a
    float32 [F_out] tensor; the dW + dX form of a whole square graph, no max)
    receives the column sums of dY itself -- the layer's own bias gradient --
    from the same launch (``mgcn_spmm_xw_bwd_hcs``).  Returns
    (dW, dX or None, colsum or None).  ``dY`` may be a :class:`PackedTable`
    (128- or 256-wide, dX-only form X = None; ``mgcn_spmm_xw_bwd_packed``)."""
    lib = L.load()
    if isinstance(dY, PackedTable):
        return _spmm_xw_bwd_packed(view_t, w_t, row_scale, dY, X, W, want_dx, relu_mask, row_div,
                                   win_mask, dx_out, colsum_acc, dy_colsum_out)
    dY = _contig_f32(dY, "dY")
    if dY.stride(0) % 4 or dY.data_ptr() % 16:
        dY = dY.contiguous()
    dx_only = X is None  # dW formed by the caller (Z^T dY, :func:`gemm_bwd`)
    if not dx_only:
        X = _contig_f32(X, "X")
        if X.stride(0) % 4 or X.data_ptr() % 16:
            X = X.contiguous()
    W = W.detach()
    # (the warp-specialised adjoint copies W into LDS with 16-byte loads)
    if W.dtype != torch.float32 or W.stride(1) != 1 or W.stride(0) % 4 or W.data_ptr() % 16:
        W = W.to(torch.float32).contiguous()
    dev = L.require_device(dY, X, W, view_t.rowptr, w_t, row_scale, relu_mask, row_div)
    F_in, F_out = W.shape
    M = view_t.n_rows if dx_only else X.size(0)
    if dx_only and (not want_dx or win_mask is not None):
        raise ValueError("spmm_xw_bwd: X=None (dX only) needs want_dx and no win_mask")
    if (not dx_only and X.size(1) != F_in) or M != view_t.n_rows or \
            dY.size(0) != view_t.n_cols or dY.size(1) != F_out:
        raise ValueError(f"spmm_xw_bwd: X {None if dx_only else tuple(X.shape)}, dY "
                         f"{tuple(dY.shape)} do not fit the "
                         f"graph ({view_t.n_rows} sources, {view_t.n_cols} destinations)")
    if (win_mask is None) != (slot_map is None):
        raise ValueError("spmm_xw_bwd: win_mask and slot_map go together (max adjoint)")
    if win_mask is not None and (win_mask.dtype != torch.int32 or win_mask.dim() != 2
                                 or win_mask.size(1) != (F_out + 31) // 32):
        raise ValueError("spmm_xw_bwd: win_mask must be int32 [nnz, ceil(F/32)]")
    dW = None if dx_only else torch.empty(F_in, F_out, dtype=torch.float32, device=dev)
    dX = None
    if want_dx:
        dX = dx_out if dx_out is not None else torch.empty(M, F_in, dtype=torch.float32,
                                                           device=dev)
        if (dX.dtype != torch.float32 or dX.dim() != 2 or tuple(dX.shape) != (M, F_in) or
                dX.stride(1) != 1 or dX.stride(0) < F_in):
            raise ValueError(f"spmm_xw_bwd: dx_out must be float32 [{M}, {F_in}], row-major")
    colsum = None
    if relu_mask is not None:
        if not want_dx:
            raise ValueError("spmm_xw_bwd: relu_mask needs want_dx")
        mw = mask_words(F_in)
        if relu_mask.shape != (M, mw) or relu_mask.dtype != torch.int32:
            raise ValueError(f"spmm_xw_bwd: relu_mask must be int32 [{M}, {mw}]")
        relu_mask = relu_mask.contiguous()
        if colsum_acc is not None:
            if not dx_only or colsum_acc.dtype != torch.float32 or \
                    tuple(colsum_acc.shape) != (F_in,) or not colsum_acc.is_contiguous():
                raise ValueError(f"spmm_xw_bwd: colsum_acc must be a contiguous float32 [{F_in}] "
                                 f"tensor (dX-only form)")
            L.require_device(colsum_acc)
            colsum = colsum_acc
        else:
            colsum = torch.empty(F_in, dtype=torch.float32, device=dev)
    elif colsum_acc is not None:
        raise ValueError("spmm_xw_bwd: colsum_acc needs relu_mask")
    acc_flag = 1 if colsum_acc is not None else 0
    if dy_colsum_out is not None:
        if (dx_only or not want_dx or win_mask is not None or view_t.n_rows != view_t.n_cols or
                dy_colsum_out.dtype != torch.float32 or
                tuple(dy_colsum_out.shape) != (F_out,) or not dy_colsum_out.is_contiguous()):
            raise ValueError("spmm_xw_bwd: dy_colsum_out needs the dW + dX form of a square "
                             f"graph (no max) and a contiguous float32 [{F_out}] tensor")
        L.require_device(dy_colsum_out)
    ws_bytes = int(lib.mgcn_spmm_xw_bwd_workspace_bytes(M, F_in, F_out))
    ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
    tname = "spmm_xw_bwd_dx" if dx_only else "spmm_xw_bwd" if want_dx else "spmm_xw_bwd_dw"
    if _TIMER is not None:
        _TIMER(tname, True, view_t.n_rows, view_t.edges)
    if dy_colsum_out is not None:
        with L.device_guard(dev):
            rc = lib.mgcn_spmm_xw_bwd_hcs(M, view_t.n_cols, L.ptr(view_t.rowptr), L.ptr(view_t.col),
                                          L.ptr(w_t), L.ptr(row_scale), L.ptr(dY), dY.stride(0),
                                          L.ptr(X), X.stride(0), L.ptr(W), W.stride(0), L.ptr(dW),
                                          dW.stride(0), 0, L.ptr(dX), dX.stride(0),
                                          L.ptr(relu_mask), L.ptr(row_div), L.ptr(colsum),
                                          L.ptr(dy_colsum_out), L.ptr(ws), ws_bytes,
                                          L.stream_of(dev))
        if _TIMER is not None:
            _TIMER(tname, False)
        L.check(rc, "mgcn_spmm_xw_bwd_hcs")
        return dW, dX, colsum
    with L.device_guard(dev):
        rc = lib.mgcn_spmm_xw_bwd(M, view_t.n_cols, F_in, F_out, L.ptr(view_t.rowptr),
                                  L.ptr(view_t.col), L.ptr(w_t), L.ptr(row_scale), L.ptr(dY),
                                  dY.stride(0), L.ptr(X), 0 if dx_only else X.stride(0),
                                  L.ptr(W), W.stride(0), L.ptr(dW),
                                  0 if dx_only else dW.stride(0), acc_flag, L.ptr(dX),
                                  dX.stride(0) if dX is not None else 0, L.ptr(relu_mask),
                                  L.ptr(row_div), L.ptr(colsum), L.ptr(win_mask),
                                  L.ptr(slot_map), L.ptr(ws), ws_bytes, L.stream_of(dev))
    if _TIMER is not None:
        _TIMER(tname, False)
    L.check(rc, "mgcn_spmm_xw_bwd")
    return dW, dX, colsum


def _spmm_xw_bwd_packed(view_t, w_t, row_scale, dY, X, W, want_dx, relu_mask, row_div,
                        win_mask, dx_out, colsum_acc, dy_colsum_out):
    """:func:`spmm_xw_bwd`'s dX-only form gathering dY from a PackedTable."""
    lib = L.load()
    if X is not None or not want_dx or win_mask is not None or dy_colsum_out is not None:
        raise ValueError("spmm_xw_bwd: a packed dY takes the dX-only form (X = None, no max)")
    W = W.detach()
    if W.dtype != torch.float32 or W.stride(1) != 1 or W.stride(0) % 4 or W.data_ptr() % 16:
        W = W.to(torch.float32).contiguous()
    dev = L.require_device(dY.words, W, view_t.rowptr, w_t, row_scale, relu_mask, row_div)
    F_in, F_out = W.shape
    M = view_t.n_rows
    if dY.F != F_out:
        raise ValueError(f"spmm_xw_bwd: packed dY of F = {dY.F}, W is [{F_in}, {F_out}]")
    dX = dx_out if dx_out is not None else torch.empty(M, F_in, dtype=torch.float32, device=dev)
    if (dX.dtype != torch.float32 or dX.dim() != 2 or tuple(dX.shape) != (M, F_in) or
            dX.stride(1) != 1 or dX.stride(0) % 4 or dX.data_ptr() % 16):
        raise ValueError(f"spmm_xw_bwd: dx_out must be float32 [{M}, {F_in}], 16-byte rows")
    colsum = None
    if relu_mask is not None:
        mw = mask_words(F_in)
        if relu_mask.shape != (M, mw) or relu_mask.dtype != torch.int32:
            raise ValueError(f"spmm_xw_bwd: relu_mask must be int32 [{M}, {mw}]")
        relu_mask = relu_mask.contiguous()
        colsum = colsum_acc if colsum_acc is not None else torch.empty(F_in, dtype=torch.float32,
                                                                         device=dev)
    elif colsum_acc is not None:
        raise ValueError("spmm_xw_bwd: colsum_acc needs relu_mask")
    ws_bytes = int(lib.mgcn_spmm_xw_bwd_workspace_bytes(M, F_in, F_out))
    ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
    if _TIMER is not None:
        _TIMER("spmm_xw_bwd_dx_pk", True, view_t.n_rows, view_t.edges)
    pk = dY.c_struct()
    with L.device_guard(dev):
        rc = lib.mgcn_spmm_xw_bwd_packed(M, F_in, F_out, L.ptr(view_t.rowptr), L.ptr(view_t.col),
                                         L.ptr(w_t), L.ptr(row_scale), L.byref(pk), L.ptr(W),
                                         W.stride(0), L.ptr(dX), dX.stride(0), L.ptr(relu_mask),
                                         L.ptr(row_div), L.ptr(colsum),
                                         1 if colsum_acc is not None else 0, L.ptr(ws), ws_bytes,
                                         L.stream_of(dev))
    if _TIMER is not None:
        _TIMER("spmm_xw_bwd_dx_pk", False)
    L.check(rc, "mgcn_spmm_xw_bwd_packed")
    return None, dX, colsum


def spmm_bwd(view_t: CSRView, w_t: torch.Tensor | None, row_scale: torch.Tensor | None,
             dY: torch.Tensor, reduce: int, cnt: torch.Tensor | None = None,
             argmax: torch.Tensor | None = None, out: torch.Tensor | None = None,
             accumulate: bool = False, win_mask: torch.Tensor | None = None,
             slot_map: torch.Tensor | None = None) -> torch.Tensor:
    """dH[view_t.n_rows, F] = sum_k g(dY[col_k]) * w_k  [* row_scale]."""
    lib = L.load()
    dY = _contig_f32(dY, "dY")
    dev = L.require_device(dY, view_t.rowptr, w_t, row_scale)
    F = dY.size(1)
    dH = out if out is not None else torch.empty(view_t.n_rows, F, dtype=torch.float32,
                                                 device=dev)
    if _TIMER is not None:
        _TIMER("spmm_bwd", True, view_t.n_rows, view_t.edges)
    with L.device_guard(dev):
        rc = lib.mgcn_spmm_bwd(view_t.n_rows, F, L.ptr(view_t.rowptr), L.ptr(view_t.col),
                               L.ptr(view_t.eid), L.ptr(w_t), L.ptr(row_scale), L.ptr(dY),
                               dY.stride(0), L.ptr(dH), dH.stride(0), reduce, L.ptr(cnt),
                               L.ptr(argmax), L.ptr(win_mask), L.ptr(slot_map),
                               int(bool(accumulate)),
                               L.ptr(view_t.order),
                               view_t.n_heavy, view_t.n_giant, L.stream_of(dev))
    if _TIMER is not None:
        _TIMER("spmm_bwd", False)
    L.check(rc, "mgcn_spmm_bwd")
    return dH


def relu_bwd_colsum(dZ: torch.Tensor, Z: torch.Tensor | None, relu: bool, want_db: bool,
                    row_div: torch.Tensor | None = None):
    """(dY, db): dY = Z > 0 ? dZ : 0 (dZ itself when not relu), divided by
    ``row_div`` per row when given (mean aggregation); db = sum_i of the
    undivided dY."""
    lib = L.load()
    dZ = dZ.contiguous()
    dev = L.require_device(dZ, Z, row_div)
    n, F = dZ.shape
    write = relu or row_div is not None
    dY = torch.empty_like(dZ) if write else dZ
    db = torch.empty(F, dtype=torch.float32, device=dev) if want_db else None
    if not write and not want_db:
        return dY, None
    ws_bytes = int(lib.mgcn_colsum_workspace_bytes(n, F)) if want_db else 0
    ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev) if want_db else None
    if _TIMER is not None:
        _TIMER("relu_bwd_colsum", True, n)
    with L.device_guard(dev):
        rc = lib.mgcn_relu_bwd_colsum(n, F, L.ptr(dZ), L.ptr(Z.contiguous() if relu else None),
                                      int(bool(relu)), L.ptr(row_div), L.ptr(dY if write else None),
                                      L.ptr(db),
                                      L.ptr(ws), ws_bytes, L.stream_of(dev))
    if _TIMER is not None:
        _TIMER("relu_bwd_colsum", False)
    L.check(rc, "mgcn_relu_bwd_colsum")
    return dY, db


def gemm_tn(A: torch.Tensor, B: torch.Tensor, out: torch.Tensor | None = None,
            accumulate: bool = False) -> torch.Tensor:
    """C = A^T B on fp32 MFMA with split-K (libmgcn ``mgcn_gemm_tn``)."""
    lib = L.load()
    A = _contig_f32(A, "A")
    B = _contig_f32(B, "B")
    dev = L.require_device(A, B)
    K, M = A.shape
    if B.size(0) != K:
        raise ValueError(f"gemm_tn: A has {K} rows, B has {B.size(0)}")
    N = B.size(1)
    C = out if out is not None else torch.empty(M, N, dtype=torch.float32, device=dev)
    ws_bytes = int(lib.mgcn_gemm_tn_workspace_bytes(K, M, N))
    ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
    if _TIMER is not None:
        _TIMER("gemm_tn", True, K)
    with L.device_guard(dev):
        rc = lib.mgcn_gemm_tn(K, M, N, L.ptr(A), A.stride(0), L.ptr(B), B.stride(0), L.ptr(C),
                              C.stride(0), int(bool(accumulate)), L.ptr(ws), ws_bytes,
                              L.stream_of(dev))
    if _TIMER is not None:
        _TIMER("gemm_tn", False)
    L.check(rc, "mgcn_gemm_tn")
    return C


def gemm_tn_split(A: torch.Tensor, B: torch.Tensor, n1: int):
    """(C1, C2t) with A^T B = [C1 | C2t^T]: columns [0, n1) as C1 [M, n1],
    the rest transposed as C2t [N - n1, M], both contiguous, from one
    ``mgcn_gemm_tn_split`` pass (two parameter gradients in their own
    layouts, no copies)."""
    lib = L.load()
    A = _contig_f32(A, "A")
    B = _contig_f32(B, "B")
    dev = L.require_device(A, B)
    K, M = A.shape
    N = B.size(1)
    if B.size(0) != K or not 0 <= n1 <= N:
        raise ValueError(f"gemm_tn_split: A {tuple(A.shape)}, B {tuple(B.shape)}, n1 {n1}")
    C1 = torch.empty(M, n1, dtype=torch.float32, device=dev)
    C2 = torch.empty(N - n1, M, dtype=torch.float32, device=dev)
    ws_bytes = int(lib.mgcn_gemm_tn_workspace_bytes(K, M, N))
    ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
    if _TIMER is not None:
        _TIMER("gemm_tn", True, K)
    with L.device_guard(dev):
        rc = lib.mgcn_gemm_tn_split(K, M, N, n1, L.ptr(A), A.stride(0), L.ptr(B), B.stride(0),
                                    L.ptr(C1), max(n1, 1), L.ptr(C2), max(M, 1), 0, L.ptr(ws),
                                    ws_bytes, L.stream_of(dev))
    if _TIMER is not None:
        _TIMER("gemm_tn", False)
    L.check(rc, "mgcn_gemm_tn_split")
    return C1, C2


def gemm_nn_supported(K: int, N: int) -> bool:
    return bool(L.load().mgcn_gemm_nn_supported(int(K), int(N)))


def gemm_nn_epi_supported(K: int, N: int) -> bool:
    """The fused ReLU-mask / bias-gradient epilogue of mgcn_gemm_nn (the tuned
    kernel, N <= 128)."""
    return bool(L.load().mgcn_gemm_nn_epi_supported(int(K), int(N)))


def make_relu_mask(Z: torch.Tensor) -> torch.Tensor:
    """int32 [rows, 4]: bit b of word v set iff Z[i, 4 b + v] > 0 (F <= 128;
    ``mgcn_relu_mask``)."""
    lib = L.load()
    Z = _contig_f32(Z, "Z")
    dev = L.require_device(Z)
    n, F = Z.shape
    m = torch.empty(n, 4, dtype=torch.int32, device=dev)
    with L.device_guard(dev):
        rc = lib.mgcn_relu_mask(n, F, L.ptr(Z), Z.stride(0), L.ptr(m), L.stream_of(dev))
    L.check(rc, "mgcn_relu_mask")
    return m


def gemm_nn(A: torch.Tensor, W: torch.Tensor, transpose_w: bool = False,
            Z: torch.Tensor | None = None, row_div: torch.Tensor | None = None,
            relu_mask: torch.Tensor | None = None):
    """C = A @ W (or A @ W^T) on libmgcn's tall-skinny MFMA kernel
    (``mgcn_gemm_nn``).  With ``relu_mask`` (from :func:`spmm_fwd` or
    :func:`make_relu_mask`) or ``Z``: C = Z > 0 ? A @ W^T : 0 and the column sums
    of C are returned too (fused ReLU backward + bias gradient).  Returns
    (C, colsum or None)."""
    lib = L.load()
    A = _contig_f32(A, "A")
    if A.stride(0) % 4 or A.data_ptr() % 16:
        A = A.contiguous()
    W = W.detach()
    dev = L.require_device(A, W, Z, relu_mask)
    if relu_mask is None and Z is not None:
        relu_mask = make_relu_mask(Z)
    M, K = A.shape
    if transpose_w:
        N, Kw = W.shape
        sbk, sbn = W.stride(1), W.stride(0)
    else:
        Kw, N = W.shape
        sbk, sbn = W.stride(0), W.stride(1)
    if Kw != K:
        raise ValueError(f"gemm_nn: A is [{M}, {K}], W gives K = {Kw}")
    C = torch.empty(M, N, dtype=torch.float32, device=dev)
    colsum = ws = None
    ws_bytes = 0
    if relu_mask is not None:
        if relu_mask.shape != (M, 4) or relu_mask.dtype != torch.int32:
            raise ValueError(f"gemm_nn: relu_mask must be int32 [{M}, 4]")
        relu_mask = relu_mask.contiguous()
        colsum = torch.empty(N, dtype=torch.float32, device=dev)
        ws_bytes = int(lib.mgcn_gemm_nn_workspace_bytes(M, N))
        ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
    if _TIMER is not None:
        _TIMER("gemm_nn", True, M)
    with L.device_guard(dev):
        rc = lib.mgcn_gemm_nn(M, K, N, L.ptr(A), A.stride(0), L.ptr(W), sbk, sbn, L.ptr(C),
                              C.stride(0), L.ptr(relu_mask),
                              L.ptr(row_div), L.ptr(colsum), L.ptr(ws), ws_bytes,
                              L.stream_of(dev))
    if _TIMER is not None:
        _TIMER("gemm_nn", False)
    L.check(rc, "mgcn_gemm_nn")
    return C, colsum


def gemm_bwd_supported(F_in: int, F_out: int) -> bool:
    return bool(L.load().mgcn_gemm_bwd_supported(int(F_in), int(F_out)))


def gemm_bwd(x: torch.Tensor, dH: torch.Tensor, W: torch.Tensor, want_dx: bool = True,
             relu_mask: torch.Tensor | None = None, row_div: torch.Tensor | None = None,
             dW_out: torch.Tensor | None = None, accumulate: bool = False,
             dh_colsum: bool = False):
    """Both adjoints of H = x @ W in one pass (``mgcn_gemm_bwd``, F_in = F_out
    = 128): dW = x^T dH and dX = dH W^T -- with ``relu_mask`` the lower
    layer's ReLU backward and bias-gradient column sums fused as in
    :func:`gemm_nn`.  ``dh_colsum`` (dW only): colsum = the column sums of dH
    (a bias gradient) from the same pass.  Returns (dW, dX or None, colsum or
    None)."""
    lib = L.load()
    x = _contig_f32(x, "x")
    dH = _contig_f32(dH, "dH")
    if x.stride(0) % 4 or x.data_ptr() % 16:
        x = x.contiguous()
    if dH.stride(0) % 4 or dH.data_ptr() % 16:
        dH = dH.contiguous()
    W = W.detach().contiguous()
    dev = L.require_device(x, dH, W, relu_mask, row_div)
    M, F_in = x.shape
    F_out = dH.size(1)
    if dH.size(0) != M or tuple(W.shape) != (F_in, F_out):
        raise ValueError(f"gemm_bwd: x {tuple(x.shape)}, dH {tuple(dH.shape)}, W {tuple(W.shape)}")
    dW = dW_out if dW_out is not None else torch.empty(F_in, F_out, dtype=torch.float32,
                                                       device=dev)
    dX = torch.empty(M, F_in, dtype=torch.float32, device=dev) if want_dx else None
    colsum = None
    if dh_colsum:
        if want_dx or relu_mask is not None:
            raise ValueError("gemm_bwd: dh_colsum is the dW-only form's")
        colsum = torch.empty(F_out, dtype=torch.float32, device=dev)
    if relu_mask is not None:
        if not want_dx:
            raise ValueError("gemm_bwd: relu_mask needs want_dx")
        if relu_mask.shape != (M, 4) or relu_mask.dtype != torch.int32:
            raise ValueError(f"gemm_bwd: relu_mask must be int32 [{M}, 4]")
        relu_mask = relu_mask.contiguous()
        colsum = torch.empty(F_in, dtype=torch.float32, device=dev)
    ws_bytes = int(lib.mgcn_gemm_bwd_workspace_bytes(M, F_in, F_out))
    ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
    if _TIMER is not None:
        _TIMER("gemm_bwd" if want_dx else "gemm_bwd_dw", True, M)
    with L.device_guard(dev):
        rc = lib.mgcn_gemm_bwd(M, F_in, F_out, L.ptr(x), x.stride(0), L.ptr(dH), dH.stride(0),
                               L.ptr(W), W.stride(0), L.ptr(dW), dW.stride(0),
                               int(bool(accumulate)), L.ptr(dX),
                               dX.stride(0) if dX is not None else F_in, L.ptr(relu_mask),
                               L.ptr(row_div), L.ptr(colsum), L.ptr(ws), ws_bytes,
                               L.stream_of(dev))
    if _TIMER is not None:
        _TIMER("gemm_bwd" if want_dx else "gemm_bwd_dw", False)
    L.check(rc, "mgcn_gemm_bwd")
    return dW, dX, colsum


def dw_pass_supported(F_in: int, F_out: int) -> bool:
    """The dense dW = Z^T dY pass of the reassociated backward: mgcn_gemm_bwd
    (dW-only) at 128 x 128, mgcn_gemm_tn (bf16x6, 128 x 128 output tiles)
    for other multiples of 128 (256 x 256: config 5)."""
    return gemm_bwd_supported(F_in, F_out) or (int(F_in) % 128 == 0 and int(F_out) % 128 == 0)


def dw_pass_cs(Z: torch.Tensor, dY: torch.Tensor, S: torch.Tensor):
    """(dW = Z^T dY, the column sums of S) in one pass (``mgcn_gemm_bwd_dw_cs``,
    128 x 128): S [M, 128] is streamed beside Z and dY -- a stack's top-layer
    bias gradient folded into its bottom layer's dW pass."""
    lib = L.load()
    Z = _contig_f32(Z, "Z")
    dY = _contig_f32(dY, "dY")
    S = _contig_f32(S, "S")
    for name, t in (("Z", Z), ("dY", dY), ("S", S)):
        if t.dim() != 2 or t.size(1) != 128 or t.stride(0) % 4 or t.data_ptr() % 16:
            raise ValueError(f"dw_pass_cs: {name} must be a [M, 128] float32 with 16-byte rows")
    M = Z.size(0)
    if dY.size(0) != M or S.size(0) != M:
        raise ValueError(f"dw_pass_cs: Z, dY, S rows {M}, {dY.size(0)}, {S.size(0)}")
    dev = L.require_device(Z, dY, S)
    dW = torch.empty(128, 128, dtype=torch.float32, device=dev)
    scs = torch.empty(128, dtype=torch.float32, device=dev)
    ws_bytes = int(lib.mgcn_gemm_bwd_dw_cs_workspace_bytes(M))
    ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
    if _TIMER is not None:
        _TIMER("gemm_bwd_dw_cs", True, M)
    with L.device_guard(dev):
        rc = lib.mgcn_gemm_bwd_dw_cs(M, L.ptr(Z), Z.stride(0), L.ptr(dY), dY.stride(0), L.ptr(dW),
                                     dW.stride(0), 0, None, L.ptr(S), S.stride(0), L.ptr(scs),
                                     L.ptr(ws), ws_bytes, L.stream_of(dev))
    if _TIMER is not None:
        _TIMER("gemm_bwd_dw_cs", False)
    L.check(rc, "mgcn_gemm_bwd_dw_cs")
    return dW, scs


def dw_pass(Z: torch.Tensor, dY: torch.Tensor, W: torch.Tensor, dh_colsum: bool = False):
    """(dW = Z^T dY, the column sums of dY or None) -- :func:`dw_pass_supported`."""
    if gemm_bwd_supported(W.size(0), W.size(1)):
        dW, _, cs = gemm_bwd(Z, dY, W, want_dx=False, dh_colsum=dh_colsum)
        return dW, cs
    dW = gemm_tn(Z, dY)
    cs = relu_bwd_colsum(dY, None, False, True)[1] if dh_colsum else None
    return dW, cs


SMALL_K = 8  # mgcn_gemm_small_k: K <= 8, N <= 128


def gemm_small_k(A: torch.Tensor, W: torch.Tensor, transpose_w: bool = False) -> torch.Tensor:
    """A @ W (or A @ W^T) for a contraction of at most SMALL_K features
    (``mgcn_gemm_small_k``: k-ordered fma, HBM-bound)."""
    lib = L.load()
    A = _contig_f32(A, "A")
    W = W.detach().to(torch.float32)
    dev = L.require_device(A, W)
    K = A.size(1)
    N = W.size(0) if transpose_w else W.size(1)
    if (W.size(1) if transpose_w else W.size(0)) != K:
        raise ValueError(f"gemm_small_k: A {tuple(A.shape)}, W {tuple(W.shape)}")
    sbk, sbn = (W.stride(1), W.stride(0)) if transpose_w else (W.stride(0), W.stride(1))
    C = torch.empty(A.size(0), N, dtype=torch.float32, device=dev)
    with L.device_guard(dev):
        rc = lib.mgcn_gemm_small_k(A.size(0), K, N, L.ptr(A), A.stride(0), L.ptr(W), sbk, sbn,
                                   L.ptr(C), C.stride(0), L.stream_of(dev))
    L.check(rc, "mgcn_gemm_small_k")
    return C


# Dense products that left libmgcn for torch.matmul (hipBLASLt), by shape:
# only non-2-D or non-fp32 operands do (every 2-D fp32 shape has a libmgcn
# kernel since ABI v15).  tests/test_host.py holds configs 2-4 to zero.
VENDOR_GEMMS: "Counter[tuple]" = Counter()


def mm_route(K: int, N: int, dim: int = 2, dtype=torch.float32) -> str:
    """Which kernel takes C[M, N] = A[M, K] B[K, N]: 'nn' (mgcn_gemm_nn: the
    tuned kernel for K in {32, 64, 128, 256}, the generic tiled one for the
    rest), 'small_k' (mgcn_gemm_small_k: K <= SMALL_K, N <= 128, k-ordered
    fma) or 'vendor' (torch.matmul: non-2-D / non-fp32 operands only)."""
    if dim != 2 or dtype != torch.float32 or K < 1 or N < 1:
        return "vendor"
    if K <= SMALL_K and N <= 128:
        return "small_k"
    return "nn"


def _mm(x: torch.Tensor, W: torch.Tensor) -> torch.Tensor:
    """x @ W on libmgcn (:func:`mm_route`)."""
    route = mm_route(W.size(0), W.size(1), x.dim(), x.dtype if W.dtype == torch.float32 else None)
    if route == "nn":
        return gemm_nn(x, W)[0]
    if route == "small_k":
        return gemm_small_k(x, W)
    VENDOR_GEMMS[("mm", tuple(x.shape), tuple(W.shape), str(x.dtype))] += 1
    return torch.matmul(x, W.detach())


def _mm_t(dH: torch.Tensor, W: torch.Tensor) -> torch.Tensor:
    """dH @ W^T on libmgcn (:func:`mm_route`)."""
    route = mm_route(W.size(1), W.size(0), dH.dim(),
                     dH.dtype if W.dtype == torch.float32 else None)
    if route == "nn":
        return gemm_nn(dH, W, transpose_w=True)[0]
    if route == "small_k":
        return gemm_small_k(dH, W, transpose_w=True)
    VENDOR_GEMMS[("mm_t", tuple(dH.shape), tuple(W.shape), str(dH.dtype))] += 1
    return torch.matmul(dH, W.detach().t())


def _gemm_batched(A: torch.Tensor, B: torch.Tensor, C: torch.Tensor,
                  a_str, b_str, c_str, M: int, N: int, K: int, batch: int,
                  accumulate: bool = False) -> None:
    """C (+)= A B per batch through explicit (batch, row, col) element strides
    (``mgcn_gemm_batched``)."""
    lib = L.load()
    dev = L.require_device(A, B, C)
    with L.device_guard(dev):
        rc = lib.mgcn_gemm_batched(batch, M, N, K, L.ptr(A), *a_str, L.ptr(B), *b_str, L.ptr(C),
                                   *c_str, 1 if accumulate else 0, L.stream_of(dev))
    L.check(rc, "mgcn_gemm_batched")


def _bstr(t: torch.Tensor):
    """(batch, row, col) strides of a 3-D tensor or a broadcast 2-D one."""
    return (t.stride(0), t.stride(1), t.stride(2)) if t.dim() == 3 else (0, t.stride(0), t.stride(1))


class _Bmm(torch.autograd.Function):
    """a [B, M, K] @ b ([B, K, N] or a broadcast [K, N]) on mgcn_gemm_batched,
    with its adjoints dA = dC b^T, db = a^T dC (summed over the batch for a
    broadcast b) through transposed strides -- no copies."""

    @staticmethod
    def forward(ctx, a, b):
        Bn, M, K = a.shape
        N = b.shape[-1]
        out = torch.empty(Bn, M, N, dtype=torch.float32, device=a.device)
        _gemm_batched(a, b, out, _bstr(a), _bstr(b), _bstr(out), M, N, K, Bn)
        ctx.save_for_backward(a, b)
        return out

    @staticmethod
    def backward(ctx, dC):
        a, b = ctx.saved_tensors
        dC = dC.to(torch.float32)  # any strides: the kernel addresses them
        Bn, M, K = a.shape
        N = b.shape[-1]
        da = db = None
        if ctx.needs_input_grad[0]:
            da = torch.empty_like(a, memory_format=torch.contiguous_format)
            sb = _bstr(b)
            _gemm_batched(dC, b, da, _bstr(dC), (sb[0], sb[2], sb[1]), _bstr(da), M, K, N, Bn)
        if ctx.needs_input_grad[1]:
            sa = _bstr(a)
            if b.dim() == 3:
                db = torch.empty(Bn, K, N, dtype=torch.float32, device=a.device)
                _gemm_batched(a, dC, db, (sa[0], sa[2], sa[1]), _bstr(dC), _bstr(db), K, N, M, Bn)
            else:  # broadcast weight: one product over the flattened batch rows
                a2 = a.reshape(Bn * M, K)
                d2 = dC.reshape(Bn * M, N)
                db = torch.empty(K, N, dtype=torch.float32, device=a.device)
                _gemm_batched(a2, d2, db, (0, a2.stride(1), a2.stride(0)), (0, d2.stride(0),
                              d2.stride(1)), (0, db.stride(0), db.stride(1)), K, N, Bn * M, 1)
        return da, db


def bmm(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """Batched dense product of DiffPool's dense operators (PyG 1.3
    DenseSAGEConv / dense_diff_pool; reference kernel/diff_pool.py:13-14, 68,
    76): a [B, M, K] @ b [B, K, N] (or a [K, N] weight broadcast over the
    batch) on libmgcn's MFMA kernel, differentiable in both operands."""
    if a.dtype != torch.float32 or b.dtype != torch.float32:
        raise TypeError(f"bmm: float32 operands (the reference computes in fp32), got "
                        f"{a.dtype} @ {b.dtype}")
    if a.dim() != 3 or b.dim() not in (2, 3) or a.size(2) != b.size(-2) or \
            (b.dim() == 3 and b.size(0) != a.size(0)):
        raise ValueError(f"bmm: shapes {tuple(a.shape)} @ {tuple(b.shape)}")
    L.require_device(a, b)
    return _Bmm.apply(a, b)


class _Linear(torch.autograd.Function):
    """H = x @ W (gcn_base_models.py:201) with all three products on libmgcn's
    MFMA kernels: forward on mgcn_gemm_nn (tall-skinny); backward dW = x^T dH
    (a K = num_nodes reduction) and dX = dH W^T together in one pass of
    mgcn_gemm_bwd at F = 128, else mgcn_gemm_tn (split-K) + mgcn_gemm_nn."""

    @staticmethod
    def forward(ctx, x, W):
        ctx.save_for_backward(x, W)
        return _mm(x, W)

    @staticmethod
    def backward(ctx, dH):
        x, W = ctx.saved_tensors
        dx = dW = None
        dH = dH.contiguous()
        if ctx.needs_input_grad[1] and gemm_bwd_supported(W.size(0), W.size(1)):
            dW, dx, _ = gemm_bwd(x, dH, W, want_dx=bool(ctx.needs_input_grad[0]))
            return dx, dW
        if ctx.needs_input_grad[0]:
            dx = _mm_t(dH, W)
        if ctx.needs_input_grad[1]:
            dW = gemm_tn(x, dH)
        return dx, dW


class _LinearBias(torch.autograd.Function):
    """torch.nn.functional.linear(x, W, b) = x W^T + b with W [out, in] on the
    libmgcn GEMMs (dW = dy^T x is the K = num_nodes reduction that hipBLASLt
    runs at ~18 TFLOP/s: GCNModel's residual and final Linear layers,
    gcn_model.py:64-73)."""

    @staticmethod
    def forward(ctx, x, W, b):
        ctx.save_for_backward(x, W)
        ctx.has_b = b is not None
        y = _mm_t(x, W)
        return y.add_(b.detach()) if b is not None else y

    @staticmethod
    def backward(ctx, dy):
        x, W = ctx.saved_tensors
        dy = dy.contiguous()
        dx = dW = db = None
        if ctx.needs_input_grad[0]:
            dx = _mm(dy, W)
        if ctx.needs_input_grad[1]:
            dW = gemm_tn(dy, x)
        if ctx.has_b and ctx.needs_input_grad[2]:
            db = relu_bwd_colsum(dy, None, False, True)[1]
        return dx, dW, db


def linear_bias(x: torch.Tensor, W: torch.Tensor, b: torch.Tensor | None) -> torch.Tensor:
    """F.linear on libmgcn for 2-D fp32 inputs (other ranks / dtypes: torch's
    F.linear on the same HIP device).  CPU tensors raise: no CPU path."""
    L.require_device(x, W, b)
    if x.dim() != 2 or x.dtype != torch.float32:
        VENDOR_GEMMS[("linear", tuple(x.shape), tuple(W.shape), str(x.dtype))] += 1
        return torch.nn.functional.linear(x, W, b)
    return _LinearBias.apply(x, W, b)


def linear(x: torch.Tensor, W: torch.Tensor) -> torch.Tensor:
    """``torch.matmul(x, W)`` with the libmgcn weight-gradient kernel.  CPU
    tensors raise: no CPU path."""
    L.require_device(x, W)
    if x.dim() != 2 or x.dtype != torch.float32 or W.dtype != torch.float32:
        VENDOR_GEMMS[("matmul", tuple(x.shape), tuple(W.shape), str(x.dtype))] += 1
        return torch.matmul(x, W)
    return _Linear.apply(x, W)


def max_mask(plan: GraphPlan, argmax: torch.Tensor) -> torch.Tensor:
    """Winner bits of every edge at its fwd slot (mgcn_max_mask): int32
    [nnz, ceil(F/32)] (bit patterns), replacing argmax in the backward."""
    lib = L.load()
    F = argmax.size(1)
    W = (F + 31) // 32
    dev = argmax.device
    mask = torch.empty(max(plan.nnz, 1), W, dtype=torch.int32, device=dev)
    with L.device_guard(dev):
        rc = lib.mgcn_max_mask(plan.fwd.n_rows, F, L.ptr(plan.fwd.rowptr), L.ptr(plan.fwd.eid),
                               L.ptr(argmax), L.ptr(mask), L.stream_of(dev))
    L.check(rc, "mgcn_max_mask")
    return mask


class _Aggregate(torch.autograd.Function):
    """y = epi(A_norm (x) H) with bias and ReLU fused; see module docstring.
    Max saves the per-edge winner bits (max_mask), not the argmax rows."""

    @staticmethod
    def forward(ctx, H, bias, plan: GraphPlan, norm: NormPlan, reduce: int, relu: bool):
        Y, mask = spmm_fwd(plan.fwd, norm.w_fwd, H, reduce, bias, relu, mask_plan=plan)
        ctx.plan, ctx.norm, ctx.reduce, ctx.relu = plan, norm, reduce, relu
        ctx.has_bias = bias is not None
        ctx.save_for_backward(Y if relu else None, mask)  # max: winner bits per edge
        return Y

    @staticmethod
    def backward(ctx, dZ):
        Y, mask = ctx.saved_tensors
        plan, norm = ctx.plan, ctx.norm
        need_h = ctx.needs_input_grad[0]
        need_b = ctx.has_bias and ctx.needs_input_grad[1]
        mean = ctx.reduce == L.REDUCE_MEAN
        # mean: dY rows divided by their count once here (bitwise the same as
        # dividing every gathered copy), so the adjoint is a plain sum
        dY, db = relu_bwd_colsum(dZ, Y, ctx.relu, need_b,
                                 row_div=plan.in_cnt if (mean and need_h) else None)
        dH = None
        if need_h:
            dH = spmm_bwd(plan.bwd, norm.w_bwd, norm.row_scale_bwd, dY,
                          L.REDUCE_SUM if mean else ctx.reduce, win_mask=mask,
                          slot_map=plan.slot_map() if mask is not None else None)
        return dH, db, None, None, None, None


def aggregate(H: torch.Tensor, edge_index: torch.Tensor, aggr: str = "add",
              deg_norm: str | None = None, deg: torch.Tensor | None = None,
              edge_weight: torch.Tensor | None = None, bias: torch.Tensor | None = None,
              relu: bool = False, num_nodes: int | None = None) -> torch.Tensor:
    """Fused gather -> scale -> reduce -> (+bias) -> (ReLU) over ``edge_index``.

    Semantics of NodeModelAdditive.forward after its matmul
    (gcn_base_models.py:209-241): messages flow ``edge_index[0] -> [1]``;
    ``deg_norm`` in {None, 'sm', 'rw'} as degnorm_const; ``aggr`` in
    {'add', 'mean', 'max'} as common.scatter_.
    """
    if aggr not in L.REDUCE_CODES:
        raise ValueError(f"aggr must be one of add/mean/max, got {aggr!r}")
    if deg_norm not in L.NORM_CODES:
        raise ValueError(f"deg_norm must be None, 'sm' or 'rw', got {deg_norm!r}")
    n = H.size(0) if num_nodes is None else int(num_nodes)
    plan = plan_for(edge_index, n)
    norm = plan.norm(deg_norm, deg=deg, edge_weight=edge_weight)
    return aggregate_plan(H, plan, norm, aggr, bias, relu)


def edge_weight_grad(view: CSRView, H: torch.Tensor, dY: torch.Tensor,
                     win_mask: torch.Tensor | None = None) -> torch.Tensor:
    """dw[k] = sum_f dY[row(k), f] * H[col[k], f] for every slot k of the fwd
    view (``mgcn_edge_weight_grad``; max: the features slot k won), in slot
    order: the gradient of the aggregation with respect to its per-slot edge
    weights (the reference's ``x_j * norm.view(-1, 1)`` adjoint,
    gcn_base_models.py:217-224)."""
    lib = L.load()
    H = _contig_f32(H, "H")
    dY = _contig_f32(dY, "dY")
    dev = L.require_device(H, dY, view.rowptr)
    F = H.size(1)
    if dY.size(1) != F or H.size(0) != view.n_cols or dY.size(0) != view.n_rows:
        raise ValueError(f"edge_weight_grad: H {tuple(H.shape)}, dY {tuple(dY.shape)} do not fit "
                         f"the view ({view.n_rows} rows, {view.n_cols} columns)")
    dw = torch.empty(view.nnz, dtype=torch.float32, device=dev)
    with L.device_guard(dev):
        rc = lib.mgcn_edge_weight_grad(view.n_rows, F, L.ptr(view.rowptr), L.ptr(view.col),
                                       L.ptr(H), H.stride(0), L.ptr(dY), dY.stride(0),
                                       L.ptr(win_mask), L.ptr(dw), L.stream_of(dev))
    L.check(rc, "mgcn_edge_weight_grad")
    return dw


class _AggregateW(torch.autograd.Function):
    """:class:`_Aggregate` with the fwd per-slot weights as an autograd input
    (a :class:`NormPlan` built with ``grad``): the backward also returns their
    gradient, from which autograd reaches edge_weight / deg through the
    differentiable degnorm_const of graph._grad_norm."""

    @staticmethod
    def forward(ctx, H, w_fwd, bias, plan: GraphPlan, norm: NormPlan, reduce: int, relu: bool):
        Y, mask = spmm_fwd(plan.fwd, w_fwd.detach(), H, reduce, bias, relu, mask_plan=plan)
        ctx.plan, ctx.norm, ctx.reduce, ctx.relu = plan, norm, reduce, relu
        ctx.has_bias = bias is not None
        ctx.save_for_backward(H, Y if relu else None, mask)
        return Y

    @staticmethod
    def backward(ctx, dZ):
        H, Y, mask = ctx.saved_tensors
        plan, norm = ctx.plan, ctx.norm
        need_h = ctx.needs_input_grad[0]
        need_w = ctx.needs_input_grad[1]
        need_b = ctx.has_bias and ctx.needs_input_grad[2]
        mean = ctx.reduce == L.REDUCE_MEAN
        # mean: dY divided by the counts once, for the adjoint gather and for
        # the weights' gradient alike (scatter_mean's backward, common.py:59)
        dY, db = relu_bwd_colsum(dZ, Y, ctx.relu, need_b,
                                 row_div=plan.in_cnt if (mean and (need_h or need_w)) else None)
        dH = dw = None
        if need_h:
            dH = spmm_bwd(plan.bwd, norm.w_bwd, norm.row_scale_bwd, dY,
                          L.REDUCE_SUM if mean else ctx.reduce, win_mask=mask,
                          slot_map=plan.slot_map() if mask is not None else None)
        if need_w:
            dw = edge_weight_grad(plan.fwd, H, dY, win_mask=mask)
        return dH, dw, db, None, None, None, None


def aggregate_plan(H: torch.Tensor, plan: GraphPlan, norm: NormPlan, aggr: str = "add",
                   bias: torch.Tensor | None = None, relu: bool = False) -> torch.Tensor:
    """:func:`aggregate` on an already-built plan (no cache lookup)."""
    if norm.grad:
        return _AggregateW.apply(H, norm.w_fwd, bias, plan, norm, L.REDUCE_CODES[aggr],
                                 bool(relu))
    return _Aggregate.apply(H, bias, plan, norm, L.REDUCE_CODES[aggr], bool(relu))


class _LayerXW(torch.autograd.Function):
    """One GCN layer  y = epi((A_norm x) W + b)  on the fused kernels: the
    forward is one mgcn_spmm_xw_fwd launch, the backward one relu_bwd_colsum
    (this layer's ReLU / bias gradient; mean's division) and one
    mgcn_spmm_xw_bwd (dW and dx from on-chip dH).  Same gradients as
    linear() + aggregate_plan() up to the association of the forward sums."""

    @staticmethod
    def forward(ctx, x, W, bias, plan: GraphPlan, norm: NormPlan, reduce: int, relu: bool):
        # Z = the aggregate before W: dW = Z^T dY needs no second gather
        want_z = bool(ctx.needs_input_grad[1]) and dw_pass_supported(W.size(0), W.size(1))
        Y = spmm_xw_fwd(plan.fwd, norm.w_fwd, x, W, reduce, bias, relu, want_z=want_z)
        Y, Z = Y if want_z else (Y, None)
        ctx.plan, ctx.norm, ctx.reduce, ctx.relu = plan, norm, reduce, relu
        ctx.has_bias = bias is not None
        ctx.save_for_backward(x, W, Y if relu else None, Z)
        return Y

    @staticmethod
    def backward(ctx, dZ):
        x, W, Y, Z = ctx.saved_tensors
        plan, norm = ctx.plan, ctx.norm
        need_b = ctx.has_bias and ctx.needs_input_grad[2]
        mean = ctx.reduce == L.REDUCE_MEAN
        if Z is None:
            dY, db = relu_bwd_colsum(dZ.contiguous(), Y, ctx.relu, need_b,
                                     row_div=plan.in_cnt if mean else None)
            if not xw_full_supported(W.size(0), W.size(1)):  # 256: W needs no grad here
                dx = None
                if ctx.needs_input_grad[0]:
                    dx = spmm_xw_bwd(plan.bwd, norm.w_bwd, norm.row_scale_bwd, dY, None, W)[1]
                return dx, None, db, None, None, None, None
            dW, dx, _ = spmm_xw_bwd(plan.bwd, norm.w_bwd, norm.row_scale_bwd, dY, x, W,
                                    want_dx=ctx.needs_input_grad[0])
            return dx, dW, db, None, None, None, None
        # reassociated: dW = Z^T dY (mean: undivided Z, dY / count) on the
        # dense dW pass, the gather only for dx
        hcs = need_b and not ctx.relu and not mean  # db from the dW pass
        if hcs:
            dY, db = dZ.contiguous(), None
        else:
            dY, db = relu_bwd_colsum(dZ.contiguous(), Y, ctx.relu, need_b,
                                     row_div=plan.in_cnt if mean else None)
        dW, cs = dw_pass(Z, dY, W, dh_colsum=hcs)
        if hcs:
            db = cs
        dx = None
        if ctx.needs_input_grad[0]:
            dx = spmm_xw_bwd(plan.bwd, norm.w_bwd, norm.row_scale_bwd, dY, None, W)[1]
        return dx, dW, db, None, None, None, None


def gcn_layer(x: torch.Tensor, W: torch.Tensor, plan: GraphPlan, norm: NormPlan,
              aggr: str = "add", bias: torch.Tensor | None = None,
              relu: bool = False, aggregate_first: bool = False) -> torch.Tensor:
    """``aggregate_plan(x @ W, plan, norm, aggr, bias, relu)`` -- the
    reference's ``x @ weight_node`` then gather / scale / scatter (+ bias,
    ReLU) (gcn_base_models.py:201-241) -- as one fused launch per direction
    where the kernels apply (128 -> 128, sum / mean, no heavy rows in either
    view, gathered tables within 4 GiB); otherwise the GEMM and the
    aggregation run as separate launches, in the order the caller's
    reference uses: ``aggregate_first`` (PyG SAGEConv: mean_j x_j, then
    @ W + b) or x @ W first (the default)."""
    reduce = L.REDUCE_CODES[aggr]
    if _FUSE_XW and not norm.grad and layer_fusable(plan, x, W, reduce):
        return _LayerXW.apply(x, W, bias, plan, norm, reduce, bool(relu))
    if aggregate_first:
        out = linear(aggregate_plan(x, plan, norm, aggr), W)
        if bias is not None:
            out = out + bias
        return torch.relu(out) if relu else out
    return aggregate_plan(linear(x, W), plan, norm, aggr, bias, relu)


class _GCNStack(torch.autograd.Function):
    """A chain of GCN layers  Z_l = act_l(A_norm (Z_{l-1} W_l) + b_l)  as one
    autograd node, so the backward can fuse across layer boundaries: the
    ReLU mask and bias gradient of layer l-1 are computed in the epilogue of
    layer l's dX GEMM (mgcn_gemm_nn with Z), instead of a separate pass.
    Per layer: GEMM -> SpMM(+bias, ReLU) forward; SpMM^T, dW (split-K), dX
    (+ fused ReLU/bias of the layer below) backward.  Same math and the same
    per-edge summation order as the layer-by-layer modules.
    128 -> 128 sum / mean layers run fused: the forward aggregates then
    multiplies ((A h) W, one launch) and keeps Z = A h; the backward forms
    dW = Z^T dY in one dense pass (the top layer's bias gradient from the
    same pass) and gathers A^T dY only for dX, so the bottom layer runs no
    gather.  Max keeps the GEMM + SpMM launches (max does not commute with W)."""

    @staticmethod
    def forward(ctx, x, plan, norm, reduce, relus, *params):
        Ws, bs = params[0::2], params[1::2]
        h = x
        inputs, outs, args, rmasks, zs = [], [], [], [], []
        for i, (W, b, relu) in enumerate(zip(Ws, bs, relus)):
            z = None
            inputs.append(h)
            # the ReLU mask the next layer's dX GEMM reads (16 B per row)
            nxt = Ws[i + 1] if i + 1 < len(Ws) else None
            rm = None
            xw = _FUSE_XW and spmm_xw_supported(plan.fwd, W.size(0), W.size(1), reduce,
                                                h.stride(0))
            if relu and nxt is not None and (
                    gemm_nn_epi_supported(nxt.size(1), nxt.size(0)) or
                    (xw and W.size(1) > 128 and
                     spmm_xw_supported(plan.bwd, nxt.size(1), nxt.size(0), L.REDUCE_SUM))):
                # (the 8-word masks of a 256-wide layer only from its fused
                # forward, for the fused dX-only adjoint of the next layer)
                rm = torch.empty(plan.fwd.n_rows, mask_words(W.size(1)), dtype=torch.int32,
                                 device=h.device)
            if xw:
                # (A h) W in one launch: h @ W is never written (sum / mean);
                # the aggregate A h is kept for dW = (A h)^T dY when the
                # backward takes that form (same predicate as its z_path):
                # the bottom layer, or one whose lower layer left a ReLU
                # mask, with the dX-only gather possible on the bwd view;
                # middle layers keep the dW + dX gather kernel (_Z_MIDDLE)
                below = i == 0 or (relus[i - 1] and rmasks[i - 1] is not None)
                middle = 0 < i < len(Ws) - 1 and relus[i - 1]
                top_full = (_TOP_FULL and i == len(Ws) - 1 and i > 0 and relus[i - 1] and
                            rmasks[i - 1] is not None and not relu and
                            reduce in (L.REDUCE_SUM, L.REDUCE_MEAN) and
                            plan.bwd.n_rows == plan.bwd.n_cols and xw_full_supported(*W.shape))
                want_z = (bool(ctx.needs_input_grad[5 + 2 * i]) and below and not top_full and
                          (_Z_MIDDLE or not middle or
                           not xw_full_supported(*W.shape)) and
                          dw_pass_supported(W.size(0), W.size(1)) and
                          spmm_xw_supported(plan.bwd, W.size(1), W.size(0), L.REDUCE_SUM))
                h, am = spmm_xw_fwd(plan.fwd, norm.w_fwd, h, W, reduce, b, relu,
                                    relu_mask=rm, want_z=want_z), None
                if want_z:
                    h, z = h
            else:
                H = _mm(h, W)
                h, am = spmm_fwd(plan.fwd, norm.w_fwd, H, reduce, b, relu, mask_plan=plan,
                                 relu_mask=rm)
            outs.append(h)
            args.append(am)  # max: winner bits per edge (adjoint slot order)
            rmasks.append(rm)
            zs.append(z)
        ctx.plan, ctx.norm, ctx.reduce, ctx.relus = plan, norm, reduce, relus
        ctx.n_layers = len(Ws)
        ctx.has_bias = [b is not None for b in bs]
        ctx.save_for_backward(*inputs, *outs, *[a if a is not None else torch.empty(0)
                                                for a in args], *Ws,
                              *[m if m is not None else torch.empty(0) for m in rmasks],
                              *[z if z is not None else torch.empty(0) for z in zs])
        return h

    @staticmethod
    def backward(ctx, dZ):
        n = ctx.n_layers
        saved = ctx.saved_tensors
        inputs, outs = saved[:n], saved[n:2 * n]
        args, Ws, rmasks = saved[2 * n:3 * n], saved[3 * n:4 * n], saved[4 * n:5 * n]
        zs = saved[5 * n:6 * n]
        plan, norm, reduce, relus = ctx.plan, ctx.norm, ctx.reduce, ctx.relus
        gW = [None] * n
        gb = [None] * n
        top = n - 1
        # mean: every layer's dY is produced divided by the row counts (fused
        # into relu_bwd_colsum / the dX GEMM epilogue); the adjoint is a sum
        mean = reduce == L.REDUCE_MEAN
        rd = plan.in_cnt if mean else None
        adj = L.REDUCE_SUM if mean else reduce

        def z_path(l):  # dW = Z^T dY from the forward's aggregate (below)
            fused = l > 0 and relus[l - 1] and rmasks[l - 1].numel() > 0
            return bool(zs[l].numel() and (fused or l == 0) and
                        dw_pass_supported(Ws[l].size(0), Ws[l].size(1)) and
                        spmm_xw_supported(plan.bwd, Ws[l].size(1), Ws[l].size(0),
                                          L.REDUCE_SUM))

        top_z = z_path(top) and not relus[top] and rd is None
        # the top layer's bias gradient from its dW + dX adjoint (mgcn_spmm_xw_bwd_hcs):
        # the forward kept no Z for it (top_full there); same predicate here
        top_hcs = (_TOP_FULL and _TOP_HCS and not zs[top].numel() and top > 0 and not relus[top] and
                   rd is None and args[top].numel() == 0 and relus[top - 1] and
                   rmasks[top - 1].numel() > 0 and ctx.needs_input_grad[5 + 2 * top] and
                   ctx.has_bias[top] and plan.bwd.n_rows == plan.bwd.n_cols and
                   _FUSE_XW and xw_full_supported(*Ws[top].shape) and
                   spmm_xw_supported(plan.bwd, Ws[top].size(0), Ws[top].size(1), L.REDUCE_SUM))
        # or from the bottom layer's dW = Z^T dY pass, which streams dZ beside
        # its own operands (mgcn_gemm_bwd_dw_cs): no separate pass over dZ
        top_defer = (not top_z and not top_hcs and _TOP_CS_DEFER and top > 0 and
                     not relus[top] and rd is None and ctx.has_bias[top] and
                     ctx.needs_input_grad[5] and z_path(0) and
                     gemm_bwd_supported(*Ws[0].shape) and tuple(dZ.shape) == (zs[0].size(0), 128))
        top_S = None
        if top_z or top_hcs or top_defer:
            # dY = dZ as it is: its column sums (the top bias gradient) come
            # from the dW = Z^T dY pass below, from the top layer's dW + dX
            # adjoint (top_hcs) or from the bottom layer's dW pass (top_defer),
            # no separate read of dZ
            dY = dZ.contiguous()
            if top_defer:
                top_S = dY
        else:
            dY, db = relu_bwd_colsum(dZ.contiguous(), outs[top], relus[top], ctx.has_bias[top],
                                     row_div=rd)
            gb[top] = db
        dx = None

        def adjoint_dx(l, dY):
            """Layer l's dX-only adjoint -> the lower layer's dY (with its ReLU
            mask, bias gradient and mean divisor)."""
            W = Ws[l]
            _, dYn, db = spmm_xw_bwd(plan.bwd, norm.w_bwd, norm.row_scale_bwd, dY, None, W,
                                     relu_mask=rmasks[l - 1], row_div=rd)
            gb[l - 1] = db if ctx.has_bias[l - 1] else None
            return dYn

        for l in range(top, -1, -1):
            am = args[l] if args[l].numel() else None
            W = Ws[l]
            fused = l > 0 and relus[l - 1] and rmasks[l - 1].numel() > 0
            if not ctx.needs_input_grad[5 + 2 * l]:
                # a frozen weight: no dW; only dX (with the lower layer's ReLU
                # / bias gradient) is wanted -- the dX-only adjoint, which
                # also takes the 8-word masks of a 256-wide layer
                if l == 0 and not ctx.needs_input_grad[0]:
                    continue
                if am is None and (fused or l == 0) and _FUSE_XW and \
                        spmm_xw_supported(plan.bwd, W.size(1), W.size(0), L.REDUCE_SUM):
                    if fused:
                        dY = adjoint_dx(l, dY)
                    else:
                        dx = spmm_xw_bwd(plan.bwd, norm.w_bwd, norm.row_scale_bwd, dY, None, W)[1]
                    continue
            if z_path(l):
                # dW = Z^T dY from the forward's aggregate Z = A h (a dense
                # pass over Z and dY, no gather); mean: Z is the undivided sum
                # and dY arrives divided by the counts, so Z^T dY is the same
                # product.  The gather runs only for dX (+ the lower layer's
                # ReLU / bias gradient); the bottom layer needs no gather at all.
                hcs = bool(top_z and l == top and ctx.has_bias[top])
                if gW[l] is None and top_S is not None and l == 0:
                    gW[l], gb[top] = dw_pass_cs(zs[l], dY, top_S)  # + the top bias gradient
                elif gW[l] is None:
                    gW[l], cs = dw_pass(zs[l], dY, W, dh_colsum=hcs)
                    if hcs:
                        gb[top] = cs
                if fused:
                    dY = adjoint_dx(l, dY)
                elif ctx.needs_input_grad[0]:
                    dx = spmm_xw_bwd(plan.bwd, norm.w_bwd, norm.row_scale_bwd, dY, None, W)[1]
                continue
            if (_FUSE_XW and xw_full_supported(W.size(0), W.size(1)) and
                    spmm_xw_supported(plan.bwd, W.size(0), W.size(1), L.REDUCE_SUM)):
                # adjoint SpMM + dW + dX (+ the lower layer's ReLU / bias
                # gradient) in one pass: dH never leaves the chip (max: the
                # adjoint routes dY through the forward's winner bits; with dX
                # the two-phase kernel measured slower than the two launches,
                # 1.53 vs 1.42 ms at config 4; the warp-specialised one is
                # faster, _MAX_FULL)
                sm = plan.slot_map() if am is not None else None
                if fused and (am is None or _MAX_FULL):
                    hcs = None
                    if top_hcs and l == top:
                        hcs = gb[top] = torch.empty(W.size(1), dtype=torch.float32,
                                                    device=dY.device)
                    gW[l], dY, db = spmm_xw_bwd(plan.bwd, norm.w_bwd, norm.row_scale_bwd, dY,
                                                inputs[l], W, relu_mask=rmasks[l - 1],
                                                row_div=rd, win_mask=am, slot_map=sm,
                                                dy_colsum_out=hcs)
                    gb[l - 1] = db if ctx.has_bias[l - 1] else None
                    continue
                if l == 0 and not ctx.needs_input_grad[0]:
                    gW[l] = spmm_xw_bwd(plan.bwd, norm.w_bwd, norm.row_scale_bwd, dY, inputs[l],
                                        W, want_dx=False, win_mask=am, slot_map=sm)[0]
                    continue
            dH = spmm_bwd(plan.bwd, norm.w_bwd, norm.row_scale_bwd, dY, adj, win_mask=am,
                          slot_map=plan.slot_map() if am is not None else None)
            if fused and gemm_bwd_supported(W.size(0), W.size(1)):
                # dW and dX (+ the lower layer's ReLU / bias gradient) in one pass
                gW[l], dY, db = gemm_bwd(inputs[l], dH, W, relu_mask=rmasks[l - 1], row_div=rd)
                gb[l - 1] = db if ctx.has_bias[l - 1] else None
                continue
            if l == 0 and not ctx.needs_input_grad[0] and gemm_bwd_supported(W.size(0), W.size(1)):
                gW[l] = gemm_bwd(inputs[l], dH, W, want_dx=False)[0]  # dW alone, same pass shape
                continue
            if ctx.needs_input_grad[5 + 2 * l]:
                gW[l] = gemm_tn(inputs[l], dH)
            if l > 0:
                if fused:
                    dY, db = gemm_nn(dH, W, transpose_w=True, relu_mask=rmasks[l - 1],
                                     row_div=rd)
                    if not ctx.has_bias[l - 1]:
                        db = None
                else:
                    dY, db = relu_bwd_colsum(_mm_t(dH, W), outs[l - 1], relus[l - 1],
                                             ctx.has_bias[l - 1], row_div=rd)
                gb[l - 1] = db
            elif ctx.needs_input_grad[0]:
                dx = _mm_t(dH, W)
        grads = []
        for w, b in zip(gW, gb):
            grads += [w, b]
        return (dx, None, None, None, None, *grads)


def gcn_stack(x: torch.Tensor, plan: GraphPlan, norm: NormPlan, Ws, bs, relus,
              aggr: str = "add") -> torch.Tensor:
    """Run len(Ws) fused GCN layers (see :class:`_GCNStack`)."""
    if norm.grad:  # weights with autograd history: layer by layer (_AggregateW)
        for W, b, r in zip(Ws, bs, relus):
            x = aggregate_plan(linear(x, W), plan, norm, aggr, b, bool(r))
        return x
    params = []
    for W, b in zip(Ws, bs):
        params += [W, b]
    return _GCNStack.apply(x, plan, norm, L.REDUCE_CODES[aggr], tuple(bool(r) for r in relus),
                           *params)


# ------------------------------------------------------- residual GCN layer
def residual_act(Z1: torch.Tensor, R: torch.Tensor, rbias: torch.Tensor | None,
                 relu: bool) -> torch.Tensor:
    """Z = act(Z1 + (R + rbias)) (``mgcn_residual_act``)."""
    lib = L.load()
    dev = L.require_device(Z1, R, rbias)
    n, F = Z1.shape
    Z = torch.empty(n, F, dtype=torch.float32, device=dev)
    rb = rbias.detach().contiguous() if rbias is not None else None
    with L.device_guard(dev):
        rc = lib.mgcn_residual_act(n, F, L.ptr(Z1), Z1.stride(0), L.ptr(R), R.stride(0), L.ptr(rb),
                                   int(bool(relu)), L.ptr(Z), Z.stride(0), L.stream_of(dev))
    L.check(rc, "mgcn_residual_act")
    return Z


def residual_act_bwd(dZ, Z, relu, Z1, relu1, dA, dS, row_div=None, want_sums=True):
    """dS / dA / their column sums (``mgcn_residual_act_bwd``); returns the
    [2F] sums (dA | dS) or None."""
    lib = L.load()
    dev = L.require_device(dZ, dA)
    n, F = dZ.shape
    sums = torch.empty(2 * F, dtype=torch.float32, device=dev) if want_sums else None
    ws_bytes = int(lib.mgcn_residual_act_bwd_workspace_bytes(n, F)) if want_sums else 0
    ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev) if want_sums else None
    with L.device_guard(dev):
        rc = lib.mgcn_residual_act_bwd(
            n, F, L.ptr(dZ), dZ.stride(0), L.ptr(Z), Z.stride(0) if Z is not None else F,
            int(bool(relu)), L.ptr(Z1), Z1.stride(0) if Z1 is not None else F, int(bool(relu1)),
            L.ptr(row_div), L.ptr(dA), dA.stride(0), L.ptr(dS),
            dS.stride(0) if dS is not None else F, L.ptr(sums), L.ptr(ws), ws_bytes,
            L.stream_of(dev))
    L.check(rc, "mgcn_residual_act_bwd")
    return sums


class _ResidualGCNLayer(torch.autograd.Function):
    """One GCNModel layer with its residual Linear (gcn_model.py:92-105,
    residual_hop = 1) as a single autograd node:

        [H | R] = x @ [W | Wr^T]                 one GEMM, x read once
        Z1 = relu1(A_norm H + b)                 SpMM, bias/ReLU epilogue
        Z  = relu2(Z1 + (R + br))                mgcn_residual_act

    backward: mgcn_residual_act_bwd gives dA (into the adjoint SpMM), dS and
    both bias gradients in one pass; the adjoint SpMM writes dH beside dS,
    so dx = [dH | dS] @ [W | Wr^T]^T and [dW | dWr^T] = x^T [dH | dS] are one
    GEMM each.  Forward values are the layer-by-layer path's bit for bit;
    gradients agree within fp32 GEMM tolerance (different summation order)."""

    @staticmethod
    def forward(ctx, x, plan, norm, reduce, relu1, relu2, W, b, Wr, br):
        F_out = W.size(1)
        Wc = torch.cat([W.detach(), Wr.detach().t()], dim=1)
        HR = _mm(x, Wc)
        Z1, mask = spmm_fwd(plan.fwd, norm.w_fwd, HR[:, :F_out], reduce, b, relu1, mask_plan=plan)
        Z = residual_act(Z1, HR[:, F_out:], br, relu2)
        ctx.plan, ctx.norm, ctx.reduce, ctx.relu1, ctx.relu2 = plan, norm, reduce, relu1, relu2
        ctx.has_b, ctx.has_br = b is not None, br is not None
        ctx.save_for_backward(x, Z1, Z, Wc, mask)
        return Z

    @staticmethod
    def backward(ctx, dZ):
        x, Z1, Z, Wc, mask = ctx.saved_tensors
        plan, norm = ctx.plan, ctx.norm
        n, F_out = Z.shape
        dZ = dZ.contiguous()
        mean = ctx.reduce == L.REDUCE_MEAN
        DH = torch.empty(n, 2 * F_out, dtype=torch.float32, device=dZ.device)
        dA = torch.empty(n, F_out, dtype=torch.float32, device=dZ.device)
        sums = residual_act_bwd(dZ, Z, ctx.relu2, Z1, ctx.relu1, dA, DH[:, F_out:],
                                row_div=plan.in_cnt if mean else None)
        spmm_bwd(plan.bwd, norm.w_bwd, norm.row_scale_bwd, dA,
                 L.REDUCE_SUM if mean else ctx.reduce, out=DH[:, :F_out], win_mask=mask,
                 slot_map=plan.slot_map() if mask is not None else None)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = _mm_t(DH, Wc)
        # [dW | dWr^T] = x^T [dH | dS] in one pass, dWr written transposed
        dW, dWr = gemm_tn_split(x, DH, F_out)
        db = sums[:F_out] if ctx.has_b else None
        dbr = sums[F_out:] if ctx.has_br else None
        return (dx, None, None, None, None, None, dW, db, dWr, dbr)


def _aligned_rows(t: torch.Tensor) -> torch.Tensor:
    """Contiguous fp32 with 16-byte aligned rows (the fused kernels' float4 accesses)."""
    t = _contig_f32(t, "x")
    if t.stride(0) % 4 or t.data_ptr() % 16 or t.stride(1) != 1:
        t = t.contiguous()
    return t


def residual_layer_supported(plan: GraphPlan, x: torch.Tensor, W: torch.Tensor, Wr: torch.Tensor,
                             reduce: int) -> bool:
    """True when :class:`_ResidualLayerFused` takes this layer: 32 -> 32 with a
    32 -> 32 residual Linear, sum or mean, fp32, on a square graph plan."""
    return (_FUSE_XW and x.dim() == 2 and x.dtype == torch.float32 and x.is_cuda and
            W.dtype == torch.float32 and Wr.dtype == torch.float32 and
            tuple(W.shape) == (x.size(1), x.size(1)) and tuple(Wr.shape) == tuple(W.shape) and
            x.size(0) == plan.fwd.n_rows == plan.fwd.n_cols and
            bool(L.load().mgcn_residual_layer_supported(x.size(1), W.size(1), int(reduce))))


class _ResidualLayerFused(torch.autograd.Function):
    """One GCNModel layer with its residual Linear (gcn_model.py:89-105,
    residual_hop = 1), F = 32, on libmgcn's fused residual-layer kernels
    (residual.hip): the forward is one pass over the rows (aggregation of x,
    both 32 x 32 products, bias, ReLU, join, ReLU; ReLU masks kept instead of
    the activations), the backward one mask pass + one pass that gathers the
    adjoint and forms dX = dH W^T + dS Wr, then [dW | dWr^T] = x^T [dH | dS]
    as one GEMM.  (A x) W instead of A (x W): the same layer to fp32
    rounding; the adjoint dH is the SpMM's bit for bit."""

    @staticmethod
    def forward(ctx, x, plan, norm, reduce, relu1, relu2, W, b, Wr, br):
        lib = L.load()
        x = _aligned_rows(x)
        dev = L.require_device(x, W, Wr, b, br)
        n, F = x.shape
        Wd = W.detach().to(torch.float32).contiguous()
        Wrd = Wr.detach().to(torch.float32).contiguous()
        bd = None if b is None else b.detach().to(torch.float32).contiguous()
        brd = None if br is None else br.detach().to(torch.float32).contiguous()
        Z = torch.empty(n, F, dtype=torch.float32, device=dev)
        masks = torch.empty(n, 2, dtype=torch.int32, device=dev)
        v = plan.fwd
        if _TIMER is not None:
            _TIMER("residual_layer_fwd", True, v.n_rows, v.edges)
        with L.device_guard(dev):
            rc = lib.mgcn_residual_layer_fwd(n, F, L.ptr(v.rowptr), L.ptr(v.col), L.ptr(v.eid),
                                             L.ptr(norm.w_fwd), L.ptr(x), x.stride(0), L.ptr(Wd),
                                             F, L.ptr(bd), L.ptr(Wrd), F, L.ptr(brd), int(reduce),
                                             int(bool(relu1)), int(bool(relu2)), L.ptr(Z), F,
                                             L.ptr(masks), L.ptr(v.order), v.n_heavy, v.n_giant,
                                             L.stream_of(dev))
        if _TIMER is not None:
            _TIMER("residual_layer_fwd", False)
        L.check(rc, "mgcn_residual_layer_fwd")
        ctx.plan, ctx.norm, ctx.reduce, ctx.relu1, ctx.relu2 = plan, norm, reduce, relu1, relu2
        ctx.has_b, ctx.has_br = b is not None, br is not None
        ctx.save_for_backward(x, Wd, Wrd, masks)
        return Z

    @staticmethod
    def backward(ctx, dZ):
        lib = L.load()
        x, Wd, Wrd, masks = ctx.saved_tensors
        plan, norm = ctx.plan, ctx.norm
        dZ = _aligned_rows(dZ)
        dev = dZ.device
        n, F = x.shape
        dX = torch.empty(n, F, dtype=torch.float32, device=dev)
        DH = torch.empty(n, 2 * F, dtype=torch.float32, device=dev)
        sums = torch.empty(2 * F, dtype=torch.float32, device=dev)
        ws_bytes = int(lib.mgcn_residual_layer_bwd_workspace_bytes(n, F))
        ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
        v = plan.bwd
        rd = plan.in_cnt if ctx.reduce == L.REDUCE_MEAN else None
        if _TIMER is not None:
            _TIMER("residual_layer_bwd", True, v.n_rows, v.edges)
        with L.device_guard(dev):
            rc = lib.mgcn_residual_layer_bwd(n, F, L.ptr(v.rowptr), L.ptr(v.col), L.ptr(v.eid),
                                             L.ptr(norm.w_bwd), L.ptr(norm.row_scale_bwd),
                                             L.ptr(rd), L.ptr(dZ), dZ.stride(0), L.ptr(masks),
                                             int(bool(ctx.relu1)), int(bool(ctx.relu2)),
                                             L.ptr(Wd), F, L.ptr(Wrd), F, L.ptr(dX), F,
                                             L.ptr(DH), 2 * F, L.ptr(sums), L.ptr(v.order),
                                             v.n_heavy, v.n_giant, L.ptr(ws), ws_bytes,
                                             L.stream_of(dev))
        if _TIMER is not None:
            _TIMER("residual_layer_bwd", False)
        L.check(rc, "mgcn_residual_layer_bwd")
        # [dW | dWr^T] = x^T [dH | dS] in one pass, dWr written transposed
        dW, dWr = gemm_tn_split(x, DH, F)
        db = sums[:F] if ctx.has_b else None
        dbr = sums[F:] if ctx.has_br else None
        dx = dX if ctx.needs_input_grad[0] else None
        return (dx, None, None, None, None, None, dW, db, dWr, dbr)


def _ptr_array(ts):
    """Host array of device pointers (NULL for None) for the stack entry points."""
    import ctypes
    arr = (ctypes.c_void_p * max(len(ts), 1))(*[None if t is None else t.data_ptr() for t in ts])
    return ctypes.cast(arr, ctypes.c_void_p), arr


def _int_array(vals):
    import ctypes
    arr = (ctypes.c_int32 * max(len(vals), 1))(*[int(bool(v)) for v in vals])
    return ctypes.cast(arr, ctypes.c_void_p), arr


def _param_f32(t):
    if t is None:
        return None
    t = t.detach()
    return t if (t.dtype == torch.float32 and t.is_contiguous()) else t.to(torch.float32).contiguous()


class _ResidualStack(torch.autograd.Function):
    """Consecutive 32 -> 32 GCNModel layers with their residual Linears
    (:class:`_ResidualLayerFused` each) as ONE autograd node and one host call
    per direction (``mgcn_residual_stack_fwd`` / ``_bwd``): bitwise the
    layer-by-layer fused path, without ~40 us of Python and ctypes work per
    layer and direction (the 12-layer config-3 step was bound by host issue).
    params = (W, b, Wr, br) per layer."""

    @staticmethod
    def forward(ctx, x0, plan, norm, reduce, relu1s, relu2s, *params):
        lib = L.load()
        nl = len(relu1s)
        x0 = _aligned_rows(x0)
        dev = x0.device
        n, F = x0.shape
        Ws = [_param_f32(p) for p in params[0::4]]
        bs = [_param_f32(p) for p in params[1::4]]
        Wrs = [_param_f32(p) for p in params[2::4]]
        brs = [_param_f32(p) for p in params[3::4]]
        Z = torch.empty(nl, n, F, dtype=torch.float32, device=dev)
        masks = torch.empty(nl, n, 2, dtype=torch.int32, device=dev)
        pw, aw = _ptr_array(Ws)
        pb, ab = _ptr_array(bs)
        pwr, awr = _ptr_array(Wrs)
        pbr, abr = _ptr_array(brs)
        pr1, ar1 = _int_array(relu1s)
        pr2, ar2 = _int_array(relu2s)
        v = plan.fwd
        if _TIMER is not None:
            _TIMER("residual_stack_fwd", True, v.n_rows, v.edges)
        with L.device_guard(dev):
            rc = lib.mgcn_residual_stack_fwd(n, F, nl, L.ptr(v.rowptr), L.ptr(v.col), L.ptr(v.eid),
                                             L.ptr(norm.w_fwd), L.ptr(x0), x0.stride(0), pw, pb,
                                             pwr, pbr, int(reduce), pr1, pr2, L.ptr(Z),
                                             L.ptr(masks), L.ptr(v.order), v.n_heavy, v.n_giant,
                                             L.stream_of(dev))
        if _TIMER is not None:
            _TIMER("residual_stack_fwd", False)
        L.check(rc, "mgcn_residual_stack_fwd")
        ctx.plan, ctx.norm, ctx.reduce = plan, norm, reduce
        ctx.relu1s, ctx.relu2s = relu1s, relu2s
        ctx.has_b = [b is not None for b in bs]
        ctx.has_br = [b is not None for b in brs]
        ctx.save_for_backward(x0, Z, masks, *Ws, *Wrs)
        return Z[nl - 1]

    @staticmethod
    def backward(ctx, dZ):
        lib = L.load()
        nl = len(ctx.relu1s)
        saved = ctx.saved_tensors
        x0, Z, masks = saved[:3]
        Ws, Wrs = saved[3:3 + nl], saved[3 + nl:3 + 2 * nl]
        plan, norm = ctx.plan, ctx.norm
        dZ = _aligned_rows(dZ)
        dev = dZ.device
        n, F = x0.shape
        G = torch.empty(nl, 2, F, F, dtype=torch.float32, device=dev)  # dW[l] | dWr[l]
        sums = torch.empty(nl, 2 * F, dtype=torch.float32, device=dev)
        dX0 = torch.empty(n, F, dtype=torch.float32, device=dev) if ctx.needs_input_grad[0] \
            else None
        ws_bytes = int(lib.mgcn_residual_stack_bwd_workspace_bytes(n, F))
        ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
        pw, aw = _ptr_array(Ws)
        pwr, awr = _ptr_array(Wrs)
        pdw, adw = _ptr_array([G[l, 0] for l in range(nl)])
        pdwr, adwr = _ptr_array([G[l, 1] for l in range(nl)])
        pr1, ar1 = _int_array(ctx.relu1s)
        pr2, ar2 = _int_array(ctx.relu2s)
        v = plan.bwd
        rd = plan.in_cnt if ctx.reduce == L.REDUCE_MEAN else None
        if _TIMER is not None:
            _TIMER("residual_stack_bwd", True, v.n_rows, v.edges)
        with L.device_guard(dev):
            rc = lib.mgcn_residual_stack_bwd(n, F, nl, L.ptr(v.rowptr), L.ptr(v.col), L.ptr(v.eid),
                                             L.ptr(norm.w_bwd), L.ptr(norm.row_scale_bwd),
                                             L.ptr(rd), L.ptr(dZ), dZ.stride(0), L.ptr(x0),
                                             x0.stride(0), L.ptr(Z), L.ptr(masks), pr1, pr2, pw,
                                             pwr, L.ptr(dX0), pdw, pdwr, L.ptr(sums),
                                             L.ptr(v.order), v.n_heavy, v.n_giant, L.ptr(ws),
                                             ws_bytes, L.stream_of(dev))
        if _TIMER is not None:
            _TIMER("residual_stack_bwd", False)
        L.check(rc, "mgcn_residual_stack_bwd")
        grads = []
        for l in range(nl):
            grads += [G[l, 0], sums[l, :F] if ctx.has_b[l] else None, G[l, 1],
                      sums[l, F:] if ctx.has_br[l] else None]
        return (dX0, None, None, None, None, None, *grads)


def residual_stack(x, plan: GraphPlan, norm: NormPlan, aggr: str, relu1s, relu2s, params):
    """Layers of :class:`_ResidualStack`; params = [(W, b, Wr, br), ...]."""
    flat = []
    for p in params:
        flat += list(p)
    return _ResidualStack.apply(x, plan, norm, L.REDUCE_CODES[aggr],
                                tuple(bool(r) for r in relu1s), tuple(bool(r) for r in relu2s),
                                *flat)


def input_layer_supported(plan: GraphPlan, x: torch.Tensor, W: torch.Tensor, Wr: torch.Tensor,
                          reduce: int) -> bool:
    """True when :class:`_InputLayer` takes this layer: in_channels = 1 with a
    1 -> F residual Linear, sum or mean, fp32, on a square graph plan."""
    return (_FUSE_XW and x.dim() == 2 and x.size(1) == 1 and x.dtype == torch.float32 and
            x.is_cuda and W.dtype == torch.float32 and Wr.dtype == torch.float32 and
            W.dim() == 2 and W.size(0) == 1 and tuple(Wr.shape) == (W.size(1), 1) and
            reduce in (L.REDUCE_SUM, L.REDUCE_MEAN) and
            x.size(0) == plan.fwd.n_rows == plan.fwd.n_cols and
            bool(L.load().mgcn_input_layer_supported(1, W.size(1))))


class _InputLayer(torch.autograd.Function):
    """GCNModel's input layer with its residual Linear when in_channels = 1
    (config 3's botnet node feature; gcn_model.py:89-105, residual_hop = 1),
    associated as (A x) W: a = A x is a 1-wide aggregation (mgcn_spmm_fwd,
    4 gathered bytes per edge instead of 4 F) and everything after it is
    elementwise (mgcn_input_layer_fwd):

        Z = relu2( relu1(a W + b) + (x Wr^T + br) )

    backward: one pass over dZ (mgcn_input_layer_bwd) gives dW, db, dWr, dbr
    as fixed-order column sums -- no adjoint gather at all unless x itself
    needs a gradient (then dx = A^T (dA W^T) + dS Wr, a 1-wide adjoint SpMM).
    The reference's A (x W) to fp32 rounding (a different association)."""

    @staticmethod
    def forward(ctx, x, plan, norm, reduce, relu1, relu2, W, b, Wr, br):
        lib = L.load()
        dev = L.require_device(x, W, b, Wr, br)
        x = x.contiguous()
        n, F = x.size(0), W.size(1)
        a, _ = spmm_fwd(plan.fwd, norm.w_fwd, x, reduce)
        Wd, Wrd = W.detach().contiguous(), Wr.detach().contiguous()
        bd = b.detach().contiguous() if b is not None else None
        brd = br.detach().contiguous() if br is not None else None
        Z = torch.empty(n, F, dtype=torch.float32, device=dev)
        if _TIMER is not None:
            _TIMER("input_layer_fwd", True, n)
        with L.device_guard(dev):
            rc = lib.mgcn_input_layer_fwd(n, F, L.ptr(a), L.ptr(x), L.ptr(Wd), L.ptr(bd),
                                          L.ptr(Wrd), L.ptr(brd), int(relu1), int(relu2),
                                          L.ptr(Z), Z.stride(0), L.stream_of(dev))
        if _TIMER is not None:
            _TIMER("input_layer_fwd", False)
        L.check(rc, "mgcn_input_layer_fwd")
        ctx.plan, ctx.norm, ctx.reduce, ctx.relu1, ctx.relu2 = plan, norm, reduce, relu1, relu2
        ctx.has_b, ctx.has_br = b is not None, br is not None
        ctx.save_for_backward(x, a, Z, Wd, bd if bd is not None else torch.empty(0), Wrd)
        return Z

    @staticmethod
    def backward(ctx, dZ):
        lib = L.load()
        x, a, Z, W, b, Wr = ctx.saved_tensors
        plan, norm = ctx.plan, ctx.norm
        n, F = Z.shape
        dev = Z.device
        dZ = _aligned_rows(dZ)
        need_x = bool(ctx.needs_input_grad[0])
        da = torch.empty(n, dtype=torch.float32, device=dev) if need_x else None
        dxr = torch.empty(n, dtype=torch.float32, device=dev) if need_x else None
        grads = torch.empty(4 * F, dtype=torch.float32, device=dev)
        mean = ctx.reduce == L.REDUCE_MEAN
        ws_bytes = int(lib.mgcn_input_layer_bwd_workspace_bytes(n, F))
        ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
        if _TIMER is not None:
            _TIMER("input_layer_bwd", True, n)
        with L.device_guard(dev):
            rc = lib.mgcn_input_layer_bwd(
                n, F, L.ptr(dZ), dZ.stride(0), L.ptr(Z), Z.stride(0), L.ptr(a), L.ptr(x),
                L.ptr(W), L.ptr(b if b.numel() else None), L.ptr(Wr), int(ctx.relu1),
                int(ctx.relu2), L.ptr(plan.in_cnt if (mean and need_x) else None), L.ptr(da),
                L.ptr(dxr), L.ptr(grads), L.ptr(ws), ws_bytes, L.stream_of(dev))
        if _TIMER is not None:
            _TIMER("input_layer_bwd", False)
        L.check(rc, "mgcn_input_layer_bwd")
        dx = None
        if need_x:
            dx = spmm_bwd(plan.bwd, norm.w_bwd, norm.row_scale_bwd, da.view(n, 1), L.REDUCE_SUM)
            dx.add_(dxr.view(n, 1))
        dW = grads[:F].view(1, F)
        db = grads[F:2 * F] if ctx.has_b else None
        dWr = grads[2 * F:3 * F].view(F, 1)
        dbr = grads[3 * F:] if ctx.has_br else None
        return (dx, None, None, None, None, None, dW, db, dWr, dbr)


def residual_gcn_layer(x, plan: GraphPlan, norm: NormPlan, aggr: str, relu1: bool, relu2: bool,
                       W, b, Wr, br):
    """One GCNModel layer + residual join: :class:`_ResidualLayerFused` where
    it applies (32 -> 32, sum / mean), :class:`_InputLayer` for an
    in_channels = 1 input layer, else :class:`_ResidualGCNLayer`."""
    reduce = L.REDUCE_CODES[aggr]
    if input_layer_supported(plan, x, W, Wr, reduce):
        return _InputLayer.apply(x, plan, norm, reduce, bool(relu1), bool(relu2), W, b, Wr, br)
    if residual_layer_supported(plan, x, W, Wr, reduce):
        return _ResidualLayerFused.apply(x, plan, norm, reduce, bool(relu1), bool(relu2), W, b,
                                         Wr, br)
    return _ResidualGCNLayer.apply(x, plan, norm, reduce, bool(relu1), bool(relu2), W, b, Wr, br)


# ---------------------------------------------------------------- scatter_
class _SegmentReduce(torch.autograd.Function):
    """torch_scatter 1.x scatter_{add,mean,max}(src, index, 0, None, dim_size)
    on an explicit [E, F] ``src`` (common.py:37-66), as a SpMM whose k-th slot
    gathers src row eid_k; the adjoint gathers dY[index[e]] back per edge."""

    @staticmethod
    def forward(ctx, src, index, dim_size: int, reduce: int):
        dev = L.require_device(src, index)
        E = src.size(0)
        from .graph import build_view
        ids = torch.arange(E, dtype=torch.int64, device=dev)
        view = build_view(index, ids, dim_size, E)
        Y, argmax = spmm_fwd(view, None, src, reduce)
        # adjoint view: one slot per edge e, pointing at row index[e]
        view_t = CSRView(rowptr=torch.arange(E + 1, dtype=torch.int64, device=dev),
                         col=index.to(torch.int32).contiguous(),
                         eid=ids.to(torch.int32), n_rows=E, n_cols=dim_size)
        cnt = (view.rowptr[1:] - view.rowptr[:-1]).clamp_(min=1).to(torch.float32)
        ctx.view_t, ctx.reduce, ctx.cnt = view_t, reduce, cnt
        ctx.save_for_backward(argmax)
        return Y

    @staticmethod
    def backward(ctx, dY):
        (argmax,) = ctx.saved_tensors
        d_src = spmm_bwd(ctx.view_t, None, None, dY, ctx.reduce,
                         cnt=ctx.cnt if ctx.reduce == L.REDUCE_MEAN else None, argmax=argmax)
        return d_src, None, None, None


def scatter_(name: str, src: torch.Tensor, index: torch.Tensor, dim_size: int | None = None,
             out: torch.Tensor | None = None) -> torch.Tensor:
    """Drop-in for src/gcn_meta/models/common.py:37-66 ``scatter_``.

    'max' fills empty rows with -1e38 and then replaces exact fill values by 0
    (:57, :63-64); 'mean' divides by ``max(count, 1)``.  ``out`` is accepted
    for signature compatibility; like the reference's only caller (which
    passes none) it must be None.
    """
    assert name in ["add", "mean", "max"]
    if out is not None:
        raise NotImplementedError("scatter_(out=...) is not supported; the reference never uses it")
    if dim_size is None:
        dim_size = int(index.max().item()) + 1 if index.numel() else 0
    squeeze = src.dim() == 1
    x = src.unsqueeze(1) if squeeze else src
    y = _SegmentReduce.apply(x, index, int(dim_size), L.REDUCE_CODES[name])
    return y.squeeze(1) if squeeze else y


def segment_mean(x: torch.Tensor, ptr: torch.Tensor) -> torch.Tensor:
    """Mean of contiguous row segments [ptr[g], ptr[g+1]) (global_mean_pool)."""
    return _SegmentMean.apply(x, ptr)


class _SegmentMean(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, ptr):
        lib = L.load()
        x = _contig_f32(x, "x")
        ptr = ptr.to(torch.int64).contiguous()
        dev = L.require_device(x, ptr)
        G = ptr.numel() - 1
        out = torch.empty(G, x.size(1), dtype=torch.float32, device=dev)
        with L.device_guard(dev):
            rc = lib.mgcn_segment_mean(G, x.size(1), L.ptr(ptr), L.ptr(x), x.stride(0), L.ptr(out),
                                       out.stride(0), L.stream_of(dev))
        L.check(rc, "mgcn_segment_mean")
        ctx.save_for_backward(ptr)
        ctx.n = x.size(0)
        return out

    @staticmethod
    def backward(ctx, dout):
        (ptr,) = ctx.saved_tensors
        counts = (ptr[1:] - ptr[:-1])
        seg = torch.repeat_interleave(torch.arange(counts.numel(), device=ptr.device), counts,
                                      output_size=ctx.n)
        scale = counts.clamp(min=1).to(dout.dtype)
        return (dout / scale.unsqueeze(1))[seg], None


# ------------------------------------------------- packed table exchange
def pack_rows_count(rows: torch.Tensor, hdr: torch.Tensor, counts: torch.Tensor) -> None:
    """hdr[i, 2 w] = mask word w of rows[i] (its not-+0.0 bits), counts[i] =
    their number (``mgcn_pack_rows_count``; mgcn.dist's packed exchange).
    ``hdr`` is the [n, 2 F/32] int32 header of the packed chunk."""
    lib = L.load()
    rows = _contig_f32(rows, "rows")
    n, F = rows.shape
    dev = L.require_device(rows, hdr, counts)
    if hdr.shape != (n, 2 * (F // 32)) or hdr.dtype != torch.int32 or not hdr.is_contiguous() \
            or counts.shape != (n,) or counts.dtype != torch.int32:
        raise ValueError("pack_rows_count: hdr int32 [n, 2 F/32] contiguous, counts int32 [n]")
    if _TIMER is not None:
        _TIMER("pack_rows_count", True, n)
    with L.device_guard(dev):
        rc = lib.mgcn_pack_rows_count(n, F, L.ptr(rows), rows.stride(0), L.ptr(hdr),
                                      L.ptr(counts), L.stream_of(dev))
    if _TIMER is not None:
        _TIMER("pack_rows_count", False)
    L.check(rc, "mgcn_pack_rows_count")


def pack_rows_values(rows: torch.Tensor, offs: torch.Tensor, hdr: torch.Tensor,
                     vals: torch.Tensor) -> None:
    """vals[offs[i] ...] = the not-+0.0 words of rows[i] in order, and the
    header's value positions hdr[i, 2 w + 1] (``mgcn_pack_rows_values``)."""
    lib = L.load()
    rows = _contig_f32(rows, "rows")
    n, F = rows.shape
    dev = L.require_device(rows, offs, hdr, vals)
    if offs.shape != (n,) or offs.dtype != torch.int32 or vals.dtype != torch.int32 or \
            hdr.shape != (n, 2 * (F // 32)) or hdr.dtype != torch.int32 or not hdr.is_contiguous():
        raise ValueError("pack_rows_values: offs int32 [n], hdr int32 [n, 2 F/32], vals int32")
    if _TIMER is not None:
        _TIMER("pack_rows_values", True, n)
    with L.device_guard(dev):
        rc = lib.mgcn_pack_rows_values(n, F, L.ptr(rows), rows.stride(0), L.ptr(offs),
                                       L.ptr(hdr), L.ptr(vals), L.stream_of(dev))
    if _TIMER is not None:
        _TIMER("pack_rows_values", False)
    L.check(rc, "mgcn_pack_rows_values")


@dataclass
class PackedTable:
    """An exchange table as the zero-skipping exchange delivered it
    (``mgcn_packed_table``): C x P packed segments of ``seg_rows`` rows each
    (pack.hip's layout), segment s at word ``seg_off[s]`` of buffer
    ``bufs[seg_buf[s]]`` (one receive buffer per row chunk, or one for all).
    The fused 128- and 256-wide layer kernels gather from it in place
    (:func:`spmm_xw_fwd` / :func:`spmm_xw_bwd` with a PackedTable for X / dY,
    over a view whose columns are packed positions (s << row_bits) | i:
    :func:`packed_cols`).  At F = 128 every segment must lie within 2 GiB of
    the lowest buffer (the kernels read the table through one range: in
    practice, one buffer)."""
    bufs: list               # int32 tensors holding the segments (kept alive here)
    seg_buf: list            # segment s -> index into bufs
    seg_off: list            # segment s -> word offset in that buffer
    seg_rows: int
    row_bits: int
    F: int

    @property
    def n_seg(self) -> int:
        return len(self.seg_off)

    @property
    def words(self) -> torch.Tensor:
        return self.bufs[0]

    def c_struct(self):
        """The C descriptor: every segment's offset counted from the lowest
        buffer address (one device address space)."""
        if self.n_seg > 64:
            raise ValueError(f"PackedTable: {self.n_seg} segments (at most 64)")
        ptrs = [b.data_ptr() for b in self.bufs]
        anchor = min(ptrs)
        if any((p - anchor) % 4 for p in ptrs):
            raise ValueError("PackedTable: buffers must be 4-byte aligned")
        rel = [(p - anchor) // 4 for p in ptrs]
        t = L.PackedTableC()
        t.words = anchor
        t.n_words = max(r + b.numel() for r, b in zip(rel, self.bufs))
        t.n_seg = self.n_seg
        t.seg_rows = int(self.seg_rows)
        t.row_bits = int(self.row_bits)
        t.F = int(self.F)
        for s_, (bi, off) in enumerate(zip(self.seg_buf, self.seg_off)):
            t.seg_base[s_] = rel[bi] + int(off)
        return t


def packed_row_bits(seg_rows: int) -> int:
    return max(int(seg_rows - 1).bit_length(), 0)


def packed_cols(col: torch.Tensor, seg_rows: int, row_bits: int) -> torch.Tensor:
    """Table positions t (row t % seg_rows of segment t // seg_rows) ->
    packed positions (s << row_bits) | i, int32."""
    t = col.to(torch.int64)
    s_ = torch.div(t, seg_rows, rounding_mode="floor")
    return ((s_ << row_bits) | (t - s_ * seg_rows)).to(torch.int32)


PACK_ROWS_WIDTHS = (32, 64, 128, 256)  # mgcn_pack_rows: one 256-word segment per row


def pack_rows(rows: torch.Tensor, hdr: torch.Tensor, vals: torch.Tensor,
              total: torch.Tensor) -> None:
    """The packed chunk in one pass (``mgcn_pack_rows``): hdr as
    pack_rows_count + pack_rows_values write it, vals, and total[0] = the
    number of values (device int64) -- no counts, no scan."""
    lib = L.load()
    rows = _contig_f32(rows, "rows")
    n, F = rows.shape
    dev = L.require_device(rows, hdr, vals, total)
    if F not in PACK_ROWS_WIDTHS or hdr.shape != (n, 2 * (F // 32)) or hdr.dtype != torch.int32 \
            or not hdr.is_contiguous() or vals.dtype != torch.int32 or total.dtype != torch.int64 \
            or total.numel() < 1:
        raise ValueError("pack_rows: F in (32, 64, 128, 256), hdr int32 [n, 2 F/32] contiguous, "
                         "vals int32, total int64")
    ws_bytes = int(lib.mgcn_pack_rows_workspace_bytes(n, F))
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev) if ws_bytes else None
    if _TIMER is not None:
        _TIMER("pack_rows", True, n)
    with L.device_guard(dev):
        rc = lib.mgcn_pack_rows(n, F, L.ptr(rows), rows.stride(0), L.ptr(hdr), L.ptr(vals),
                                L.ptr(total), L.ptr(ws), ws_bytes, L.stream_of(dev))
    if _TIMER is not None:
        _TIMER("pack_rows", False)
    L.check(rc, "mgcn_pack_rows")


def unpack_rows(buf: torch.Tensor, n_seg: int, n: int, seg_words: int, out: torch.Tensor) -> None:
    """out[p n + i] = row i of packed segment p of ``buf`` (``mgcn_unpack_rows``)."""
    lib = L.load()
    dev = L.require_device(buf, out)
    F = out.size(1)
    if buf.dtype != torch.int32 or not buf.is_contiguous() or buf.numel() < n_seg * seg_words or \
            out.dtype != torch.float32 or out.size(0) < n_seg * n or out.stride(1) != 1:
        raise ValueError("unpack_rows: buf int32 [n_seg * seg_words], out float32 [n_seg * n, F]")
    if _TIMER is not None:
        _TIMER("unpack_rows", True, n_seg * n)
    with L.device_guard(dev):
        rc = lib.mgcn_unpack_rows(n_seg, n, F, L.ptr(buf), seg_words, L.ptr(out), out.stride(0),
                                  L.stream_of(dev))
    if _TIMER is not None:
        _TIMER("unpack_rows", False)
    L.check(rc, "mgcn_unpack_rows")

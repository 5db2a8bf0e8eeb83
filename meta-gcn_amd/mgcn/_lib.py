"""ctypes binding of libmgcn.so (the C ABI declared in include/mgcn.h).

The product path has exactly one implementation: the HIP kernels in this
library.  If the library is missing, or a tensor is not on a HIP device, the
call raises -- there is no CPU fallback anywhere in :mod:`mgcn`.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libmgcn.so")

# constants mirrored from include/mgcn.h
ABI_VERSION = 22
OK, EINVAL, EINDEX, EHIP, EWORKSPACE, EDEVICE = 0, 1, 2, 3, 4, 5
REDUCE_SUM, REDUCE_MEAN, REDUCE_MAX = 0, 1, 2
NORM_NONE, NORM_SM, NORM_RW = 0, 1, 2
MAX_FILL = -1e38

REDUCE_CODES = {"add": REDUCE_SUM, "sum": REDUCE_SUM, "mean": REDUCE_MEAN, "max": REDUCE_MAX}
NORM_CODES = {None: NORM_NONE, "sm": NORM_SM, "rw": NORM_RW}

_vp = ctypes.c_void_p
_i64 = ctypes.c_int64
_i32 = ctypes.c_int32
_int = ctypes.c_int
_sz = ctypes.c_size_t

# name -> (restype, argtypes); every symbol include/mgcn.h declares
SIGNATURES = {
    "mgcn_abi_version": (_int, []),
    "mgcn_last_error": (ctypes.c_char_p, []),
    "mgcn_set_option": (_int, [ctypes.c_char_p, _int]),
    "mgcn_check_device": (_int, [_vp, _int]),
    "mgcn_csr_workspace_bytes": (_sz, [_i64, _i64]),
    "mgcn_csr_build": (_int, [_vp, _vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _sz, _vp]),
    "mgcn_degree_norm": (_int, [_i64, _vp, _vp, _vp, _vp, _int, _vp, _vp, _vp]),
    "mgcn_edge_norm": (_int, [_i64, _i64, _vp, _vp, _vp, _int, _vp, _vp, _int, _vp, _vp]),
    "mgcn_spmm_fwd": (_int, [_i64, _i32, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _i64, _int, _vp,
                             _int, _vp, _vp, _vp, _vp, _i64, _i64, _vp]),
    "mgcn_relu_mask": (_int, [_i64, _i32, _vp, _i64, _vp, _vp]),
    "mgcn_spmm_bwd": (_int, [_i64, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _i64, _int,
                             _vp, _vp, _vp, _vp, _int, _vp, _i64, _i64, _vp]),
    "mgcn_slot_map_workspace_bytes": (_sz, [_i64]),
    "mgcn_slot_map": (_int, [_i64, _vp, _vp, _vp, _vp, _sz, _vp]),
    "mgcn_max_mask": (_int, [_i64, _i32, _vp, _vp, _vp, _vp, _vp]),
    "mgcn_row_schedule_workspace_bytes": (_sz, [_i64]),
    "mgcn_row_schedule": (_int, [_i64, _vp, _i64, _vp, ctypes.POINTER(ctypes.c_int64),
                                 ctypes.POINTER(ctypes.c_int64), _vp, _sz, _vp]),
    "mgcn_gemm_tn_workspace_bytes": (_sz, [_i64, _i32, _i32]),
    "mgcn_gemm_tn": (_int, [_i64, _i32, _i32, _vp, _i64, _vp, _i64, _vp, _i64, _int, _vp, _sz,
                            _vp]),
    "mgcn_gemm_tn_split": (_int, [_i64, _i32, _i32, _i32, _vp, _i64, _vp, _i64, _vp, _i64, _vp,
                                  _i64, _int, _vp, _sz, _vp]),
    "mgcn_gemm_small_k": (_int, [_i64, _i32, _i32, _vp, _i64, _vp, _i64, _i64, _vp, _i64, _vp]),
    "mgcn_gemm_nn_supported": (_int, [_i32, _i32]),
    "mgcn_gemm_nn_fast": (_int, [_i32, _i32]),
    "mgcn_gemm_nn_epi_supported": (_int, [_i32, _i32]),
    "mgcn_gemm_nn_workspace_bytes": (_sz, [_i64, _i32]),
    "mgcn_gemm_nn": (_int, [_i64, _i32, _i32, _vp, _i64, _vp, _i64, _i64, _vp, _i64, _vp,
                            _vp, _vp, _vp, _sz, _vp]),
    "mgcn_gemm_bwd_supported": (_int, [_i32, _i32]),
    "mgcn_gemm_bwd_workspace_bytes": (_sz, [_i64, _i32, _i32]),
    "mgcn_gemm_bwd": (_int, [_i64, _i32, _i32, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _i64, _int,
                             _vp, _i64, _vp, _vp, _vp, _vp, _sz, _vp]),
    "mgcn_gemm_bwd_dw_cs_workspace_bytes": (_sz, [_i64]),
    "mgcn_gemm_bwd_dw_cs": (_int, [_i64, _vp, _i64, _vp, _i64, _vp, _i64, _int, _vp, _vp, _i64, _vp,
                                   _vp, _sz, _vp]),
    "mgcn_edge_weight_grad": (_int, [_i64, _i32, _vp, _vp, _vp, _i64, _vp, _i64, _vp, _vp, _vp]),
    "mgcn_edge_merge_workspace_bytes": (_sz, [_i64, _i64]),
    "mgcn_edge_merge_greedy": (_int, [_i64, _i64, _vp, _vp, _vp, _vp, _sz, _vp, _vp, _vp, _vp]),
    "mgcn_spmm_xw_supported": (_int, [_i32, _i32, _int]),
    "mgcn_spmm_xw_bwd_full_supported": (_int, [_i32, _i32]),
    "mgcn_spmm_xw_fwd_workspace_bytes": (_sz, [_i32, _i32]),
    "mgcn_spmm_xw_fwd": (_int, [_i64, _i64, _i32, _i32, _vp, _vp, _vp, _vp, _i64, _vp, _i64, _vp, _vp,
                                _i64, _int, _int, _vp, _vp, _i64, _vp, _sz, _vp]),
    "mgcn_spmm_xw_bwd_workspace_bytes": (_sz, [_i64, _i32, _i32]),
    "mgcn_spmm_xw_bwd": (_int, [_i64, _i64, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _i64,
                                _vp, _i64, _vp, _i64, _int, _vp, _i64, _vp, _vp, _vp, _vp, _vp,
                                _vp, _sz, _vp]),
    "mgcn_spmm_xw_bwd_hcs": (_int, [_i64, _i64, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _i64, _vp,
                                    _i64, _vp, _i64, _int, _vp, _i64, _vp, _vp, _vp, _vp, _vp,
                                    _sz, _vp]),
    "mgcn_gemm_batched": (_int, [_i64, _i32, _i32, _i32, _vp, _i64, _i64, _i64, _vp, _i64, _i64,
                                 _i64, _vp, _i64, _i64, _i64, _int, _vp]),
    "mgcn_colsum_workspace_bytes": (_sz, [_i64, _i32]),
    "mgcn_relu_bwd_colsum": (_int, [_i64, _i32, _vp, _vp, _int, _vp, _vp, _vp, _vp, _sz, _vp]),
    "mgcn_residual_act": (_int, [_i64, _i32, _vp, _i64, _vp, _i64, _vp, _int, _vp, _i64, _vp]),
    "mgcn_residual_act_bwd_workspace_bytes": (_sz, [_i64, _i32]),
    "mgcn_input_layer_supported": (_int, [_i32, _i32]),
    "mgcn_input_layer_fwd": (_int, [_i64, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _int, _int, _vp,
                                    _i64, _vp]),
    "mgcn_input_layer_bwd_workspace_bytes": (_sz, [_i64, _i32]),
    "mgcn_input_layer_bwd": (_int, [_i64, _i32, _vp, _i64, _vp, _i64, _vp, _vp, _vp, _vp, _vp,
                                    _int, _int, _vp, _vp, _vp, _vp, _vp, _sz, _vp]),
    "mgcn_residual_act_bwd": (_int, [_i64, _i32, _vp, _i64, _vp, _i64, _int, _vp, _i64, _int, _vp,
                                     _vp, _i64, _vp, _i64, _vp, _vp, _sz, _vp]),
    "mgcn_segment_mean": (_int, [_i64, _i32, _vp, _vp, _i64, _vp, _i64, _vp]),
    "mgcn_residual_layer_supported": (_int, [_i32, _i32, _int]),
    "mgcn_residual_layer_fwd": (_int, [_i64, _i32, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _i64, _vp,
                                       _vp, _i64, _vp, _int, _int, _int, _vp, _i64, _vp, _vp,
                                       _i64, _i64, _vp]),
    "mgcn_residual_stack_fwd": (_int, [_i64, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp,
                                       _vp, _vp, _int, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _vp]),
    "mgcn_residual_stack_bwd_workspace_bytes": (_sz, [_i64, _i32]),
    "mgcn_residual_stack_bwd": (_int, [_i64, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64,
                                       _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                       _vp, _vp, _i64, _i64, _vp, _sz, _vp]),
    "mgcn_pack_rows_count": (_int, [_i64, _i32, _vp, _i64, _vp, _vp, _vp]),
    "mgcn_pack_rows_values": (_int, [_i64, _i32, _vp, _i64, _vp, _vp, _vp, _vp]),
    "mgcn_unpack_rows": (_int, [_i64, _i64, _i32, _vp, _i64, _vp, _i64, _vp]),
    "mgcn_pack_rows_workspace_bytes": (_sz, [_i64, _i32]),
    "mgcn_pack_rows": (_int, [_i64, _i32, _vp, _i64, _vp, _vp, _vp, _vp, _sz, _vp]),
    "mgcn_spmm_xw_fwd_packed": (_int, [_i64, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp,
                                       _i64, _int, _int, _vp, _vp, _i64, _vp, _sz, _vp]),
    "mgcn_spmm_xw_bwd_packed": (_int, [_i64, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp,
                                       _i64, _vp, _vp, _vp, _int, _vp, _sz, _vp]),
    "mgcn_residual_layer_bwd_workspace_bytes": (_sz, [_i64, _i32]),
    "mgcn_residual_layer_bwd": (_int, [_i64, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp,
                                       _int, _int, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _i64, _vp,
                                       _vp, _i64, _i64, _vp, _sz, _vp]),
}

class PackedTableC(ctypes.Structure):
    """include/mgcn.h mgcn_packed_table."""
    _fields_ = [("words", ctypes.c_void_p), ("n_words", ctypes.c_int64),
                ("n_seg", ctypes.c_int32), ("seg_rows", ctypes.c_int32),
                ("row_bits", ctypes.c_int32), ("F", ctypes.c_int32),
                ("seg_base", ctypes.c_int64 * 64)]


byref = ctypes.byref

_lock = threading.Lock()
_lib = None


class MgcnError(RuntimeError):
    """A libmgcn call failed (bad argument, bad index, HIP error)."""


def load(path: str | None = None) -> ctypes.CDLL:
    """Load libmgcn.so (after torch, so the HIP runtime torch already mapped
    is the one the library binds to) and declare every C signature."""
    global _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        p = path or os.environ.get("MGCN_LIB") or LIB_PATH  # MGCN_LIB: experiment builds
        if not os.path.exists(p):
            raise MgcnError(
                f"libmgcn.so not found at {p}: build it with "
                "`make -C meta-gcn_amd/csrc` (or __graft_entry__.build()); "
                "mgcn has no CPU fallback")
        lib = ctypes.CDLL(p)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.mgcn_abi_version() != ABI_VERSION:
            raise MgcnError(f"libmgcn ABI {lib.mgcn_abi_version()} != expected {ABI_VERSION}")
        # tuning knobs from the environment: MGCN_OPTIONS="name=value,..."
        for item in filter(None, os.environ.get("MGCN_OPTIONS", "").split(",")):
            name, _, value = item.partition("=")
            rc = lib.mgcn_set_option(name.strip().encode(), int(value))
            if rc != OK:
                raise MgcnError(f"MGCN_OPTIONS {item!r}: "
                                f"{lib.mgcn_last_error().decode(errors='replace')}")
        if path is None:
            _lib = lib
        return lib


def check(rc: int, what: str) -> None:
    if rc != OK:
        msg = load().mgcn_last_error().decode(errors="replace")
        if rc == EINDEX:
            raise IndexError(f"{what}: {msg}")
        raise MgcnError(f"{what} failed (code {rc}): {msg}")


def ptr(t: torch.Tensor | None):
    """Raw device address of a tensor (None -> NULL)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


def require_device(*tensors: torch.Tensor | None) -> torch.device:
    """All tensors must live on one HIP device; returns it.  Raises for CPU
    tensors: the engine is GPU-only and never falls back to a CPU path."""
    dev = None
    for t in tensors:
        if t is None:
            continue
        if t.device.type != "cuda":
            raise MgcnError(
                f"mgcn kernels run on a HIP device only; got a tensor on {t.device} "
                "(move the graph and features to 'cuda')")
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise MgcnError(f"tensors on different devices: {dev} vs {t.device}")
    if dev is None:
        raise MgcnError("no tensor given")
    return dev


def stream_of(device: torch.device):
    """The caller's current HIP stream on `device` (kernels launch there).
    The raw handle straight from the C++ stream registry: a torch Stream
    object per launch costs more host time than the launch (config 3 issues
    ~200 launches a step and is bound by host issue)."""
    return ctypes.c_void_p(torch._C._cuda_getCurrentRawStream(device.index))


class _NoGuard:
    __slots__ = ()

    def __enter__(self):
        return None

    def __exit__(self, *exc):
        return False


_NO_GUARD = _NoGuard()


def device_guard(device: torch.device):
    """torch.cuda.device(device) when it differs from the current device,
    else a no-op context (the common case; the full guard costs two device
    switches of host time per launch)."""
    if device.index is None or device.index == torch._C._cuda_getDevice():
        return _NO_GUARD
    return torch.cuda.device(device)


def check_device(device: torch.device | None = None, sync: bool = True) -> None:
    """Raise if a libmgcn kernel reported a failure from the device
    (``mgcn_check_device``; MGCN_EDEVICE: a warp-specialised kernel left a
    hand-off at its spin bound, so that launch's outputs are invalid).
    ``sync`` first synchronises the current stream of ``device`` (default:
    the current device), covering every launch issued on it so far."""
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device())
    check(load().mgcn_check_device(stream_of(device), 1 if sync else 0), "mgcn_check_device")


def set_option(name: str, value: int) -> None:
    check(load().mgcn_set_option(name.encode(), int(value)), f"mgcn_set_option({name})")

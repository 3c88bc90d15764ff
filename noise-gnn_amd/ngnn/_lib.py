"""ctypes binding of libngnn.so (C ABI declared in include/ngnn.h).

The library is built in-tree by ``noise-gnn_amd/csrc/Makefile`` into
``noise-gnn_amd/ngnn/lib/libngnn.so``.  There is no fallback: if the library
is missing, every op raises.  Loading the library needs no GPU (it only links
libamdhip64), so CPU tests can check the exported symbols.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# NGNN_LIB: an alternative build of the same ABI (A/B kernel experiments);
# read once, at import
LIB_PATH = os.environ.get("NGNN_LIB") or os.path.join(_HERE, "lib", "libngnn.so")
ABI_VERSION = 21

OK = 0
SLOT_UNSORTED = 1  # ngnn_slot_load's err bits (include/ngnn.h NGNN_SLOT_*)
SLOT_RANGE = 2
E_ARG, E_DTYPE, E_SHAPE, E_ALIGN, E_RANGE, E_WORKSPACE = -1, -2, -3, -4, -5, -6
REDUCE = {"sum": 0, "add": 0, "mean": 1, "max": 2}
MATH_EXACT_F32 = 0x100  # OR-ed into ngnn_sage_fwd_raw's reduce (include/ngnn.h)
FWD_NARROW = 0x200      # same: output layer aggregated in the F_out-wide space
X_BF16 = 0x400          # same: x rows are bf16 (read as bf16, widened exactly)
W_BF16 = 0x800          # same: weights are bf16-exact (one split part)
WL_PREPACKED = 0x1000   # same: ws already holds ngnn_pack_weight(wl)
OUT_BF16 = 0x2000   # same: out rows bf16 (a bf16 model's hidden activations)
SAGE2_PREP, SAGE2_EDGE, SAGE2_MAIN, SAGE2_NARROW, SAGE2_ALL = 1, 2, 4, 8, 15  # ngnn_sage2_fwd stages
F32, BF16 = 0, 1

# name -> (restype, argtypes); mirrors include/ngnn.h one to one
_i64, _i32, _sz, _p, _int = ctypes.c_int64, ctypes.c_int32, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int
SIGNATURES = {
    "ngnn_abi_version": (_int, []),
    "ngnn_strerror": (ctypes.c_char_p, [_int]),
    "ngnn_edge_probe": (_int, [_p, _i64, _i64, _i64, _p, _p]),
    "ngnn_csr_workspace_bytes": (_sz, [_i64, _i64]),
    "ngnn_csr_build": (_int, [_p, _p, _i64, _i64, _int, _p, _p, _p, _p, _sz, _p]),
    "ngnn_seg_agg_fwd": (_int, [_p, _i64, _i64, _p, _p, _i64, _int, _int, _p, _i64, _p]),
    "ngnn_seg_agg_bwd_workspace_bytes": (_sz, [_i64, _i64, _int]),
    "ngnn_seg_agg_bwd": (_int, [_p, _i64, _i64, _p, _p, _i64, _p, _p, _i64, _int, _int,
                                _p, _i64, _p, _i64, _p, _i64, _p, _sz, _p]),
    "ngnn_sample_hop": (_int, [_p, _p, _p, _i64, _int, ctypes.c_uint64, _p, _p, _p]),
    "ngnn_sample_block_workspace_bytes": (_sz, [_i64, _p, _int]),
    "ngnn_sample_block": (_int, [_p, _p, _i64, _p, _i64, _p, _int, ctypes.c_uint64, _p, _p, _sz, _p,
                                 _p]),
    "ngnn_sample_block_finish": (_int, [_p, _int, _i64, _i64, _i64, _p, _i64, _p, _sz, _p, _p, _p,
                                        _p, _p, _i64, _i64, _p, _i64, _i64, _p, _p, _p, _p]),
    "ngnn_pack_weight_bytes": (_sz, [_i64, _i64]),
    "ngnn_pack_weight": (_int, [_p, _i64, _i64, _i64, _p, _p]),
    "ngnn_pack_weight_ex": (_int, [_p, _p, _i64, _i64, _i64, _i64, _int, _p, _p]),
    "ngnn_seed_xent_workspace_bytes": (_sz, [_i64]),
    "ngnn_seed_xent_fwd": (_int, [_p, _i64, _i64, _i64, _p, _i64, _p, _p, _p, _sz, _p]),
    "ngnn_seed_xent_bwd": (_int, [_p, _i64, _i64, _i64, _p, _i64, _p, _p, _p, _p, _i64, _p]),
    "ngnn_seed_xent_fwd_grad": (_int, [_p, _i64, _i64, _i64, _p, _i64, _p, _p, _p, _i64, _p, _sz,
                                       _p]),
    "ngnn_ct_loss_workspace_bytes": (_sz, [_i64]),
    "ngnn_ct_loss_fwd": (_int, [_p, _i64, _p, _i64, _i64, _i64, _p, _i64, _i64, _p, _p, _i64, _p,
                                _p, _p, _p, _sz, _p, _p]),
    "ngnn_ct_loss_bwd": (_int, [_int, _p, _i64, _i64, _i64, _p, _i64, _p, _p, _p, _i64, _p]),
    "ngnn_adam_step": (_int, [_int, _p, _p, _p, _p, _p, _p, _p, _p, ctypes.c_float, ctypes.c_float,
                              ctypes.c_float, ctypes.c_float, ctypes.c_float, _p, _p, _p]),
    "ngnn_slot_load": (_int, [_p, _i64, _i64, _i64, _p, _i64, _i64, _p, _i64, _p, _i64, _i64,
                              _p, _i64, _p, _p, _p, _p, _p, _p, _p, ctypes.c_uint32, _p, _p, _p,
                              _p, _p, _i64, _i64, _i64, _p, _p, _p, _p, _p]),
    "ngnn_sage_fwd": (_int, [_p, _i64, _i64, _i64, _p, _p, _p, _int, _p, _p, _p, _i64, _p, _i64,
                             _int, ctypes.c_float, ctypes.c_uint64, _p, _p, _i64, _p, _i64,
                             ctypes.c_float, _p]),
    "ngnn_sage_fwd_raw_workspace_bytes": (_sz, [_i64, _i64, _i64]),
    "ngnn_sage_wide_preferred": (_int, [_i64, _i64, _int]),
    "ngnn_sage_fwd_raw": (_int, [_p, _p, _p, _p, _i64, _i64, _i64, _i64, _p, _i64, _p, _p, _p, _p, _int, _p, _p,
                                 _i64, _p, _i64,
                                 _p, _i64, _int, ctypes.c_float, ctypes.c_uint64, _p, _p, _i64, _p,
                                 _sz, _p]),
    "ngnn_cast_tensors": (_int, [_int, _p, _p, _p, _int, _p]),
    "ngnn_cast_tensors_ex": (_int, [_int, _p, _p, _p, _p, _p, ctypes.c_float, _p]),
    "ngnn_sage2_bwd_workspace_bytes": (_sz, [_i64, _i64, _i64]),
    "ngnn_sage2_bwd": (_int, [_p, _i64, _i64, _p, _p, _i64, _p, _i64, ctypes.c_float, _p, _p, _p, _p, _i64, _i64,
                              _i64, _p, _i64, _p, _p, _i64, _p, _p, _int, _p, _p, _p, _p, _p, _p, _p, _p,
                              _p, _sz, _p]),
    "ngnn_sage2_supported": (_int, [_i64, _i64, _i64, _int]),
    "ngnn_sage2_workspace_bytes": (_sz, [_i64, _i64, _i64]),
    "ngnn_sage2_fwd": (_int, [_p, _p, _p, _p, _i64, _i64, _i64, _i64, _p, _i64, _p, _p, _p, _p, _int,
                              _p, _p, _p, _i64,
                              _i64, _p, _p, _p, _i64, _i64, ctypes.c_float, ctypes.c_uint64, _p, _p,
                              _i64, _i64, _p, _p, _i64, _p, _i64, _p, _int, _p, _sz, _p]),
    "ngnn_xent_head_workspace_bytes": (_sz, [_i64]),
    "ngnn_gcn_agg_fwd": (_int, [_p, _i64, _i64, _p, _p, _i64, _p, _p, _int, ctypes.c_float,
                                ctypes.c_uint64, _p, _p, _i64, _p]),
    "ngnn_row_extent": (_int, [_p, _i64, _i64, _i64, _p, _p]),
    "ngnn_block_prefix_stats": (_int, [_p, _p, _p, _p, _p, _i64, _p]),
    "ngnn_sage_wgrad_workspace_bytes": (_sz, [_i64, _i64]),
    "ngnn_cast_f32_bf16": (_int, [_p, _p, _i64, _p]),
    "ngnn_cast_f32_bf16_rows": (_int, [_p, _p, _i64, _i64, _p, _p]),
    "ngnn_widen_bf16_rows": (_int, [_p, _i64, _i64, _i64, _p, _p, _i64, _p]),
    "ngnn_sage_wgrad": (_int, [_p, _i64, _p, _i64, ctypes.c_float, _p, _p, _p, _p, _i64, _int, _i64, _p,
                               _i64, _p, _i64,
                               _p, _i64, _i64, _p, _p, _p, _p, _sz, _p]),
    "ngnn_sage_dgrad_workspace_bytes": (_sz, [_i64, _i64, _int]),
    "ngnn_sage_dgrad_gather": (_int, [_p, _i64, _p, _i64, _p, _p, _p, _p, _i64, _p, _p, _i64,
                                      _int, _p, _i64, _p, _i64, _p, _i64, _int, _p, _sz, _p]),
    "ngnn_sage_dgrad_scatter": (_int, [_p, _i64, _p, _i64, _p, _p, _i64, _p, _p, _i64, _int, _p,
                                       _i64, _p, _i64, _p, _i64, _int, _p]),
    "ngnn_sage_dgrad_fused": (_int, [_p, _i64, _p, _i64, ctypes.c_float, _p, _p, _i64, _i64, _p,
                                     _p, _i64, _p, _p, _int, _p, _i64, _p, _i64, _p, _i64, _int,
                                     _p]),
    "ngnn_sage_dgrad_lowdim_workspace_bytes": (_sz, [_i64, _i64, _i64]),
    "ngnn_sage_dgrad_lowdim": (_int, [_p, _i64, _p, _i64, ctypes.c_float, _p, _p, _i64, _i64,
                                      _i64, _p, _p, _i64, _p, _p, _int, _p, _i64, _int, _p, _sz,
                                      _p]),
}

_lib = None
_lock = threading.Lock()


class NGNNError(RuntimeError):
    pass


def load() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise NGNNError(
                    f"libngnn.so not found at {LIB_PATH}: build it with "
                    "`make -C noise-gnn_amd/csrc` (or __graft_entry__.build()); "
                    "there is no CPU fallback")
            lib = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(lib, name)
                fn.restype, fn.argtypes = res, args
            v = lib.ngnn_abi_version()
            if v != ABI_VERSION:
                raise NGNNError(f"libngnn ABI {v} != expected {ABI_VERSION}; rebuild")
            _lib = lib
    return _lib


def check(rc: int, what: str = "") -> None:
    if rc != OK:
        msg = load().ngnn_strerror(rc).decode()
        raise NGNNError(f"{what}: {msg} (rc={rc})" if what else f"{msg} (rc={rc})")


class XentHead(ctypes.Structure):
    """include/ngnn.h ngnn_xent_head (ngnn_sage2_fwd's loss head, ABI 15; src_count ABI 17)."""
    _fields_ = [("y", _p), ("B", _i64), ("ignore_index", _i64), ("loss", _p), ("count", _p),
                ("dy", _p), ("ldd", _i64), ("g", _p), ("g_rows", _i64), ("g_rows_dev", _p),
                ("ws", _p), ("ws_bytes", _sz), ("src_count", _p)]


class AdamFold(ctypes.Structure):
    """include/ngnn.h ngnn_adam_fold (ngnn_sage2_bwd's optimizer step, ABI 15; the gate ABI 20)."""
    _fields_ = [("param", _p * 6), ("exp_avg", _p * 6), ("exp_avg_sq", _p * 6), ("step", _p),
                ("lr", ctypes.c_float), ("beta1", ctypes.c_float),
                ("beta2", ctypes.c_float), ("eps", ctypes.c_float), ("weight_decay", ctypes.c_float),
                ("gate", _p), ("gate_gen", _p)]  # (ABI 20: the slot's contract gate)


def ptr(t) -> int:
    """Device address of a tensor (0 for None)."""
    return 0 if t is None else t.data_ptr()


_raw_stream = None


def stream_handle(device=None) -> int:
    """The raw hipStream_t of torch's current stream on `device` (torch's C
    accessor: torch.cuda.current_stream builds a Stream object per call,
    a few us of the host-bound eager step each)."""
    global _raw_stream
    import torch
    if _raw_stream is None:
        _raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None) or (
            lambda i: torch.cuda.current_stream(i).cuda_stream)
    if device is None:
        idx = torch.cuda.current_device()
    elif isinstance(device, int):
        idx = device
    else:
        idx = device.index if device.index is not None else torch.cuda.current_device()
    return _raw_stream(idx)

"""ctypes wrapper for oracle/seg_agg.c — ORACLE / TEST INFRASTRUCTURE ONLY."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "build", "liboracle_agg.so")
_lib = None

REDUCE = {"sum": 0, "add": 0, "mean": 1, "max": 2}


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _SO


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        lib = ctypes.CDLL(_SO)
        i64, p = ctypes.c_int64, ctypes.c_void_p
        lib.oracle_agg_fwd.argtypes = [p, i64, i64, p, p, i64, i64, ctypes.c_int, p, i64]
        lib.oracle_agg_bwd.argtypes = [p, i64, i64, p, p, i64, i64, i64, ctypes.c_int,
                                       p, i64, p, i64, p, i64]
        _lib = lib
    return _lib


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def _i64(a):
    return np.ascontiguousarray(a, dtype=np.int64)


def agg_fwd(x, edge_index, n_dst: int, reduce: str) -> np.ndarray:
    x, ei = _f32(x), _i64(edge_index)
    F = x.shape[1]
    out = np.empty((n_dst, F), np.float32)
    src, dst = np.ascontiguousarray(ei[0]), np.ascontiguousarray(ei[1])
    rc = _load().oracle_agg_fwd(x.ctypes.data, F, F, src.ctypes.data, dst.ctypes.data,
                                src.shape[0], n_dst, REDUCE[reduce], out.ctypes.data, F)
    assert rc == 0
    return out


def agg_bwd(grad_out, edge_index, n_src: int, reduce: str, x=None, agg=None) -> np.ndarray:
    g, ei = _f32(grad_out), _i64(edge_index)
    n_dst, F = g.shape
    src, dst = np.ascontiguousarray(ei[0]), np.ascontiguousarray(ei[1])
    gx = np.empty((n_src, F), np.float32)
    xp = _f32(x) if x is not None else np.zeros((1, F), np.float32)
    ap = _f32(agg) if agg is not None else np.zeros((1, F), np.float32)
    rc = _load().oracle_agg_bwd(g.ctypes.data, F, F, src.ctypes.data, dst.ctypes.data,
                                src.shape[0], n_src, n_dst, REDUCE[reduce], xp.ctypes.data, F,
                                ap.ctypes.data, F, gx.ctypes.data, F)
    assert rc == 0
    return gx

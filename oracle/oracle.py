"""CPU ORACLE bindings (test infrastructure only).

Thin ctypes/numpy front-end over ``oracle/libpcm_oracle.so`` (the scalar C
restatement in ``pcm_oracle.c``).  Only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg may import this module, and only as the
checker / the timed CPU baseline -- never as the product path.

Parity status: Chamfer pinned by tests/golden (reference utils/utils.py:246-290);
EMD partially pinned (reference invariant metric/emd/test.py:24-28 only; the rest
is "parity unpinned" beyond this deterministic restatement).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libpcm_oracle.so")
_lib = None

_f32p = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_i64p = np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS")


def build() -> None:
    """Compile the oracle (gcc) if the .so is missing or stale."""
    src = os.path.join(_HERE, "pcm_oracle.c")
    if (not os.path.exists(_LIB_PATH)) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src):
        subprocess.run(["make", "-C", _HERE], check=True, stdout=subprocess.DEVNULL)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        c_int, c_float = ctypes.c_int, ctypes.c_float
        L.pcm_oracle_chamfer_nn.argtypes = [_f32p, _f32p, c_int, c_int, c_int, _f32p, _i32p, c_int, c_int]
        L.pcm_oracle_chamfer_forward.argtypes = [_f32p, _f32p, c_int, c_int, c_int,
                                                 _f32p, _f32p, _i32p, _i32p, c_int]
        L.pcm_oracle_chamfer_backward.argtypes = [_f32p, _f32p, c_int, c_int, c_int, _f32p, _f32p,
                                                  _i32p, _i32p, _f32p, _f32p, c_int]
        L.pcm_oracle_emd_forward.argtypes = [_f32p, _f32p, c_int, c_int, c_float, c_int,
                                             _f32p, _i32p, ctypes.c_void_p, ctypes.c_void_p, c_int]
        L.pcm_oracle_emd_backward.argtypes = [_f32p, _f32p, c_int, c_int, _f32p, _i32p, _f32p]
        L.pcm_oracle_emd_values.argtypes = [_f32p, _f32p, _f32p, c_int, _f32p]
        L.pcm_oracle_emd_bid.argtypes = [_f32p, _f32p, _f32p, c_int, c_int, _i32p, _f32p, _f32p]
        L.pcm_oracle_emd_values.restype = None
        L.pcm_oracle_emd_bid.restype = None
        L.pcm_oracle_num_threads.restype = c_int
        for name in ("pcm_oracle_chamfer_nn", "pcm_oracle_chamfer_forward",
                     "pcm_oracle_chamfer_backward", "pcm_oracle_emd_forward",
                     "pcm_oracle_emd_backward"):
            getattr(L, name).restype = None
        _lib = L
    return _lib


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def _i32(a):
    return np.ascontiguousarray(a, dtype=np.int32)


def num_threads() -> int:
    return int(lib().pcm_oracle_num_threads())


def chamfer_nn(xyz, xyz2, order: int = 0, nthreads: int = 0):
    """One direction of NmDistanceKernel (chamfer3D.cu:12-134)."""
    xyz, xyz2 = _f32(xyz), _f32(xyz2)
    b, n, _ = xyz.shape
    m = xyz2.shape[1]
    dist = np.zeros((b, n), np.float32)
    idx = np.zeros((b, n), np.int32)
    lib().pcm_oracle_chamfer_nn(xyz, xyz2, b, n, m, dist, idx, order, nthreads)
    return dist, idx


def chamfer_forward(xyz1, xyz2, nthreads: int = 0):
    """chamfer_cuda_forward (chamfer3D.cu:136-154) -> dist1, dist2, idx1, idx2."""
    xyz1, xyz2 = _f32(xyz1), _f32(xyz2)
    b, n, _ = xyz1.shape
    m = xyz2.shape[1]
    d1 = np.zeros((b, n), np.float32)
    d2 = np.zeros((b, m), np.float32)
    i1 = np.zeros((b, n), np.int32)
    i2 = np.zeros((b, m), np.int32)
    lib().pcm_oracle_chamfer_forward(xyz1, xyz2, b, n, m, d1, d2, i1, i2, nthreads)
    return d1, d2, i1, i2


def chamfer_backward(xyz1, xyz2, graddist1, graddist2, idx1, idx2, nthreads: int = 0):
    """chamfer_cuda_backward (chamfer3D.cu:176-195), deterministic order."""
    xyz1, xyz2 = _f32(xyz1), _f32(xyz2)
    b, n, _ = xyz1.shape
    m = xyz2.shape[1]
    g1 = np.zeros((b, n, 3), np.float32)
    g2 = np.zeros((b, m, 3), np.float32)
    lib().pcm_oracle_chamfer_backward(xyz1, xyz2, b, n, m, _f32(graddist1), _f32(graddist2),
                                      _i32(idx1), _i32(idx2), g1, g2, nthreads)
    return g1, g2


def emd_forward(xyz1, xyz2, eps: float, iters: int, with_stats: bool = False, nthreads: int = 0):
    """emd_cuda_forward (emd_cuda.cu:228-282), deterministic tie rule.

    Returns (dist, assignment) or, with_stats, (dist, assignment, price, unass_hist)."""
    xyz1, xyz2 = _f32(xyz1), _f32(xyz2)
    b, n, _ = xyz1.shape
    dist = np.zeros((b, n), np.float32)
    ass = np.zeros((b, n), np.int32)
    price = np.zeros((b, n), np.float32)
    hist = np.zeros(max(iters, 1), np.int64)
    lib().pcm_oracle_emd_forward(xyz1, xyz2, b, n, float(eps), int(iters), dist, ass,
                                 price.ctypes.data, hist.ctypes.data if with_stats else None,
                                 nthreads)
    if with_stats:
        return dist, ass, price, hist[:iters]
    return dist, ass


def emd_values(p, xyz2, price):
    """Bid's value of every object for one bidder p (emd_cuda.cu:142-146)."""
    xyz2, price = _f32(xyz2), _f32(price)
    v = np.zeros(xyz2.shape[0], np.float32)
    lib().pcm_oracle_emd_values(_f32(p), xyz2, price, xyz2.shape[0], v)
    return v


def emd_bid(p, xyz2, price, nu):
    """One bidder's (best_i, best, better) with nu unassigned points (the
    reference's exact-tie order, emd_cuda.cu:95-179)."""
    xyz2, price = _f32(xyz2), _f32(price)
    bi = np.zeros(1, np.int32)
    b1 = np.zeros(1, np.float32)
    b2 = np.zeros(1, np.float32)
    lib().pcm_oracle_emd_bid(_f32(p), xyz2, price, xyz2.shape[0], int(nu), bi, b1, b2)
    return int(bi[0]), b1[0], b2[0]


def emd_backward(xyz1, xyz2, graddist, assignment):
    """emd_cuda_backward (emd_cuda.cu:284-316)."""
    xyz1, xyz2 = _f32(xyz1), _f32(xyz2)
    b, n, _ = xyz1.shape
    g = np.zeros((b, n, 3), np.float32)
    lib().pcm_oracle_emd_backward(xyz1, xyz2, b, n, _f32(graddist), _i32(assignment), g)
    return g

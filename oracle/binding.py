"""ctypes binding of oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg, as the checker / CPU baseline.  See oracle.h for what the C code restates
(reference file:line) and how it is pinned.
"""
from __future__ import annotations

import ctypes
import os
import time

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liboracle.so")

F32, F64 = 0, 1
STAR, BOX = 0, 1
NAIVE, DMA, LEX = 0, 1, 2


class Problem(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in ("dims", "dtype", "shape", "radius", "order", "reserved")] + \
               [(n, ctypes.c_int64) for n in ("nx", "ny", "nz")]


_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} missing: run `make -C oracle`")
        lib = ctypes.CDLL(LIB_PATH)
        P = ctypes.POINTER(Problem)
        lib.oracle_elems.restype = ctypes.c_int64
        lib.oracle_elems.argtypes = [P]
        lib.oracle_check.argtypes = [P]
        lib.oracle_init.argtypes = [P, ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p]
        lib.oracle_sweep.argtypes = [P, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int]
        lib.oracle_run.argtypes = [P, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        lib.oracle_fnv1a64_interior.restype = ctypes.c_uint64
        lib.oracle_fnv1a64_interior.argtypes = [P, ctypes.c_void_p]
        lib.oracle_sum_interior.restype = ctypes.c_double
        lib.oracle_sum_interior.argtypes = [P, ctypes.c_void_p]
        _lib = lib
    return _lib


def problem(dims=2, dtype="fp32", shape="star", radius=1, order="naive", nx=1, ny=1, nz=1) -> Problem:
    return Problem(dims, F64 if dtype == "fp64" else F32, BOX if shape == "box" else STAR, radius,
                   {"dma": DMA, "lex": LEX}.get(order, NAIVE), 0, nx, ny, nz if dims == 3 else 1)


def dense_shape(p: Problem):
    r = p.radius
    if p.dims == 3:
        return (p.nz + 2 * r, p.ny + 2 * r, p.nx + 2 * r)
    return (p.ny + 2 * r, p.nx + 2 * r)


def np_dtype(p: Problem):
    return np.float64 if p.dtype == F64 else np.float32


def _ptr(a: np.ndarray):
    assert a.flags["C_CONTIGUOUS"]
    return ctypes.c_void_p(a.ctypes.data)


def init(p: Problem, kind: str = "reference", seed: int = 0) -> np.ndarray:
    lib = load()
    a = np.empty(dense_shape(p), dtype=np_dtype(p))
    rc = lib.oracle_init(ctypes.byref(p), 1 if kind == "random" else 0, ctypes.c_uint64(seed & (2**64 - 1)), _ptr(a))
    if rc:
        raise ValueError(f"oracle_init: {rc}")
    return a


def sweep(p: Problem, src: np.ndarray, dst: np.ndarray, begin: int, end: int, threads: int = 1) -> None:
    rc = load().oracle_sweep(ctypes.byref(p), _ptr(src), _ptr(dst), begin, end, threads)
    if rc:
        raise ValueError(f"oracle_sweep: {rc}")


def run(p: Problem, iterations: int, kind: str = "reference", seed: int = 0, threads: int = 1) -> np.ndarray:
    """Final ghost-padded grid after `iterations` sweeps."""
    a = init(p, kind, seed)
    b = a.copy()
    w = load().oracle_run(ctypes.byref(p), iterations, _ptr(a), _ptr(b), threads)
    if w < 0:
        raise ValueError(f"oracle_run: {w}")
    return b if w == 1 else a


def timed_run(p: Problem, iterations: int, threads: int = 1):
    a = init(p)
    b = a.copy()
    t0 = time.perf_counter()
    load().oracle_run(ctypes.byref(p), iterations, _ptr(a), _ptr(b), threads)
    return time.perf_counter() - t0


def interior(p: Problem, g: np.ndarray) -> np.ndarray:
    r = p.radius
    if p.dims == 3:
        return g[r:-r, r:-r, r:-r]
    return g[r:-r, r:-r]


def fnv1a64(p: Problem, g: np.ndarray) -> int:
    return int(load().oracle_fnv1a64_interior(ctypes.byref(p), _ptr(g)))


def interior_sum(p: Problem, g: np.ndarray) -> float:
    return float(load().oracle_sum_interior(ctypes.byref(p), _ptr(g)))

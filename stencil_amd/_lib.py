"""ctypes binding of libstencil_hip.so (include/stencil_hip.h).

The shared library is the product: every sweep runs as a gfx950 HIP kernel
behind the C-ABI.  There is no Python or CPU fallback; if the library is
missing or cannot be loaded this module raises immediately.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, Structure, c_char_p, c_double, c_float, c_int, c_int32, c_int64, c_uint32, c_uint64, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libstencil_hip.so")
# The same kernels linked with the experiment knobs enabled (Makefile,
# csrc/knobs.cpp): loaded when a STENCIL_* variable other than the documented
# ones is set, i.e. by the shape-sweep tests and the A/B tools.
DEBUG_LIB_PATH = os.path.join(_HERE, "libstencil_hip_debug.so")
API_KNOBS = ("STENCIL_TK_STEPS", "STENCIL_BOX_STEPS", "STENCIL_TK_PACK", "STENCIL_BOXK_PACK", "STENCIL_SLAB_SIGNAL",
             "STENCIL_SLAB_CPWAIT", "STENCIL_SLAB_SERIAL", "STENCIL_SLAB_XCU", "STENCIL_SLAB_XCU_EXCL",
             "STENCIL_SLAB_TIMEOUT_MS", "STENCIL_SLAB_ROLLING_OVERLAP", "STENCIL_SLAB_STAGED", "STENCIL_SLAB_GATE",
             "STENCIL_SLAB_PLACEMENTS", "STENCIL_SLAB_XCU_ALT")

STENCIL_OK = 0
ETIMEOUT = -6
SLAB_FORMS = {0: "boundary + interior launches", 1: "face-signalled launches", 2: "rolling passes",
              3: "serial launches (whole slab, then the exchange)",
              4: "staged launches (the face quarters, then the middle beside the exchange)"}
F32, F64 = 0, 1
STAR, BOX = 0, 1
ORDER_NAIVE, ORDER_DMA = 0, 1
KERNEL_AUTO, KERNEL_DIRECT, KERNEL_ZMARCH, KERNEL_TEMPORAL2, KERNEL_TEMPORALK, KERNEL_PERSISTENT = 0, 1, 2, 3, 4, 5
INIT_REFERENCE, INIT_RANDOM = 0, 1
HALO_LO, HALO_HI = 1, 2
EXCHANGE_RCCL, EXCHANGE_COPY = 0, 1
SLAB_PERIODIC, SLAB_ROLLING = 1, 2
SLAB_ID_BYTES = 128

KERNEL_NAMES = {"auto": KERNEL_AUTO, "direct": KERNEL_DIRECT, "zmarch": KERNEL_ZMARCH, "temporal2": KERNEL_TEMPORAL2,
                "temporalk": KERNEL_TEMPORALK, "persistent": KERNEL_PERSISTENT}

# Every symbol include/stencil_hip.h declares (checked by tests/test_abi.py).
EXPORTED_SYMBOLS = (
    "stencil_strerror", "stencil_last_error_message", "stencil_last_error", "stencil_debug_knobs",
    "stencil_iterate_dma", "stencil_iterate_dma_static_unroll", "stencil_iterate_dma_slave_pack",
    "stencil_iterate_rma",
    "stencil_layout_init", "stencil_slow_extent", "stencil_device_count", "stencil_set_device",
    "stencil_synchronize", "stencil_alloc", "stencil_free", "stencil_fill_initial", "stencil_upload",
    "stencil_download", "stencil_copy_planes", "stencil_sweep", "stencil_sweep2", "stencil_sweepk", "stencil_iterate",
    "stencil_prepare", "stencil_rolling_bytes", "stencil_rolling_init_margin", "stencil_rolling_iterate",
    "stencil_pack_plan", "stencil_plan", "stencil_plane_sums", "stencil_copy_bandwidth", "stencil_sweepk_geometry", "stencil_sweepk_signal",
    "stencil_wait_counters", "stencil_face_signal_create", "stencil_face_signal_destroy",
    "stencil_face_signal_reset", "stencil_face_signal_read", "stencil_wait_face_signal",
    "stencil_slab_create", "stencil_slab_destroy", "stencil_slab_info", "stencil_slab_fill_initial",
    "stencil_slab_upload", "stencil_slab_download", "stencil_slab_run", "stencil_slab_plane_sums",
    "stencil_slab_kernel_timing", "stencil_slab_kernel_time", "stencil_slab_unique_id", "stencil_slab_create_rank",
    "stencil_slab_create2", "stencil_slab_create_rank2", "stencil_slab_rolling_info", "stencil_slab_round_form",
    "stencil_slab_set_timeout", "stencil_prepare2", "stencil_slab_exchange_time",
    "stencil_sweepk_signal_gated", "stencil_exchange_done", "stencil_slab_round_info", "stencil_pack_table",
    "stencil_slab_exchange_budget",
)


class Problem(Structure):
    _fields_ = [("dims", c_int32), ("dtype", c_int32), ("shape", c_int32), ("radius", c_int32),
                ("order", c_int32), ("kernel", c_int32), ("halo", c_int32), ("flags", c_int32),
                ("nx", c_int64), ("ny", c_int64), ("nz", c_int64)]


class Layout(Structure):
    _fields_ = [("prob", Problem), ("row", c_int64), ("plane", c_int64), ("planes", c_int64),
                ("zghost", c_int64), ("rows", c_int64), ("origin", c_int64), ("elems", c_int64),
                ("bytes", c_int64)]


class MatrixView(Structure):
    """Layout of detail::BoundaryMatrix<float,false> (boundary_matrix.hpp:225-237)."""
    _fields_ = [("actual_width", ctypes.c_size_t), ("actual_height", ctypes.c_size_t),
                ("boundary_width", ctypes.c_uint), ("boundary_height", ctypes.c_uint),
                ("data_stride", ctypes.c_size_t), ("data", POINTER(c_float))]


class Arguments(Structure):
    """Layout of struct Arguments (stencil_slave.hpp:13-24)."""
    _fields_ = [("block_size", ctypes.c_uint), ("iterations", ctypes.c_uint),
                ("input", MatrixView), ("output", MatrixView)]


class StencilError(RuntimeError):
    def __init__(self, code: int, where: str, message: str):
        super().__init__(f"{where}: error {code}: {message}")
        self.code = code


_libs: dict = {}


def debug_knobs_requested() -> bool:
    """Is an experiment knob (a STENCIL_* variable the product ignores) set?"""
    return any(k.startswith("STENCIL_") and k not in API_KNOBS for k in os.environ)


def load(debug: bool | None = None) -> ctypes.CDLL:
    """Load libstencil_hip.so (or, with experiment knobs set / debug=True, its
    debug twin) once; raise if it is absent (no fallback)."""
    if debug is None:
        debug = debug_knobs_requested()
    if debug in _libs:
        return _libs[debug]
    path = DEBUG_LIB_PATH if debug else LIB_PATH
    if not os.path.exists(path):
        raise ImportError(
            f"{path} is missing: the HIP extension has not been built "
            "(run `make` or `python -c 'import __graft_entry__ as g; g.build()'`)")
    lib = ctypes.CDLL(path)
    for name, (res, args) in signatures().items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    for name in ("stencil_iterate_dma", "stencil_iterate_dma_static_unroll",
                 "stencil_iterate_dma_slave_pack", "stencil_iterate_rma"):
        fn = getattr(lib, name)
        fn.restype = None
        fn.argtypes = [POINTER(Arguments)]
    _libs[debug] = lib
    return lib


def signatures() -> dict:
    """(restype, argtypes) of every C-ABI function but the four reference
    entry points (tests/cpu_slab/binding.py reuses the stencil_slab_* ones)."""
    P, L = POINTER(Problem), POINTER(Layout)
    return {
        "stencil_strerror": (c_char_p, [c_int]),
        "stencil_last_error_message": (c_char_p, []),
        "stencil_last_error": (c_int, []),
        "stencil_debug_knobs": (c_int, []),
        "stencil_layout_init": (c_int, [P, L]),
        "stencil_slow_extent": (c_int64, [L]),
        "stencil_device_count": (c_int, [POINTER(c_int)]),
        "stencil_set_device": (c_int, [c_int]),
        "stencil_synchronize": (c_int, [c_void_p]),
        "stencil_alloc": (c_int, [L, POINTER(c_void_p)]),
        "stencil_free": (c_int, [c_void_p]),
        "stencil_fill_initial": (c_int, [L, c_void_p, c_int, c_uint64, c_void_p]),
        "stencil_upload": (c_int, [L, c_void_p, c_void_p, c_int64, c_int64, c_void_p]),
        "stencil_download": (c_int, [L, c_void_p, c_void_p, c_int64, c_int64, c_void_p]),
        "stencil_copy_planes": (c_int, [L, c_void_p, c_int64, c_void_p, c_int64, c_int64, c_void_p]),
        "stencil_sweep": (c_int, [L, c_void_p, c_void_p, c_int64, c_int64, c_void_p]),
        "stencil_sweep2": (c_int, [L, c_void_p, c_void_p, c_int64, c_int64, c_void_p]),
        "stencil_sweepk": (c_int, [L, c_void_p, c_void_p, c_int64, c_int64, c_int32, c_void_p]),
        "stencil_iterate": (c_int, [L, c_void_p, c_void_p, c_uint32, c_void_p, POINTER(c_int), POINTER(c_float)]),
        "stencil_prepare": (c_int, [L, c_void_p, c_void_p, c_void_p]),
        "stencil_prepare2": (c_int, [L, c_void_p, c_void_p, c_void_p, POINTER(c_int64), POINTER(c_float)]),
        "stencil_rolling_bytes": (c_int, [L, c_int64, POINTER(c_int64), POINTER(c_int32)]),
        "stencil_rolling_init_margin": (c_int, [L, c_void_p, c_int64, c_void_p]),
        "stencil_rolling_iterate": (c_int, [L, c_void_p, c_int64, c_uint32, POINTER(c_int32), c_void_p,
                                            POINTER(c_int64), POINTER(c_float)]),
        "stencil_pack_plan": (c_int, [c_int64, c_int64, c_int32, c_int32, c_int32, POINTER(c_int64),
                                      POINTER(c_int64), POINTER(c_int64)]),
        "stencil_pack_table": (c_int, [c_int64, c_int64, c_int64, c_int32, c_int32, c_int32, c_int32, POINTER(c_int32),
                                       c_int64, POINTER(c_int64)]),
        "stencil_plan": (c_int, [L, c_uint32, POINTER(c_int64), POINTER(c_int32)]),
        "stencil_plane_sums": (c_int, [L, c_void_p, POINTER(c_double), c_void_p]),
        "stencil_copy_bandwidth": (c_int, [c_void_p, c_void_p, c_int64, c_int, c_void_p, POINTER(c_float)]),
        "stencil_sweepk_geometry": (c_int, [L, c_int64, c_int64, c_int32, POINTER(c_int64), POINTER(c_int32),
                                            POINTER(c_int32)]),
        "stencil_sweepk_signal": (c_int, [L, c_void_p, c_void_p, c_int64, c_int64, c_int32, c_void_p, c_void_p,
                                          POINTER(c_int32), c_void_p]),
        "stencil_wait_counters": (c_int, [c_void_p, c_uint32, c_uint32, c_void_p, c_void_p]),
        "stencil_sweepk_signal_gated": (c_int, [L, c_void_p, c_void_p, c_int64, c_int64, c_int32, c_void_p, c_void_p,
                                                c_uint32, c_void_p, POINTER(c_int32), c_void_p]),
        "stencil_exchange_done": (c_int, [c_void_p, c_uint32, c_void_p]),
        "stencil_face_signal_create": (c_int, [POINTER(c_void_p)]),
        "stencil_face_signal_destroy": (c_int, [c_void_p]),
        "stencil_face_signal_reset": (c_int, [c_void_p, c_void_p]),
        "stencil_face_signal_read": (c_int, [c_void_p, POINTER(c_uint64)]),
        "stencil_wait_face_signal": (c_int, [c_void_p, c_uint64, c_void_p]),
        "stencil_slab_create": (c_int, [POINTER(Problem), c_int32, POINTER(c_int32), c_int32, c_int32,
                                        POINTER(c_void_p)]),
        "stencil_slab_destroy": (c_int, [c_void_p]),
        "stencil_slab_unique_id": (c_int, [c_void_p, c_int64]),
        "stencil_slab_create_rank": (c_int, [POINTER(Problem), c_int32, c_int32, c_int32, c_void_p, c_int64, c_int32,
                                             POINTER(c_void_p)]),
        "stencil_slab_create2": (c_int, [POINTER(Problem), c_int32, POINTER(c_int32), c_int32, c_int32, c_int64,
                                         POINTER(c_void_p)]),
        "stencil_slab_create_rank2": (c_int, [POINTER(Problem), c_int32, c_int32, c_int32, c_void_p, c_int64, c_int32,
                                              c_int64, POINTER(c_void_p)]),
        "stencil_slab_rolling_info": (c_int, [c_void_p, POINTER(c_int64), POINTER(c_int64)]),
        "stencil_slab_info": (c_int, [c_void_p, c_int32, POINTER(c_int64), POINTER(c_int64), POINTER(c_int32),
                                      POINTER(c_int32)]),
        "stencil_slab_fill_initial": (c_int, [c_void_p, c_int32, c_uint64]),
        "stencil_slab_upload": (c_int, [c_void_p, c_void_p, c_int64, c_int64]),
        "stencil_slab_download": (c_int, [c_void_p, c_void_p, c_int64, c_int64]),
        "stencil_slab_run": (c_int, [c_void_p, c_uint32, POINTER(c_float)]),
        "stencil_slab_plane_sums": (c_int, [c_void_p, POINTER(c_double)]),
        "stencil_slab_kernel_timing": (c_int, [c_void_p, c_int32]),
        "stencil_slab_kernel_time": (c_int, [c_void_p, POINTER(c_float), POINTER(c_int64), POINTER(c_int64),
                                             POINTER(c_int32)]),
        "stencil_slab_round_form": (c_int, [c_void_p, POINTER(c_int32)]),
        "stencil_slab_round_info": (c_int, [c_void_p, POINTER(c_int32), POINTER(c_int32), POINTER(c_int32)]),
        "stencil_slab_exchange_budget": (c_int, [c_void_p, POINTER(c_int32), POINTER(c_int32), POINTER(c_float),
                                                 POINTER(c_float)]),
        "stencil_slab_set_timeout": (c_int, [c_void_p, c_int64]),
        "stencil_slab_exchange_time": (c_int, [c_void_p, POINTER(c_float), POINTER(c_float), POINTER(c_int64)]),
    }


def check(rc: int, where: str, lib: ctypes.CDLL | None = None) -> None:
    """Raise StencilError for a failed call; `lib` = the library that made it
    (its per-thread error message)."""
    if rc != STENCIL_OK:
        lib = lib or load()
        msg = (lib.stencil_last_error_message() or b"").decode(errors="replace")
        raise StencilError(rc, where, msg or lib.stencil_strerror(rc).decode())


def make_problem(dims=3, dtype=F64, shape=STAR, radius=1, order=ORDER_NAIVE, kernel=KERNEL_AUTO,
                 nx=1, ny=1, nz=1, halo=0, flags=0) -> Problem:
    return Problem(dims, dtype, shape, radius, order, kernel, halo, flags, nx, ny, nz if dims == 3 else 1)


def make_layout(prob: Problem) -> Layout:
    lib = load()
    lay = Layout()
    check(lib.stencil_layout_init(ctypes.byref(prob), ctypes.byref(lay)), "stencil_layout_init")
    return lay

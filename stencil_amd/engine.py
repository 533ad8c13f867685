"""Device-resident Jacobi engine: torch owns HBM and streams, every sweep is a
HIP kernel launched through the C-ABI (stencil_amd/_lib.py).

This is the Python counterpart of the C++ host engine (csrc/host/stencil.cpp,
itself the mirror of the reference's class Stencil, src/stencil/stencil.cpp).
It exposes what the benchmark and the tests need:
two ping-pong grids in the engine's padded layout, the reference initial
condition, single sweeps over slow-axis ranges, the whole-job iterate, and
views of whole planes for halo exchange.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib

_TORCH_DTYPE = {_lib.F32: torch.float32, _lib.F64: torch.float64}
_NP_DTYPE = {_lib.F32: np.float32, _lib.F64: np.float64}


@dataclass(frozen=True)
class StencilSpec:
    dims: int = 3
    dtype: str = "fp64"          # "fp32" | "fp64"
    shape: str = "star"          # "star" | "box"
    radius: int = 1
    order: str = "naive"         # "naive" | "dma"
    kernel: str = "auto"         # "auto" | "direct" | "zmarch" | "temporal2" | "temporalk" | "persistent"
    halo: int = 0                # 3D ghost planes per z side (0 = radius); 2 for fused slabs

    def problem(self, nx: int, ny: int, nz: int, flags: int = 0) -> _lib.Problem:
        return _lib.make_problem(
            dims=self.dims, dtype=_lib.F64 if self.dtype == "fp64" else _lib.F32,
            shape=_lib.BOX if self.shape == "box" else _lib.STAR, radius=self.radius,
            order=_lib.ORDER_DMA if self.order == "dma" else _lib.ORDER_NAIVE,
            kernel=_lib.KERNEL_NAMES[self.kernel], nx=nx, ny=ny, nz=nz if self.dims == 3 else 1,
            halo=self.halo, flags=flags)

    @property
    def fusable(self) -> bool:
        """Does the fused two-step kernel cover this stencil?"""
        if self.dims != 3 or self.radius != 1 or self.order != "naive":
            return False
        # AUTO fuses both: TEMPORALK for the 7-point star, the 2-step BOXK kernel for the box
        return self.kernel in ("temporal2", "temporalk", "auto")

    @property
    def elem_bytes(self) -> int:
        return 8 if self.dtype == "fp64" else 4


def _stream_handle(stream) -> ctypes.c_void_p:
    if stream is None:
        stream = torch.cuda.current_stream()
    return ctypes.c_void_p(stream.cuda_stream)


class JacobiEngine:
    """Two grids (a, b) of one problem on one GPU."""

    def __init__(self, spec: StencilSpec, nx: int, ny: int, nz: int = 1, device: int | torch.device = 0,
                 allocate: bool = True, flags: int = 0):
        self.lib = _lib.load()
        self.spec = spec
        self.prob = spec.problem(nx, ny, nz, flags)
        self.layout = _lib.make_layout(self.prob)
        self.device = torch.device("cuda", device) if isinstance(device, int) else device
        self.torch_dtype = _TORCH_DTYPE[self.prob.dtype]
        self.r = spec.radius
        # ghost/halo units per side of the slow axis (what a slab exchanges)
        self.depth = int(self.layout.zghost) if spec.dims == 3 else spec.radius
        self.fused = spec.fusable
        # sweeps one fused launch performs (the library's own launch plan):
        # 4 or 5 for the 7-point star (TEMPORALK), 3 or 4 for the 27-point box
        self.fuse_steps = 1
        if self.fused:
            # sweeps per fused launch: the most sweeps stencil_iterate runs as one launch
            self.fuse_steps = next((k for k in (8, 5, 4, 3, 2) if self.plan(k)[0] == 1), 2)
        self.slow_extent = int(self.lib.stencil_slow_extent(ctypes.byref(self.layout)))
        # one slow-axis unit = a whole plane (3D) or a whole padded row (2D)
        self.unit = int(self.layout.plane if spec.dims == 3 else self.layout.row)
        if allocate:
            n = int(self.layout.elems) + 256 // spec.elem_bytes  # tail pad, as stencil_alloc
            self.a = torch.empty(n, dtype=self.torch_dtype, device=self.device)
            self.b = torch.empty(n, dtype=self.torch_dtype, device=self.device)

    # ------------------------------------------------------------------ init
    def fill_initial(self, grid: torch.Tensor, kind: str = "reference", seed: int = 0, stream=None) -> None:
        k = _lib.INIT_RANDOM if kind == "random" else _lib.INIT_REFERENCE
        _lib.check(self.lib.stencil_fill_initial(ctypes.byref(self.layout), ctypes.c_void_p(grid.data_ptr()), k,
                                                 ctypes.c_uint64(seed & 0xFFFFFFFFFFFFFFFF), _stream_handle(stream)),
                   "stencil_fill_initial", lib=self.lib)

    def reset(self, kind: str = "reference", seed: int = 0) -> None:
        self.fill_initial(self.a, kind, seed)
        self.fill_initial(self.b, kind, seed)

    def place(self, trials: int = 6, max_bytes: int | None = None, passes: int = 2, sweeps: int | None = None) -> dict:
        """Choose where the two grids live.  The same launch
        runs up to 8 % apart depending on which physical pages its grids land
        on (512^3 fp64: 1184-1278 Gcell/s over 18 placements in one process;
        a physically contiguous grid is no better), so: allocate up to
        `trials` candidate pairs -- each while the earlier ones are held, so
        each lands elsewhere --, time one fused whole-grid launch on each
        (reference initial condition; `passes` interleaved passes, best of 2
        per pass), keep the fastest pair and free the rest.  The grids'
        contents are undefined afterwards: call reset().  Candidates are
        limited to `max_bytes` (default a quarter of the free memory).
        `sweeps`: the sweeps each timed call runs (default one fused launch).
        Returns the per-candidate ms per call and the choice."""
        if not hasattr(self, "a"):
            raise ValueError("place() needs the engine's grids (allocate=True)")
        grid_bytes = self.a.numel() * self.a.element_size()
        free = torch.cuda.mem_get_info(self.device)[0]
        budget = max_bytes if max_bytes is not None else free // 4
        n = max(1, min(int(trials), 1 + int(budget // max(1, 2 * grid_bytes))))
        if n == 1:
            return {"candidates": 1, "ms_per_launch": [], "chosen": 0, "sweeps_per_launch": self.fuse_steps}
        cands = [(self.a, self.b)]
        for _ in range(n - 1):
            try:
                cands.append((torch.empty_like(self.a), torch.empty_like(self.b)))
            except torch.OutOfMemoryError:  # fewer candidates
                break
        if len(cands) == 1:
            return {"candidates": 1, "ms_per_launch": [], "chosen": 0, "sweeps_per_launch": self.fuse_steps}
        k = int(sweeps) if sweeps else (self.fuse_steps if self.fused else 1)
        fin, ms = ctypes.c_int(0), ctypes.c_float(0.0)
        stream = _stream_handle(None)

        def run(a, b, timed):
            _lib.check(self.lib.stencil_iterate(ctypes.byref(self.layout), ctypes.c_void_p(a.data_ptr()),
                                                ctypes.c_void_p(b.data_ptr()), k, stream, ctypes.byref(fin),
                                                ctypes.byref(ms) if timed else None), "stencil_iterate", lib=self.lib)
            return ms.value

        for a, b in cands:
            self.fill_initial(a, "reference")
            self.fill_initial(b, "reference")
        for _ in range(8):  # clock up before the first candidate is timed
            run(*cands[0], False)
        best = [float("inf")] * len(cands)
        for _ in range(max(1, passes)):
            for i, (a, b) in enumerate(cands):
                run(a, b, False)
                best[i] = min(best[i], run(a, b, True), run(a, b, True))
        pick = min(range(len(cands)), key=lambda i: best[i])
        self.a, self.b = cands[pick]
        a = b = None  # drop every reference to the other candidates before returning their memory
        cands.clear()
        torch.cuda.empty_cache()
        return {"candidates": len(best), "ms_per_launch": [round(v, 5) for v in best], "chosen": pick,
                "sweeps_per_launch": k}

    # ---------------------------------------------------------------- sweeps
    def sweep(self, src: torch.Tensor, dst: torch.Tensor, begin: int, end: int, stream=None) -> None:
        _lib.check(self.lib.stencil_sweep(ctypes.byref(self.layout), ctypes.c_void_p(src.data_ptr()),
                                          ctypes.c_void_p(dst.data_ptr()), begin, end, _stream_handle(stream)),
                   "stencil_sweep", lib=self.lib)

    def sweep2(self, src: torch.Tensor, dst: torch.Tensor, begin: int, end: int, stream=None) -> None:
        _lib.check(self.lib.stencil_sweep2(ctypes.byref(self.layout), ctypes.c_void_p(src.data_ptr()),
                                           ctypes.c_void_p(dst.data_ptr()), begin, end, _stream_handle(stream)),
                   "stencil_sweep2", lib=self.lib)

    def sweepk(self, src: torch.Tensor, dst: torch.Tensor, begin: int, end: int, steps: int, stream=None) -> None:
        """dst = S^steps(src) on [begin, end) in one launch (steps 1..5; box: 1..3)."""
        _lib.check(self.lib.stencil_sweepk(ctypes.byref(self.layout), ctypes.c_void_p(src.data_ptr()),
                                           ctypes.c_void_p(dst.data_ptr()), begin, end, steps,
                                           _stream_handle(stream)), "stencil_sweepk", lib=self.lib)

    def sweepk_geometry(self, steps: int, begin: int = 0, end: int | None = None) -> dict:
        """How sweepk(steps) over [begin, end) would launch the K-step strip
        kernel: workgroups, planes per z-chunk, packed schedule or not."""
        wg, zc, packed = ctypes.c_int64(0), ctypes.c_int32(0), ctypes.c_int32(0)
        end = self.slow_extent if end is None else end
        _lib.check(self.lib.stencil_sweepk_geometry(ctypes.byref(self.layout), begin, end, steps, ctypes.byref(wg),
                                                    ctypes.byref(zc), ctypes.byref(packed)), "stencil_sweepk_geometry", lib=self.lib)
        return {"workgroups": int(wg.value), "zchunk": int(zc.value), "packed": bool(packed.value)}

    @property
    def supports_signal(self) -> bool:
        """Face-signalled K-step launches (stencil_sweepk_signal): the 3D 7-point
        star (K = 3..5) and the 27-point box (K = 2..4)."""
        s = self.spec
        if not (s.dims == 3 and s.radius == 1 and s.order == "naive" and self.fused):
            return False
        return 3 <= self.fuse_steps <= 5 if s.shape == "star" else 2 <= self.fuse_steps <= 4

    def sweepk_signal(self, src: torch.Tensor, dst: torch.Tensor, begin: int, end: int, steps: int,
                      counters: torch.Tensor, stream=None, face_signal: "FaceSignal | None" = None) -> int:
        """sweepk over [begin, end) as one launch that adds to counters[0] / [1]
        once the low / high face planes are stored; returns adds per face.
        With face_signal, it also grows by 2 once both faces are complete."""
        n = ctypes.c_int32(0)
        _lib.check(self.lib.stencil_sweepk_signal(ctypes.byref(self.layout), ctypes.c_void_p(src.data_ptr()),
                                                  ctypes.c_void_p(dst.data_ptr()), begin, end, steps,
                                                  ctypes.c_void_p(counters.data_ptr()),
                                                  face_signal.ptr if face_signal is not None else None,
                                                  ctypes.byref(n), _stream_handle(stream)), "stencil_sweepk_signal", lib=self.lib)
        return int(n.value)

    def face_signal(self) -> "FaceSignal":
        return FaceSignal()

    def wait_counters(self, counters: torch.Tensor, target_lo: int, target_hi: int, stream=None) -> None:
        """Queue on `stream` a wait until counters[0] >= target_lo and
        counters[1] >= target_hi (counters[2] is set on a 10 s timeout)."""
        _lib.check(self.lib.stencil_wait_counters(ctypes.c_void_p(counters.data_ptr()), target_lo, target_hi,
                                                  ctypes.c_void_p(counters.data_ptr() + 8), _stream_handle(stream)),
                   "stencil_wait_counters", lib=self.lib)

    def iterate(self, iterations: int, stream=None, timed: bool = False):
        """Whole job a -> ... ; returns (final grid tensor, device ms or None)."""
        fin = ctypes.c_int(0)
        ms = ctypes.c_float(0.0)
        _lib.check(self.lib.stencil_iterate(ctypes.byref(self.layout), ctypes.c_void_p(self.a.data_ptr()),
                                            ctypes.c_void_p(self.b.data_ptr()), iterations, _stream_handle(stream),
                                            ctypes.byref(fin), ctypes.byref(ms) if timed else None),
                   "stencil_iterate", lib=self.lib)
        return (self.b if fin.value else self.a), (ms.value if timed else None)

    def prepare(self, stream=None) -> dict:
        """stencil_prepare2: settle the job's one-time per-shape choices (the
        z-chunk schedule trial) by one fused launch a -> b, then the same
        launch for ~25 ms of device time so the GPU's clock has settled
        (DESIGN.md §6); `a` is unchanged.  Returns what ran: launches and
        their estimated device ms."""
        n, ms = ctypes.c_int64(0), ctypes.c_float(0.0)
        _lib.check(self.lib.stencil_prepare2(ctypes.byref(self.layout), ctypes.c_void_p(self.a.data_ptr()),
                                             ctypes.c_void_p(self.b.data_ptr()), _stream_handle(stream),
                                             ctypes.byref(n), ctypes.byref(ms)),
                   "stencil_prepare2", lib=self.lib)
        return {"launches": int(n.value), "device_ms": float(ms.value)}

    def plan(self, iterations: int):
        launches = ctypes.c_int64(0)
        kernel = ctypes.c_int32(0)
        _lib.check(self.lib.stencil_plan(ctypes.byref(self.layout), iterations, ctypes.byref(launches),
                                         ctypes.byref(kernel)), "stencil_plan", lib=self.lib)
        return int(launches.value), int(kernel.value)

    # ----------------------------------------------------------------- views
    def plane_view(self, grid: torch.Tensor, first: int, count: int) -> torch.Tensor:
        """Contiguous 1-D view of slow-axis units [first, first+count), ghost
        units included (first may be -r .. n+r-count)."""
        if self.spec.dims == 3:
            base = int(self.layout.zghost) * int(self.layout.plane)
        else:
            base = int(self.layout.origin) - int(self.layout.origin) % int(self.layout.row)
        start = base + first * self.unit
        return grid[start:start + count * self.unit]

    def interior(self, grid: torch.Tensor) -> torch.Tensor:
        """Strided (nz, ny, nx) / (ny, nx) view of the interior."""
        p, lay = self.prob, self.layout
        base = grid.storage_offset()  # as_strided offsets are absolute in the storage
        if self.spec.dims == 3:
            return grid.as_strided((p.nz, p.ny, p.nx), (lay.plane, lay.row, 1), base + lay.origin)
        return grid.as_strided((p.ny, p.nx), (lay.row, 1), base + lay.origin)

    def with_ghosts(self, grid: torch.Tensor) -> torch.Tensor:
        """Strided view of interior + ghost ring, the oracle's dense shape."""
        p, lay, r = self.prob, self.layout, self.r
        corner = grid.storage_offset() + lay.origin - r * lay.row - r - (r * lay.plane if self.spec.dims == 3 else 0)
        if self.spec.dims == 3:
            return grid.as_strided((p.nz + 2 * r, p.ny + 2 * r, p.nx + 2 * r), (lay.plane, lay.row, 1), corner)
        return grid.as_strided((p.ny + 2 * r, p.nx + 2 * r), (lay.row, 1), corner)

    def to_numpy(self, grid: torch.Tensor) -> np.ndarray:
        """Dense host copy with ghosts (oracle layout)."""
        torch.cuda.synchronize(self.device)
        return self.with_ghosts(grid).cpu().numpy().copy()

    def plane_sums(self, grid: torch.Tensor, stream=None) -> np.ndarray:
        out = np.zeros(self.slow_extent, dtype=np.float64)
        _lib.check(self.lib.stencil_plane_sums(ctypes.byref(self.layout), ctypes.c_void_p(grid.data_ptr()),
                                               out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                               _stream_handle(stream)), "stencil_plane_sums", lib=self.lib)
        return out


class RollingGrid:
    """ONE resident grid plus `shift` spare planes (stencil_rolling_*): the
    job stencil_iterate runs on two grids, bitwise, for grids whose two
    copies do not fit the GPU (BASELINE config 3: 4096^3 fp32)."""

    def __init__(self, spec: StencilSpec, nx: int, ny: int, nz: int, shift: int, device: int | torch.device = 0):
        self.lib = _lib.load()
        self.spec = spec
        self.prob = spec.problem(nx, ny, nz)
        self.layout = _lib.make_layout(self.prob)
        self.device = torch.device("cuda", device) if isinstance(device, int) else device
        self.shift = int(shift)
        nbytes, k = ctypes.c_int64(0), ctypes.c_int32(0)
        _lib.check(self.lib.stencil_rolling_bytes(ctypes.byref(self.layout), self.shift, ctypes.byref(nbytes),
                                                  ctypes.byref(k)), "stencil_rolling_bytes", lib=self.lib)
        self.bytes, self.sweeps_per_pass = int(nbytes.value), int(k.value)
        es = spec.elem_bytes
        self.buf = torch.empty(-(-self.bytes // es), dtype=_TORCH_DTYPE[self.prob.dtype], device=self.device)
        self.position = 0  # 0: the grid is at home (slot offset shift), 1: shifted to the allocation's start
        self._grid_elems = int(self.layout.elems) + 256 // es
        self._eng = JacobiEngine(spec, nx, ny, nz, device=self.device, allocate=False)

    @staticmethod
    def bytes_needed(spec: StencilSpec, nx: int, ny: int, nz: int, shift: int) -> int:
        lib = _lib.load()
        lay = _lib.make_layout(spec.problem(nx, ny, nz))
        nbytes = ctypes.c_int64(0)
        _lib.check(lib.stencil_rolling_bytes(ctypes.byref(lay), shift, ctypes.byref(nbytes), None),
                   "stencil_rolling_bytes", lib=lib)
        return int(nbytes.value)

    @property
    def grid(self) -> torch.Tensor:
        """The current grid, as a tensor in the engine layout."""
        start = 0 if self.position else self.shift * int(self.layout.plane)
        return self.buf[start:start + self._grid_elems]

    def reset(self, kind: str = "reference", seed: int = 0, stream=None) -> None:
        self.position = 0
        self._eng.fill_initial(self.grid, kind, seed, stream)
        self.init_margin(stream)

    def init_margin(self, stream=None) -> None:
        _lib.check(self.lib.stencil_rolling_init_margin(ctypes.byref(self.layout), ctypes.c_void_p(self.buf.data_ptr()),
                                                        self.shift, _stream_handle(stream)),
                   "stencil_rolling_init_margin", lib=self.lib)

    def iterate(self, iterations: int, stream=None, timed: bool = False):
        """`iterations` sweeps; returns (current grid, device ms or None, launches)."""
        pos = ctypes.c_int32(self.position)
        n, ms = ctypes.c_int64(0), ctypes.c_float(0.0)
        _lib.check(self.lib.stencil_rolling_iterate(ctypes.byref(self.layout), ctypes.c_void_p(self.buf.data_ptr()),
                                                    self.shift, iterations, ctypes.byref(pos), _stream_handle(stream),
                                                    ctypes.byref(n), ctypes.byref(ms) if timed else None),
                   "stencil_rolling_iterate", lib=self.lib)
        self.position = int(pos.value)
        return self.grid, (ms.value if timed else None), int(n.value)

    def interior(self, grid: torch.Tensor | None = None) -> torch.Tensor:
        return self._eng.interior(self.grid if grid is None else grid)

    def with_ghosts(self, grid: torch.Tensor | None = None) -> torch.Tensor:
        return self._eng.with_ghosts(self.grid if grid is None else grid)

    def to_numpy(self) -> np.ndarray:
        return self._eng.to_numpy(self.grid)

    def plane_sums(self, stream=None) -> np.ndarray:
        return self._eng.plane_sums(self.grid, stream)


class FaceSignal:
    """A uint64 count in HIP signal memory that stencil_sweepk_signal bumps
    once per completed face and a stream can wait on in the command
    processor (stencil_wait_face_signal): no wait kernel on the GPU."""

    def __init__(self):
        self.lib = _lib.load()
        self.ptr = ctypes.c_void_p()
        _lib.check(self.lib.stencil_face_signal_create(ctypes.byref(self.ptr)), "stencil_face_signal_create", lib=self.lib)

    def reset(self, stream=None) -> None:
        _lib.check(self.lib.stencil_face_signal_reset(self.ptr, _stream_handle(stream)), "stencil_face_signal_reset", lib=self.lib)

    def wait(self, target: int, stream=None) -> None:
        _lib.check(self.lib.stencil_wait_face_signal(self.ptr, ctypes.c_uint64(target), _stream_handle(stream)),
                   "stencil_wait_face_signal", lib=self.lib)

    def value(self) -> int:
        v = ctypes.c_uint64(0)
        _lib.check(self.lib.stencil_face_signal_read(self.ptr, ctypes.byref(v)), "stencil_face_signal_read", lib=self.lib)
        return int(v.value)

    def close(self) -> None:
        if self.ptr and self.ptr.value:
            self.lib.stencil_face_signal_destroy(self.ptr)
            self.ptr = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def copy_bandwidth(nbytes: int, reps: int = 20, device: int = 0) -> float:
    """Attainable HBM bandwidth (GB/s, read+write) of a plain float4 copy."""
    lib = _lib.load()
    src = torch.empty(nbytes // 4, dtype=torch.float32, device=torch.device("cuda", device))
    dst = torch.empty_like(src)
    src.fill_(1.0)
    ms = ctypes.c_float(0.0)
    _lib.check(lib.stencil_copy_bandwidth(ctypes.c_void_p(dst.data_ptr()), ctypes.c_void_p(src.data_ptr()),
                                          nbytes, 2, _stream_handle(None), ctypes.byref(ms)), "copy warmup", lib=lib)
    _lib.check(lib.stencil_copy_bandwidth(ctypes.c_void_p(dst.data_ptr()), ctypes.c_void_p(src.data_ptr()),
                                          nbytes, reps, _stream_handle(None), ctypes.byref(ms)), "copy", lib=lib)
    return 2.0 * nbytes * reps / (ms.value * 1e-3) / 1e9


class SlabJob:
    """A multi-GPU z-slab job run by the C++ host (stencil_slab_*: the rounds
    in csrc/slab_core.hpp, bound to HIP + RCCL in csrc/slab.hip): one process
    and `devices` one slab each, halos over RCCL (or device copies, which let
    several slabs share a GPU), or -- rank mode -- this process's one slab of
    a job whose other slabs live in other processes."""

    def __init__(self, spec: StencilSpec, nx: int, ny: int, nz: int, devices, exchange: str = "rccl",
                 periodic: bool = False, rank=None, rolling: bool = False, margin: int = 0, lib=None):
        """rank=(nranks, rank, unique_id): rank mode (stencil_slab_create_rank),
        this process's one slab on devices[0], the others in other processes
        that make the same call with the same id (SlabJob.unique_id on one rank,
        handed to the rest by the caller).  rolling: ONE grid per slab plus
        `margin` spare planes (0: as deep as free memory allows).  lib: the
        library whose stencil_slab_* entry points run the job (default the
        product; the CPU tests pass tests/cpu_slab's fake device)."""
        self.lib = lib if lib is not None else _lib.load()
        self.spec = spec
        self.shape = (nx, ny, nz)
        prob = spec.problem(nx, ny, nz)
        job = ctypes.c_void_p()
        flags = (_lib.SLAB_PERIODIC if periodic else 0) | (_lib.SLAB_ROLLING if rolling else 0)
        if rank is not None:
            nranks, r, uid = rank
            if exchange != "rccl" or len(devices) != 1:
                raise ValueError("rank mode: one device per rank, RCCL exchange")
            buf = ctypes.create_string_buffer(bytes(uid), len(uid))
            _lib.check(self.lib.stencil_slab_create_rank2(ctypes.byref(prob), nranks, r, devices[0], buf, len(uid),
                                                          flags, margin, ctypes.byref(job)),
                       "stencil_slab_create_rank", lib=self.lib)
        else:
            devs = (ctypes.c_int32 * len(devices))(*devices)
            kind = _lib.EXCHANGE_RCCL if exchange == "rccl" else _lib.EXCHANGE_COPY
            _lib.check(self.lib.stencil_slab_create2(ctypes.byref(prob), len(devices), devs, kind, flags, margin,
                                                     ctypes.byref(job)),
                       "stencil_slab_create", lib=self.lib)
        self.job = job
        self.nslabs = len(devices)

    @staticmethod
    def unique_id(lib=None) -> bytes:
        """A fresh RCCL id for a rank-mode job (make it on one rank only)."""
        lib = lib if lib is not None else _lib.load()
        buf = ctypes.create_string_buffer(_lib.SLAB_ID_BYTES)
        _lib.check(lib.stencil_slab_unique_id(buf, _lib.SLAB_ID_BYTES), "stencil_slab_unique_id", lib=lib)
        return buf.raw

    def close(self) -> None:
        if self.job:
            self.lib.stencil_slab_destroy(self.job)
            self.job = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def info(self, slab: int) -> dict:
        first, planes = ctypes.c_int64(0), ctypes.c_int64(0)
        dev, k = ctypes.c_int32(0), ctypes.c_int32(0)
        _lib.check(self.lib.stencil_slab_info(self.job, slab, ctypes.byref(first), ctypes.byref(planes),
                                              ctypes.byref(dev), ctypes.byref(k)), "stencil_slab_info", lib=self.lib)
        return {"first": int(first.value), "planes": int(planes.value), "device": int(dev.value),
                "sweeps_per_round": int(k.value)}

    def rolling_info(self) -> dict:
        """Rolling slabs: the margin (0: two grids) and the most z-range
        launches one pass makes on a slab of this process."""
        m, n = ctypes.c_int64(0), ctypes.c_int64(0)
        _lib.check(self.lib.stencil_slab_rolling_info(self.job, ctypes.byref(m), ctypes.byref(n)),
                   "stencil_slab_rolling_info", lib=self.lib)
        return {"margin": int(m.value), "launches_per_pass": int(n.value)}

    def fill_initial(self, kind: str = "reference", seed: int = 0) -> None:
        k = _lib.INIT_RANDOM if kind == "random" else _lib.INIT_REFERENCE
        _lib.check(self.lib.stencil_slab_fill_initial(self.job, k, seed), "stencil_slab_fill_initial", lib=self.lib)

    def _dense(self) -> np.ndarray:
        nx, ny, nz = self.shape
        r = self.spec.radius
        dt = np.float64 if self.spec.dtype == "fp64" else np.float32
        return np.zeros((nz + 2 * r, ny + 2 * r, nx + 2 * r), dtype=dt)

    def upload(self, dense: np.ndarray) -> None:
        a = np.ascontiguousarray(dense)
        _lib.check(self.lib.stencil_slab_upload(self.job, ctypes.c_void_p(a.ctypes.data), a.shape[2], a.shape[1]),
                   "stencil_slab_upload", lib=self.lib)

    def download(self) -> np.ndarray:
        """The current global grid, dense with ghosts (oracle layout)."""
        a = self._dense()
        _lib.check(self.lib.stencil_slab_download(self.job, ctypes.c_void_p(a.ctypes.data), a.shape[2], a.shape[1]),
                   "stencil_slab_download", lib=self.lib)
        return a

    def run(self, iterations: int) -> float:
        """`iterations` sweeps; returns the host wall time of the rounds (ms)."""
        ms = ctypes.c_float(0.0)
        _lib.check(self.lib.stencil_slab_run(self.job, iterations, ctypes.byref(ms)), "stencil_slab_run", lib=self.lib)
        return float(ms.value)

    def kernel_timing(self, enable: bool) -> None:
        """Record hipEvents around slab 0's compute launch of every round from
        now on (the whole slab in face-signalled rounds, else its interior)."""
        _lib.check(self.lib.stencil_slab_kernel_timing(self.job, 1 if enable else 0), "stencil_slab_kernel_timing", lib=self.lib)

    def kernel_time(self) -> dict:
        ms, n, cells, sig = ctypes.c_float(0.0), ctypes.c_int64(0), ctypes.c_int64(0), ctypes.c_int32(0)
        _lib.check(self.lib.stencil_slab_kernel_time(self.job, ctypes.byref(ms), ctypes.byref(n), ctypes.byref(cells),
                                                     ctypes.byref(sig)), "stencil_slab_kernel_time", lib=self.lib)
        form = self.round_form()
        return {"total_ms": float(ms.value), "launches": int(n.value), "cells_per_launch": int(cells.value),
                "signalled": int(sig.value) == 1, "rolling": form == 2, "serial": form == 3, "form": form}

    def exchange_time(self) -> dict:
        """The timed rounds' exchanges (kernel timing on): summed transfer time
        on slab 0's exchange stream, the part of it beside the same round's
        timed launches, and the count (stencil_slab_exchange_time)."""
        t, b, n = ctypes.c_float(0.0), ctypes.c_float(0.0), ctypes.c_int64(0)
        _lib.check(self.lib.stencil_slab_exchange_time(self.job, ctypes.byref(t), ctypes.byref(b), ctypes.byref(n)),
                   "stencil_slab_exchange_time", lib=self.lib)
        return {"transfer_ms": float(t.value), "beside_ms": float(b.value), "exchanges": int(n.value)}

    def round_form(self) -> int:
        """0 boundary + interior launches, 1 face-signalled, 2 rolling passes, 3 serial, 4 staged."""
        f = ctypes.c_int32(-1)
        _lib.check(self.lib.stencil_slab_round_form(self.job, ctypes.byref(f)), "stencil_slab_round_form", lib=self.lib)
        return int(f.value)

    def round_info(self) -> dict:
        """The form plus whether face-signalled launches are halo-gated (no
        event wait between rounds) and whether the exchange is confined to
        CUs of its own (stencil_slab_round_info)."""
        f, g, c = ctypes.c_int32(-1), ctypes.c_int32(0), ctypes.c_int32(0)
        _lib.check(self.lib.stencil_slab_round_info(self.job, ctypes.byref(f), ctypes.byref(g), ctypes.byref(c)),
                   "stencil_slab_round_info", lib=self.lib)
        return {"form": int(f.value), "gated": bool(g.value), "confined": bool(c.value)}

    def exchange_budget(self) -> dict:
        """Staged rounds with a confined exchange: the CUs per XCD the
        exchange uses, the alternative budget tried in the tuning rounds and
        both tuning rounds' times (stencil_slab_exchange_budget)."""
        c, a, r0, r1 = ctypes.c_int32(0), ctypes.c_int32(0), ctypes.c_float(0.0), ctypes.c_float(0.0)
        _lib.check(self.lib.stencil_slab_exchange_budget(self.job, ctypes.byref(c), ctypes.byref(a), ctypes.byref(r0),
                                                         ctypes.byref(r1)), "stencil_slab_exchange_budget", lib=self.lib)
        return {"cus_per_xcd": int(c.value), "alt_cus_per_xcd": int(a.value), "round_ms": round(float(r0.value), 4),
                "alt_round_ms": round(float(r1.value), 4)}

    def set_timeout(self, ms: int) -> None:
        """The job's deadline for every device wait (stencil_slab_set_timeout):
        past it the job fails with STENCIL_ETIMEOUT and aborts its communicators."""
        _lib.check(self.lib.stencil_slab_set_timeout(self.job, int(ms)), "stencil_slab_set_timeout", lib=self.lib)

    def plane_sums(self) -> np.ndarray:
        out = np.zeros(self.shape[2], dtype=np.float64)
        _lib.check(self.lib.stencil_slab_plane_sums(self.job, out.ctypes.data_as(ctypes.POINTER(ctypes.c_double))),
                   "stencil_slab_plane_sums", lib=self.lib)
        return out

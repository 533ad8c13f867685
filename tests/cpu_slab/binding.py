"""ctypes binding of tests/cpu_slab/libslab_fake.so -- TEST INFRASTRUCTURE ONLY.

The library runs csrc/slab_core.hpp (the multi-GPU slab job's round and
exchange logic, the same code csrc/slab.hip binds to HIP and RCCL) on a CPU
fake device whose sweeps are the oracle's (fake_dev.cpp).  `load()` returns
an object with the product's stencil_slab_* names, so
stencil_amd.engine.SlabJob(..., lib=load()) drives it unchanged.
"""
from __future__ import annotations

import ctypes
import os

from stencil_amd import _lib

HERE = os.path.dirname(os.path.abspath(__file__))
PATH = os.path.join(HERE, "libslab_fake.so")

_cached = None


class FakeSlabLib:
    """stencil_slab_* -> fake_slab_*, plus the error-message calls _lib.check uses."""

    def __init__(self, cdll: ctypes.CDLL):
        self._cdll = cdll
        for name, (res, args) in _lib.signatures().items():
            if not name.startswith("stencil_slab_"):
                continue
            fn = getattr(cdll, "fake_" + name[len("stencil_"):])
            fn.restype, fn.argtypes = res, args
            setattr(self, name, fn)
        cdll.fake_slab_last_error_message.restype = ctypes.c_char_p
        cdll.fake_slab_set_k.argtypes = [ctypes.c_int32]
        cdll.fake_slab_set_signal.argtypes = [ctypes.c_int32]
        cdll.fake_slab_set_free_bytes.argtypes = [ctypes.c_int64]
        cdll.fake_slab_stats.argtypes = [ctypes.POINTER(ctypes.c_int64), ctypes.c_int32]
        cdll.fake_slab_gate_stats.argtypes = [ctypes.POINTER(ctypes.c_int64), ctypes.c_int32]
        cdll.fake_slab_layout_init.argtypes = [ctypes.POINTER(_lib.Problem), ctypes.POINTER(_lib.Layout)]

    # what _lib.check calls on failure
    def stencil_last_error_message(self):
        return self._cdll.fake_slab_last_error_message()

    @staticmethod
    def stencil_strerror(code):
        return b"fake slab error %d" % code

    # test knobs of the fake device
    def set_k(self, k: int) -> None:
        """Sweeps per round (0: the library's own rule)."""
        self._cdll.fake_slab_set_k(k)

    def set_signal(self, on: bool) -> None:
        self._cdll.fake_slab_set_signal(1 if on else 0)

    def set_free_bytes(self, b: int) -> None:
        self._cdll.fake_slab_set_free_bytes(b)

    def layout(self, prob) -> "_lib.Layout":
        """The fake device's padded layout of `prob` (its copy of api.hip's rule)."""
        lay = _lib.Layout()
        rc = self._cdll.fake_slab_layout_init(ctypes.byref(prob), ctypes.byref(lay))
        if rc:
            raise _lib.StencilError(rc, "fake_slab_layout_init", self._cdll.fake_slab_last_error_message().decode())
        return lay

    def stats(self, reset: bool = False) -> dict:
        out = (ctypes.c_int64 * 5)()
        self._cdll.fake_slab_stats(out, 1 if reset else 0)
        return dict(zip(("sweeps", "signal_sweeps", "sends", "recvs", "peer_copies"), list(out)))

    def gate_stats(self, reset: bool = False) -> dict:
        """Halo-gated launches, gate numbering violations (a launch whose
        awaited exchange number is not the last completed one, an exchange
        completion out of order) and exchange-completion stores."""
        out = (ctypes.c_int64 * 3)()
        self._cdll.fake_slab_gate_stats(out, 1 if reset else 0)
        return dict(zip(("gated", "violations", "completions"), list(out)))


def available() -> bool:
    return os.path.exists(PATH)


def load() -> FakeSlabLib:
    global _cached
    if _cached is None:
        if not available():
            raise ImportError(f"{PATH} is missing: run `make` (Makefile target tests/cpu_slab/libslab_fake.so)")
        _cached = FakeSlabLib(ctypes.CDLL(PATH))
    return _cached

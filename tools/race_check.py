#!/usr/bin/env python3
"""One-off check of the round-1 slab stream race.

Runs tests/test_gpu_slab.py's large-plane case twice: with SlabJacobi.finish
disabled (the round-1 behaviour: the remainder pair after face-signalled
rounds launches on the caller's stream without joining the round streams)
and with the fixed code.  Prints whether each equals the boundary+interior
rounds.  Device-wide synchronisation before every read keeps the readback
itself ordered in both runs."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from stencil_amd.engine import JacobiEngine, StencilSpec  # noqa: E402
from stencil_amd.slab import LoopbackExchanger, SlabJacobi  # noqa: E402
from tests.test_gpu_slab import _periodic_run_sig  # noqa: E402


def main():
    for dtype in ("fp64", "fp32"):
        nx = ny = 2048
        fuse = JacobiEngine(StencilSpec(dims=3, dtype=dtype), nx, ny, 8, device=0, allocate=False).fuse_steps
        nz, it = 2 * fuse, 2 * fuse + 2
        want = _periodic_run_sig(0, LoopbackExchanger(), nx, ny, nz, it, False, dtype=dtype)
        ib = torch.int64 if dtype == "fp64" else torch.int32
        for label in ("no-join (round 1)", "fixed"):
            saved = SlabJacobi.finish
            if label.startswith("no-join"):
                SlabJacobi.finish = lambda self: None
            try:
                got = _periodic_run_sig(0, LoopbackExchanger(), nx, ny, nz, it, True, False, dtype=dtype)
            finally:
                SlabJacobi.finish = saved
            eq = torch.equal(got.view(ib), want.view(ib))
            ndiff = int((got.view(ib) != want.view(ib)).sum())
            print(f"{dtype} K={fuse} nz={nz} it={it} {label}: {'EQUAL' if eq else 'MISMATCH'} ({ndiff} cells differ)",
                  flush=True)


if __name__ == "__main__":
    main()

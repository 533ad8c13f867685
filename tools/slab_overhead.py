"""Host-side cost of one slab round (no communication): the overlap path of
stencil_amd/slab.py with a no-op exchanger on one GPU, against the same sweeps
issued by stencil_iterate.  If a round's host time exceeded its GPU time the
multi-GPU bench would be host-bound."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from stencil_amd import _lib  # noqa: E402
from stencil_amd.engine import JacobiEngine, StencilSpec  # noqa: E402
from stencil_amd.slab import SlabInfo, SlabJacobi  # noqa: E402


class NullExchanger:
    def exchange(self, *views):
        return []


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    rounds = 100
    eng = JacobiEngine(StencilSpec(dims=3, dtype="fp64", halo=2), n, n, n,
                       flags=_lib.HALO_LO | _lib.HALO_HI)
    slab = SlabJacobi(eng, SlabInfo(1, 3, n, n), NullExchanger())
    eng.reset()
    slab.run(4)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    slab.run(2 * rounds)
    t_host = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    ref = JacobiEngine(StencilSpec(dims=3, dtype="fp64"), n, n, n)
    ref.reset()
    ref.iterate(4)
    _, ms = ref.iterate(2 * rounds, timed=True)
    print(f"slab path: host issue {t_host / rounds * 1e6:.0f} us/round, wall {t_all / rounds * 1e6:.0f} us/round; "
          f"single-grid GPU {ms * 1e3 / rounds:.0f} us per 2 sweeps")


if __name__ == "__main__":
    main()

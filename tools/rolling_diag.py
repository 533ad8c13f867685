#!/usr/bin/env python3
"""Where does the rolling job differ from the two-grid job?  Per-plane
mismatch counts for a few shapes / shifts (diagnostic)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(nx, ny, nz, it, shift, dtype="fp32"):
    import torch
    from stencil_amd.engine import JacobiEngine, RollingGrid, StencilSpec
    sp = StencilSpec(dims=3, dtype=dtype)
    e = JacobiEngine(sp, nx, ny, nz)
    e.reset()
    fin, _ = e.iterate(it)
    want = e.interior(fin).clone()
    del e, fin
    torch.cuda.empty_cache()
    g = RollingGrid(sp, nx, ny, nz, shift)
    g.reset()
    _, _, n = g.iterate(it)
    got = g.interior()
    bad = torch.tensor([int((got[z] != want[z]).sum()) for z in range(nz)])
    planes = [int(z) for z in torch.nonzero(bad).flatten()]
    whole = torch.equal(got, want)
    print(f"{nx}x{ny}x{nz} {dtype} it={it} shift={shift} launches={n}: {len(planes)} planes differ"
          f"{': ' + str(planes[:12]) + (' ...' if len(planes) > 12 else '') if planes else ''}"
          f"{' counts ' + str([int(bad[z]) for z in planes[:6]]) if planes else ''}; torch.equal(whole) = {whole}", flush=True)
    del g, got, want
    torch.cuda.empty_cache()


if __name__ == "__main__":
    run(2048, 2048, 256, 10, 40)
    run(4096, 4096, 1024, 10, 395)
    run(4096, 4096, 1024, 40, 395)

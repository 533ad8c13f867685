#!/usr/bin/env python3
"""Which path is wrong at 4096^2 x 1024 fp32 (K = 5): after t = 10 sweeps
planes 0 .. 53 depend only on planes <= 63 and the bottom ghost plane, so a
4096^2 x 64 two-grid run gives their exact values.  Compare the two-grid and
the rolling runs of the deep grid against it, plane by plane, and report the
rows that differ (diagnostic)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from stencil_amd.engine import JacobiEngine, RollingGrid, StencilSpec
    sp = StencilSpec(dims=3, dtype="fp32")
    nx = ny = 4096
    it = 10
    e = JacobiEngine(sp, nx, ny, 64)
    e.reset()
    fin, _ = e.iterate(it)
    ref = e.interior(fin)[:54].clone()
    del e, fin
    torch.cuda.empty_cache()

    def report(tag, got):
        bad = []
        for z in range(54):
            d = got[z] != ref[z]
            n = int(d.sum())
            if n:
                rows = torch.nonzero(d.any(dim=1)).flatten().tolist()
                cols = torch.nonzero(d.any(dim=0)).flatten().tolist()
                bad.append((z, n, rows[:12], len(rows), cols[:6], len(cols)))
        print(f"{tag}: {len(bad)} of planes 0..53 differ from the 4096^2 x 64 run", flush=True)
        for b in bad[:6]:
            print(f"   plane {b[0]}: {b[1]} cells; rows {b[2]} ({b[3]} rows), cols {b[4]} ({b[5]} cols)", flush=True)

    for nz, zc in ((1024, None), (1024, "390"), (400, None)):
        if zc:
            os.environ["STENCIL_TK_ZCHUNK"] = zc
        e = JacobiEngine(sp, nx, ny, nz)
        print("geometry", e.sweepk_geometry(5), "knobs", e.lib.stencil_debug_knobs(), flush=True)
        e.reset()
        fin, _ = e.iterate(it)
        report(f"two-grid {nx}x{ny}x{nz} zchunk={zc}", e.interior(fin))
        del e, fin
        torch.cuda.empty_cache()
        os.environ.pop("STENCIL_TK_ZCHUNK", None)
    for shift in (395, 200):
        g = RollingGrid(sp, nx, ny, 1024, shift)
        g.reset()
        _, _, n = g.iterate(it)
        report(f"rolling 1024 planes shift {shift} ({n} launches)", g.interior())
        del g
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

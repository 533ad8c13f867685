"""Host-timed C++ slab jobs (stencil_slab_run) on one GPU: a periodic ring of
one slab (an interior rank's structure: both faces cross the exchange every
round), face-signalled rounds vs boundary + interior launches, device-copy and
RCCL exchange.  usage: python tools/slab_job_time.py [n] [star|box] [sweeps]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stencil_amd.engine import SlabJob, StencilSpec  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    shape = sys.argv[2] if len(sys.argv) > 2 else "star"
    sweeps = int(sys.argv[3]) if len(sys.argv) > 3 else 400
    spec = StencilSpec(dims=3, dtype="fp64", shape=shape)
    out = {}
    for rnd in range(2):
        for exchange in ("copy", "rccl"):
            for sig in ("1", "0"):
                os.environ["STENCIL_SLAB_SIGNAL"] = sig
                job = SlabJob(spec, n, n, n, devices=[0], exchange=exchange, periodic=True)
                k = job.info(0)["sweeps_per_round"]
                job.fill_initial("reference", 0)
                job.run(4 * k)
                ms = job.run(sweeps // k * k)
                job.close()
                key = f"{exchange} signal={sig}"
                out.setdefault(key, []).append(round(n ** 3 * (sweeps // k * k) / (ms * 1e-3) / 1e9, 1))
    print(json.dumps({"grid": [n, n, n], "shape": shape, "sweeps": sweeps, "Gcell_per_s": out}), flush=True)


if __name__ == "__main__":
    main()

"""The two-tier 7-point launch (kernels_strip.hip TIER):
8 sweeps per launch, producer workgroups handing the grid after 4 sweeps to
consumer workgroups through a ring of plane slots (sc1 stores / loads and
per-plane flags).  Still an experiment (STENCIL_TK_TIER=1, debug library);
whatever its speed, its results must be bitwise the oracle's."""
import numpy as np
import pytest

from oracle import binding as ob
from stencil_amd import _lib
from stencil_amd.engine import JacobiEngine, StencilSpec

pytestmark = pytest.mark.gpu


@pytest.fixture()
def tier_env(monkeypatch):
    monkeypatch.setenv("STENCIL_TK_TIER", "1")


def _engine(gpu, shape):
    e = JacobiEngine(StencilSpec(dims=3, dtype="fp64"), *shape, device=gpu)
    assert e.lib.stencil_debug_knobs() == 1
    return e


@pytest.mark.parametrize("shape,it,init", [
    ((56, 48, 9), 8, "random"),      # one tile: one producer, one consumer, 9 planes
    ((100, 90, 37), 8, "random"),    # 2 x 2 tiles, one launch
    ((100, 90, 37), 19, "random"),   # two launches + a K = 4 launch + a pair + a single
    ((64, 64, 64), 16, "reference"),
    ((130, 97, 50), 27, "random"),   # ragged tiles in x and y
    ((300, 250, 20), 24, "random"),  # 6 x 6 tiles, fewer planes than the slot ring holds twice
])
def test_tier_matches_oracle(gpu, tier_env, shape, it, init):
    e = _engine(gpu, shape)
    launches, kernel = e.plan(8)
    assert (launches, kernel) == (1, _lib.KERNEL_TEMPORALK), "8 sweeps = one two-tier launch"
    assert e.fuse_steps == 8
    e.reset(init, 3)
    fin, _ = e.iterate(it)
    got = e.to_numpy(fin)
    p = ob.problem(3, "fp64", "star", 1, "naive", *shape)
    want = ob.run(p, it, init, 3)
    assert np.array_equal(got.view(np.uint8), want.view(np.uint8)), np.argwhere(got != want)[:5]


def test_tier_c2_whole_job(gpu, tier_env):
    """BASELINE config 2 through the two-tier launches: 512^3 fp64 from the
    reference initial condition, 1000 sweeps = 125 launches, bitwise the
    16-thread oracle."""
    import torch
    n, it = 512, 1000
    e = _engine(gpu, (n, n, n))
    assert e.plan(it) == (125, _lib.KERNEL_TEMPORALK)
    e.reset()
    e.prepare()
    fin, ms = e.iterate(it, timed=True)
    got = e.interior(fin).cpu().numpy()
    del e, fin
    torch.cuda.empty_cache()
    p = ob.problem(3, "fp64", "star", 1, "naive", n, n, n)
    want = ob.interior(p, ob.run(p, it, threads=16))
    assert np.array_equal(got.view(np.uint8), np.ascontiguousarray(want).view(np.uint8))
    print(f"two-tier C2: {ms:.2f} ms for {it} sweeps = {n ** 3 * it / ms / 1e6:.1f} Gcell/s")


def test_tier_not_used_on_large_planes(gpu, tier_env):
    """Grids whose tiles do not fit twice on the device keep the K = 4 launches."""
    e = JacobiEngine(StencilSpec(dims=3, dtype="fp64"), 2048, 2048, 16, device=gpu, allocate=False)
    assert e.plan(8)[0] == 2

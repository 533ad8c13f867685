"""The packed z-chunk schedule's dispatcher model (kernels_strip.hip
pack_search, exported as stencil_pack_plan) on the CPU: the shapes measured
on MI355X (profiles/r02gg_pack.log, r02hh_pick.log) and a plain-Python
restatement of the model over random shapes.  No GPU: the model is host code."""
import ctypes
import math
import random

import pytest

from stencil_amd import _lib


def plan(tiles, nz, fill, slots, zc):
    lib = _lib.load()
    eq, pk, wg = ctypes.c_int64(0), ctypes.c_int64(0), ctypes.c_int64(0)
    rc = lib.stencil_pack_plan(tiles, nz, fill, slots, zc, ctypes.byref(eq), ctypes.byref(pk), ctypes.byref(wg))
    return rc, eq.value, pk.value, wg.value


def model(tiles, nz, fill, slots, zc):
    """Workgroup i goes to XCD i % 8, there to the slot that frees first; a
    chunk of n planes costs n + fill steps; chunks longest first."""
    def makespan(lens):
        per = max(1, slots // 8)
        free = [[0] * per for _ in range(8)]
        span = 0
        for i, n in enumerate(lens):
            f = free[i % 8]
            j = min(range(per), key=f.__getitem__)
            f[j] += n + fill
            span = max(span, f[j])
        return span

    def build(lc):
        items = []
        for t in range(tiles):
            z, c = 0, 0
            while z < nz:
                items.append((min(lc, nz - z), c, t))
                z += lc
                c += 1
        items.sort(key=lambda it: (-it[0], it[1], it[2]))
        return makespan([it[0] for it in items]), len(items)

    base, _ = build(zc)
    best, best_n = base, 0
    lc = max(fill, nz // 16)
    while lc <= nz:
        m, n = build(lc)
        if m < best:
            best, best_n = m, n
        lc += max(1, nz // 256)
    return base, best, (best_n if best_n and best * 50 < base * 49 else 0)


def equal_chunk(tiles, nz, fill, slots):
    """kernels_strip.hip launch_st: the chunk count minimising rounds x (chunk + fill)."""
    best_c, best = 1, None
    for c in range(1, nz + 1):
        z = math.ceil(nz / c)
        if c > 1 and z < fill:
            break
        cost = math.ceil(tiles * c / slots) * (z + fill)
        if best is None or cost <= best:
            best, best_c = cost, c
    return math.ceil(nz / best_c)


@pytest.mark.parametrize("shape,want", [
    ((512, 512, 512), (260, 240, 330)),   # C2: packed kept by the trial (0.456 vs 0.487 ms)
    ((504, 512, 512), (222, 216, 297)),   # the model packs; measured 0.566 vs 0.423 ms: equal chunks win
    ((256, 256, 256), (40, 39, 270)),     # likewise (-17 % packed)
    ((320, 320, 320), (62, 62, 0)),       # no gain predicted: equal chunks
    ((768, 768, 256), (264, 238, 448)),
])
def test_model_at_measured_shapes(shape, want):
    nx, ny, nz = shape
    tiles = math.ceil(nx / 56) * math.ceil(ny / 48)  # fp64 K = 4 strip tile: 56 x 48 outputs
    zc = equal_chunk(tiles, nz, 8, 256)
    rc, eq, pk, wg = plan(tiles, nz, 8, 256, zc)
    assert rc == 0
    assert (eq, pk, wg) == want


def test_model_matches_python_restatement():
    rng = random.Random(7)
    for _ in range(12):
        tiles, nz = rng.randint(1, 300), rng.randint(1, 700)
        fill, slots = rng.choice([6, 8, 9, 12]), rng.choice([64, 128, 256])
        zc = equal_chunk(tiles, nz, fill, slots)
        rc, eq, pk, wg = plan(tiles, nz, fill, slots, zc)
        assert rc == 0
        assert (eq, pk, wg) == model(tiles, nz, fill, slots, zc), (tiles, nz, fill, slots, zc)


def test_invalid_arguments():
    lib = _lib.load()
    for args in [(0, 10, 8, 256, 5), (10, 0, 8, 256, 5), (10, 10, -1, 256, 5), (10, 10, 8, 0, 5), (10, 10, 8, 256, 0)]:
        rc, *_ = plan(*args)
        assert rc != 0
        assert b"pack plan" in lib.stencil_last_error_message()

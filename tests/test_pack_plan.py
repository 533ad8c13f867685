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


def table(tiles, tiles_x, nz, fill, slots, zc, w):
    lib = _lib.load()
    n = ctypes.c_int64(0)
    assert lib.stencil_pack_table(tiles, tiles_x, nz, fill, slots, zc, w, None, 0, ctypes.byref(n)) == 0
    buf = (ctypes.c_int32 * (3 * n.value))()
    assert lib.stencil_pack_table(tiles, tiles_x, nz, fill, slots, zc, w, buf, n.value, ctypes.byref(n)) == 0
    return [tuple(buf[3 * i:3 * i + 3]) for i in range(n.value)]


@pytest.mark.parametrize("w", [2, 3, 5, 10])
def test_xcd_patch_order_permutes_generations_into_patches(w):
    """stencil_pack_table with an XCD-patch width: C2's packed
    grid (10 x 11 tiles of 512 planes, K = 4, 256 slots) keeps every
    position's chunk length and first plane -- the same makespan -- and only
    permutes tiles within each generation; the tiles one XCD holds in a
    generation (workgroup i -> XCD i % 8) then have same-XCD x/y neighbours,
    where the tile-major table has none."""
    tx, ty = 10, 11
    base = table(tx * ty, tx, 512, 8, 256, 256, 0)
    pat = table(tx * ty, tx, 512, 8, 256, 256, w)
    assert len(base) == len(pat) == 330
    assert [(z, n) for _, z, n in base] == [(z, n) for _, z, n in pat]
    gens = {}
    for i, (t, z, n) in enumerate(pat):
        gens.setdefault((z, n), []).append((i, t))
    assert sorted(t for t, _, _ in base) == sorted(t for t, _, _ in pat)

    def shared_neighbours(tab):
        xcd = {}
        for i, (t, z, n) in enumerate(tab):
            xcd[(t, z, n)] = i % 8
        pairs = 0
        for (t, z, n), x in xcd.items():
            bx, by = t % tx, t // tx
            for dx, dy in ((1, 0), (0, 1)):
                if bx + dx < tx and by + dy < ty and xcd.get((t + dx + dy * tx, z, n)) == x:
                    pairs += 1
        return pairs

    for key, ent in gens.items():
        assert len({t for _, t in ent}) == len(ent)  # a permutation: every tile once per generation
    assert shared_neighbours(base) == 0
    assert shared_neighbours(pat) >= 100 if w > 2 else shared_neighbours(pat) >= 60


def test_auto_patch_width_for_c2():
    """xcd_width = -1 (what long jobs launch): the width with the most same-XCD
    neighbour tiles -- 5 for C2's 10 x 11 tiles (451 of 597 pairs)."""
    tx, ty = 10, 11
    assert table(tx * ty, tx, 512, 8, 256, 256, -1) == table(tx * ty, tx, 512, 8, 256, 256, 5)

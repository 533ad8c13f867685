"""The C-ABI library loads, exports every symbol include/stencil_hip.h
declares, keeps the reference's struct layouts, and validates problems --
all without touching a GPU."""
import ctypes
import os
import re

import pytest

from stencil_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "stencil_hip.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?\w+\s*\**\s*(stencil_\w+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_header_declares_what_binding_knows():
    decl = declared_functions()
    assert len(decl) >= 20
    assert set(decl) == set(_lib.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    for name in declared_functions():
        assert hasattr(lib, name), name


def test_library_has_gfx950_code_object():
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_reference_struct_layouts():
    # struct Arguments is 88 bytes on LP64; each
    # BoundaryMatrixView<float> is 40 bytes.
    assert ctypes.sizeof(_lib.MatrixView) == 40
    assert ctypes.sizeof(_lib.Arguments) == 88
    assert _lib.Arguments.input.offset == 8 and _lib.Arguments.output.offset == 48
    assert ctypes.sizeof(_lib.Problem) == 56


@pytest.mark.parametrize("dims,dtype,r,n", [(2, _lib.F32, 1, (1024, 1024, 1)), (3, _lib.F64, 1, (512, 512, 512)),
                                            (3, _lib.F32, 2, (70, 19, 6)), (2, _lib.F64, 40, (5, 3, 1))])
def test_layout_alignment(dims, dtype, r, n):
    lay = _lib.make_layout(_lib.make_problem(dims=dims, dtype=dtype, radius=r, nx=n[0], ny=n[1], nz=n[2]))
    es = 8 if dtype == _lib.F64 else 4
    align = 128 // es
    ox = lay.origin % lay.row
    assert ox % align == 0 and ox >= r                      # interior x=0 is 128-B aligned, ghosts fit
    assert lay.row % align == 0 and lay.row >= ox + n[0] + r
    assert lay.rows == n[1] + 2 * r
    assert lay.plane == lay.row * lay.rows
    assert lay.planes == (n[2] + 2 * r if dims == 3 else 1)
    assert lay.bytes == lay.elems * es == lay.plane * lay.planes * es
    lib = _lib.load()
    assert lib.stencil_slow_extent(ctypes.byref(lay)) == (n[2] if dims == 3 else n[1])


@pytest.mark.parametrize("kw,code", [
    (dict(dims=4), _lib.STENCIL_OK - 1),
    (dict(radius=0), -1),
    (dict(dims=3, order=_lib.ORDER_DMA), -1),
    (dict(dims=2, shape=_lib.BOX, order=_lib.ORDER_DMA), -1),
    (dict(nx=-3), -1),
    (dict(dims=2, nz=5), -1),
    (dict(dims=2, nz=1, kernel=_lib.KERNEL_ZMARCH), -5),
    (dict(dims=3, shape=_lib.BOX, radius=2, kernel=_lib.KERNEL_ZMARCH), -5),
    (dict(dims=3, radius=2, kernel=_lib.KERNEL_TEMPORAL2), -5),
    (dict(dims=3, radius=2, halo=1), -1),
    (dict(dims=2, nz=1, halo=2), -1),
    (dict(dims=3, flags=4), -1),
])
def test_layout_rejects_invalid(kw, code):
    base = dict(dims=3, dtype=_lib.F64, nx=8, ny=8, nz=8)
    base.update(kw)
    prob = _lib.Problem(dims=base.get("dims"), dtype=base.get("dtype"), shape=base.get("shape", 0),
                        radius=base.get("radius", 1), order=base.get("order", 0), kernel=base.get("kernel", 0),
                        halo=base.get("halo", 0), flags=base.get("flags", 0),
                        nx=base.get("nx"), ny=base.get("ny"), nz=base.get("nz"))
    lib = _lib.load()
    lay = _lib.Layout()
    rc = lib.stencil_layout_init(ctypes.byref(prob), ctypes.byref(lay))
    assert rc == code
    assert lib.stencil_last_error_message()


def test_halo_depth_layout():
    lay = _lib.make_layout(_lib.make_problem(dims=3, nx=16, ny=8, nz=10, halo=2, flags=_lib.HALO_LO))
    assert lay.zghost == 2 and lay.planes == 14
    assert lay.origin // lay.plane == 2


def test_error_strings():
    lib = _lib.load()
    for code in (0, -1, -2, -3, -4, -5, -99):
        assert lib.stencil_strerror(code)
    with pytest.raises(_lib.StencilError):
        _lib.make_layout(_lib.make_problem(dims=2, radius=0, nx=4, ny=4))


def test_plan_counts_launches(monkeypatch):
    lib = _lib.load(debug=True)  # STENCIL_NO_TK below is an experiment knob
    lay2 = _lib.make_layout(_lib.make_problem(dims=2, nx=64, ny=64))
    launches, kernel = ctypes.c_int64(), ctypes.c_int32()
    assert lib.stencil_plan(ctypes.byref(lay2), 100, ctypes.byref(launches), ctypes.byref(kernel)) == 0
    assert launches.value == 1 and kernel.value == _lib.KERNEL_TEMPORAL2  # 2D, fits one workgroup: one launch
    lay2 = _lib.make_layout(_lib.make_problem(dims=2, nx=300, ny=300))
    assert lib.stencil_plan(ctypes.byref(lay2), 100, ctypes.byref(launches), ctypes.byref(kernel)) == 0
    # 2D: 8 sweeps per launch without a GPU to query; up to 16 where one round of tiles fits the CUs
    assert launches.value in {-(-100 // k) for k in range(8, 17)} and kernel.value == _lib.KERNEL_TEMPORAL2
    lay = _lib.make_layout(_lib.make_problem(dims=3, nx=8, ny=8, nz=8))
    launches, kernel = ctypes.c_int64(), ctypes.c_int32()
    assert lib.stencil_plan(ctypes.byref(lay), 7, ctypes.byref(launches), ctypes.byref(kernel)) == 0
    assert launches.value == 3 and kernel.value == _lib.KERNEL_TEMPORALK  # AUTO: 3 + 3 fused, 1 single
    monkeypatch.setenv("STENCIL_TK_STEPS", "4")
    assert lib.stencil_plan(ctypes.byref(lay), 11, ctypes.byref(launches), ctypes.byref(kernel)) == 0
    assert launches.value == 4 and kernel.value == _lib.KERNEL_TEMPORALK  # 4 + 4 + pair + single
    monkeypatch.setenv("STENCIL_NO_TK", "1")
    assert lib.stencil_plan(ctypes.byref(lay), 7, ctypes.byref(launches), ctypes.byref(kernel)) == 0
    assert launches.value == 4 and kernel.value == _lib.KERNEL_TEMPORAL2  # pairs + single
    monkeypatch.delenv("STENCIL_NO_TK")
    monkeypatch.delenv("STENCIL_TK_STEPS")
    lay = _lib.make_layout(_lib.make_problem(dims=3, nx=8, ny=8, nz=8, kernel=_lib.KERNEL_ZMARCH))
    assert lib.stencil_plan(ctypes.byref(lay), 7, ctypes.byref(launches), ctypes.byref(kernel)) == 0
    assert launches.value == 7 and kernel.value == _lib.KERNEL_ZMARCH
    lay = _lib.make_layout(_lib.make_problem(dims=3, shape=_lib.BOX, nx=8, ny=8, nz=8))
    assert lib.stencil_plan(ctypes.byref(lay), 7, ctypes.byref(launches), ctypes.byref(kernel)) == 0
    assert launches.value == 3 and kernel.value == _lib.KERNEL_TEMPORAL2  # 27-point: 2 x 3-step launches + single
    monkeypatch.setenv("STENCIL_BOX_STEPS", "2")
    assert lib.stencil_plan(ctypes.byref(lay), 7, ctypes.byref(launches), ctypes.byref(kernel)) == 0
    assert launches.value == 4 and kernel.value == _lib.KERNEL_TEMPORAL2  # pairs + single
    monkeypatch.delenv("STENCIL_BOX_STEPS")
    lay = _lib.make_layout(_lib.make_problem(dims=3, radius=2, nx=8, ny=8, nz=8))
    assert lib.stencil_plan(ctypes.byref(lay), 7, ctypes.byref(launches), ctypes.byref(kernel)) == 0
    assert launches.value == 7 and kernel.value == _lib.KERNEL_DIRECT


def test_product_library_ignores_experiment_knobs(monkeypatch):
    """The shipped library runs AUTO's plan only: experiment knobs (here
    STENCIL_NO_TK, which turns the K-step kernel off) are read by the debug
    twin alone; the documented STENCIL_TK_STEPS is read by both."""
    prod, dbg = _lib.load(debug=False), _lib.load(debug=True)
    assert prod.stencil_debug_knobs() == 0 and dbg.stencil_debug_knobs() == 1
    lay = _lib.make_layout(_lib.make_problem(dims=3, nx=8, ny=8, nz=8))
    launches, kernel = ctypes.c_int64(), ctypes.c_int32()
    monkeypatch.setenv("STENCIL_NO_TK", "1")
    assert _lib.load() is dbg  # an experiment knob is set: the debug twin
    assert prod.stencil_plan(ctypes.byref(lay), 8, ctypes.byref(launches), ctypes.byref(kernel)) == 0
    assert (launches.value, kernel.value) == (2, _lib.KERNEL_TEMPORALK)
    assert dbg.stencil_plan(ctypes.byref(lay), 8, ctypes.byref(launches), ctypes.byref(kernel)) == 0
    assert (launches.value, kernel.value) == (4, _lib.KERNEL_TEMPORAL2)
    monkeypatch.delenv("STENCIL_NO_TK")
    monkeypatch.setenv("STENCIL_TK_STEPS", "3")
    assert _lib.load() is prod  # documented knobs keep the product
    assert prod.stencil_plan(ctypes.byref(lay), 9, ctypes.byref(launches), ctypes.byref(kernel)) == 0
    assert launches.value == 3


def test_row_pitch_rule():
    """stencil_layout_init's row-pitch rule: pitches of
    32 KiB or more within [-512, +256] B of a multiple of 32 KiB move to
    residue 384 (from [-256, 256]) or 128 B up (from [-512, -384]); every other
    pitch is the 128-B-aligned minimum.  Every preset width is covered."""
    from stencil_amd import _lib
    cases = {  # (dtype, nx): row pitch in bytes
        ("fp64", 512): 4352, ("fp64", 2048): 16640, ("fp32", 4096): 16640,  # C2, C4/C5/NS, C3: no padding
        ("fp64", 4096): 33152,   # NS4096: 33024 (r 256) -> 33152
        ("fp64", 4000): 32384,   # 32256 (r -512) -> +128
        ("fp64", 4032): 33152,   # 32512 (r -256) -> r 384 (+128 would land on r -128)
        ("fp64", 4048): 33152,   # 32640 (r -128) -> r 384 (+128 would land on r 0)
        ("fp32", 8112): 33152,   # 32640 (r -128) -> r 384
        ("fp64", 4128): 33280,   # r 512: unpadded
        ("fp64", 8160): 65920,   # 65536 (r 0) -> r 384
        ("fp64", 8192): 65920,   # 65792 (r 256) -> r 384
        ("fp32", 8160): 33152,   # 32896 (r 128) -> r 384
        ("fp32", 8192): 33152,   # 33024 (r 256) -> r 384
        ("fp64", 12288): 98688,  # 98560 (r 256) -> r 384
    }
    for (dt, nx), want in cases.items():
        es = 8 if dt == "fp64" else 4
        lay = _lib.make_layout(_lib.make_problem(dims=3, dtype=_lib.F64 if dt == "fp64" else _lib.F32, nx=nx, ny=4, nz=4))
        assert lay.row * es == want, (dt, nx, lay.row * es, want)

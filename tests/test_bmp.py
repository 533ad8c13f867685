"""The BMP dump: header layout and colour map of the
reference's BMPImage / Stencil::to_bmp, checked by compiling the header into a
tiny host program (no GPU)."""
import os
import struct
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(ROOT, "stencil_amd", "csrc", "host")

PROG = r'''
#include "bmp.hpp"
#include <cstdio>
int main(int argc, char** argv) {
    std::vector<BmpPixel> px;
    const double vals[6] = {0.0, 0.2, 0.3, 0.6, 0.9, 1.0};
    for (double v : vals) px.push_back(heat_color(v));
    if (!write_bmp24(argv[1], 3, 2, px)) return 1;
    for (double v : vals) { BmpPixel p = heat_color(v); std::printf("%d %d %d\n", p.r, p.g, p.b); }
    return 0;
}
'''


@pytest.fixture(scope="module")
def prog(tmp_path_factory):
    d = tmp_path_factory.mktemp("bmp")
    src = d / "t.cpp"
    src.write_text(PROG)
    exe = d / "t"
    subprocess.run(["g++", "-std=c++17", "-O1", "-I", HOST, str(src), "-o", str(exe)], check=True)
    return exe, d


def test_bmp_layout(prog):
    exe, d = prog
    out = d / "img.bmp"
    r = subprocess.run([str(exe), str(out)], capture_output=True, text=True, check=True)
    data = out.read_bytes()
    row = 3 * 3 + 3  # 9 bytes of pixels padded to 12
    assert data[:2] == b"BM"
    assert struct.unpack("<I", data[2:6])[0] == len(data) == 54 + 2 * row
    assert struct.unpack("<I", data[10:14])[0] == 54
    assert struct.unpack("<IiiHH", data[14:30]) == (40, 3, 2, 1, 24)
    # first pixel (value 0): pure blue, stored B, G, R
    assert data[54:57] == bytes([255, 0, 0])
    assert data[54 + 9:54 + 12] == b"\0\0\0"  # row padding
    colours = [tuple(map(int, line.split())) for line in r.stdout.split("\n") if line]
    # quarter-wise heat map (stencil.cpp:163-186): r, g, b
    assert colours[0] == (0, 0, 255)
    assert colours[1] == (0, int(4 * 0.2 * 255), 255)
    assert colours[2] == (0, 255, int((1 + 4 * (0.25 - 0.3)) * 255))
    assert colours[3] == (int(4 * (0.6 - 0.5) * 255), 255, 0)
    assert colours[5] == (255, 0, 0)


def test_cli_accepts_bmp_flag():
    cli = os.path.join(ROOT, "build", "bin", "stencil_main")
    p = subprocess.run([cli, "-s", "8", "-b", "1", "-i", "1", "-m", "HIP", "--bmp", "x.bmp", "--print-config"],
                       capture_output=True, text=True)
    assert p.returncode == 0

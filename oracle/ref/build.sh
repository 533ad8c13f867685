#!/bin/bash
# Build the reference's own naive CPU loop into oracle/_ref/ (TEST
# INFRASTRUCTURE ONLY; this container only -- /root/reference does not exist
# on the GPU box, and nothing built here is used by the product).
#
#   oracle/_ref/ref_naive   Stencil::check_result's loop (stencil.cpp:77-131)
#                           and generate_initialized_matrix (190-207), compiled
#                           from the reference's source lines with its real
#                           headers; emits the final interior (tests/golden/
#                           make_ref_golden.py turns it into fixtures)
#   oracle/_ref/abi_check   static_asserts: include/stencil_hip.h's
#                           StencilArguments / StencilMatrixView against the
#                           reference's Arguments / BoundaryMatrixView<float>
#
# The reference lines are piped straight into the compiler; no copy of them is
# written anywhere.  The kernels (src/stencil/slave/*.cpp) and the full
# stencil.cpp need the Sunway athread SDK and cannot be built here.
set -euo pipefail
HERE=$(cd "$(dirname "$0")" && pwd)
ROOT=$(cd "$HERE/../.." && pwd)
REF=${REF:-/root/reference}
OUT=$ROOT/oracle/_ref
CXX=${CXX:-g++}
# IEEE arithmetic as written: no FMA contraction, no fast-math
# (x86-64 SSE2 float/double, like the survey's probe at -O2)
FLAGS=(-std=c++17 -O2 -ffp-contract=off -fno-fast-math -Wno-unused-result -I"$REF/include" -I"$ROOT/include")
if [ ! -f "$REF/src/stencil/stencil.cpp" ]; then
    echo "reference tree not found at $REF: oracle/_ref not built" >&2
    exit 0
fi
mkdir -p "$OUT"
SRC=$REF/src/stencil/stencil.cpp
{
    cat "$HERE/head.inc"
    sed -n '190,207p' "$SRC"
    cat "$HERE/mid.inc"
    sed -n '77,131p' "$SRC"
    cat "$HERE/mid2.inc"
    sed -n '85,131p' "$SRC" | sed 's/\bfloat\b/double/g'
    cat "$HERE/tail.inc"
} | "$CXX" "${FLAGS[@]}" -x c++ - -o "$OUT/ref_naive"
{
    cat "$HERE/abi_head.inc"
    sed -n '13,24p' "$REF/src/stencil/slave/stencil_slave.hpp"
    cat "$HERE/abi_tail.inc"
} | "$CXX" "${FLAGS[@]}" -x c++ - -o "$OUT/abi_check"
"$OUT/abi_check"
echo "built $OUT/ref_naive"

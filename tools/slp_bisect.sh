#!/bin/bash
# Build variants of the debug library whose box probe object (kernels_boxk_probe.hip,
# SLP vectorisation ON) is compiled with extra compiler flags, to find which
# compilation step makes the fp32 one-cell-per-lane box shapes compute wrong values
# (DESIGN.md §9.2b).  Every variant lands in build/slp/libdbg_<tag>.so; tools/slp_bisect.py
# runs a probe shape through one of them against the oracle.
#   usage: tools/slp_bisect.sh tag "extra flags" [tag "extra flags" ...]
set -euo pipefail
cd "$(dirname "$0")/.."
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-gpu-flush-denormals-to-zero -Wno-pass-failed -Iinclude -Istencil_amd/csrc -fslp-vectorize"
mkdir -p build/slp
OTHERS=$(ls build/obj/*.o | grep -v -e '/kernels_boxk_probe.o$' -e '/knobs.o$')
while [ $# -ge 2 ]; do
  tag=$1; extra=$2; shift 2
  # shellcheck disable=SC2086
  $HIPCC $FLAGS $extra -c stencil_amd/csrc/kernels_boxk_probe.hip -o build/slp/probe_$tag.o 2> build/slp/probe_$tag.err
  # shellcheck disable=SC2086
  $HIPCC --offload-arch=gfx950 -shared -fPIC -o build/slp/libdbg_$tag.so $OTHERS build/slp/probe_$tag.o
  echo "built build/slp/libdbg_$tag.so ($extra)"
done

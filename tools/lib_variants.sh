#!/bin/bash
# Build variants of the product library in which ONE kernel source is compiled with extra compiler
# flags (scheduler choices and the like), for A/B runs of bench.py through tools/bench_lib.py.
#   usage: tools/lib_variants.sh <source.hip> tag "extra flags" [tag "extra flags" ...]
#   -> build/variants/lib_<tag>.so (+ build/variants/<tag>.info: VGPRs / spills of the source's kernels)
set -euo pipefail
cd "$(dirname "$0")/.."
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
SRC=$1; shift
BASE=$(basename "$SRC" .hip)
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -fno-gpu-flush-denormals-to-zero -Wno-pass-failed -Iinclude -Istencil_amd/csrc"
mkdir -p build/variants
OTHERS=$(ls build/obj/*.o | grep -v -e "/$BASE.o\$" -e '/knobs_debug.o$')
while [ $# -ge 2 ]; do
  tag=$1; extra=$2; shift 2
  # shellcheck disable=SC2086
  $HIPCC $FLAGS $extra -c "$SRC" -o build/variants/${BASE}_$tag.o -Rpass-analysis=kernel-resource-usage 2> build/variants/$tag.info
  # shellcheck disable=SC2086
  $HIPCC --offload-arch=gfx950 -shared -fPIC -o build/variants/lib_$tag.so $OTHERS build/variants/${BASE}_$tag.o
  echo "built build/variants/lib_$tag.so ($extra)"
done

#!/bin/bash
# Build variants of the product library in which kernel sources are compiled with extra compiler
# flags (scheduler choices, -D switches and the like), for A/B runs through tools/bench_lib.py /
# tools/time_lib.py.
#   usage: tools/lib_variants.sh <source.hip>[,<source.hip>...] tag "extra flags" [tag "extra flags" ...]
#   -> build/variants/lib_<tag>.so (+ build/variants/<tag>.info: VGPRs / spills of the sources' kernels)
# Each source keeps its Makefile flags (kernels_strip_ilp.hip: the max-ILP scheduler) plus the extra ones.
set -euo pipefail
cd "$(dirname "$0")/.."
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
IFS=',' read -r -a SRCS <<< "$1"; shift
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -fno-gpu-flush-denormals-to-zero -Wno-pass-failed -Iinclude -Istencil_amd/csrc"
mkdir -p build/variants
EXCL=(-e '/knobs_debug.o$' -e '/kernels_boxk_probe' -e '/kernels_strip_probe')
for src in "${SRCS[@]}"; do EXCL+=(-e "/$(basename "$src" .hip).o\$"); done
OTHERS=$(ls build/obj/*.o | grep -v "${EXCL[@]}")
per_file_flags() {  # the Makefile's per-file device flags
  case "$(basename "$1" .hip)" in
    kernels_strip_ilp|kernels_tb2d) echo "-Xarch_device -mllvm=-misched=gcn-max-ilp" ;;
    kernels_boxk) echo "-Xarch_device -mllvm=-amdgpu-disable-unclustered-high-rp-reschedule" ;;
  esac
}
while [ $# -ge 2 ]; do
  tag=$1; extra=$2; shift 2
  objs=()
  : > build/variants/$tag.info
  for src in "${SRCS[@]}"; do
    base=$(basename "$src" .hip)
    # shellcheck disable=SC2086
    $HIPCC $FLAGS $(per_file_flags "$src") $extra -c "$src" -o build/variants/${base}_$tag.o \
      -Rpass-analysis=kernel-resource-usage 2>> build/variants/$tag.info
    objs+=(build/variants/${base}_$tag.o)
  done
  # shellcheck disable=SC2086
  $HIPCC --offload-arch=gfx950 -shared -fPIC -o build/variants/lib_$tag.so $OTHERS "${objs[@]}"
  echo "built build/variants/lib_$tag.so ($extra)"
done

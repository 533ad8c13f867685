#!/bin/bash
# Final-tree PMC picture (FETCH/WRITE, SQ waits/VALU/LDS, TCC hit rate) of the
# default C2 kernel (512^3 fp64, K = 4 strip, packed) and of the box K = 4
# strip at the C5 slab (2048^2 x 256 fp64); tools/pmc_table.py summarises
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/pmc_variants.sh r02qq_c2 "STENCIL_TK_PACK=1" || exit 1
TUNE_KERNEL=auto TUNE_STENCIL=box TUNE_SWEEPK=4 TUNE_SHAPE=2048,2048,256 TUNE_ITERS=8 \
  bash tools/pmc_variants.sh r02qq_box "STENCIL_BOX_STEPS=4" || exit 1

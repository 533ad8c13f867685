#!/bin/bash
# PMC passes of the box kernel shapes (fp64 K=3): 2048^2 x 256 and 512^3
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TUNE_STENCIL=box TUNE_SWEEPK=3 TUNE_DTYPE=fp64 TUNE_ITERS=6 TUNE_KERNEL=auto
TUNE_SHAPE=2048,2048,256 bash tools/pmc_variants.sh box2048 STENCIL_BOXK_CFG=10308 STENCIL_BOXK_CFG=910216 STENCIL_BOXK_CFG=910408 || exit 1
TUNE_SHAPE=512,512,512 bash tools/pmc_variants.sh box512 STENCIL_BOXK_CFG=10308 STENCIL_BOXK_CFG=910408 || exit 1

#!/bin/bash
# Counterpart of the reference's run.sh (run.sh:3).  The reference submits one
# Sunway job through bsub with a stale flag (-m 400 meant the matrix size,
# SURVEY.md §4); this runs the drop-in binary directly on the local GPU with
# the current CLI: 400 x 400 grid, 50-cell blocks, 1000 iterations, radius 1;
# CPU (the reference's own naive loop on the host) runs beside the GPU methods.
set -e
cd "$(dirname "$0")"
[ -x build/bin/stencil_main ] || make -j8
exec ./build/bin/stencil_main -s 400 -b 50 -i 1000 -r 1 -m DMA DMAStaticUnroll DMASlavePack RMA HIP CPU "$@"

#!/bin/bash
# round 3, call as: the driver's own bench command on the final tree, twice; and the single-process 2-slab
# rehearsal through the C-ABI (slabs sharing GPU 0, device-copy halos)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03as_driver_cmd.json 2>/dev/null &&
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline >> gpurun_out/r03as_driver_cmd.json 2>/dev/null &&
timeout -k 10 300 python3 bench.py --gpus 2 --share-device --exchange copy --steps 40 --warmup 8 > gpurun_out/r03as_rehearse_2slab.json 2>/dev/null

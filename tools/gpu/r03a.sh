#!/bin/bash
# round 3, call a: the whole benched C2 job and the C5 slab against the oracle; HBM capacity probe
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python3 -c "
import torch
f, t = torch.cuda.mem_get_info(0)
p = torch.cuda.get_device_properties(0)
print('mem_get_info free', f, 'total', t, 'GiB', f/2**30, t/2**30, 'props total', p.total_memory)
" > gpurun_out/r03a_mem.txt 2>&1 &&
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "c2_whole_benched_job or c5_slab_reference_job or full_size_c2_1000" \
  > gpurun_out/r03a_tests.txt 2>&1

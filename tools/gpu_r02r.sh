#!/bin/bash
# C++ slab jobs with face-signalled rounds: slab-job + CLI tests, host-timed rings (signal on/off, copy/RCCL)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_slab_job.py tests/test_gpu_parity.py -k "slab_job or multi_gpu or cli" -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_r02r.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests_r02r.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/slab_job_time.py 512 star 400 || exit 1
timeout -k 10 300 python -u tools/slab_job_time.py 1024 box 60 || exit 1

#!/bin/bash
# round 3, call c: rolling-vs-two-grid diagnostic at large planes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u tools/rolling_diag.py > gpurun_out/r03c_rolling_diag.txt 2>&1

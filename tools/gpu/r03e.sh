#!/bin/bash
# round 3, call e: rolling-vs-two-grid diagnostic, then call d's A/B + PMC + probe + rehearsal + default bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 420 python3 -u tools/rolling_diag.py > gpurun_out/r03c_rolling_diag.txt 2>&1
bash tools/gpu/r03d.sh

# decomposition of the persistent 2D kernel's time (DIAG builds give wrong results)
set -o pipefail
for d in 0 1 2; do
  echo "== DIAG $d"
  STENCIL_TB2DP_DIAG=$d TUNE_DIMS=2 TUNE_ITERS=96 timeout -k 5 120 python tools/tune.py 1024 '[{}, {"STENCIL_TB2DP": 1}, {"STENCIL_TB2DP": 1, "STENCIL_TB2DP_K": 16}, {"STENCIL_TB2DP": 1, "STENCIL_TB2DP_K": 4}]' || exit 1
done

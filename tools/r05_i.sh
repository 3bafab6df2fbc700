#!/bin/bash
# round-5 pass i: -m gpu suite on the build with FastDiv in the camera stage only + precomputed
# Gaussian filter weights, then same-box A/B against the unit_quot build (variants/quot)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r05/i
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
A="--pmc off --steps 20 --warmup 2 --nanovdb-leg 0 --tune-walk off"
Q="AVR_LIB=variants/quot/libavr_hip.so"
bash tools/gpu_ab.sh "cam1||$A" "quot1|$Q|$A" "cam2||$A" "quot2|$Q|$A" "cam3||$A" "quot3|$Q|$A" || exit 2
mv gpurun_out/ab_*.json gpurun_out/ab_*.err $O/ 2>/dev/null
true

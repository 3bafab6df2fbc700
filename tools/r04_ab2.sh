#!/bin/bash
# A/B at the driver command (--steps 20): in-tree library (round-3 code) vs the pass-table variant
# (64 / 0 dims), the pass table + machine-LICM off, and the current source (pass table, wave
# counters, cooperative draws through LDS, gray sigma as scalars) at 3 waves and at 4 waves with
# machine LICM off; then the GPU suite on the two current-source builds
set -o pipefail
cd "$GRAFT_REPO_ROOT"
A="--steps 20 --warmup 2 --pmc off"
L() { echo "AVR_LIB=variants/$1/libavr_hip.so"; }
bash tools/gpu_ab.sh "base|$(L base)|$A" "pt64|$(L ptab)|$A" "pt0|$(L ptab)|$A --zsobol-pass-table 0" "licm|$(L ptlicm)|$A" \
  "r4a|$(L r4a)|$A" "r4l4|$(L r4l4)|$A" || exit 1
for v in r4a r4l4; do
  AVR_LIB=variants/$v/libavr_hip.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_$v.log 2>&1 || { tail -30 gpurun_out/tests_$v.log; exit 2; }
  tail -2 gpurun_out/tests_$v.log
done

#!/bin/bash
# A/B at the driver command (--steps 20): round-3 library (variants/base) vs the pass-table build
# (64 / 0 dims), the pass table + machine-LICM off, the current in-tree source (pass table, wave
# counters, cooperative draws through LDS, gray sigma as scalars) with the fat and the bricked
# grid layouts, and the current source at 4 waves/SIMD with machine LICM off; then the GPU suite
set -o pipefail
cd "$GRAFT_REPO_ROOT"
A="--steps 20 --warmup 2 --pmc off"
L() { echo "AVR_LIB=variants/$1/libavr_hip.so"; }
bash tools/gpu_ab.sh "base|$(L base)|$A" "pt64|$(L ptab)|$A" "pt0|$(L ptab)|$A --zsobol-pass-table 0" "licm|$(L ptlicm)|$A" \
  "cur||$A" "brick||$A --grid-layout brick" "r4l4|$(L r4l4)|$A" || exit 1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_cur.log 2>&1 || { tail -30 gpurun_out/tests_cur.log; exit 2; }
tail -2 gpurun_out/tests_cur.log
AVR_LIB=variants/r4l4/libavr_hip.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_r4l4.log 2>&1 || { tail -30 gpurun_out/tests_r4l4.log; exit 3; }
tail -2 gpurun_out/tests_r4l4.log
for lay in fat brick; do
  timeout -k 10 300 python tools/fetch_probe.py --layout $lay > gpurun_out/fetch_$lay.json 2> gpurun_out/fetch_$lay.err || { tail -5 gpurun_out/fetch_$lay.err; exit 4; }
  cat gpurun_out/fetch_$lay.json
done

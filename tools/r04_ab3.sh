#!/bin/bash
# A/B at the driver command (--steps 20): round-3 library vs the current source at 3 waves/SIMD
# (machine LICM on / off) and 4 waves/SIMD (off / on), the bricked layout; then the GPU suite on
# the 4-wave LICM-off build and the fetch probes of the fat and bricked layouts
set -o pipefail
cd "$GRAFT_REPO_ROOT"
A="--steps 20 --warmup 2 --pmc off"
L() { echo "AVR_LIB=variants/$1/libavr_hip.so"; }
bash tools/gpu_ab.sh "base|$(L base)|$A" "c3|$(L c3)|$A" "c3l|$(L c3l)|$A" "c4l|$(L c4l)|$A" "c4|$(L c4)|$A" \
  "c4lbrick|$(L c4l)|$A --grid-layout brick" "base2|$(L base)|$A" || exit 1
AVR_LIB=variants/c4l/libavr_hip.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_c4l.log 2>&1 || { tail -30 gpurun_out/tests_c4l.log; exit 2; }
tail -2 gpurun_out/tests_c4l.log
for lay in fat brick; do
  AVR_LIB=variants/c4l/libavr_hip.so timeout -k 10 300 python tools/fetch_probe.py --layout $lay > gpurun_out/fetch_$lay.json 2> gpurun_out/fetch_$lay.err || { tail -5 gpurun_out/fetch_$lay.err; exit 4; }
  cat gpurun_out/fetch_$lay.json
done

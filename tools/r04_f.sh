#!/bin/bash
# A/B at the driver command (--steps 20): pass table 64 vs 96 dimensions (two-level build,
# alternating), and the camera stage without its filter-table sampling (variants/camx3,
# measurement only: breaks replay)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
A="--steps 20 --warmup 2 --pmc off"
L() { echo "AVR_LIB=variants/$1/libavr_hip.so"; }
bash tools/gpu_ab.sh "f64a||$A" "f96a||$A --zsobol-pass-table 96" "camx3|$(L camx3)|$A" "f64b||$A" "f96b||$A --zsobol-pass-table 96" \
  "f80||$A --zsobol-pass-table 80" || exit 1

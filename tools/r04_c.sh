#!/bin/bash
# round-4 pass C: -m gpu suite on the paired camera draws, then A/B of the pass-table size
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04/c
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
A="--steps 20 --warmup 2 --pmc off --tune-walk off"
bash tools/gpu_ab.sh "cc8f|AVR_LIB=variants/c8f/libavr_hip.so|$A" "cpair||$A" "cpt32||$A --zsobol-pass-table 32" "cpt48||$A --zsobol-pass-table 48" "cpair2||$A" || exit 2

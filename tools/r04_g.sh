#!/bin/bash
# the guided filter search (camera stage) + pass table 96 by default: bench lines at the
# driver command, then the GPU suite
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
A="--steps 20 --warmup 2 --pmc off"
bash tools/gpu_ab.sh "g96a||$A" "g64||$A --zsobol-pass-table 64" "g96b||$A" || exit 1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_g.log 2>&1 || { tail -30 gpurun_out/tests_g.log; exit 3; }
tail -2 gpurun_out/tests_g.log

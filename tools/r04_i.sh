#!/bin/bash
# FastDiv index splits (camera stage + k_paths refill) and the Gaussian filter cell weights
# precomputed on the host: the GPU suite, then bench lines at the
# driver command; pass size 64 vs 128 / 32 sample indices (the drain's share of k_paths)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_i.log 2>&1 || { tail -30 gpurun_out/tests_i.log; exit 3; }
tail -1 gpurun_out/tests_i.log
A="--warmup 2 --pmc off --tune-walk off"
bash tools/gpu_ab.sh "i64a||--steps 20 $A" "i128p16k||--steps 10 --spp-per-step 128 --max-paths 134217728 --pixelsamples 16384 $A" \
  "i32p16k||--steps 20 --spp-per-step 32 --pixelsamples 16384 $A" "i64b||--steps 20 $A" || exit 1

#!/bin/bash
# pass size: k_paths per-sample time at 64 vs 128 sample indices per pass (the drain's share),
# at the driver's pixelsamples (16384) and at the plan's own for 128 (32768)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
A="--warmup 2 --pmc off --tune-walk off"
bash tools/gpu_ab.sh "s64||--steps 20 $A" "s128p16k||--steps 10 --spp-per-step 128 --max-paths 134217728 --pixelsamples 16384 $A" \
  "s128||--steps 20 --spp-per-step 128 --max-paths 134217728 $A" "s32p16k||--steps 20 --spp-per-step 32 --pixelsamples 16384 $A" || exit 1

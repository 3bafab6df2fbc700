#!/bin/bash
# round-5 pass t: what k_paths' correctly rounded float divisions cost (measurement builds, replay
# breaks, the paths' work is unchanged): Spec / float as a multiply by the hardware reciprocal
# (fsdiv, -DAVR_MEASURE_FAST_SDIV) and every f32 division and sqrt in the fast hardware sequence
# (fdivall, -fno-hip-fp32-correctly-rounded-divide-sqrt), against in-tree
# build first (CPU): python -m acceleratedvolrenderer_amd.build fsdiv -DAVR_MEASURE_FAST_SDIV;
#   python -m acceleratedvolrenderer_amd.build fdivall -fno-hip-fp32-correctly-rounded-divide-sqrt
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
A="--pmc off --tune-walk off --nanovdb-leg 0"
bash tools/gpu_ab.sh "base1||$A" "fs1|AVR_LIB=variants/fsdiv/libavr_hip.so|$A" "fa1|AVR_LIB=variants/fdivall/libavr_hip.so|$A" \
                     "base2||$A" "fs2|AVR_LIB=variants/fsdiv/libavr_hip.so|$A" "fa2|AVR_LIB=variants/fdivall/libavr_hip.so|$A"

#!/bin/bash
# round-5 pass l: upper bounds of two latency sources in k_paths' handlers (measurement-only
# builds whose samples are wrong but statistically the same work): the ZSobol pass-table reads
# of the cooperative draws (-DAVR_MEASURE_NO_PTAB) and the NEE spawn's two MurmurHash64A
# (-DAVR_MEASURE_CHEAP_HASH), against the in-tree build, alternating
# build first (CPU): python -m acceleratedvolrenderer_amd.build noptab -DAVR_MEASURE_NO_PTAB
#                   python -m acceleratedvolrenderer_amd.build cheaphash -DAVR_MEASURE_CHEAP_HASH
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
A="--pmc off --tune-walk off --nanovdb-leg 0"
bash tools/gpu_ab.sh "base1||$A" "noptab1|AVR_LIB=variants/noptab/libavr_hip.so|$A" "cheap1|AVR_LIB=variants/cheaphash/libavr_hip.so|$A" \
                     "base2||$A" "noptab2|AVR_LIB=variants/noptab/libavr_hip.so|$A" "cheap2|AVR_LIB=variants/cheaphash/libavr_hip.so|$A"

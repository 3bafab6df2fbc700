#!/bin/bash
# round-5 pass p: k_film occupancy after it took over the wavelength pdfs (127 VGPRs, 4 waves/SIMD,
# 14 waves of pixels per SIMD): batches of 2 samples (fb2: 90 VGPRs, 5 waves), + launch bounds
# for 6 / 8 waves (fw6b2: 80 VGPRs, 16 B scratch; fw8b2: 64 VGPRs, 108 B scratch), against in-tree
# build first (CPU): python -m acceleratedvolrenderer_amd.build fb2 -DAVR_FILM_BATCH=2 (fw6b2 / fw8b2:
#   also -DAVR_FILM_WAVES=6 / 8)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
A="--pmc off --tune-walk off --nanovdb-leg 0"
bash tools/gpu_ab.sh "base1||$A" "fb2a|AVR_LIB=variants/fb2/libavr_hip.so|$A" "fw6a|AVR_LIB=variants/fw6b2/libavr_hip.so|$A" "fw8a|AVR_LIB=variants/fw8b2/libavr_hip.so|$A" \
                     "base2||$A" "fb2b|AVR_LIB=variants/fb2/libavr_hip.so|$A" "fw6b|AVR_LIB=variants/fw6b2/libavr_hip.so|$A" "fw8b|AVR_LIB=variants/fw8b2/libavr_hip.so|$A"

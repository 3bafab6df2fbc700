#!/bin/bash
# round-5 pass r: where the camera stage's 2.47 ms go after the pdfs moved to k_film — measurement
# builds (replay broken, same work otherwise): AVR_CAM_EXPERIMENT=1 wavelengths without
# transcendentals, =2 no sampler work, =3 no filter-table sampling; camera ms against in-tree
# build first (CPU): python -m acceleratedvolrenderer_amd.build camx1 -DAVR_CAM_EXPERIMENT=1 (camx2, camx3 likewise)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
A="--pmc off --tune-walk off --nanovdb-leg 0"
bash tools/gpu_ab.sh "base1||$A" "x1a|AVR_LIB=variants/camx1/libavr_hip.so|$A" "x2a|AVR_LIB=variants/camx2/libavr_hip.so|$A" "x3a|AVR_LIB=variants/camx3/libavr_hip.so|$A" \
                     "base2||$A" "x1b|AVR_LIB=variants/camx1/libavr_hip.so|$A" "x2b|AVR_LIB=variants/camx2/libavr_hip.so|$A" "x3b|AVR_LIB=variants/camx3/libavr_hip.so|$A"

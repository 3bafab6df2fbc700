#!/bin/bash
# round-5 pass w: pixel orders more compact than scanline rows for a wave's 64 camera rays
# (bench --pixel-order tile4 / tile8 / tile16 / morton via avr_set_pixel_order; results unchanged)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
A="--pmc off --tune-walk off --nanovdb-leg 0"
bash tools/gpu_ab.sh "base1||$A" "t8a||$A --pixel-order tile8" "t4a||$A --pixel-order tile4" "t16a||$A --pixel-order tile16" "mo_a||$A --pixel-order morton" \
                     "base2||$A" "t8b||$A --pixel-order tile8" "t4b||$A --pixel-order tile4" "t16b||$A --pixel-order tile16" "mo_b||$A --pixel-order morton"

#!/bin/bash
# round-5 pass v: the drain — scanline pixel order with the least-majorant pixels last (bench
# --pixel-order tail, integrator.tail_order), so each XCD's work queue ends on the cheapest
# paths; against the default scanline order, same library
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
A="--pmc off --tune-walk off --nanovdb-leg 0"
bash tools/gpu_ab.sh "base1||$A" "t05a||$A --pixel-order tail --tail-frac 0.05" "t15a||$A --pixel-order tail --tail-frac 0.15" \
                     "base2||$A" "t05b||$A --pixel-order tail --tail-frac 0.05" "t15b||$A --pixel-order tail --tail-frac 0.15"

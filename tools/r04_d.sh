#!/bin/bash
# round-4 pass D: pass-table size 64 / 96 / 128 at the driver's command
set -o pipefail
cd "$GRAFT_REPO_ROOT"
A="--steps 20 --warmup 2 --pmc off --tune-walk off"
bash tools/gpu_ab.sh "dpt64||$A" "dpt96||$A --zsobol-pass-table 96" "dpt128||$A --zsobol-pass-table 128" "dpt64b||$A" || exit 2

#!/bin/bash
# pass j (NanoVDB majorant L2 vs LDS) then the measurement pass, in one call
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/r05_j.sh || exit 1
R05_PASS=mid bash tools/r05_final.sh

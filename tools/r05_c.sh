#!/bin/bash
# round-5 pass c: -m gpu suite on the current build (light pick in cam1.w), then same-box A/B lines:
# in-tree build vs the block-barrier measurement variant (bsync) vs the light pick in its own array (ulsep)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r05/c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -20 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
A="--pmc off --steps 20 --warmup 2 --nanovdb-leg 0 --tune-walk off"
bash tools/gpu_ab.sh "base1||$A" "bsync1|AVR_LIB=variants/bsync/libavr_hip.so|$A" "ulsep1|AVR_LIB=variants/ulsep/libavr_hip.so|$A" \
  "base2||$A" "bsync2|AVR_LIB=variants/bsync/libavr_hip.so|$A" "ulsep2|AVR_LIB=variants/ulsep/libavr_hip.so|$A" || exit 2
mv gpurun_out/ab_*.json gpurun_out/ab_*.err $O/ 2>/dev/null
true

#!/bin/bash
# round-5 pass q: ZSobol cam3 carrying {h0, h1, morton, hi} (-DAVR_CAM_MORTON=1, variants/cammorton):
# k_paths' refill hashes h0 / h1 instead of four divisions + a Morton encode; parity of the
# variant (replay suite + full-size replays through AVR_LIB), then A/B against in-tree
# build first (CPU): python -m acceleratedvolrenderer_amd.build cammorton -DAVR_CAM_MORTON=1
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r05/q
mkdir -p $O
export TMPDIR=/tmp
AVR_LIB=variants/cammorton/libavr_hip.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_fullsize.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
A="--pmc off --tune-walk off --nanovdb-leg 0"
bash tools/gpu_ab.sh "base1||$A" "cm1|AVR_LIB=variants/cammorton/libavr_hip.so|$A" "base2||$A" "cm2|AVR_LIB=variants/cammorton/libavr_hip.so|$A" \
                     "base3||$A" "cm3|AVR_LIB=variants/cammorton/libavr_hip.so|$A"

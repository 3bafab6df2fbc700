#!/bin/bash
# round-5 pass z (reused for each small change of this kind against variants/prevlib): the's digit permutations from a 24-byte LDS table (one byte read +
# bit-field extract) instead of selecting among three 64-bit words; GPU parity, then A/B against
# the previous build (variants/prevlib)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r05/z
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fullsize.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
A="--pmc off --tune-walk off --nanovdb-leg 0"
bash tools/gpu_ab.sh "prev1|AVR_LIB=variants/prevlib/libavr_hip.so|$A" "new1||$A" "prev2|AVR_LIB=variants/prevlib/libavr_hip.so|$A" "new2||$A" \
                     "prev3|AVR_LIB=variants/prevlib/libavr_hip.so|$A" "new3||$A"

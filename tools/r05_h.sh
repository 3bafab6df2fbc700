#!/bin/bash
# round-5 pass h: -m gpu suite (gray x/x quotients without the division), then same-box A/B against
# the build before it (variants/noovl: round-5 code with k_film on the context stream) and the FastDiv +
# precomputed Gaussian filter weights build on top (variants/fastdiv)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r05/h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
A="--pmc off --steps 20 --warmup 2 --nanovdb-leg 0 --tune-walk off"
F="AVR_LIB=variants/fastdiv/libavr_hip.so"
B="AVR_LIB=variants/noovl/libavr_hip.so"
bash tools/gpu_ab.sh "quot1||$A" "base1|$B|$A" "fdiv1|$F|$A" "quot2||$A" "base2|$B|$A" "fdiv2|$F|$A" || exit 2
mv gpurun_out/ab_*.json gpurun_out/ab_*.err $O/ 2>/dev/null
true

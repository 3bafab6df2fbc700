#!/bin/bash
# round-5 pass f: -m gpu suite with k_film on the film stream (overlap), then same-box A/B lines
# against the single-stream build (variants/noovl, -DAVR_FILM_OVERLAP=0)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r05/f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
A="--pmc off --steps 20 --warmup 2 --nanovdb-leg 0 --tune-walk off"
bash tools/gpu_ab.sh "ovl1||$A" "noovl1|AVR_LIB=variants/noovl/libavr_hip.so|$A" "ovl2||$A" "noovl2|AVR_LIB=variants/noovl/libavr_hip.so|$A" || exit 2
mv gpurun_out/ab_*.json gpurun_out/ab_*.err $O/ 2>/dev/null
true

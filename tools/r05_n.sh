#!/bin/bash
# round-5 pass n: phase requests pooled across a block's waves (-DAVR_POOL_PHASE=1, variants
# pool32 / pool16 = AVR_POOL_MIN): replay parity of the variant (the GPU parity suite and the
# driver-configuration full-size replay through AVR_LIB), then A/B bench lines against in-tree
# build first (CPU): python -m acceleratedvolrenderer_amd.build pool32 -DAVR_POOL_PHASE=1 -DAVR_POOL_MIN=32 (pool16: 16;
#   poolboth32: also -DAVR_POOL_NEE=1)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r05/n
mkdir -p $O
export TMPDIR=/tmp
AVR_LIB=variants/pool32/libavr_hip.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py "tests/test_gpu_fullsize.py::test_fullsize_replay_at_the_driver_headline_configuration" \
  "tests/test_gpu_fullsize.py::test_fullsize_nanovdb_replay_at_the_driver_configuration" > $O/pool32_tests.log 2>&1 || { tail -30 $O/pool32_tests.log; exit 1; }
tail -3 $O/pool32_tests.log
AVR_LIB=variants/poolboth32/libavr_hip.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py "tests/test_gpu_fullsize.py::test_fullsize_replay_at_the_driver_headline_configuration" > $O/poolboth32_tests.log 2>&1 || { tail -30 $O/poolboth32_tests.log; exit 1; }
tail -3 $O/poolboth32_tests.log
A="--pmc off --tune-walk off --nanovdb-leg 0"
bash tools/gpu_ab.sh "base1||$A" "pool32a|AVR_LIB=variants/pool32/libavr_hip.so|$A" "pool16a|AVR_LIB=variants/pool16/libavr_hip.so|$A" "both32a|AVR_LIB=variants/poolboth32/libavr_hip.so|$A" \
                     "base2||$A" "pool32b|AVR_LIB=variants/pool32/libavr_hip.so|$A" "pool16b|AVR_LIB=variants/pool16/libavr_hip.so|$A" "both32b|AVR_LIB=variants/poolboth32/libavr_hip.so|$A"

#!/bin/bash
# round-5 pass o: the ZSobol pass table built one thread per pair of dimensions (16-B loads and
# stores, multiply-shift index splits) and the wavelength pdfs evaluated by k_film instead of
# carried in cam4 (AVR_FILM_PDF): GPU parity (replay suite incl. the pass-table identity tests
# and the per-sample L / lambda / pdf comparisons) and the bench A/B against the previous build
# (variants/prevlib: a copy of the in-tree library before both changes) and the pass-table change
# alone (variants/ptonly: -DAVR_FILM_PDF=0)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r05/o
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fullsize.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
A="--pmc off --tune-walk off --nanovdb-leg 0"
bash tools/gpu_ab.sh "prev1|AVR_LIB=variants/prevlib/libavr_hip.so|$A" "pt1|AVR_LIB=variants/ptonly/libavr_hip.so|$A" "new1||$A" \
                     "prev2|AVR_LIB=variants/prevlib/libavr_hip.so|$A" "pt2|AVR_LIB=variants/ptonly/libavr_hip.so|$A" "new2||$A"

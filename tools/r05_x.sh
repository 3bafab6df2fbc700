#!/bin/bash
# round-5 pass x: XCD bands — the pass's record ids band-major (AVR_XCD_BANDS=1), so each XCD's
# work range of k_paths is 1/8 of the image's rows for all 64 sample indices instead of 8 sample
# indices of every pixel; same library, against the default layout
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r05/x
timeout -k 10 200 python tools/band_check.py gpurun_out/r05/x/film_default.npy && \
AVR_XCD_BANDS=1 timeout -k 10 200 python tools/band_check.py gpurun_out/r05/x/film_bands.npy || exit 1
cmp gpurun_out/r05/x/film_default.npy gpurun_out/r05/x/film_bands.npy && echo "films bit-identical" || { echo "films DIFFER"; exit 2; }
A="--pmc off --tune-walk off --nanovdb-leg 0"
bash tools/gpu_ab.sh "base1||$A" "band1|AVR_XCD_BANDS=1|$A" "base2||$A" "band2|AVR_XCD_BANDS=1|$A" "base3||$A" "band3|AVR_XCD_BANDS=1|$A"

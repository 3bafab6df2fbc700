#!/bin/bash
# round-5 pass y: XCD-grouped chunks — each XCD's work range laid out 64 pixels x its 8 sample
# indices at a time (AVR_PIXEL_CHUNKS=1), so an XCD's waves trace the same pixels' samples
# together; film bit-identity check, then A/B against the default layout (same library)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r05/y
timeout -k 10 200 python tools/band_check.py gpurun_out/r05/y/film_default.npy && \
AVR_PIXEL_CHUNKS=1 timeout -k 10 200 python tools/band_check.py gpurun_out/r05/y/film_chunks.npy || exit 1
cmp gpurun_out/r05/y/film_default.npy gpurun_out/r05/y/film_chunks.npy && echo "films bit-identical" || { echo "films DIFFER"; exit 2; }
A="--pmc off --tune-walk off --nanovdb-leg 0"
bash tools/gpu_ab.sh "base1||$A" "ch1|AVR_PIXEL_CHUNKS=1|$A" "base2||$A" "ch2|AVR_PIXEL_CHUNKS=1|$A" "base3||$A" "ch3|AVR_PIXEL_CHUNKS=1|$A"

#!/bin/bash
# round-5 end: k_paths section profiles (variants/prof, -DAVR_PROFILE_SECTIONS) of the final code,
# grid and NanoVDB
# build first (CPU): python tools/section_profile.py --build
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r05/sec
timeout -k 10 300 python tools/section_profile.py > gpurun_out/r05/sec/grid.json 2> gpurun_out/r05/sec/grid.err || { tail -5 gpurun_out/r05/sec/grid.err; exit 1; }
timeout -k 10 300 python tools/section_profile.py --medium nanovdb > gpurun_out/r05/sec/nanovdb.json 2> gpurun_out/r05/sec/nanovdb.err || { tail -5 gpurun_out/r05/sec/nanovdb.err; exit 2; }
cat gpurun_out/r05/sec/grid.json gpurun_out/r05/sec/nanovdb.json

#!/bin/bash
# round-5 pass m: how the phase handler's cycles split between its cooperative ZSobol draws and
# the per-lane rest (section profiles prof / profsplit), and an upper bound for cheapening the
# per-lane rest (-DAVR_MEASURE_CHEAP_PHASE: hardware transcendentals + multiply-xor seeds)
# build first (CPU): python tools/section_profile.py --build; python tools/section_profile.py --build --variant profsplit
#   --define=-DAVR_SEC_SPLIT_PHASE; python -m acceleratedvolrenderer_amd.build cheapphase -DAVR_MEASURE_CHEAP_PHASE
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r05/m
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python tools/section_profile.py --variant prof > $O/sec_prof.json 2> $O/sec_prof.err || { tail -5 $O/sec_prof.err; exit 1; }
timeout -k 10 300 python tools/section_profile.py --variant profsplit > $O/sec_split.json 2> $O/sec_split.err || { tail -5 $O/sec_split.err; exit 2; }
cat $O/sec_prof.json $O/sec_split.json
A="--pmc off --tune-walk off --nanovdb-leg 0"
bash tools/gpu_ab.sh "base1||$A" "cphase1|AVR_LIB=variants/cheapphase/libavr_hip.so|$A" "base2||$A" "cphase2|AVR_LIB=variants/cheapphase/libavr_hip.so|$A"

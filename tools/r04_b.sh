#!/bin/bash
# round-4 pass B: -m gpu suite, A/B of the 32-bit pass-table kernel, rocprofv3 kernel stats
# (CSV) of the driver's command, section profiles (grid, NanoVDB) at the bench configuration
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04/b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
A="--steps 20 --warmup 2 --pmc off --tune-walk off"
bash tools/gpu_ab.sh "bc8f|AVR_LIB=variants/c8f/libavr_hip.so|$A" "bcur||$A" || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 2 --pmc off --no-cpu-baseline --fast-leg 0 --tune-walk off > $O/bench_prof.json 2> $O/bench_prof.err || { tail -10 $O/bench_prof.err; exit 3; }
timeout -k 10 300 python tools/section_profile.py --steps 3 > $O/sections_grid.json 2> $O/sections_grid.err || { tail -10 $O/sections_grid.err; exit 4; }
cat $O/sections_grid.json
timeout -k 10 400 python tools/section_profile.py --steps 3 --medium nanovdb > $O/sections_vdb.json 2> $O/sections_vdb.err || { tail -10 $O/sections_vdb.err; exit 5; }
cat $O/sections_vdb.json
# camera-stage decomposition (measurement-only variants; replay broken by design)
bash tools/gpu_ab.sh "camx1|AVR_LIB=variants/camx1/libavr_hip.so|$A" "camx2|AVR_LIB=variants/camx2/libavr_hip.so|$A" || exit 6
timeout -k 10 600 python bench.py --steps 20 --warmup 2 --fast-leg 0 --no-cpu-baseline > $O/bench_pmc.json 2> $O/bench_pmc.err || { tail -10 $O/bench_pmc.err; exit 7; }

#!/bin/bash
# round-4 full pass on the in-tree build: -m gpu suite, smoke, the driver's bench command (PMC
# child passes + CPU baseline), its rocprofv3 kernel stats, and NanoVDB lines (round-3 library,
# 3-wave build and the default)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04/full
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -10 $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py --steps 20 --warmup 2 > $O/bench_line.json 2> $O/bench_line.err || { tail -10 $O/bench_line.err; exit 3; }
cat $O/bench_line.json | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 2 --pmc off --no-cpu-baseline --fast-leg 0 --tune-walk off > $O/bench_prof.json 2> $O/bench_prof.err || { tail -10 $O/bench_prof.err; exit 4; }
A="--steps 20 --warmup 2 --pmc off"
bash tools/gpu_ab.sh "gc8f|AVR_LIB=variants/c8f/libavr_hip.so|$A --tune-walk off" "gcur||$A --tune-walk off" "gcurt||$A" \
  "gcam5l|AVR_LIB=variants/cam5l/libavr_hip.so|$A --tune-walk off" || exit 5
A="--medium nanovdb --steps 20 --warmup 2 --pmc off"
bash tools/gpu_ab.sh "vdbbase|AVR_LIB=variants/base/libavr_hip.so|$A --tune-walk off" "vdbc3|AVR_LIB=variants/c3/libavr_hip.so|$A --tune-walk off" "vdbc8f|AVR_LIB=variants/c8f/libavr_hip.so|$A --tune-walk off" "vdbcur||$A --tune-walk off" "vdbcurt||$A" || exit 6

#!/bin/bash
# round-4 first GPU pass: the -m gpu suite, the driver's bench command, rocprofv3 kernel stats
set -o pipefail
O=gpurun_out/r04
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --steps 20 --warmup 2 > $O/bench_default.json 2> $O/bench_default.err || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 2 --pmc off --no-cpu-baseline --fast-leg 0 > $O/bench_prof.json 2> $O/bench_prof.err || exit 3

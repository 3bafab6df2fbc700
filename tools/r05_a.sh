#!/bin/bash
# round-5 first pass: the -m gpu suite with printed replay counts (-s), then the driver's bench
# command (NanoVDB leg, PMC child passes, CPU baseline)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r05/a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
tail -5 $O/gpu_tests.log
grep -E "FAILED|ERROR|Timeout" $O/gpu_tests.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_line.json 2> $O/bench_line.err || { tail -10 $O/bench_line.err; exit 3; }
cut -c1-400 $O/bench_line.json

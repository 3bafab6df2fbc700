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
timeout -k 10 300 python tools/walk_sweep.py --medium grid --ddas 0,16,32 --exits 0,4,8,12,16,24 --steps 4 --rounds 2 > $O/sweep_grid.json 2> $O/sweep_grid.err || { tail -5 $O/sweep_grid.err; exit 4; }
timeout -k 10 400 python tools/walk_sweep.py --medium nanovdb --ddas 0,48 --exits 0,4,8,12,16 --steps 4 --rounds 2 > $O/sweep_vdb.json 2> $O/sweep_vdb.err || { tail -5 $O/sweep_vdb.err; exit 5; }
cut -c1-1500 $O/sweep_grid.json; cut -c1-800 $O/sweep_vdb.json

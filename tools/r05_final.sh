#!/bin/bash
# round-5 final pass on the in-tree build: -m gpu suite, smoke, the driver's bench command (PMC
# child passes, CPU baseline, NanoVDB leg) and its rocprofv3 kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r05/${R05_PASS:-final}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -10 $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_line.json 2> $O/bench_line.err || { tail -10 $O/bench_line.err; exit 3; }
cut -c1-300 $O/bench_line.json
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --pmc off --no-cpu-baseline --fast-leg 0 --tune-walk off > $O/bench_prof.json 2> $O/bench_prof.err || { tail -10 $O/bench_prof.err; exit 4; }
echo "kernel stats done"

#!/bin/bash
# round-5 measurement pass: the driver's bench command (PMC child passes, CPU baseline, NanoVDB
# leg), its rocprofv3 kernel stats, and the section profiles (grid, NanoVDB) at the current build
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r05/${R05_PASS:-g}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_line.json 2> $O/bench_line.err || { tail -10 $O/bench_line.err; exit 1; }
cut -c1-300 $O/bench_line.json
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --pmc off --no-cpu-baseline --fast-leg 0 > $O/bench_prof.json 2> $O/bench_prof.err || { tail -10 $O/bench_prof.err; exit 2; }
echo "kernel stats done"
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/section_profile.py --medium grid --steps 3 > $O/section_grid.json 2> $O/section_grid.err || { tail -5 $O/section_grid.err; exit 3; }
timeout -k 10 300 python tools/section_profile.py --medium nanovdb --steps 3 > $O/section_vdb.json 2> $O/section_vdb.err || { tail -5 $O/section_vdb.err; exit 4; }
cat $O/section_grid.json $O/section_vdb.json

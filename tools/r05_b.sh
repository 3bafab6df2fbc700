#!/bin/bash
# round-5 probes: walk occupancy, zero-majorant steps and distinct gather lines per collision
# round (variants/probe, -DAVR_PROBE_STATS) on the grid and NanoVDB S-cloud
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r05/b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python tools/probe_stats.py --medium grid --steps 3 > $O/probe_grid.json 2> $O/probe_grid.err || { tail -5 $O/probe_grid.err; exit 1; }
cat $O/probe_grid.json
timeout -k 10 300 python tools/probe_stats.py --medium nanovdb --steps 3 > $O/probe_vdb.json 2> $O/probe_vdb.err || { tail -5 $O/probe_vdb.err; exit 2; }
cat $O/probe_vdb.json

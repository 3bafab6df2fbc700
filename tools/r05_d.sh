#!/bin/bash
# round-5 pass d: k_paths schedule re-sweep at the current build (NanoVDB and grid)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r05/d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python tools/walk_sweep.py --medium nanovdb --refills 8,12,16,20 --ddas 20,28,36 --steps 3 --rounds 2 > $O/sweep_vdb.json 2> $O/sweep_vdb.err || { tail -5 $O/sweep_vdb.err; exit 1; }
timeout -k 10 400 python tools/walk_sweep.py --medium grid --refills 24,28,32,36 --ddas 8,10,12 --steps 3 --rounds 2 > $O/sweep_grid.json 2> $O/sweep_grid.err || { tail -5 $O/sweep_grid.err; exit 2; }
python - <<'PY'
import json
for f in ("sweep_vdb", "sweep_grid"):
    d = json.load(open(f"gpurun_out/r05/d/{f}.json"))
    for r in sorted(d["rows"], key=lambda r: -r["Msamples_s"])[:6]:
        print(f, r)
PY

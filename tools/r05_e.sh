#!/bin/bash
# round-5 pass e: pass-size (drain) measurement — 64 vs 128 sample indices per k_paths launch over
# the same samples — and the NanoVDB leg at the new default refill (16)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r05/e
mkdir -p $O
export TMPDIR=/tmp
A="--pmc off --no-cpu-baseline --fast-leg 0 --tune-walk off"
timeout -k 10 400 python bench.py $A --steps 20 --warmup 2 --pixelsamples 16384 > $O/p64.json 2> $O/p64.err || { tail -5 $O/p64.err; exit 1; }
timeout -k 10 400 python bench.py $A --steps 10 --warmup 1 --spp-per-step 128 --max-paths 134217728 --pixelsamples 16384 --nanovdb-leg 0 > $O/p128.json 2> $O/p128.err || { tail -5 $O/p128.err; exit 2; }
timeout -k 10 400 python bench.py $A --steps 40 --warmup 4 --spp-per-step 32 --pixelsamples 16384 --nanovdb-leg 0 > $O/p32.json 2> $O/p32.err || { tail -5 $O/p32.err; exit 3; }
python - <<'PY'
import json
for t in ("p64", "p128", "p32"):
    d = json.loads(open(f"gpurun_out/r05/e/{t}.json").read().strip().split("\n")[-1])
    de, r = d["detail"], d["roofline"]
    n = d["steps"]
    print(t, round(d["value"], 1), "step", d["ms_per_step"], "k_paths", round(r["avg_launch_ms"], 3), "camera", round(de["ms_camera"] / n, 3),
          "film", round(de["ms_film"] / n, 3), "simd", round(d["simd_utilisation"], 4), "vdb", (d.get("nanovdb") or {}).get("value"))
PY

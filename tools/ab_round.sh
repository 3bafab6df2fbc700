#!/bin/bash
# One A/B session (through gpurun): optional replay-parity check of variant libraries, then
# alternating bench lines.  usage: bash tools/ab_round.sh <outdir> "<variants to parity-check>" <tag|env|args> ...
# e.g. bash tools/ab_round.sh r06/ab1 "wl" "base||$A" "wl|AVR_LIB=variants/wl/libavr_hip.so|$A"
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; shift
mkdir -p $O; export TMPDIR=/tmp
for v in $1; do
  AVR_LIB=variants/$v/libavr_hip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_$v.log 2>&1 || { echo "parity $v failed"; tail -20 $O/tests_$v.log; exit 1; }
  echo "parity $v: $(tail -1 $O/tests_$v.log)"
done
shift
for spec in "$@"; do
  IFS='|' read -r tag envs args <<< "$spec"
  env $envs timeout -k 10 400 python bench.py --no-cpu-baseline $args > $O/ab_$tag.json 2> $O/ab_$tag.err || { echo "$tag failed"; tail -5 $O/ab_$tag.err; exit 2; }
  python - "$O" "$tag" <<'PY'
import json, sys
o, t = sys.argv[1], sys.argv[2]
d = json.load(open(f"{o}/ab_{t}.json"))
de, r, n = d["detail"], d["roofline"], d["steps"]
v = d.get("nanovdb") or {}
f = d.get("fast_mode") or {}
print(f"{t}: {d['value']:.1f} Msamples/s, step {d['ms_per_step']:.3f} ms, k_paths {r['avg_launch_ms']:.3f}, camera {de['ms_camera'] / n:.3f}, "
      f"film {de['ms_film'] / n:.3f}, nanovdb {v.get('value')}, fast {f.get('value')}")
PY
done

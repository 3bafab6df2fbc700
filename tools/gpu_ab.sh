#!/bin/bash
# A/B bench lines on one GPU box: each argument is "<tag>|<env assignments>|<bench args>"; every
# line runs bench.py once under its own time limit, and the script stops at the first failure.
# usage (through gpurun): bash tools/gpu_ab.sh "base||--pmc off" "cam6|AVR_LIB=variants/cam6/libavr_hip.so|--pmc off"
mkdir -p gpurun_out
for spec in "$@"; do
  IFS='|' read -r tag envs args <<< "$spec"
  env $envs timeout -k 10 400 python bench.py --no-cpu-baseline --fast-leg 0 $args > gpurun_out/ab_$tag.json 2> gpurun_out/ab_$tag.err || { echo "$tag failed"; tail -5 gpurun_out/ab_$tag.err; exit 1; }
  python - "$tag" <<'PY'
import json, sys
t = sys.argv[1]
d = json.load(open(f"gpurun_out/ab_{t}.json"))
de, r = d["detail"], d["roofline"]
n = d["steps"]
print(f"{t}: {d['value']:.1f} Msamples/s, step {d['ms_per_step']:.3f} ms, k_paths {r['avg_launch_ms']:.3f}, "
      f"camera {de['ms_camera'] / n:.3f}, film {de['ms_film'] / n:.3f}")
PY
done

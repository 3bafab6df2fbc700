#!/bin/bash
# round-5 pass aa: the NanoVDB leg before / after the LDS permutation table in k_paths'
# cooperative draws (variants/prevlib: the commit before it, built from a git worktree)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for k in 1 2 3; do
  for v in prev new; do
    if [ $v = prev ]; then E="AVR_LIB=variants/prevlib/libavr_hip.so"; else E=""; fi
    env $E timeout -k 10 400 python bench.py --no-cpu-baseline --fast-leg 0 --pmc off --tune-walk off --nanovdb-leg 1 --nanovdb-steps 8 > gpurun_out/aa_${v}$k.json 2> gpurun_out/aa_${v}$k.err || { tail -5 gpurun_out/aa_${v}$k.err; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/aa_${v}$k.json')); n=d['nanovdb']
print('${v}$k', round(d['value'],1), 'k_paths', round(d['roofline']['avg_launch_ms'],3), 'vdb', round(n['value'],1), 'vdb k_paths', round(n['roofline']['avg_launch_ms'],3))"
  done
done

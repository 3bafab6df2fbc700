#!/bin/bash
# GPU pass al: majorant prefetch in the k_paths DDA — full gpu suite, grid + nanovdb benches.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/al
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || { echo "stop: $name rc=$rc"; tail -40 $O/$name.log; exit $rc; }
}
step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
step grid 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline
step vdb512p 400 python bench.py --res 512 --medium nanovdb --steps 6 --warmup 2 --no-cpu-baseline
exit 0

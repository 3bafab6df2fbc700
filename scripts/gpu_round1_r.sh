#!/bin/bash
# GPU pass r: temperature (blackbody) emission + full parity suite.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || { echo "stop: $name rc=$rc"; tail -30 $O/$name.log; exit $rc; }
}
step gpu_tests 900 python -m pytest tests -m gpu -x -q -s -rA
step zs_gauss 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline
exit 0

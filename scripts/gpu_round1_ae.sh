#!/bin/bash
# GPU pass ae: FLIP on the device, then the suite.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ae
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || { echo "stop: $name rc=$rc"; tail -30 $O/$name.log; exit $rc; }
}
step flip_tests 300 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -s -rA -k flip
step gpu_tests 900 python -m pytest tests -m gpu -x -q -s -rA
exit 0

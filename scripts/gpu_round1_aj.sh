#!/bin/bash
# GPU pass aj: lighting-graph parity tests.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/aj
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || { echo "stop: $name rc=$rc"; tail -40 $O/$name.log; exit $rc; }
}
step graph 400 python -u -m pytest tests/test_graph.py -m gpu -x -v -s --timeout 120 --timeout-method thread
exit 0

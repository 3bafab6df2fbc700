#!/bin/bash
# GPU pass ah (re-entry check): full -m gpu suite, smoke(), default bench.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ah
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || { echo "stop: $name rc=$rc"; tail -30 $O/$name.log; exit $rc; }
}
step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 400 python bench.py
exit 0

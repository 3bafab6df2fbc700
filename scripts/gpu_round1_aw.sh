#!/bin/bash
# GPU pass aw: full gpu suite + smoke + default bench (with CPU baseline) + NanoVDB bench.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/aw
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || { echo "stop: $name rc=$rc"; tail -30 $O/$name.log; exit $rc; }
}
step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 500 python bench.py
step bench_vdb 500 python bench.py --res 512 --medium nanovdb --cpu-seconds 10
exit 0

#!/bin/bash
# GPU pass ad: bench with a run long enough to wrap the ZSobol index range.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ad
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || { echo "stop: $name rc=$rc"; tail -30 $O/$name.log; exit $rc; }
}
step bench_long 400 python bench.py --steps 100 --warmup 2 --no-cpu-baseline
exit 0

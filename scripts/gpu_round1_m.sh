#!/bin/bash
# GPU pass m: refill-threshold x walk-budget sweep.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/m
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || { echo "stop: $name rc=$rc"; tail -20 $O/$name.log; exit $rc; }
}
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline"
for r in 16 24 32 40 48; do
  for b in 12 24; do
    step r${r}_b${b} 300 $B --refill-min $r --dda-budget $b
  done
done
step r32_b8 300 $B --refill-min 32 --dda-budget 8
step r32_b16 300 $B --refill-min 32 --dda-budget 16
exit 0

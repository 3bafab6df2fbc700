#!/bin/bash
# GPU pass y: experiment — cost of the ZSobol sample digits (variants skip the top 2 / all 4).
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/y
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || { echo "stop: $name rc=$rc"; tail -30 $O/$name.log; exit $rc; }
}
step base 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline
AVR_LIB=$R/variants/libavr_skip2.so step skip2 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline
AVR_LIB=$R/variants/libavr_skip4.so step skip4 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline
exit 0

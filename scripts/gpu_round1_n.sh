#!/bin/bash
# GPU pass n: shared segment-start block (one SampleT_maj prologue per batch), refill 32.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/n
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || { echo "stop: $name rc=$rc"; tail -20 $O/$name.log; exit $rc; }
}
step gpu_tests 900 python -m pytest tests -m gpu -x -q -s -rA
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline"
step ab_base 300 $B
step ab_prev 300 env AVR_LIB=$R/variants/libavr_prev.so $B --refill-min 32
step ab_r24 300 $B --refill-min 24
step ab_r40 300 $B --refill-min 40
step ab_b8 300 $B --dda-budget 8
step ab_base2 300 $B
exit 0

#!/bin/bash
# GPU pass h: DDA walk budget sweep (tests first, stop on any failure).
set -u
mkdir -p gpurun_out/h
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -m pytest tests -m gpu -x -q -s -rA > gpurun_out/h/gpu_tests.log 2>&1; rc=$?
echo "pytest rc=$rc"
[ $rc -eq 0 ] || { echo "stop: pytest rc=$rc"; exit $rc; }
B="python bench.py --steps 3 --warmup 1 --spp-per-step 16 --no-cpu-baseline"
run() {
  local name=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/h/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || { echo "stop: $name rc=$rc"; exit $rc; }
}
run b1 AVR_X=0 $B --dda-budget 1
run b2 AVR_X=0 $B --dda-budget 2
run b4 AVR_X=0 $B --dda-budget 4
run b8 AVR_X=0 $B --dda-budget 8
run binf AVR_X=0 $B --dda-budget 1000
run b2r32 AVR_X=0 $B --dda-budget 2 --refill-min 32
run b4r8 AVR_X=0 $B --dda-budget 4 --refill-min 8
exit 0

#!/bin/bash
# GPU pass g: fat-layout fix — parity tests first (stop on any failure), then A/B benches.
set -u
mkdir -p gpurun_out/g
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -m pytest tests -m gpu -x -q -s -rA > gpurun_out/g/gpu_tests.log 2>&1; rc=$?
echo "pytest rc=$rc"
[ $rc -eq 0 ] || { echo "stop: pytest rc=$rc"; exit $rc; }
B="python bench.py --steps 3 --warmup 1 --spp-per-step 16 --no-cpu-baseline"
run() {
  local name=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/g/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || { echo "stop: $name rc=$rc"; exit $rc; }
}
run fat AVR_X=0 $B
run linear AVR_X=0 $B --grid-layout linear
run w2fat AVR_LIB=$PWD/variants/libavr_w2.so $B
run w4fat AVR_LIB=$PWD/variants/libavr_w4.so $B
exit 0

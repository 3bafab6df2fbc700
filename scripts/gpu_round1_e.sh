#!/bin/bash
# GPU pass e: batched-event k_paths — parity tests, occupancy variants, refill/batch threshold sweep.
set -u
mkdir -p gpurun_out/e
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -m pytest tests -m gpu -q -s -rA > gpurun_out/e/gpu_tests.log 2>&1; rc=$?
echo "pytest rc=$rc"
case $rc in 0|1) ;; *) echo "stop: pytest rc=$rc"; exit $rc;; esac
B="python bench.py --steps 3 --warmup 1 --spp-per-step 16 --no-cpu-baseline"
run() {
  local name=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/e/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"
  case $rc in 0|1) return 0;; *) echo "stop: $name rc=$rc"; exit $rc;; esac
}
run base AVR_X=0 $B
run b8 AVR_X=0 $B --refill-min 8
run b32 AVR_X=0 $B --refill-min 32
run b48 AVR_X=0 $B --refill-min 48
run w2 AVR_LIB=$PWD/variants/libavr_w2.so $B
run w4 AVR_LIB=$PWD/variants/libavr_w4.so $B
run w4b32 AVR_LIB=$PWD/variants/libavr_w4.so $B --refill-min 32
exit 0

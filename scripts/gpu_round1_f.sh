#!/bin/bash
# GPU pass f: gray/fast-reject DDA loop + fat grid layout — parity tests, layout and occupancy A/B.
set -u
mkdir -p gpurun_out/f
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -m pytest tests -m gpu -q -s -rA > gpurun_out/f/gpu_tests.log 2>&1; rc=$?
echo "pytest rc=$rc"
case $rc in 0|1) ;; *) echo "stop: pytest rc=$rc"; exit $rc;; esac
B="python bench.py --steps 3 --warmup 1 --spp-per-step 16 --no-cpu-baseline"
run() {
  local name=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/f/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"
  case $rc in 0|1) return 0;; *) echo "stop: $name rc=$rc"; exit $rc;; esac
}
run fat AVR_X=0 $B
run linear AVR_X=0 $B --grid-layout linear
run w2fat AVR_LIB=$PWD/variants/libavr_w2.so $B
run w4fat AVR_LIB=$PWD/variants/libavr_w4.so $B
run fat_spp32 AVR_X=0 python bench.py --steps 2 --warmup 1 --spp-per-step 32 --no-cpu-baseline
exit 0

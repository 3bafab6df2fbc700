#!/bin/bash
# GPU pass ai: 4 waves/SIMD k_paths (128 VGPRs + scratch) vs default 3 waves.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ai
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || { echo "stop: $name rc=$rc"; tail -30 $O/$name.log; exit $rc; }
}
step base 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline
AVR_LIB=$R/variants/libavr_w4.so step w4 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline
exit 0

#!/bin/bash
# GPU pass ag: 8x8 tiled pixel hand-out in k_paths — replay tests, bench A/B against scanline order.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ag
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || { echo "stop: $name rc=$rc"; tail -30 $O/$name.log; exit $rc; }
}
step tests 600 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -s -rA -k "persistent or uniform_box or samplers"
step tiled 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline
AVR_LIB=$R/variants/libavr_linear.so step linear 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline
step tiled_ind 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --sampler independent --filter box
AVR_LIB=$R/variants/libavr_linear.so step linear_ind 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --sampler independent --filter box
exit 0

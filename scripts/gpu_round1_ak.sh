#!/bin/bash
# GPU pass ak: k_paths NanoVDB specialisation — parity (both kernels), grid regression bench,
# NanoVDB S-cloud bench persistent vs wavefront.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ak
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || { echo "stop: $name rc=$rc"; tail -40 $O/$name.log; exit $rc; }
}
step vdbtests 400 python -u -m pytest tests/test_gpu_parity.py -k "nanovdb" -x -v -s --timeout 120 --timeout-method thread
step grid 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline
step vdb512p 400 python bench.py --res 512 --medium nanovdb --steps 6 --warmup 2 --no-cpu-baseline
step vdb512w 400 python bench.py --res 512 --medium nanovdb --kernel wavefront --steps 4 --warmup 1 --no-cpu-baseline
step grid512 300 python bench.py --res 512 --steps 6 --warmup 2 --no-cpu-baseline
exit 0

#!/bin/bash
# GPU pass am: SpectralFilm — full gpu suite, default bench regression.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/am
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || { echo "stop: $name rc=$rc"; tail -40 $O/$name.log; exit $rc; }
}
step spectral 300 python -u -m pytest tests/test_gpu_parity.py -k spectral -x -v -s --timeout 120 --timeout-method thread
step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
step grid 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline
exit 0

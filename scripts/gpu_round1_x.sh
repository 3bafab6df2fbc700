#!/bin/bash
# GPU pass x: ZSobol seed-hash table — identity tests, then bench.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/x
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || { echo "stop: $name rc=$rc"; tail -30 $O/$name.log; exit $rc; }
}
step zs_tests 300 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -s -rA -k "zsobol or sampler"
step bench_table 400 python bench.py --steps 6 --warmup 2 --no-cpu-baseline
exit 0

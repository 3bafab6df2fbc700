#!/bin/bash
# GPU pass ab: ZSobol table dimension-major by linear pixel — tests, bench.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || { echo "stop: $name rc=$rc"; tail -30 $O/$name.log; exit $rc; }
}
step zs_tests 300 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -s -rA -k "zsobol or sampler"
step bench 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline
step bench_notable 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --zsobol-table 0
exit 0

#!/bin/bash
# GPU pass q: Integrator::Tr, homogeneous/cloud media, 32-bit ZSobol index — tests + bench.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/q
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || { echo "stop: $name rc=$rc"; tail -30 $O/$name.log; exit $rc; }
}
step gpu_tests 900 python -m pytest tests -m gpu -x -q -s -rA
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline"
step zs_gauss 300 $B
step ind_box 300 $B --sampler independent --filter box
exit 0

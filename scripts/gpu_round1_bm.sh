#!/bin/bash
# GPU pass bm (final): suite, smoke, benches, kernel trace + PMC passes.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/bm
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || { echo "stop: $name rc=$rc"; tail -20 $O/$name.log; exit $rc; }
}
step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 500 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 500 python bench.py
step bench_vdb 500 python bench.py --res 512 --medium nanovdb --cpu-seconds 10
cd /tmp && export TMPDIR=/tmp
P="python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline"
step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- $P
step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- $P
step pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- $P
step pmc_sq1 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O/pmc_sq1 -o run -- $P
step pmc_sq2 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_VALU --output-format csv -d $O/pmc_sq2 -o run -- $P
step prof_vdb 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_vdb -o run -- python3 $R/bench.py --res 512 --medium nanovdb --steps 3 --warmup 1 --no-cpu-baseline
exit 0

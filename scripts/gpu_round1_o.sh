#!/bin/bash
# GPU pass o: asynchronous render passes (device PCG advance table, lazy stats), shared
# segment starts; parity, smoke, full bench with CPU baseline, A/B, kernel trace + PMC.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/o
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || { echo "stop: $name rc=$rc"; tail -20 $O/$name.log; exit $rc; }
}
step gpu_tests 900 python -m pytest tests -m gpu -x -q -s -rA
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline"
step ab_base 300 $B
step ab_base2 300 $B
step ab_steps10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline
step bench 400 python bench.py
cd /tmp && export TMPDIR=/tmp
step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline
step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline
step pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline
step pmc_sq1 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O/pmc_sq1 -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline
step pmc_sq2 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_VALU --output-format csv -d $O/pmc_sq2 -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline
exit 0

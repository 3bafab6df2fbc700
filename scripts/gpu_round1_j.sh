#!/bin/bash
# GPU pass j: exact free-flight test hoisted out of the DDA walk, budget 8 default —
# parity tests, A/B (budget, float-libm cost), SQ instruction counters.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/j
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {   # name timeout cmd... ; stops the script on any nonzero status
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || { echo "stop: $name rc=$rc"; tail -20 $O/$name.log; exit $rc; }
}
step gpu_tests 900 python -m pytest tests -m gpu -x -q -s -rA
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline"
step ab_base 300 $B
step ab_b4 300 $B --dda-budget 4
step ab_b12 300 $B --dda-budget 12
step ab_b16 300 $B --dda-budget 16
step ab_fl 300 env AVR_LIB=$R/variants/libavr_fl.so $B
step ab_base2 300 $B
cd /tmp && export TMPDIR=/tmp
P="python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline"
step pmc_sq1 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O/pmc_sq1 -o run -- $P
step pmc_sq2 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_VALU --output-format csv -d $O/pmc_sq2 -o run -- $P
exit 0

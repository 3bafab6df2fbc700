#!/bin/bash
# GPU pass i: gray-specialised k_paths — parity tests (incl. chromatic/emissive), default bench
# with CPU baseline, A/B variants, rocprofv3 kernel stats and HBM PMC passes.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/i
mkdir -p $O
export PYTHONUNBUFFERED=1
step() {   # name timeout cmd... ; stops the script on any nonzero status
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || { echo "stop: $name rc=$rc"; tail -20 $O/$name.log; exit $rc; }
}
step gpu_tests 900 python -m pytest tests -m gpu -x -q -s -rA
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 400 python bench.py
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline"
step ab_base 300 $B
step ab_g4 300 env AVR_LIB=$R/variants/libavr_g4.so $B
step ab_b8 300 $B --dda-budget 8
step ab_b6 300 $B --dda-budget 6
step ab_linear 300 $B --grid-layout linear
step ab_base2 300 $B
step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline
step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline
step pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline
exit 0

#!/bin/bash
# GPU pass d: k_paths tuning experiments (occupancy variants, refill threshold) + PMC counters.
set -u
mkdir -p gpurun_out/d
export PYTHONUNBUFFERED=1
B="python bench.py --steps 3 --warmup 1 --spp-per-step 16 --no-cpu-baseline"
run() { # name, env, args
  local name=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/d/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"
  case $rc in 0|1) return 0;; *) echo "stop: $name rc=$rc"; exit $rc;; esac
}
run base AVR_X=0 $B
run refill1 AVR_X=0 $B --refill-min 1
run refill32 AVR_X=0 $B --refill-min 32
run refill48 AVR_X=0 $B --refill-min 48
run w3 AVR_LIB=$PWD/variants/libavr_w3.so $B
run w4 AVR_LIB=$PWD/variants/libavr_w4.so $B
run wavefront AVR_X=0 $B --kernel wavefront
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
P="python3 $R/bench.py --steps 1 --warmup 1 --spp-per-step 16 --no-cpu-baseline"
for ctr in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_VALU" "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  tag=$(echo $ctr | tr ' ' '_' | cut -c1-40)
  timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d $R/gpurun_out/d/pmc_$tag -o run -- $P > $R/gpurun_out/d/pmc_$tag.log 2>&1; rc=$?
  echo "pmc $tag rc=$rc"
  case $rc in 0|1) ;; *) echo "stop: pmc rc=$rc"; exit $rc;; esac
done
exit 0

#!/bin/bash
# GPU pass b: parity tests, smoke, bench at 16 spp/step, rocprofv3 kernel trace of the bench.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -m pytest tests -m gpu -q -s -rA > gpurun_out/gpu_tests_b.log 2>&1; rc=$?
echo "pytest rc=$rc"
case $rc in 0|1) ;; *) echo "stop: pytest rc=$rc"; exit $rc;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_b.log 2>&1; rc=$?
echo "smoke rc=$rc"
case $rc in 0|1) ;; *) echo "stop: smoke rc=$rc"; exit $rc;; esac
timeout -k 10 600 python bench.py --steps 4 --warmup 1 --spp-per-step 16 --cpu-seconds 15 > gpurun_out/bench_b.log 2>&1; rc=$?
echo "bench rc=$rc"
case $rc in 0|1) ;; *) echo "stop: bench rc=$rc"; exit $rc;; esac
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_b -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --spp-per-step 16 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_b.log 2>&1; rc=$?
echo "rocprof rc=$rc"
exit 0

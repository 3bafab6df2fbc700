#!/bin/bash
# GPU pass c: both kernel organisations — parity tests, smoke, bench (persistent + wavefront), rocprof stats.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -m pytest tests -m gpu -q -s -rA > gpurun_out/gpu_tests_c.log 2>&1; rc=$?
echo "pytest rc=$rc"
case $rc in 0|1) ;; *) echo "stop: pytest rc=$rc"; exit $rc;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_c.log 2>&1; rc=$?
echo "smoke rc=$rc"
case $rc in 0|1) ;; *) echo "stop: smoke rc=$rc"; exit $rc;; esac
timeout -k 10 600 python bench.py --steps 4 --warmup 1 --spp-per-step 16 --cpu-seconds 10 > gpurun_out/bench_c_persistent.log 2>&1; rc=$?
echo "bench persistent rc=$rc"
case $rc in 0|1) ;; *) echo "stop: bench rc=$rc"; exit $rc;; esac
timeout -k 10 600 python bench.py --steps 4 --warmup 1 --spp-per-step 16 --no-cpu-baseline --kernel wavefront > gpurun_out/bench_c_wavefront.log 2>&1; rc=$?
echo "bench wavefront rc=$rc"
case $rc in 0|1) ;; *) echo "stop: bench rc=$rc"; exit $rc;; esac
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_c -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --spp-per-step 16 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_c.log 2>&1; rc=$?
echo "rocprof rc=$rc"
exit 0

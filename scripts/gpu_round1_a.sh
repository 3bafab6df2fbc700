#!/bin/bash
# First GPU pass: parity tests, smoke, small bench. Each GPU step time-limited; stop on crash codes.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
rocm-smi --showproductname > gpurun_out/rocm_smi.txt 2>&1 || true
nproc > gpurun_out/nproc.txt; lscpu > gpurun_out/lscpu.txt 2>&1 || true
timeout -k 10 900 python -m pytest tests -m gpu -q -s -rA > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "pytest rc=$rc"
case $rc in 0|1) ;; *) echo "stop: pytest rc=$rc"; exit $rc;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"
case $rc in 0|1) ;; *) echo "stop: smoke rc=$rc"; exit $rc;; esac
timeout -k 10 600 python bench.py --res 256 --steps 2 --warmup 1 --cpu-seconds 5 > gpurun_out/bench_256.log 2>&1; rc=$?
echo "bench256 rc=$rc"
case $rc in 0|1) ;; *) echo "stop: bench rc=$rc"; exit $rc;; esac
timeout -k 10 900 python bench.py --steps 2 --warmup 1 --cpu-seconds 10 > gpurun_out/bench_1024.log 2>&1; rc=$?
echo "bench1024 rc=$rc"
exit 0

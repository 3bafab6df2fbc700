#!/bin/bash
# A/B at the driver command (--steps 20): the two-level ZSobol pass table (in-tree) vs the
# one-level build (variants/onelevel), at 64 and 96 pass-table dimensions; the pass-table and
# sampler parity tests first, the full GPU suite last
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
A="--steps 20 --warmup 2 --pmc off"
L() { echo "AVR_LIB=variants/$1/libavr_hip.so"; }
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "pass_table or zsobol" > gpurun_out/tests_pt.log 2>&1 || { tail -30 gpurun_out/tests_pt.log; exit 2; }
tail -2 gpurun_out/tests_pt.log
bash tools/gpu_ab.sh "two64||$A" "one64|$(L onelevel)|$A" "two96||$A --zsobol-pass-table 96" "one96|$(L onelevel)|$A --zsobol-pass-table 96" "cam5|$(L cam5)|$A" "two64b||$A" || exit 1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_cur.log 2>&1 || { tail -30 gpurun_out/tests_cur.log; exit 3; }
tail -2 gpurun_out/tests_cur.log

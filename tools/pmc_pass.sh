#!/bin/bash
# Counter passes of the default bench for tools/pmc_summary.py (through gpurun):
#   bash tools/pmc_pass.sh <outdir-under-gpurun_out> [bench args ...]
# One rocprofv3 run per counter group (FETCH_SIZE and WRITE_SIZE apart: TCC block limits),
# each under its own KILL time limit, plus a kernel-trace --stats run and one plain bench
# line. No tracing domains are combined with --pmc. Stops at the first failure.
set -o pipefail
out=$GRAFT_REPO_ROOT/gpurun_out/$1; shift
mkdir -p "$out"
bench=(python3 "$GRAFT_REPO_ROOT/bench.py" --pmc off --no-cpu-baseline --fast-leg 0 "$@")
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 "${bench[@]}" --steps 10 --warmup 3 > "$out/bench.log" 2> "$out/bench.err" || exit $?
echo "bench: $(head -c 300 "$out/bench.log")"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof" -o run -- \
  "${bench[@]}" --steps 4 --warmup 1 > "$out/prof.log" 2>&1 || exit $?
echo "kernel trace done"
pass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$out/$name" -o run -- \
    "${bench[@]}" --steps 2 --warmup 1 > "$out/$name.log" 2>&1 || exit $?
  echo "pass $name done"
}
pass pmc_fetch FETCH_SIZE
pass pmc_write WRITE_SIZE
pass pmc_sq1 SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVES SQ_WAVE_CYCLES
pass pmc_sq2 SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD
pass pmc_tcc TCC_HIT_sum TCC_MISS_sum
exit 0

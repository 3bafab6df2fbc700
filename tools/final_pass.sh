#!/bin/bash
# A round's closing GPU pass on the in-tree build (through gpurun):
#   bash tools/final_pass.sh <outdir-under-gpurun_out> [steps: tests smoke bench stats]
# tests: the whole -m gpu suite; smoke: __graft_entry__.smoke(); bench: the driver's command
# (PMC child passes, CPU baseline, NanoVDB and fast legs); stats: rocprofv3 --kernel-trace
# --stats of the same command without the counter passes. Each step has its own time limit;
# the script stops at the first failure (no retries).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/$1; shift
mkdir -p "$O"
export TMPDIR=/tmp
steps=("$@"); [ ${#steps[@]} -eq 0 ] && steps=(tests smoke bench stats)
for s in "${steps[@]}"; do
  case $s in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > "$O/gpu_tests.log" 2>&1 || { tail -30 "$O/gpu_tests.log"; exit 1; }
      tail -1 "$O/gpu_tests.log" ;;
    smoke)
      timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail -10 "$O/smoke.log"; exit 2; }
      tail -1 "$O/smoke.log" ;;
    bench)
      timeout -k 10 900 python bench.py --steps 20 --warmup 5 > "$O/bench_line.json" 2> "$O/bench_line.err" || { tail -10 "$O/bench_line.err"; exit 3; }
      cut -c1-300 "$O/bench_line.json" ;;
    stats)
      (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- \
        python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --pmc off --no-cpu-baseline --tune-walk off \
        > "$O/bench_prof.json" 2> "$O/bench_prof.err") || { tail -10 "$O/bench_prof.err"; exit 4; }
      echo "kernel stats done" ;;
    *) echo "unknown step $s"; exit 9 ;;
  esac
done

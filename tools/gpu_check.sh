#!/bin/bash
# One GPU-box session: the -m gpu tests, then bench lines. Usage (through gpurun):
#   bash tools/gpu_check.sh <tag> [bench args ...] [-- more bench args ...]
# Every bench invocation after the tests is one "--" separated group; each GPU step has its
# own time limit and the script stops at the first failure (no retries).
tag=$1; shift
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  kargs=(); [ -n "${KEXPR:-}" ] && kargs=(-k "$KEXPR")
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${TESTS:-} \
    "${kargs[@]}" > gpurun_out/${tag}_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${tag}_tests.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || [ $rc -eq 5 ] || exit $rc
fi
i=0; args=()
run_bench() {
  [ ${#args[@]} -eq 0 ] && [ $i -gt 0 ] && return 0
  timeout -k 10 400 python bench.py "${args[@]}" > gpurun_out/${tag}_b$i.json 2> gpurun_out/${tag}_b$i.err || exit $?
  echo "bench $i (${args[*]}): $(head -c 400 gpurun_out/${tag}_b$i.json)"
  i=$((i+1)); args=()
}
if [ $# -gt 0 ]; then
  for a in "$@"; do
    if [ "$a" = "--" ]; then run_bench; elif [ -n "$a" ]; then args+=("$a"); fi
  done
  run_bench
fi
exit ${rc:-0}

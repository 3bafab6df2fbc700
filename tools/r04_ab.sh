#!/bin/bash
# round-4 A/B: bench lines of the in-tree library and variant libraries at the driver's command
# (--steps 20), then the -m gpu suite on the first variant.  usage: bash tools/r04_ab.sh <variant>...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
specs=("base||--steps 20 --warmup 2 --pmc off")
for v in "$@"; do specs+=("$v|AVR_LIB=variants/$v/libavr_hip.so|--steps 20 --warmup 2 --pmc off"); done
bash tools/gpu_ab.sh "${specs[@]}" || exit 1
if [ -n "$1" ]; then
  AVR_LIB=variants/$1/libavr_hip.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_$1.log 2>&1 || { tail -30 gpurun_out/tests_$1.log; exit 2; }
  tail -3 gpurun_out/tests_$1.log
fi

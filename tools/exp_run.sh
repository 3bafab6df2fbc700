set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/f3_tests.log 2>&1 || { tail -30 gpurun_out/f3_tests.log; exit 1; }
tail -1 gpurun_out/f3_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/f3_smoke.log 2>&1 || { tail -20 gpurun_out/f3_smoke.log; exit 1; }
tail -1 gpurun_out/f3_smoke.log
B="--pmc off --no-cpu-baseline --fast-leg 0 --steps 10 --warmup 2"
for a in "" "--scene uniform --res 256 --width 512 --height 512"; do
  timeout -k 10 200 python bench.py $B $a > gpurun_out/f3_b.json 2>gpurun_out/f3_err.log || { tail gpurun_out/f3_err.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/f3_b.json')); print('$a', d['value'], d['roofline']['avg_launch_ms'])"
done

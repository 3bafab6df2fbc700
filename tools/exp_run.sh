set -o pipefail
mkdir -p gpurun_out
B="--pmc off --no-cpu-baseline --fast-leg 0 --steps 10 --warmup 2 --scene uniform --res 256 --width 512 --height 512"
for a in "--dda-budget 12" "--dda-budget 10" "--dda-budget 12" "--dda-budget 10" "--dda-budget 16"; do
  timeout -k 10 200 python bench.py $B $a > gpurun_out/e8_b.json 2>gpurun_out/e8_err.log || { tail gpurun_out/e8_err.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/e8_b.json')); print('$a', d['value'], d['roofline']['avg_launch_ms'])"
done

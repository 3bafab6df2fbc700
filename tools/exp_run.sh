set -o pipefail
mkdir -p gpurun_out
B="--pmc off --no-cpu-baseline --fast-leg 0 --steps 4 --warmup 1 --medium nanovdb"
for a in "--dda-budget 32" "--dda-budget 24" "--dda-budget 40" "--dda-budget 28" "--dda-budget 32"; do
  timeout -k 10 200 python bench.py $B $a > gpurun_out/e10_b.json 2>gpurun_out/e10_err.log || { tail gpurun_out/e10_err.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/e10_b.json')); print('$a', d['value'], d['roofline']['avg_launch_ms'])"
done

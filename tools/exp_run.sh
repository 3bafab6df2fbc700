set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/e5_tests.log 2>&1 || { tail -30 gpurun_out/e5_tests.log; exit 1; }
tail -2 gpurun_out/e5_tests.log
B="--pmc off --no-cpu-baseline --fast-leg 0 --steps 4 --warmup 1"
for sc in "" "--scene explosion" "--width 1920 --height 1080" "--scene uniform --res 256 --width 512 --height 512"; do
  timeout -k 10 200 python bench.py $B $sc > gpurun_out/e5_b.json 2>gpurun_out/e5_err.log || { tail gpurun_out/e5_err.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/e5_b.json')); print('$sc', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['detail']['ms_film']/d['steps'])"
done

set -o pipefail
mkdir -p gpurun_out
B="--pmc off --no-cpu-baseline --fast-leg 0 --steps 10 --warmup 3"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/e2_tests.log 2>&1 || { tail -20 gpurun_out/e2_tests.log; exit 1; }
tail -2 gpurun_out/e2_tests.log
timeout -k 10 200 python bench.py $B --scene explosion > gpurun_out/e2_c5.json 2>gpurun_out/e2_err.log || exit $?
python -c "import json,sys; d=json.load(open('gpurun_out/e2_c5.json')); print('c5', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['detail']['ms_film'])"
timeout -k 10 200 python bench.py $B > gpurun_out/e2_def.json 2>gpurun_out/e2_err.log || exit $?
python -c "import json; d=json.load(open('gpurun_out/e2_def.json')); print('default', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['detail']['ms_film'])"

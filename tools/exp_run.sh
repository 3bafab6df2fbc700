set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/f4_tests.log 2>&1 || { tail -30 gpurun_out/f4_tests.log; exit 1; }
tail -1 gpurun_out/f4_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/f4_smoke.log 2>&1 || { tail -20 gpurun_out/f4_smoke.log; exit 1; }
tail -1 gpurun_out/f4_smoke.log
timeout -k 10 500 python bench.py --steps 10 --warmup 2 > gpurun_out/f4_bench.json 2>gpurun_out/f4_bench.err || { tail gpurun_out/f4_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/f4_bench.json')); print(d['value'], d['fast_mode']['value'], d['roofline']['frac'], d['roofline']['avg_launch_ms'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/f4_prof -o run -- python3 bench.py --pmc off --no-cpu-baseline --fast-leg 0 --steps 10 --warmup 2 > gpurun_out/f4_prof_bench.json 2>gpurun_out/f4_prof.err || { tail gpurun_out/f4_prof.err; exit 1; }
echo prof ok

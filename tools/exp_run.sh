set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/f2_tests.log 2>&1 || { tail -30 gpurun_out/f2_tests.log; exit 1; }
tail -1 gpurun_out/f2_tests.log
timeout -k 10 500 python bench.py --steps 10 --warmup 2 > gpurun_out/f2_bench.json 2>gpurun_out/f2_bench.err || { tail gpurun_out/f2_bench.err; exit 1; }
head -c 1500 gpurun_out/f2_bench.json; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/f2_prof -o run -- python3 bench.py --pmc off --no-cpu-baseline --fast-leg 0 --steps 10 --warmup 2 > gpurun_out/f2_prof_bench.json 2>gpurun_out/f2_prof.err || { tail gpurun_out/f2_prof.err; exit 1; }
echo prof ok
B="--pmc off --no-cpu-baseline --steps 4 --warmup 1"
for sc in "--scene explosion" "--width 1920 --height 1080" "--scene uniform --res 256 --width 512 --height 512" "--medium nanovdb"; do
  n=$(echo "$sc" | tr -d ' -' | cut -c1-20)
  timeout -k 10 300 python bench.py $B $sc > gpurun_out/f2_cfg_$n.json 2>gpurun_out/f2_err.log || { tail gpurun_out/f2_err.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/f2_cfg_$n.json')); print('$sc', d['value'], (d.get('fast_mode') or {}).get('value'), d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done

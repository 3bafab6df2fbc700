set -o pipefail
mkdir -p gpurun_out
B="--pmc off --no-cpu-baseline --steps 4 --warmup 1"
for sc in "--scene explosion" "--width 1920 --height 1080" "--scene uniform --res 256 --width 512 --height 512" "--medium nanovdb"; do
  n=$(echo "$sc" | tr -d ' -' | cut -c1-20)
  timeout -k 10 300 python bench.py $B $sc > gpurun_out/f5_cfg_$n.json 2>gpurun_out/f5_err.log || { tail gpurun_out/f5_err.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/f5_cfg_$n.json')); print('$sc', d['value'], (d.get('fast_mode') or {}).get('value'), d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done

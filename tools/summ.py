"""Summarise bench logs and PMC csvs of one gpurun pass: python tools/summ.py gpurun_out/<pass>"""
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
for f in sorted(glob.glob(os.path.join(d, "*.log"))):
    lines = [x for x in open(f, errors="replace") if x.startswith("{")]
    if not lines:
        continue
    j = json.loads(lines[-1])
    r = j["roofline"]
    print(f"{os.path.basename(f)[:-4]:12s} {j['value']:9.2f} Ms/s  kern {r['avg_launch_ms']:7.3f} ms  "
          f"simd {j.get('simd_utilisation') or 0:.3f}  iters {j['detail'].get('loop_iterations')}  "
          f"cpu {j['cpu_baseline']['value'] if j.get('cpu_baseline') else '-'}")
for f in sorted(glob.glob(os.path.join(d, "pmc_*", "run_counter_collection.csv"))):
    agg = {}
    for row in csv.DictReader(open(f)):
        if "k_paths" in row["Kernel_Name"]:
            agg.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    print(os.path.basename(os.path.dirname(f)), {k: round(sum(v) / len(v) / 1e6, 2) for k, v in agg.items()})
t = os.path.join(d, "gpu_tests.log")
if os.path.exists(t):
    print([x.strip() for x in open(t) if " passed" in x or " failed" in x][-1:])

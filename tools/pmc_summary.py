"""Fold one gpurun profiling pass (rocprofv3 --kernel-trace --stats + separate --pmc passes
of bench.py) into profiles/<round>_pmc_k_paths_<sampler>_<filter>.json.

usage: python tools/pmc_summary.py gpurun_out/<pass> <sampler> <filter> [round]

Traffic rule (MI355X_MICROARCH.md, HBM section): FETCH_SIZE (kB) x 2 on gfx950 + WRITE_SIZE
(kB). VALU issue capacity: SIMD-32, a wave64 VALU op issues in 2 cycles; 1024 SIMDs at 2.4 GHz.
"""
import csv
import json
import os
import sys

d, sampler, filt = sys.argv[1], sys.argv[2], sys.argv[3]
rnd = sys.argv[4] if len(sys.argv) > 4 else "r01"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def pmc(sub):
    agg, name = {}, None
    for r in csv.DictReader(open(os.path.join(d, sub, "run_counter_collection.csv"))):
        if "k_paths" in r["Kernel_Name"]:
            name = r["Kernel_Name"]
            agg.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}, name


f, kname = pmc("pmc_fetch")
w, _ = pmc("pmc_write")
s1, _ = pmc("pmc_sq1")
s2, _ = pmc("pmc_sq2")
stats = list(csv.DictReader(open(os.path.join(d, "prof", "run_kernel_stats.csv"))))
kp = [r for r in stats if "k_paths" in r["Name"]][0]
avg_ns = float(kp["AverageNs"])
bench = None
for name in ("bench.log", "zs_gauss.log"):
    pth = os.path.join(d, name)
    if os.path.exists(pth):
        lines = [x for x in open(pth) if x.startswith("{")]
        if lines:
            bench = json.loads(lines[-1])
            break
clk, simds = 2.4e9, 1024
valu = s2["SQ_INSTS_VALU"]
out = {
    "round": int(rnd[1:]), "source": f"{d} (tools/pmc_pass.sh), MI355X, S-cloud-1024 720p, "
                                      f"16 spp per launch, {sampler} sampler, {filt} filter",
    "kernel": kname, "rocprof_kernel_stats": {k: kp[k] for k in ("Calls", "AverageNs", "MinNs", "MaxNs")},
    "rocprof_avg_launch_ns": avg_ns,
    "bench_avg_launch_ms": bench["roofline"]["avg_launch_ms"] if bench else None,
    "FETCH_SIZE_kB_per_launch": f["FETCH_SIZE"], "WRITE_SIZE_kB_per_launch": w["WRITE_SIZE"],
    "hbm_traffic_bytes_per_launch": 1024 * (2 * f["FETCH_SIZE"] + w["WRITE_SIZE"]),
    "traffic_rule": "MI355X_MICROARCH.md HBM section: FETCH_SIZE (kB) x2 on gfx950, WRITE_SIZE (kB) as is; "
                    "the x2 is calibrated for 16-B/lane streaming reads, these are 2x16-B gathers",
    "algorithmic_bytes_per_launch": bench["roofline"]["bytes_per_launch"] if bench else None,
    "SQ": {**s1, **s2},
    "valu_wave_instructions_per_launch": valu,
    "valu_issue_fraction": valu * 2 / (simds * clk * avg_ns * 1e-9),
    "valu_rule": "MI355X_MICROARCH.md: SIMD-32, a wave64 VALU op issues in 2 cycles (one wave alone sustains 4); "
                 "1024 SIMDs at 2.4 GHz",
    "wave_cycle_split": {"active_inst_any": s1["SQ_ACTIVE_INST_ANY"] / s1["SQ_WAVE_CYCLES"],
                         "wait_inst_any (dependency/issue stall)": s1["SQ_WAIT_INST_ANY"] / s1["SQ_WAVE_CYCLES"],
                         "wait_any (s_waitcnt: memory/LDS)": s1["SQ_WAIT_ANY"] / s1["SQ_WAVE_CYCLES"]},
}
if os.path.isdir(os.path.join(d, "pmc_tcc")):
    t, _ = pmc("pmc_tcc")
    hit, miss = t.get("TCC_HIT_sum", 0.0), t.get("TCC_MISS_sum", 0.0)
    out["TCC"] = {"TCC_HIT_sum": hit, "TCC_MISS_sum": miss, "hit_rate": hit / max(1.0, hit + miss)}
if bench:
    spl = bench["config"]["global_batch"]   # samples per step = per k_paths launch
    out["samples_per_launch"] = spl
    out["valu_wave_instructions_per_sample"] = valu / spl
    out["bench_value"] = bench["value"]
dst = os.path.join(ROOT, "profiles", f"{rnd}_pmc_k_paths_{sampler}_{filt}.json")
json.dump(out, open(dst, "w"), indent=1)
print(dst, round(out["valu_issue_fraction"], 3), out["wave_cycle_split"])

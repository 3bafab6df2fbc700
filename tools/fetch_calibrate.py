"""Calibrate rocprofv3's read-byte counters for k_paths' access pattern (round-6 verdict item 1).

The standalone density fetch (avr_density_fetch: SampledGrid::Lookup from the fat layout, one
16-B point read, one 32-B fat entry gathered, one 4-B result written per lookup) runs over four
lookup orders whose useful bytes are known, on S-cloud-1024's fat copy (34.5 GB, far past the
256 MiB Infinity Cache):
  stream   : consecutive fat entries, each read once (fully coalesced: the known byte count),
  random   : uniformly random entries over the whole copy (no reuse),
  trace    : the lookups of one wavefront pass in trace order (the renderer's own pattern),
  shuffled : the same lookups in random order.
Each order is dispatched once per child process, under two counter passes:
  size   : TCC_EA0_RDREQ_sum and its 32-B / 64-B / 128-B request counts (the memory-side reads
           by request size: bytes = 32 R32 + 64 R64 + 128 R128),
  fetch  : FETCH_SIZE (rocprofv3's derived KiB, which on gfx950 tallies 128-B requests at 64 B).
For each order the result gives bytes per lookup by request size, FETCH_SIZE's bytes, their
ratio (the correction FETCH_SIZE needs for this pattern) and the request-size bytes over the
known useful bytes. bench.py prices `traffic` with the request-size bytes.

usage (through gpurun): python tools/fetch_calibrate.py --out gpurun_out/r06/fetch_cal.json
"""
import argparse
import csv
import glob
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
ORDERS = ("stream", "random", "trace", "shuffled")
PASSES = (("size", ("TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum")),
          ("fetch", ("FETCH_SIZE",)), ("write", ("WRITE_SIZE",)))
POINT_BYTES, ENTRY_BYTES, OUT_BYTES = 16, 32, 4


def log(msg):
    print(f"[fetch_calibrate] {msg}", file=sys.stderr, flush=True)


def child(a):
    """One process: build the scene, trace a wavefront pass's lookups, dispatch each order once
    (plus one untimed warm-up dispatch first); prints the lookup count of each dispatch."""
    import torch
    from acceleratedvolrenderer_amd import VolPathIntegrator, scenes, capi
    n = a.res
    dens = torch.empty((n, n, n), dtype=torch.float32, device="cuda:0")
    gen = capi.Context(0)
    for first in range(0, n ** 3, n * n * 64):
        gen.generate_cloud(dens.data_ptr() + 4 * first, n, first, min(n * n * 64, n ** 3 - first))
    gen.sync()
    gen.close()
    scene = scenes.s_cloud(dens, sampler="zsobol", spp=256, filter="gaussian")
    integ = VolPathIntegrator(scene, maxdepth=scenes.CLOUD_MAXDEPTH, spp=a.spp, device=0, kernel="wavefront")
    assert integ.ctx.grid_layout_active() == 1, "the fat layout is needed"
    cap = a.lookups
    pts = torch.zeros((cap, 4), dtype=torch.float32, device="cuda:0")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda:0")
    torch.cuda.synchronize()
    integ.ctx.record_lookups(pts.data_ptr(), cap, cnt.data_ptr())
    integ.ctx.render(0, a.spp, 0, scenes.CLOUD_MAXDEPTH)
    integ.ctx.sync()
    integ.ctx.record_lookups(0, 0, 0)
    nl = min(int(cnt.item()), cap)
    trace = pts[:nl].contiguous()
    del pts
    m = nl
    e1 = n + 1

    def entries_to_points(e):
        ix = (e % e1) - 1
        iy = ((e // e1) % e1) - 1
        iz = (e // (e1 * e1)) - 1
        p = torch.zeros((len(e), 4), dtype=torch.float32, device="cuda:0")
        p[:, 0] = (ix.to(torch.float32) + 0.75) / n
        p[:, 1] = (iy.to(torch.float32) + 0.75) / n
        p[:, 2] = (iz.to(torch.float32) + 0.75) / n
        return p

    total = e1 ** 3
    g = torch.Generator(device="cuda:0")
    g.manual_seed(1)
    arrays = {
        "stream": entries_to_points(torch.arange(m, device="cuda:0", dtype=torch.int64) + total // 3),
        "random": entries_to_points(torch.randint(0, total, (m,), device="cuda:0", generator=g, dtype=torch.int64)),
        "trace": trace,
        "shuffled": trace.index_select(0, torch.randperm(m, device="cuda:0", generator=g)).contiguous(),
    }
    out = torch.empty(m, dtype=torch.float32, device="cuda:0")
    torch.cuda.synchronize()
    integ.ctx.density_fetch(arrays["shuffled"].data_ptr(), min(m, 1 << 20), out.data_ptr())   # warm-up dispatch
    res = {"lookups": m, "order": ["warmup"] + list(ORDERS), "ms": {}}
    for k in ORDERS:
        res["ms"][k] = integ.ctx.density_fetch(arrays[k].data_ptr(), m, out.data_ptr())
    integ.close()
    print(json.dumps(res), flush=True)


def parse_counters(d):
    """{counter: [value per k_density_fetch dispatch, in dispatch order]}"""
    per = {}
    for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(fn)):
            if "k_density_fetch" not in row["Kernel_Name"]:
                continue
            did = int(row.get("Dispatch_Id", 0) or 0)
            per.setdefault(row["Counter_Name"], {}).setdefault(did, 0.0)
            per[row["Counter_Name"]][did] += float(row["Counter_Value"])
    return {k: [v[i] for i in sorted(v)] for k, v in per.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--res", type=int, default=1024)
    ap.add_argument("--spp", type=int, default=16)
    ap.add_argument("--lookups", type=int, default=48 * 1024 * 1024)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    if a.child:
        return child(a)
    exe = shutil.which("rocprofv3")
    assert exe, "rocprofv3 not found"
    me = [sys.executable, os.path.abspath(__file__), "--child", "--res", str(a.res), "--spp", str(a.spp),
          "--lookups", str(a.lookups)]
    tmp = tempfile.mkdtemp(prefix="avr_fcal_", dir=os.environ.get("TMPDIR", "/tmp"))
    ctr, info = {}, None
    try:
        for name, counters in PASSES:
            d = os.path.join(tmp, name)
            log(f"pass {name}: {' '.join(counters)}")
            t0 = time.time()
            r = subprocess.run([exe, "--pmc", *counters, "-d", d, "-o", "run", "--output-format", "csv", "--"] + me,
                               capture_output=True, text=True, timeout=300)
            if r.returncode != 0:
                raise SystemExit(f"pass {name} exited {r.returncode}: {r.stderr[-400:]}")
            info = json.loads(r.stdout.strip().splitlines()[-1])
            ctr.update(parse_counters(d))
            log(f"pass {name} done in {time.time() - t0:.0f} s")
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    m = info["lookups"]
    out = {"what": __doc__.split("\n\n")[0], "lookups_per_dispatch": m, "kernel": "k_density_fetch (fat layout)",
           "known_bytes_per_lookup": {"point_read": POINT_BYTES, "fat_entry_read": ENTRY_BYTES, "result_written": OUT_BYTES},
           "orders": {}}
    for i, k in enumerate(info["order"]):
        if k == "warmup":
            continue
        g = lambda c: ctr[c][i] if c in ctr and i < len(ctr[c]) else None
        r, r32, r64, r128 = (g("TCC_EA0_RDREQ_sum"), g("TCC_EA0_RDREQ_32B_sum"), g("TCC_EA0_RDREQ_64B_sum"),
                             g("TCC_EA0_RDREQ_128B_sum"))
        fs, ws = g("FETCH_SIZE"), g("WRITE_SIZE")
        sized = 32 * r32 + 64 * r64 + 128 * r128 if None not in (r32, r64, r128) else None
        known = (POINT_BYTES + ENTRY_BYTES) * m
        out["orders"][k] = {
            "ms": round(info["ms"][k], 4),
            "rdreq": r, "rdreq_32B": r32, "rdreq_64B": r64, "rdreq_128B": r128,
            "sizes_partition_rdreq": (abs((r32 + r64 + r128) - r) <= 0.001 * r) if None not in (r, r32, r64, r128) else None,
            "read_bytes_by_request_size": sized,
            "read_bytes_per_lookup": round(sized / m, 3) if sized else None,
            "fetch_size_bytes": fs * 1024 if fs is not None else None,
            "fetch_size_bytes_per_lookup": round(fs * 1024 / m, 3) if fs is not None else None,
            "fetch_size_correction": round(sized / (fs * 1024), 4) if sized and fs else None,
            "read_over_useful": round(sized / known, 4) if sized else None,
            "write_bytes_per_lookup": round(ws * 1024 / m, 3) if ws is not None else None,
            "effective_read_GBps": round(sized / (info["ms"][k] / 1e3) / 1e9, 1) if sized else None,
        }
        log(f"{k}: {out['orders'][k]}")
    s = out["orders"].get("stream", {})
    out["formula_check"] = {
        "what": "stream order: every byte read once, fully coalesced; the request-size bytes should equal the known bytes",
        "known_read_bytes": (POINT_BYTES + ENTRY_BYTES) * m, "request_size_bytes": s.get("read_bytes_by_request_size"),
        "ratio": s.get("read_over_useful")}
    line = json.dumps(out, indent=1)
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        open(a.out, "w").write(line)
    print(line)


if __name__ == "__main__":
    main()

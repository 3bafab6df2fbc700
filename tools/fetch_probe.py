"""Staged density-fetch measurement (the opt-in `bench.py --fetch-leg`, step by step with a
device synchronisation and a progress line after every stage, so that a failure names its
stage). S-cloud at --res^3: one wavefront pass traces its GridMedium lookups, then the
standalone density-fetch kernel (avr_density_fetch) runs on them in trace order, sorted by
the trilinear footprint's voxel, and shuffled. Prints one JSON line."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def log(msg):
    print(f"[fetch_probe] {msg}", file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--res", type=int, default=1024)
    ap.add_argument("--spp", type=int, default=16)
    ap.add_argument("--cap", type=int, default=48 * 1024 * 1024)
    ap.add_argument("--layout", default="fat", choices=["fat", "linear", "brick"])
    a = ap.parse_args()
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
    integ = VolPathIntegrator(scene, maxdepth=scenes.CLOUD_MAXDEPTH, spp=a.spp, device=0, kernel="wavefront",
                              grid_layout=a.layout)
    log("scene ready")
    pts = torch.zeros((a.cap, 4), dtype=torch.float32, device="cuda:0")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda:0")
    torch.cuda.synchronize()
    integ.ctx.record_lookups(pts.data_ptr(), a.cap, cnt.data_ptr())
    integ.ctx.render(0, a.spp, 0, scenes.CLOUD_MAXDEPTH)
    integ.ctx.sync()
    integ.ctx.record_lookups(0, 0, 0)
    total = int(cnt.item())
    nl = min(total, a.cap)
    p = pts[:nl]
    lo, hi = float(p[:, :3].min().item()), float(p[:, :3].max().item())
    finite = bool(torch.isfinite(p[:, :3]).all().item())
    log(f"traced {total} lookups (kept {nl}), points in [{lo:.5f}, {hi:.5f}], finite {finite}")
    if not (finite and lo > -0.01 and hi < 1.01 and nl > 0):
        raise SystemExit("traced points outside the unit box")
    out = torch.empty(nl, dtype=torch.float32, device="cuda:0")
    torch.cuda.synchronize()
    fb = 32 + 16 + 4
    res = {"lookups": nl, "bytes_per_lookup": fb, "layout": {0: "linear", 1: "fat", 2: "brick"}[integ.ctx.grid_layout_active()],
           "peak_GBps": 8000.0}

    def run(name, arr):
        integ.ctx.density_fetch(arr.data_ptr(), nl, out.data_ptr())
        t = sorted(integ.ctx.density_fetch(arr.data_ptr(), nl, out.data_ptr()) for _ in range(3))[1]
        g = fb * nl / (t / 1e3) / 1e9
        res[name] = {"ms": round(t, 4), "GBps": round(g, 1), "frac": round(g / 8000.0, 4)}
        log(f"{name}: {res[name]}")

    run("trace_order", p)
    gx = torch.floor(p[:, 0] * n - 0.5).to(torch.int64) + 1
    gy = torch.floor(p[:, 1] * n - 0.5).to(torch.int64) + 1
    gz = torch.floor(p[:, 2] * n - 0.5).to(torch.int64) + 1
    key = (gz * (n + 1) + gy) * (n + 1) + gx
    order = torch.argsort(key)
    torch.cuda.synchronize()
    log("sorted order computed")
    ps = p.index_select(0, order).contiguous()
    torch.cuda.synchronize()
    del gx, gy, gz, key, order
    run("sorted_by_voxel", ps)
    del ps
    perm = torch.randperm(nl, device="cuda:0")
    pr = p.index_select(0, perm).contiguous()
    torch.cuda.synchronize()
    log("shuffled order computed")
    run("shuffled", pr)
    integ.close()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    t0 = time.time()
    main()
    log(f"done in {time.time() - t0:.1f} s")

"""k_paths schedule sweep (refill lanes x DDA budget) in ONE process (GPU): the bench's S-cloud-1024 (GridMedium, or the
same cloud as a NanoVDBMedium with --medium nanovdb) at 720p, ZSobol + Gaussian, pixelsamples
16384 (the driver's plan), built once; then for each (refill, dda budget) candidate
`--steps` passes of 64 sample indices are timed (HIP events of k_paths, summed, and wall time of
the steps), candidates interleaved over `--rounds` rounds so box drift averages out. Schedule
parameters never change results (tests/test_gpu_edges.py).

usage: python tools/walk_sweep.py [--medium grid|nanovdb] [--ddas 0,16] [--refills 0,24]
prints one JSON line: {"medium", "rows": [{"refill", "dda", "kpaths_ms", "step_ms", "Msamples_s"}]}"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def ints(s):
    return [int(x) for x in s.split(",") if x != ""]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--medium", default="grid", choices=["grid", "nanovdb"])
    p.add_argument("--res", type=int, default=1024)
    p.add_argument("--refills", default="0")
    p.add_argument("--ddas", default="0")
    p.add_argument("--steps", type=int, default=4)
    p.add_argument("--rounds", type=int, default=2)
    p.add_argument("--pixelsamples", type=int, default=16384)
    p.add_argument("--majorant-res", type=int, default=0, help="r^3 majorant instead of pbrt's (0)")
    p.add_argument("--mode", default="replay", choices=["replay", "fast"], help="render mode (fast: the bench's fast leg)")
    a = p.parse_args()
    import torch
    from acceleratedvolrenderer_amd import VolPathIntegrator, scenes, capi
    n = a.res
    density = torch.empty((n, n, n), dtype=torch.float32, device="cuda:0")
    gen = capi.Context(0)
    slab = n * n * 64
    for first in range(0, n ** 3, slab):
        gen.generate_cloud(density.data_ptr() + 4 * first, n, first, min(slab, n ** 3 - first))
    gen.sync()
    gen.close()
    if a.medium == "nanovdb":
        scene = scenes.s_cloud_vdb(scenes.vdb_grid(density), sampler="zsobol", spp=a.pixelsamples, filter="gaussian")
        del density
        torch.cuda.empty_cache()
    else:
        scene = scenes.s_cloud(density, sampler="zsobol", spp=a.pixelsamples, filter="gaussian")
    S = 64
    integ = VolPathIntegrator(scene, maxdepth=scenes.CLOUD_MAXDEPTH, spp=S, seed=0, device=0, mode=a.mode)
    if a.majorant_res:
        integ.ctx.set_majorant_res((a.majorant_res,) * 3)
    npix = scene.film.width * scene.film.height
    cands = [(r, d) for r in ints(a.refills) for d in ints(a.ddas)]
    acc = {c: [0.0, 0.0, 0] for c in cands}
    integ.ctx.render(0, S, 0, scenes.CLOUD_MAXDEPTH)   # one-off tables
    integ.ctx.sync()
    base = S
    for rnd in range(a.rounds):
        for c in (cands if rnd % 2 == 0 else cands[::-1]):
            r, d = c
            integ.ctx.set_refill_min(r)
            integ.ctx.set_dda_budget(d)
            integ.ctx.render(base, base + S, 0, scenes.CLOUD_MAXDEPTH)   # warm this schedule
            integ.ctx.sync()
            integ.ctx.reset_stats()
            t0 = time.perf_counter()
            for k in range(a.steps):
                integ.ctx.render(base + (k + 1) * S, base + (k + 2) * S, 0, scenes.CLOUD_MAXDEPTH)
            integ.ctx.sync()
            el = time.perf_counter() - t0
            st = integ.ctx.stats()
            acc[c][0] += st["ms_medium"]
            acc[c][1] += el * 1e3
            acc[c][2] += a.steps
            print(f"[sweep] round {rnd} refill {r} dda {d}: k_paths {st['ms_medium'] / a.steps:.3f} ms, "
                  f"step {el * 1e3 / a.steps:.3f} ms", file=sys.stderr, flush=True)
            base = (base + (a.steps + 2) * S) % (a.pixelsamples - (a.steps + 2) * S)
    rows = [{"refill": c[0], "dda": c[1], "kpaths_ms": round(v[0] / v[2], 4),
             "step_ms": round(v[1] / v[2], 4), "Msamples_s": round(npix * S / (v[1] / v[2] / 1e3) / 1e6, 2)}
            for c, v in acc.items()]
    integ.close()
    print(json.dumps({"medium": a.medium, "mode": a.mode, "res": n, "majorant_res": a.majorant_res or None, "lib": os.environ.get("AVR_LIB"), "pixelsamples": a.pixelsamples, "steps_per_round": a.steps,
                      "rounds": a.rounds, "rows": rows}))


if __name__ == "__main__":
    main()

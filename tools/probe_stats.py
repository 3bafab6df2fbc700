"""k_paths walk / gather probes on the bench workload (variant build with -DAVR_PROBE_STATS):
how full the DDA walk's trips are, how many zero-majorant cells the walk crosses, and how many
distinct 64-B / 128-B lines the lanes of one collision round gather from (N1: the coalescing an
in-wave sort of the lookups could exploit). Results are unchanged by the probes.

usage: python tools/probe_stats.py --build                  (CPU, before gpurun)
       python tools/probe_stats.py [--medium grid|nanovdb] [--steps 3] [--dda 0]
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VARIANT = os.path.join(ROOT, "variants", "probe", "libavr_hip.so")
NAMES = ["walk_trips", "walking_lanes", "collision_rounds", "collision_lanes", "distinct_128B_lines",
         "distinct_64B_lines", "zero_majorant_steps", "walks_cut_with_walkers"]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--build", action="store_true")
    p.add_argument("--res", type=int, default=1024)
    p.add_argument("--medium", default="grid", choices=["grid", "nanovdb"])
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--dda", type=int, default=0)
    p.add_argument("--pixelsamples", type=int, default=16384)
    a = p.parse_args()
    sys.path.insert(0, ROOT)
    if a.build:
        from acceleratedvolrenderer_amd import build as b
        print(b.build(variant="probe", defines=["-DAVR_PROBE_STATS"]))
        return
    os.environ["AVR_LIB"] = VARIANT
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
    else:
        scene = scenes.s_cloud(density, sampler="zsobol", spp=a.pixelsamples, filter="gaussian")
    S = 64
    integ = VolPathIntegrator(scene, maxdepth=scenes.CLOUD_MAXDEPTH, spp=S, device=0)
    if a.dda:
        integ.ctx.set_dda_budget(a.dda)
    lib = capi.load()
    lib.avr_debug_sections.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_ulonglong)]
    out = (ctypes.c_ulonglong * 8)()
    integ.ctx.render(0, S, 0, scenes.CLOUD_MAXDEPTH)
    integ.ctx.sync()
    lib.avr_debug_sections(integ.ctx.h, out)
    integ.ctx.reset_stats()
    for k in range(1, 1 + a.steps):
        integ.ctx.render(S * k, S * (k + 1), 0, scenes.CLOUD_MAXDEPTH)
    integ.ctx.sync()
    lib.avr_debug_sections(integ.ctx.h, out)
    c = {NAMES[i]: int(out[i]) for i in range(8)}
    st = integ.stats()
    npix = scene.film.width * scene.film.height
    d = {"medium": a.medium, "dda": a.dda, "counters": c,
         "loop_iterations": st.get("loop_iterations"), "dda_lane_steps": st.get("medium_dda_steps"),
         "samples": npix * S * a.steps,
         "walk_lanes_per_trip": round(c["walking_lanes"] / max(1, c["walk_trips"]), 3),
         "trips_per_iteration": round(c["walk_trips"] / max(1, st.get("loop_iterations") or 1), 3),
         "zero_majorant_step_frac": round(c["zero_majorant_steps"] / max(1, st.get("medium_dda_steps") or 1), 4),
         "collision_lanes_per_round": round(c["collision_lanes"] / max(1, c["collision_rounds"]), 3),
         "lines128_per_lookup": round(c["distinct_128B_lines"] / max(1, c["collision_lanes"]), 4),
         "lines64_per_lookup": round(c["distinct_64B_lines"] / max(1, c["collision_lanes"]), 4)}
    print(json.dumps(d))
    integ.close()


if __name__ == "__main__":
    main()

"""k_paths time split by section on the bench workload (profiling variant build).

Builds variants/prof/libavr_hip.so with -DAVR_PROFILE_SECTIONS (build.build(variant="prof"),
here on the CPU: `--build`), then
on the GPU runs S-cloud passes through it and prints, per section, the share of wave cycles
(s_memtime, summed over waves): the event handlers (NEE spawn, shadow done, phase sampling,
escape + end), refill, segment starts, DDA walk, collision (exact candidate + density fetch +
callbacks).

usage: python tools/section_profile.py --build            (CPU, before gpurun)
       python tools/section_profile.py [--res 1024] [--medium grid|nanovdb] [--steps 3]
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NAMES = ["nee spawn", "refill", "segment starts", "dda walk", "collision", "shadow done", "phase sampling",
         "escape+end"]


def build(variant="prof", extra=()):
    sys.path.insert(0, ROOT)
    from acceleratedvolrenderer_amd import build as b
    print(b.build(variant=variant, defines=["-DAVR_PROFILE_SECTIONS"] + list(extra)))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--build", action="store_true")
    p.add_argument("--res", type=int, default=1024)
    p.add_argument("--medium", default="grid", choices=["grid", "nanovdb"])
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--sampler", default="zsobol")
    p.add_argument("--filter", default="gaussian")
    p.add_argument("--pixelsamples", type=int, default=16384, help="sampler pixelsamples (bench.py --steps 20: 16384)")
    p.add_argument("--pass-size", type=int, default=64, help="sample indices per pass (bench.py: 64)")
    p.add_argument("--variant", default="prof", help="variants/<name> (e.g. profsplit)")
    p.add_argument("--define", action="append", default=[], help="extra -D for --build")
    a = p.parse_args()
    if a.build:
        return build(a.variant, a.define)
    os.environ["AVR_LIB"] = os.path.join(ROOT, "variants", a.variant, "libavr_hip.so")
    sys.path.insert(0, ROOT)
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
        scene = scenes.s_cloud_vdb(scenes.vdb_grid(density), sampler=a.sampler, spp=a.pixelsamples,
                                   filter=a.filter)
        del density
    else:
        scene = scenes.s_cloud(density, sampler=a.sampler, spp=a.pixelsamples, filter=a.filter)
    S = a.pass_size
    integ = VolPathIntegrator(scene, maxdepth=scenes.CLOUD_MAXDEPTH, spp=S, device=0)
    lib = capi.load()
    lib.avr_debug_sections.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_ulonglong)]
    out = (ctypes.c_ulonglong * 8)()
    integ.ctx.render(0, S, 0, scenes.CLOUD_MAXDEPTH)   # warmup (pixel tables)
    integ.ctx.sync()
    lib.avr_debug_sections(integ.ctx.h, out)
    t0 = time.perf_counter()
    for k in range(1, 1 + a.steps):
        integ.ctx.render(S * k, S * (k + 1), 0, scenes.CLOUD_MAXDEPTH)
    integ.ctx.sync()
    dt = time.perf_counter() - t0
    lib.avr_debug_sections(integ.ctx.h, out)
    tot = sum(out[i] for i in range(8))
    res = {NAMES[i]: round(out[i] / tot, 4) for i in range(8)}
    st = integ.stats()
    print(json.dumps({"variant": a.variant, "medium": a.medium, "res": n, "pixelsamples": a.pixelsamples, "pass_size": S,
                      "Msamples_per_s": 1280 * 720 * S * a.steps / dt / 1e6,
                      "section_share": res, "wave_cycles": tot, "loop_iterations": st.get("loop_iterations"),
                      "dda_steps": st.get("medium_dda_steps")}))
    integ.close()


if __name__ == "__main__":
    main()

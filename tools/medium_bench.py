"""Persistent vs wavefront throughput on a non-GridMedium input (GPU): an RGBGridMedium of
random sigmoid coefficients (n^3) under the S-cloud camera and lights, zsobol + gaussian.

usage: python tools/medium_bench.py [--n 128] [--steps 4] [--kernel persistent|wavefront]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=128)
    p.add_argument("--steps", type=int, default=4)
    p.add_argument("--kernel", default="persistent")
    p.add_argument("--emissive", action="store_true")
    a = p.parse_args()
    import torch  # noqa: F401
    from acceleratedvolrenderer_amd import VolPathIntegrator, scenes, RGBGridMedium
    from acceleratedvolrenderer_amd.scene import Scene
    rng = np.random.default_rng(0)
    shape = (a.n, a.n, a.n)

    def coeffs(hi):
        c = np.empty(shape + (4,), np.float32)
        c[..., 0] = rng.uniform(-2e-5, 2e-5, shape)
        c[..., 1] = rng.uniform(-0.02, 0.02, shape)
        c[..., 2] = rng.uniform(-5, 5, shape)
        c[..., 3] = rng.uniform(0.0, hi, shape)
        return c
    base = scenes.s_cloud(np.zeros((1, 1, 1), np.float32), sampler="zsobol", spp=256, filter="gaussian")
    kw = dict(sigma_a_coeffs=coeffs(0.3), sigma_s_coeffs=coeffs(4.0), g=0.877)
    if a.emissive:
        kw.update(Le_coeffs=coeffs(1.0), Lescale=0.5)
    med = RGBGridMedium(**kw)
    scene = Scene(base.camera, base.film, med, base.lights, sampler=base.sampler)
    integ = VolPathIntegrator(scene, maxdepth=scenes.CLOUD_MAXDEPTH, spp=16, device=0, kernel=a.kernel)
    integ.ctx.render(0, 16, 0, scenes.CLOUD_MAXDEPTH)
    integ.ctx.sync()
    t0 = time.perf_counter()
    for k in range(1, 1 + a.steps):
        integ.ctx.render(16 * k, 16 * (k + 1), 0, scenes.CLOUD_MAXDEPTH)
    integ.ctx.sync()
    dt = time.perf_counter() - t0
    print(json.dumps({"medium": f"RGBGridMedium {a.n}^3", "kernel": a.kernel, "emissive": a.emissive,
                      "Msamples_per_s": round(1280 * 720 * 16 * a.steps / dt / 1e6, 2)}))
    integ.close()


if __name__ == "__main__":
    main()

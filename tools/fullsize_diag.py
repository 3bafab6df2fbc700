"""Diagnose full-size replay mismatches: per configuration, the fraction of bit-identical
lambda and L over a strided pixel subset of S-cloud-n 720p (GPU vs the canonical oracle)."""
import sys, os
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from acceleratedvolrenderer_amd import VolPathIntegrator, scenes, capi
from oracle import binding

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
md = int(sys.argv[2]) if len(sys.argv) > 2 else scenes.CLOUD_MAXDEPTH
kernel = sys.argv[3] if len(sys.argv) > 3 else "persistent"
configs = [("independent", "box", "fat", 0)]
density = torch.empty((n, n, n), dtype=torch.float32, device="cuda:0")
gen = capi.Context(0)
slab = n * n * 64
for first in range(0, n ** 3, slab):
    gen.generate_cloud(density.data_ptr() + 4 * first, n, first, min(slab, n ** 3 - first))
gen.sync(); gen.close()
hd = density.cpu().numpy()
for sampler, filt, layout, table in configs:
    scene = scenes.s_cloud(density, sampler=sampler, spp=256, filter=filt)
    integ = VolPathIntegrator(scene, maxdepth=md, spp=16, device=0, grid_layout=layout, kernel=kernel)
    integ.ctx.set_sampler_table(table)
    integ.ctx.render(32, 48, 0, md)
    f = scene.film
    npix = f.width * f.height
    _, _, L, lam, _ = integ.ctx.last_pass_samples(npix, 16)
    host = scenes.s_cloud(hd, sampler=sampler, spp=256, filter=filt)
    canon = binding.OracleRun(host, max_depth=md, seed=0, libm="canonical")
    el = ell = tot = 0
    worst = None
    for pix in np.arange(0, npix, 8191):
        for s in range(16):
            Lo, lo, _, _ = canon.pixel_sample(int(pix % f.width), int(pix // f.width), 32 + s)
            g = s * npix + int(pix)
            tot += 1
            a = np.array_equal(lam[g].view(np.uint32), lo.view(np.uint32))
            b = np.array_equal(L[g].view(np.uint32), Lo.view(np.uint32))
            el += a; ell += a and b
            if a and not b and worst is None:
                worst = (int(pix), s, L[g].tolist(), Lo.tolist())
    print(f"n{n} md{md} {kernel} {sampler}/{filt}/{layout}/table{table}: lambda {el/tot:.4f}, lambda+L {ell/tot:.4f} ({tot}); first L mismatch {worst}", flush=True)
    integ.close()

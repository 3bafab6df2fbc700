"""Film sums of a small S-cloud render (ZSobol, Gaussian, 3 passes of 64 sample indices) saved
to the given .npy path: run once with AVR_XCD_BANDS=1 and once without, then compare the files
byte for byte (the record-id layout must not change a single bit of the film)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from acceleratedvolrenderer_amd import VolPathIntegrator, scenes, capi
    n = 256
    density = torch.empty((n, n, n), dtype=torch.float32, device="cuda:0")
    gen = capi.Context(0)
    gen.generate_cloud(density.data_ptr(), n, 0, n ** 3)
    gen.sync()
    gen.close()
    scene = scenes.s_cloud(density, sampler="zsobol", spp=1024, filter="gaussian", width=320, height=184)
    integ = VolPathIntegrator(scene, maxdepth=scenes.CLOUD_MAXDEPTH, spp=64, seed=0, device=0)
    integ.ctx.film_clear()
    for k in range(3):
        integ.ctx.render(64 * k, 64 * (k + 1), 0, scenes.CLOUD_MAXDEPTH)
    integ.ctx.sync()
    rgb, w = integ.film_sums()
    np.save(sys.argv[1], np.concatenate([np.asarray(rgb).ravel(), np.asarray(w).ravel()]))
    integ.close()
    print("saved", sys.argv[1])


if __name__ == "__main__":
    main()

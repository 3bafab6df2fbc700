"""Driven by tests/test_launch_gloo.py: the launcher bench.py uses (launch.ensure_world),
then the multi-GPU path's one exchange (integrator.reduce_film) over gloo on CPU. Each rank
'renders' its sample shard of a fake film (value = f(pixel, sample index), summed over its
shard in sampleIndex order); rank 0 prints one JSON line with n_gpus and the reduced film."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--spp", type=int, default=10)
    p.add_argument("--npix", type=int, default=6)
    a = p.parse_args()
    from acceleratedvolrenderer_amd import launch
    launch.ensure_world(a.gpus, os.path.abspath(__file__), sys.argv[1:])
    import numpy as np
    import torch
    import torch.distributed as dist
    from acceleratedvolrenderer_amd.integrator import film_buffer_size, reduce_film, shard_samples
    world, rank, _ = launch.world_from_env()
    if world > 1:
        dist.init_process_group("gloo", init_method="env://")
    lo, hi = shard_samples(a.spp, rank, world)
    buf = np.zeros(film_buffer_size(a.npix), np.float64)
    for s in range(lo, hi):
        for pix in range(a.npix):
            v = 0.5 + 0.25 * pix + 0.125 * s
            buf[3 * pix:3 * pix + 3] += (v, 2 * v, 3 * v)
            buf[3 * a.npix + pix] += 1.0
    t = torch.from_numpy(buf)
    if world > 1:
        out = reduce_film(t, a.npix, 0, rank)
    else:
        out = (buf[:3 * a.npix], buf[3 * a.npix:])
    if rank == 0:
        print(json.dumps({"n_gpus": world, "rgb": [float(x) for x in out[0]], "w": [float(x) for x in out[1]]}),
              flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

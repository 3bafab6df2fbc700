"""Pass cost by call pattern on one GPU: the bench's S-cloud-1024 (GridMedium, ZSobol + Gaussian,
720p, pixelsamples 16384) rendered as K one-pass calls of 64 sample indices, either consecutive
(the 1-GPU bench, pbrt's pass loop) or strided by N passes (what one rank of an N-GPU sample
shard renders: launch.sample_plan), with the ZSobol pass table built ahead (avr_set_pass_table_ahead)
on and off. Prints one JSON line of ms per pass (wall time of the K calls, synchronised).

usage: python tools/pass_stride_probe.py [--strides 1,8] [--passes 12] [--rounds 2]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--res", type=int, default=1024)
    p.add_argument("--strides", default="1,8")
    p.add_argument("--passes", type=int, default=12)
    p.add_argument("--rounds", type=int, default=2)
    a = p.parse_args()
    import torch
    from acceleratedvolrenderer_amd import VolPathIntegrator, scenes, capi
    n = a.res
    density = torch.empty((n, n, n), dtype=torch.float32, device="cuda:0")
    gen = capi.Context(0)
    for first in range(0, n ** 3, n * n * 64):
        gen.generate_cloud(density.data_ptr() + 4 * first, n, first, min(n * n * 64, n ** 3 - first))
    gen.sync()
    gen.close()
    S, spp = 64, 16384
    scene = scenes.s_cloud(density, sampler="zsobol", spp=spp, filter="gaussian")
    integ = VolPathIntegrator(scene, maxdepth=scenes.CLOUD_MAXDEPTH, spp=S, seed=0, device=0)
    integ.ctx.render(0, S, 0, scenes.CLOUD_MAXDEPTH)   # one-off tables
    integ.ctx.sync()
    strides = [int(x) for x in a.strides.split(",")]
    acc = {}
    for rnd in range(a.rounds):
        for st in strides:
            for ahead in (1, 0):
                integ.ctx.set_pass_table_ahead(ahead)
                first = (rnd * 7 + 1) * S
                bases = [(first + k * st * S) % (spp - S) for k in range(a.passes + 1)]
                integ.ctx.render(bases[0], bases[0] + S, 0, scenes.CLOUD_MAXDEPTH)   # sets the call stride
                integ.ctx.sync()
                t0 = time.perf_counter()
                for b in bases[1:]:
                    integ.ctx.render(b, b + S, 0, scenes.CLOUD_MAXDEPTH)
                integ.ctx.sync()
                ms = (time.perf_counter() - t0) * 1e3 / a.passes
                acc.setdefault(f"stride{st}_ahead{ahead}", []).append(round(ms, 3))
                print(f"[probe] round {rnd} stride {st} ahead {ahead}: {ms:.3f} ms per pass", file=sys.stderr, flush=True)
    integ.close()
    print(json.dumps({"res": n, "pixelsamples": spp, "pass": S, "passes": a.passes, "ms_per_pass": acc}))


if __name__ == "__main__":
    main()

"""Multi-process sample sharding + SUM reduce of the fp64 film (world_size 2, gloo on CPU).

The GPU path shards sample indices across ranks and reduces the film over RCCL
(VolPathIntegrator.render_distributed); here the CPU oracle renders each rank's shard
and the same reduction runs over gloo. The reduced film must equal the 1-process film
up to fp64 summation order."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _scene():
    from acceleratedvolrenderer_amd import scenes
    rng = np.random.default_rng(11)
    dens = rng.random((8, 8, 8), dtype=np.float32)
    return scenes.s_uniform(n=8, width=12, height=9, variant="scatter", density=dens)


def _worker(rank, world, port, spp, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from acceleratedvolrenderer_amd import shard_samples
    from oracle import binding
    sc = _scene()
    lo, hi = shard_samples(spp, rank, world)
    rgb, w = binding.OracleRun(sc, max_depth=5).render(lo, hi, nthreads=1)
    from acceleratedvolrenderer_amd.integrator import reduce_film
    out = reduce_film(torch.from_numpy(np.concatenate([rgb, w])), 12 * 9, 0, rank)
    if rank == 0:
        np.save(out_path, np.concatenate(out))
    dist.barrier()
    dist.destroy_process_group()


def _spectral_scene():
    from acceleratedvolrenderer_amd import SpectralFilm
    from acceleratedvolrenderer_amd.scene import Scene
    base = _scene()
    return Scene(base.camera, SpectralFilm(12, 9, nbuckets=6), base.medium, base.lights)


def _spectral_worker(rank, world, port, spp, out_path):
    """The product's reduce step (integrator.reduce_film, the same call render_distributed
    makes over RCCL) on this rank's SpectralFilm shard packed as avr_film_export_device lays
    it out."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from acceleratedvolrenderer_amd import shard_samples
    from acceleratedvolrenderer_amd.integrator import reduce_film, film_buffer_size
    from oracle import binding
    sc = _spectral_scene()
    npix, nb = 12 * 9, sc.film.nbuckets
    lo, hi = shard_samples(spp, rank, world)
    rgb, w, bs, bw = binding.OracleRun(sc, max_depth=5).render_spectral(lo, hi, nthreads=1)
    buf = torch.from_numpy(np.concatenate([rgb, w, bs.ravel(), bw.ravel()]))
    assert buf.numel() == film_buffer_size(npix, nb)
    out = reduce_film(buf, npix, nb, rank)
    if rank == 0:
        np.savez(out_path, *out)
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_spectral_film_reduces_to_single_process_film(tmp_path):
    spp, world = 5, 2
    out = str(tmp_path / "spec.npz")
    mp.spawn(_spectral_worker, args=(world, _free_port(), spp, out), nprocs=world, join=True)
    got = np.load(out)
    from oracle import binding
    ref = binding.OracleRun(_spectral_scene(), max_depth=5).render_spectral(0, spp, nthreads=1)
    for k, r in enumerate(ref):
        g = got[f"arr_{k}"]
        assert g.shape == r.shape
        assert np.allclose(g, r, rtol=1e-12, atol=0)
    assert np.array_equal(got["arr_3"], ref[3])   # bucket weights: sums of small integers


@pytest.mark.parametrize("world", [2])
def test_sharded_render_reduces_to_single_process_film(tmp_path, world):
    spp = 6
    out = str(tmp_path / "film.npy")
    mp.spawn(_worker, args=(world, _free_port(), spp, out), nprocs=world, join=True)
    reduced = np.load(out)
    from oracle import binding
    sc = _scene()
    rgb, w = binding.OracleRun(sc, max_depth=5).render(0, spp, nthreads=1)
    full = np.concatenate([rgb, w])
    npix = 12 * 9
    assert np.array_equal(reduced[3 * npix:], full[3 * npix:])
    assert np.allclose(reduced, full, rtol=1e-12, atol=0)

"""PowerLightSampler in the oracle (lightsamplers.h:63-99, lightsamplers.cpp:76-96,
util/sampling.cpp:563-645): with equal light weights the alias table picks exactly as the
BVH / uniform sampler does, and with unequal weights the power-sampled estimator converges to
the same image (both are unbiased; only the light-pick PMF differs)."""
import numpy as np
import pytest


def _scene(variant, W=16, H=12, lights=None):
    from acceleratedvolrenderer_amd import scenes
    from acceleratedvolrenderer_amd.scene import Scene
    base = scenes.s_uniform(n=6, width=W, height=H, variant=variant,
                            density=(0.2 + np.random.default_rng(4).random((6, 6, 6), dtype=np.float32)))
    return Scene(base.camera, base.film, base.medium, base.lights if lights is None else lights)


def test_power_sampler_with_equal_weights_picks_as_bvh():
    """Two identical distant lights: weights equal, every alias bin keeps q = 1, and
    AliasTable::Sample's offset min(u n, n - 1) is the BVH sampler's index -> identical films."""
    from acceleratedvolrenderer_amd import DistantLight
    from oracle import binding
    lights = [DistantLight(from_=(1, 1, -1), to=(0, 0, 0), scale=1.5), DistantLight(from_=(1, 1, -1), to=(0, 0, 0), scale=1.5)]
    scene = _scene("scatter", lights=lights)
    a = binding.OracleRun(scene, max_depth=6, seed=0, lightsampler="bvh").render(0, 8, nthreads=8)
    b = binding.OracleRun(scene, max_depth=6, seed=0, lightsampler="power").render(0, 8, nthreads=8)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("variant", ["scatter", "chromatic"])
def test_power_sampler_is_unbiased_against_bvh(variant):
    """Distant + uniform infinite lights (their Phi differ by ~4 pi): the power-sampled and the
    uniformly sampled estimators agree within 5 standard errors on the frame mean, and the
    films differ (the pick PMF changed)."""
    from oracle import binding
    scene = _scene(variant)
    spp = 64
    means = {}
    films = {}
    for ls in ("bvh", "power"):
        per_seed = []
        for seed in range(4):
            rgb, w = binding.OracleRun(scene, max_depth=8, seed=seed, lightsampler=ls).render(0, spp, nthreads=8)
            img = rgb / np.maximum(w, 1e-30)[..., None] if rgb.ndim == w.ndim + 1 else rgb
            per_seed.append(float(np.mean(img)))
            films.setdefault(ls, rgb)
        means[ls] = (np.mean(per_seed), np.std(per_seed, ddof=1) / np.sqrt(len(per_seed)))
    (mb, sb), (mp, sp) = means["bvh"], means["power"]
    print(f"{variant}: frame mean bvh {mb:.5f} +- {sb:.5f}, power {mp:.5f} +- {sp:.5f}")
    assert abs(mb - mp) <= 5 * np.hypot(sb, sp) + 1e-6
    assert not np.array_equal(films["bvh"], films["power"])

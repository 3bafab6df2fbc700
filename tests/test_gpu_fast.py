"""The "fast" render mode (avr_set_render_mode 1; SURVEY.md §7 "replay / fast").

Fast mode evaluates log / exp / sin / cos with the hardware instructions (about 1 ulp) and
decides each free-flight candidate once, instead of the canonical f64 sequences and pbrt's
CPU FastExp polynomial that replay uses. The estimator (VolPathIntegrator::Li,
cpu/integrators.cpp:962-1280) is the same, so parity is statistical. Tolerances:
  * correlated: at the same seed the fast film may differ from the platform CPU oracle's
    film by at most 0.5 x the Monte Carlo noise (relative RMS between two oracle films at
    different seeds) — the sample streams are the same and only last bits differ;
  * unbiased: the frame mean of a fast render at many more samples lies within 4 standard
    errors of the oracle's frame mean;
  * counts: every (pixel, sample) path is traced exactly once (weights bit-exact).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    torch.cuda.init()


def _rel_rms(a, b):
    return float(np.sqrt(np.mean((a - b) ** 2)) / max(1e-12, np.sqrt(np.mean(b ** 2))))


def _scene(kind):
    from acceleratedvolrenderer_amd import scenes
    from oracle import binding
    if kind == "uniform":   # C2's scene type: uniform GridMedium cube, orthographic
        n = 16
        dens = np.full((n, n, n), 0.75, np.float32)
        return scenes.s_uniform(n=n, width=32, height=32, variant="scatter", density=dens), 5
    if kind == "cloud":     # C3's stand-in: the S-cloud, perspective, ZSobol + Gaussian
        dens = binding.cloud_grid(32)
        return scenes.s_cloud(dens, width=48, height=27, sampler="zsobol", spp=1024,
                              filter="gaussian"), scenes.CLOUD_MAXDEPTH
    raise ValueError(kind)


@pytest.mark.parametrize("maj", ["pbrt", "tuned1"])
@pytest.mark.parametrize("kind", ["uniform", "cloud"])
def test_fast_mode_statistical_parity(kind, maj):
    """maj "pbrt": pbrt's own 16^3 majorant; "tuned1": the 1^3 majorant avr_tune_majorant picks
    for the bench's S-cloud (bench.py fast_mode leg) — correlated parity against the platform
    oracle built with the same majorant, unbiasedness against the oracle at pbrt's 16^3."""
    from acceleratedvolrenderer_amd import VolPathIntegrator
    from oracle import binding
    scene, maxdepth = _scene(kind)
    pbrt_scene, _ = _scene(kind)
    if maj == "tuned1":
        scene.medium.majorant_res = (1, 1, 1)
    spp = 16
    fast = VolPathIntegrator(scene, maxdepth=maxdepth, spp=spp, seed=0, device=0, mode="fast")
    if maj == "tuned1":
        assert fast.ctx.majorant(1).tolist() == binding.build_majorant(scene.medium.density, (1, 1, 1)).tolist()
    rgb_f, w_f = fast.render()
    ref = binding.OracleRun(scene, max_depth=maxdepth, seed=0)
    rgb_o, w_o = ref.render(0, spp, nthreads=8)
    assert np.array_equal(w_f, w_o), "every (pixel, sample) path traced once, same filter weights"
    rgb_1, w_1 = binding.OracleRun(scene, max_depth=maxdepth, seed=1).render(0, spp, nthreads=8)
    img_f, img_o, img_1 = fast.image(rgb_f, w_f), fast.image(rgb_o, w_o), fast.image(rgb_1, w_1)
    err, noise = _rel_rms(img_f, img_o), _rel_rms(img_1, img_o)

    # unbiasedness: 64x the samples on the device vs the frame mean of the oracle at pbrt's
    # own majorant (any conservative majorant is the same estimator in expectation)
    if maj == "tuned1":
        rgb_o, w_o = binding.OracleRun(pbrt_scene, max_depth=maxdepth, seed=0).render(0, spp, nthreads=8)
        rgb_1, w_1 = binding.OracleRun(pbrt_scene, max_depth=maxdepth, seed=1).render(0, spp, nthreads=8)
        img_o, img_1 = fast.image(rgb_o, w_o), fast.image(rgb_1, w_1)
    rgb_big, w_big = fast.render(0, 64 * spp if kind == "uniform" else 1024)
    img_big = fast.image(rgb_big, w_big)
    o_mean = 0.5 * (img_o.mean() + img_1.mean())
    # standard error of the oracle's two-seed frame mean from the per-pixel seed difference
    # (var of (o + o1) / 2 over N pixels = var(o - o1) / (4 N)); the device mean adds ~1/32 of it
    se = 1.02 * float(np.std(img_o - img_1)) / (2 * np.sqrt(img_o.size))
    print(f"fast/{kind}/{maj}: film rel RMS vs platform oracle {err:.3e} (MC noise {noise:.3e}); frame mean "
          f"{img_big.mean():.6f} vs oracle {o_mean:.6f} (se {se:.2e})")
    assert err <= 0.5 * noise
    assert abs(img_big.mean() - o_mean) <= 4 * se + 1e-6 * abs(o_mean)
    fast.close()


def test_fast_and_replay_modes_switch_on_one_context():
    """The mode is a per-render switch: replay after fast is bit-identical to replay alone."""
    from acceleratedvolrenderer_amd import VolPathIntegrator
    scene, maxdepth = _scene("uniform")
    a = VolPathIntegrator(scene, maxdepth=maxdepth, spp=8, seed=0, device=0)
    rgb_a, w_a = a.render()
    a.ctx.set_render_mode("fast")
    rgb_f, _ = a.render()
    a.ctx.set_render_mode("replay")
    rgb_b, w_b = a.render()
    assert np.array_equal(rgb_a, rgb_b) and np.array_equal(w_a, w_b)
    assert not np.array_equal(rgb_a, rgb_f)   # the fast pass really ran other arithmetic
    a.close()


def test_render_mode_argument_errors():
    from acceleratedvolrenderer_amd import capi
    lib = capi.load()
    assert lib.avr_set_render_mode(None, 0) != 0
    ctx = capi.Context(0)
    with pytest.raises(RuntimeError):
        ctx.set_render_mode(2)
    ctx.close()


def test_set_majorant_res_matches_oracle_majorant():
    """avr_set_majorant_res rebuilds SampledGrid::MaxValue cells (containers.h:838-857) at
    the new resolution: bit-exact against the oracle's majorant build."""
    from acceleratedvolrenderer_amd import scenes, VolPathIntegrator
    from oracle import binding
    rng = np.random.default_rng(11)
    dens = rng.random((20, 24, 28), dtype=np.float32)
    scene = scenes.s_uniform(n=1, width=8, height=8, variant="scatter", density=dens)
    integ = VolPathIntegrator(scene, spp=1, device=0)
    for res in [(1, 1, 1), (4, 4, 4), (3, 5, 7), (16, 16, 16)]:
        integ.ctx.set_majorant_res(res)
        got = integ.ctx.majorant(res[0] * res[1] * res[2])
        want = binding.build_majorant(dens, res)
        assert got.view(np.uint32).tolist() == want.view(np.uint32).tolist(), res
    with pytest.raises(RuntimeError):
        integ.ctx.set_majorant_res((0, 4, 4))
    integ.close()


def test_replay_at_a_tuned_majorant_resolution_is_bit_exact():
    """A non-pbrt majorant resolution changes the sample streams, not the arithmetic: replay
    against the canonical oracle built with the same resolution stays bit-exact."""
    from acceleratedvolrenderer_amd import scenes, VolPathIntegrator
    from oracle import binding
    dens = binding.cloud_grid(24)
    scene = scenes.s_cloud(dens, width=32, height=18)
    scene.medium.majorant_res = (4, 4, 4)
    integ = VolPathIntegrator(scene, maxdepth=scenes.CLOUD_MAXDEPTH, spp=4, seed=0, device=0)
    rgb, w = integ.render()
    canon = binding.OracleRun(scene, max_depth=scenes.CLOUD_MAXDEPTH, seed=0, libm="canonical")
    rgb_c, w_c = canon.render(0, 4, nthreads=8)
    assert np.array_equal(w, w_c)
    assert np.array_equal(rgb, rgb_c)
    integ.close()


def test_tune_majorant_keeps_the_film_and_picks_a_candidate():
    from acceleratedvolrenderer_amd import scenes, VolPathIntegrator
    from oracle import binding
    dens = binding.cloud_grid(32)
    scene = scenes.s_cloud(dens, width=64, height=36, sampler="zsobol", spp=64, filter="gaussian")
    integ = VolPathIntegrator(scene, maxdepth=scenes.CLOUD_MAXDEPTH, spp=4, seed=0, device=0, mode="fast")
    rgb, w = integ.render()
    chosen, ms = integ.tune_majorant(candidates=(1, 2, 4, 8, 16), probe=(4, 8))
    rgb2, w2 = integ.film_sums()
    assert np.array_equal(rgb, rgb2) and np.array_equal(w, w2)
    assert chosen[0] in (1, 2, 4, 8, 16) and chosen[0] == chosen[1] == chosen[2]
    assert all(t > 0 for t in ms.values())
    assert min(ms, key=ms.get) == chosen[0]
    got = integ.ctx.majorant(chosen[0] ** 3)
    assert got.view(np.uint32).tolist() == binding.build_majorant(dens, chosen).view(np.uint32).tolist()
    print(f"tuned majorant {chosen}, probe ms {ms}")
    integ.close()


def test_tune_majorant_failure_restores_film_and_majorant():
    """A probe that fails (here: an invalid max_depth reaches avr_render) leaves the context as
    it was: the film sums and the majorant grid at its previous resolution."""
    from acceleratedvolrenderer_amd import scenes, VolPathIntegrator
    from oracle import binding
    dens = binding.cloud_grid(24)
    scene = scenes.s_cloud(dens, width=32, height=18)
    integ = VolPathIntegrator(scene, maxdepth=scenes.CLOUD_MAXDEPTH, spp=2, seed=0, device=0)
    rgb, w = integ.render()
    maj = integ.ctx.majorant(16 ** 3)
    with pytest.raises(RuntimeError, match="sample range"):
        integ.ctx.tune_majorant([(1, 1, 1), (4, 4, 4)], 0, 2, 0, -1)
    rgb2, w2 = integ.film_sums()
    assert np.array_equal(rgb, rgb2) and np.array_equal(w, w2)
    assert integ.ctx.majorant(16 ** 3).view(np.uint32).tolist() == maj.view(np.uint32).tolist()
    # and the context still renders the same samples
    rgb3, w3 = integ.render()
    assert np.array_equal(rgb3, rgb) and np.array_equal(w3, w)
    integ.close()


def test_tune_majorant_refuses_single_segment_media():
    """HomogeneousMedium / CloudMedium have one majorant segment (no grid to tune), as
    avr_set_majorant_res refuses them."""
    from acceleratedvolrenderer_amd import scenes, VolPathIntegrator
    from acceleratedvolrenderer_amd import HomogeneousMedium
    from acceleratedvolrenderer_amd.scene import Scene
    base = scenes.s_uniform(n=4, width=8, height=8, variant="scatter")
    scene = Scene(base.camera, base.film, HomogeneousMedium(sigma_a=0.5, sigma_s=2.0, g=0.3), base.lights)
    integ = VolPathIntegrator(scene, maxdepth=5, spp=1, seed=0, device=0)
    with pytest.raises(RuntimeError, match="single majorant segment"):
        integ.ctx.tune_majorant([(1, 1, 1), (2, 2, 2)], 0, 1, 0, 5)
    with pytest.raises(RuntimeError, match="single majorant segment"):
        integ.ctx.set_majorant_res((2, 2, 2))
    integ.close()


def test_tune_walk_keeps_the_film_and_changes_no_result():
    """avr_tune_walk (k_paths' refill / DDA-budget schedule chosen by on-device probes): the film
    is restored, the choice is the fastest probe (the default unless beaten by > 2 %), the counters
    are reset, and renders under the
    chosen schedule — and under every candidate — are bit-identical to the default schedule."""
    from acceleratedvolrenderer_amd import scenes, VolPathIntegrator
    from oracle import binding
    dens = binding.cloud_grid(32)
    scene = scenes.s_cloud(dens, width=64, height=36, sampler="zsobol", spp=64, filter="gaussian")
    integ = VolPathIntegrator(scene, maxdepth=scenes.CLOUD_MAXDEPTH, spp=4, seed=0, device=0)
    rgb, w = integ.render()
    refill, dda = (0, 8, 32, 48), (0, 4, 12)
    chosen, ms = integ.ctx.tune_walk(refill, dda, 4, 8, 0, scenes.CLOUD_MAXDEPTH)
    rgb2, w2 = integ.film_sums()
    assert np.array_equal(rgb, rgb2) and np.array_equal(w, w2)
    assert ms.shape == (4, 3) and (ms > 0).all()
    # the fastest probe, except that the default (0, 0) is kept unless beaten by > 2 % (probe noise)
    # by every probe of the same effective schedule (this grid's defaults: 32 lanes, 10 cells)
    i, j = np.unravel_index(int(np.argmin(ms)), ms.shape)
    eff = lambda a, b: (a or 32, b or 10)
    t_def = min(ms[a, b] for a in range(len(refill)) for b in range(len(dda))
                if eff(refill[a], dda[b]) == eff(0, 0))
    want = (0, 0) if t_def <= ms[i, j] * 1.02 else (refill[i], dda[j])
    assert chosen == want
    assert integ.stats()["medium_lookups"] == 0
    rgb3, w3 = integ.render()
    assert np.array_equal(rgb3, rgb) and np.array_equal(w3, w)
    for r in refill[1:]:
        for d in dda[1:]:
            integ.ctx.set_refill_min(r)
            integ.ctx.set_dda_budget(d)
            rgb4, w4 = integ.render()
            assert np.array_equal(rgb4, rgb) and np.array_equal(w4, w), (r, d)
    with pytest.raises(RuntimeError, match="refill candidates"):
        integ.ctx.tune_walk((65,), (0,), 0, 1, 0, 5)
    integ.close()

"""Parity at the bench's full size (BASELINE config C3 stand-in: S-cloud-1024 GridMedium,
perspective 1280x720, ZSobol + Gaussian, maxdepth 100) through size-independent properties:
per-sample replay of a strided pixel subset against the canonical CPU oracle (every sample
bit-identical), multi-pass accumulation equal to one pass, run-to-run determinism, and the
majorant grid bit-exact. Needs ~40 GB of HBM (grid + fat copy) and ~5 GB of host memory."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def cloud():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from acceleratedvolrenderer_amd import VolPathIntegrator, scenes, capi
    n = 1024
    density = torch.empty((n, n, n), dtype=torch.float32, device="cuda:0")
    gen = capi.Context(0)
    slab = n * n * 64
    for first in range(0, n ** 3, slab):
        gen.generate_cloud(density.data_ptr() + 4 * first, n, first, min(slab, n ** 3 - first))
    gen.sync()
    gen.close()
    scene = scenes.s_cloud(density, sampler="zsobol", spp=256, filter="gaussian")
    integ = VolPathIntegrator(scene, maxdepth=scenes.CLOUD_MAXDEPTH, spp=16, device=0)
    integ.density_tensor = density   # the device grid, for scenes at other sampler settings
    host = scenes.s_cloud(density.cpu().numpy(), sampler="zsobol", spp=256, filter="gaussian")
    yield integ, host
    integ.close()


def test_fullsize_majorant_and_replay(cloud):
    from acceleratedvolrenderer_amd import scenes
    from oracle import binding
    integ, host = cloud
    canon = binding.OracleRun(host, max_depth=scenes.CLOUD_MAXDEPTH, seed=0, libm="canonical")
    assert integ.ctx.majorant(16 ** 3).view(np.uint32).tolist() == canon.majorant.view(np.uint32).tolist()
    integ.ctx.film_clear()
    integ.ctx.render(32, 48, 0, scenes.CLOUD_MAXDEPTH)
    f = host.film
    npix = f.width * f.height
    _, _, L, lam, _ = integ.ctx.last_pass_samples(npix, 16)
    pixels = np.arange(0, npix, 4099)          # ~225 pixels spread over the frame
    exact = total = 0
    for pix in pixels:
        for s in range(16):
            Lo, lo, _, _ = canon.pixel_sample(int(pix % f.width), int(pix // f.width), 32 + s)
            g = s * npix + int(pix)
            total += 1
            exact += int(np.array_equal(L[g].view(np.uint32), Lo.view(np.uint32)) and
                         np.array_equal(lam[g].view(np.uint32), lo.view(np.uint32)))
    print(f"full-size replay: {exact}/{total} samples bit-identical")
    assert exact == total


def test_fullsize_replay_at_the_driver_headline_configuration(cloud):
    """The exact configuration the driver times (`python bench.py --steps 20 --warmup 5`):
    launch.sample_plan gives pixelsamples 16384 at every world size, so at 720p Morton(pixel)
    (22 bits) << log2 spp (14) needs 36 bits and k_paths runs its 64-bit-index ZSobol
    GridMedium instantiation (samplers.h:250-254). Strided pixel subset, two 16-index passes
    (one inside the N = 1 timed range, one at the top of the N = 8 range): every sample
    bit-identical to the canonical oracle, with the instantiation checked by name."""
    from acceleratedvolrenderer_amd import VolPathIntegrator, scenes
    from acceleratedvolrenderer_amd.launch import sample_plan
    from oracle import binding
    integ256, host256 = cloud
    P = sample_plan(1, 20, 5, 64)[0]
    assert P == sample_plan(8, 20, 5, 64)[0] == 16384
    scene = scenes.s_cloud(integ256.density_tensor, sampler="zsobol", spp=P, filter="gaussian")
    integ = VolPathIntegrator(scene, maxdepth=scenes.CLOUD_MAXDEPTH, spp=16, device=0)
    try:
        host = scenes.s_cloud(host256.medium.density, sampler="zsobol", spp=P, filter="gaussian")
        canon = binding.OracleRun(host, max_depth=scenes.CLOUD_MAXDEPTH, seed=0, libm="canonical")
        f = host.film
        npix = f.width * f.height
        pixels = np.arange(0, npix, 4099)
        exact = total = 0
        for base in (640, 8 * 20 * 64 - 16):
            integ.ctx.film_clear()
            integ.ctx.render(base, base + 16, 0, scenes.CLOUD_MAXDEPTH)
            assert integ.ctx.last_kernel() == "k_paths<false, true, 3, 0, false, false>"
            _, _, L, lam, _ = integ.ctx.last_pass_samples(npix, 16)
            for pix in pixels:
                for s in range(16):
                    Lo, lo, _, _ = canon.pixel_sample(int(pix % f.width), int(pix // f.width), base + s)
                    g = s * npix + int(pix)
                    total += 1
                    exact += int(np.array_equal(L[g].view(np.uint32), Lo.view(np.uint32)) and
                                 np.array_equal(lam[g].view(np.uint32), lo.view(np.uint32)))
        print(f"headline-config replay (pixelsamples {P}, 64-bit ZSobol): {exact}/{total} samples bit-identical")
        assert exact == total
    finally:
        integ.close()


def test_fullsize_nanovdb_replay_at_the_driver_configuration(cloud):
    """disney-cloud's medium type at the bench's size: the S-cloud-1024 as a
    NanoVDBMedium (the tree classified from the device grid, pbrt's 64^3 majorant) at 720p with
    the driver's pixelsamples 16384, so k_paths runs its 64-bit-index ZSobol NanoVDB
    instantiation (checked by name). The 64^3 majorant is bit-exact against the oracle's
    (media.cpp:556-613), and a strided pixel subset of two 16-index passes (inside the N = 1
    timed range and at the top of the N = 8 range) is bit-identical to the canonical oracle,
    which walks its own hash-map tree (parity against NanoVDB itself unpinned)."""
    from acceleratedvolrenderer_amd import VolPathIntegrator, scenes
    from acceleratedvolrenderer_amd.launch import sample_plan
    from oracle import binding
    integ256, _ = cloud
    P = sample_plan(1, 20, 5, 64)[0]
    grid = scenes.vdb_grid(integ256.density_tensor)
    scene = scenes.s_cloud_vdb(grid, sampler="zsobol", spp=P, filter="gaussian")
    integ = VolPathIntegrator(scene, maxdepth=scenes.CLOUD_MAXDEPTH, spp=16, device=0)
    try:
        canon = binding.OracleRun(scene, max_depth=scenes.CLOUD_MAXDEPTH, seed=0, libm="canonical")
        assert integ.ctx.majorant(64 ** 3).view(np.uint32).tolist() == canon.majorant.view(np.uint32).tolist()
        f = scene.film
        npix = f.width * f.height
        pixels = np.arange(0, npix, 4099)
        exact = total = 0
        for base in (640, 8 * 20 * 64 - 16):
            integ.ctx.film_clear()
            integ.ctx.render(base, base + 16, 0, scenes.CLOUD_MAXDEPTH)
            assert integ.ctx.last_kernel() == "k_paths<false, true, 3, 3, false, false>"
            _, _, L, lam, _ = integ.ctx.last_pass_samples(npix, 16)
            for pix in pixels:
                for s in range(16):
                    Lo, lo, _, _ = canon.pixel_sample(int(pix % f.width), int(pix // f.width), base + s)
                    g = s * npix + int(pix)
                    total += 1
                    exact += int(np.array_equal(L[g].view(np.uint32), Lo.view(np.uint32)) and
                                 np.array_equal(lam[g].view(np.uint32), lo.view(np.uint32)))
        print(f"NanoVDB S-cloud-1024 replay ({len(grid.leaf_origins)} leaves, {len(grid.tile_values)} tiles, "
              f"pixelsamples {P}): {exact}/{total} samples bit-identical")
        assert exact == total
    finally:
        integ.close()


def test_fullsize_multipass_and_determinism(cloud):
    from acceleratedvolrenderer_amd import scenes
    integ, _ = cloud
    md = scenes.CLOUD_MAXDEPTH
    integ.ctx.film_clear()
    integ.ctx.render(0, 16, 0, md)
    integ.ctx.render(16, 32, 0, md)
    two = integ.film_sums()
    integ.ctx.film_clear()
    integ.ctx.render(0, 32, 0, md)
    one = integ.film_sums()
    integ.ctx.film_clear()
    integ.ctx.render(0, 32, 0, md)
    again = integ.film_sums()
    for a, b, c in zip(two, one, again):
        assert np.array_equal(a, b) and np.array_equal(b, c)
    assert float(one[1].sum()) > 0.9 * 1280 * 720 * 32 * 0.5   # Gaussian filter weights, every pixel sampled


def test_fullsize_fast_mode_at_the_tuned_majorant(cloud):
    """The bench's fast_mode leg at its configuration: hardware math and the 1^3 majorant
    avr_tune_majorant picks for the S-cloud-1024 (bench.py). On a strided pixel subset:
    per-pixel means of the hero-wavelength radiance track the platform oracle built with the
    same majorant (relative RMS <= 0.5 x the two-seed oracle noise), and the subset mean over
    more samples agrees with the oracle at pbrt's own 16^3 majorant within 4 standard errors."""
    import copy
    from acceleratedvolrenderer_amd import scenes
    from oracle import binding
    integ, host = cloud
    md = scenes.CLOUD_MAXDEPTH
    f = host.film
    npix = f.width * f.height
    pixels = np.arange(0, npix, 4099)
    host1 = copy.copy(host)
    host1.medium = copy.copy(host.medium)
    host1.medium.majorant_res = (1, 1, 1)
    plat = binding.OracleRun(host1, max_depth=md, seed=0)
    plat_b = binding.OracleRun(host1, max_depth=md, seed=1)
    integ.ctx.set_render_mode("fast")
    integ.ctx.set_majorant_res((1, 1, 1))
    try:
        gpu = []
        for p0 in (64, 80, 96, 112):
            integ.ctx.film_clear()
            integ.ctx.render(p0, p0 + 16, 0, md)
            _, _, L, _, _ = integ.ctx.last_pass_samples(npix, 16)
            gpu.append(np.stack([L[s * npix + pixels, 0] for s in range(16)], 1))
        gpu = np.concatenate(gpu, 1)                                      # (pixels, 64)
    finally:
        integ.ctx.set_render_mode("replay")
        integ.ctx.set_majorant_res((16, 16, 16))
    px, py = pixels % f.width, pixels // f.width
    per = lambda run, s0, n: np.array([[run.pixel_sample(int(x), int(y), s0 + s)[0][0] for s in range(n)]
                                       for x, y in zip(px, py)])
    o0, o1 = per(plat, 64, 16), per(plat_b, 64, 16)
    g, a, b = gpu[:, :16].mean(1), o0.mean(1), o1.mean(1)
    err = float(np.sqrt(np.mean((g - a) ** 2)) / np.sqrt(np.mean(a ** 2)))
    noise = float(np.sqrt(np.mean((b - a) ** 2)) / np.sqrt(np.mean(a ** 2)))
    # unbiasedness against pbrt's 16^3 majorant (replay streams of the canonical/platform oracle)
    ref = binding.OracleRun(host, max_depth=md, seed=0)
    r = per(ref, 64, 64)
    se = float(np.sqrt(gpu.var() / gpu.size + r.var() / r.size))
    print(f"full-size fast@1^3: subset rel RMS {err:.3e} (noise {noise:.3e}); mean {gpu.mean():.5f} vs "
          f"oracle@16^3 {r.mean():.5f} (se {se:.2e})")
    assert err <= 0.5 * noise
    assert abs(gpu.mean() - r.mean()) <= 4 * se

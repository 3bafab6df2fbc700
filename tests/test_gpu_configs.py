"""BASELINE.json configurations C2, C4 and C5 on the HIP path at their sizes (C3, the bench's
S-cloud-1024 at 720p, is tests/test_gpu_fullsize.py). Each is checked against the oracle on
a strided replay subset (canonical libm, every sample bit-identical, as
tests/test_gpu_parity.py) and through size-independent properties:

  C2  S-uniform 256^3 GridMedium, orthographic 512x512: Beer-Lambert mean of the absorber
      (integral of the trilinear density = 1 - 0.25/n, containers.h:822-835), white
      furnace (every sample L == 1), scatter-variant replay subset.
  C4  S-cloud-1024 at 1920x1080, ZSobol pixelsamples 1024, on ONE GPU: the eight sample
      shards [k spp/8, (k+1) spp/8) rendered one after another and summed in fp64 equal one
      unsharded render to summation order (rtol 1e-10), their last pass bit-identical, and
      a strided replay subset.
  C5  the emissive RGB-coefficient explosion as BASELINE names it — an RGBGridMedium of
      1024^3 {c0, c1, c2, scale} voxels for sigma_a / sigma_s / Le generated on the device
      (k_rgb_explosion), 1280x720 SpectralFilm, 4096 pixelsamples: majorant bit-exact and a
      replay subset; the emissive NanoVDB explosion over a 1024^3 index extent
      (scenes.explosion_vdb), same film: replay subset; and the emission-only absorber's line integral
      E[L(lambda)] = Le(lambda) (1 - exp(-sigma_a D)) through a uniform density block inside
      a uniform-temperature region (Le constant wherever sigma_a > 0).
Memory: C4 holds the 4 GiB grid, its 34.5 GB fat copy and a 4 GiB host copy for the oracle;
C5's RGB grids 48 GiB on the device and their 48 GiB host copy; C5's NanoVDB grids ~2 GB of
leaves per copy."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    torch.cuda.init()


def _replay_subset(integ, canon, first, ns, stride, max_pixels=None):
    """Fraction of bit-identical (L, lambda) samples of the last pass over every
    `stride`-th pixel, against oracle.pixel_sample."""
    f = integ.scene.film
    npix = f.width * f.height
    got_first, got_ns, L, lam, _ = integ.ctx.last_pass_samples(npix, ns)
    assert (got_first, got_ns) == (first, ns)
    pixels = np.arange(0, npix, stride)[:max_pixels]
    exact = total = 0
    for pix in pixels:
        for s in range(ns):
            Lo, lo, _, _ = canon.pixel_sample(int(pix % f.width), int(pix // f.width), first + s)
            g = s * npix + int(pix)
            total += 1
            exact += int(np.array_equal(L[g].view(np.uint32), Lo.view(np.uint32)) and
                         np.array_equal(lam[g].view(np.uint32), lo.view(np.uint32)))
    return exact, total


# ------------------------------------------------------------------------------------ C2
def test_c2_uniform_256_absorber_beer_lambert():
    from acceleratedvolrenderer_amd import VolPathIntegrator, scenes
    n, W, H, spp = 256, 512, 512, 16
    scene = scenes.s_uniform(n=n, width=W, height=H, variant="absorber")
    integ = VolPathIntegrator(scene, maxdepth=5, spp=spp, device=0)
    integ.render()
    _, ns, L, _, _ = integ.ctx.last_pass_samples(W * H, spp)
    assert ns == spp
    Lm = L.reshape(ns, H, W, 4)[:, 8:-8, 8:-8, :].astype(np.float64)
    want = np.exp(-(1 - 0.25 / n))
    cnt = Lm[..., 0].size
    tol = 4 * np.sqrt(want * (1 - want) / cnt)
    print(f"C2 absorber: mean L {Lm.mean():.6f} vs Beer-Lambert {want:.6f} (tol {tol:.2e}, {cnt} samples)")
    for c in range(4):
        assert abs(Lm[..., c].mean() - want) < tol
    rgb, w = integ.film_sums()
    assert np.all(w == spp)
    integ.close()


def test_c2_uniform_256_white_furnace():
    from acceleratedvolrenderer_amd import VolPathIntegrator, scenes
    n, W, H, spp = 256, 512, 512, 4
    scene = scenes.s_uniform(n=n, width=W, height=H, variant="furnace")
    integ = VolPathIntegrator(scene, maxdepth=1000, spp=spp, device=0)
    integ.render()
    _, ns, L, _, _ = integ.ctx.last_pass_samples(W * H, spp)
    assert ns == spp and np.all(L == 1.0)
    integ.close()


def test_c2_uniform_256_scatter_replay_subset():
    from acceleratedvolrenderer_amd import VolPathIntegrator, scenes
    from oracle import binding
    n, W, H, spp = 256, 512, 512, 4
    dens = (0.25 + np.random.default_rng(21).random((n, n, n), dtype=np.float32)).astype(np.float32)
    scene = scenes.s_uniform(n=n, width=W, height=H, variant="scatter", density=dens)
    integ = VolPathIntegrator(scene, maxdepth=5, spp=spp, device=0)
    integ.render()
    canon = binding.OracleRun(scene, max_depth=5, seed=0, libm="canonical")
    exact, total = _replay_subset(integ, canon, 0, spp, stride=521)
    print(f"C2 scatter 256^3 512x512: {exact}/{total} samples bit-identical")
    assert exact == total
    integ.close()


# ------------------------------------------------------------------------------------ C4
@pytest.fixture(scope="module")
def cloud1080():
    from acceleratedvolrenderer_amd import VolPathIntegrator, scenes, capi
    n = 1024
    density = torch.empty((n, n, n), dtype=torch.float32, device="cuda:0")
    gen = capi.Context(0)
    slab = n * n * 64
    for first in range(0, n ** 3, slab):
        gen.generate_cloud(density.data_ptr() + 4 * first, n, first, min(slab, n ** 3 - first))
    gen.sync()
    gen.close()
    scene = scenes.s_cloud(density, width=1920, height=1080, sampler="zsobol", spp=1024, filter="gaussian")
    # 16M paths per pass (the wavefront default; k_paths' own default is 64M): several passes
    # per render at 1080p, so the shard tests also cover pass splitting
    integ = VolPathIntegrator(scene, maxdepth=scenes.CLOUD_MAXDEPTH, spp=1024, device=0, max_paths=16 << 20)
    yield integ, density
    integ.close()


def test_c4_1080p_eight_sample_shards_sum_to_one_render(cloud1080):
    """C4's pixel/sample sharding over 8 GPUs, rehearsed on one: sum of the 8 shard films =
    the unsharded 1024-spp film (fp64, to summation order); each (pixel, sample) path is
    traced identically whichever shard renders it (last pass bit-identical)."""
    from acceleratedvolrenderer_amd import scenes
    from acceleratedvolrenderer_amd.integrator import shard_samples
    integ, _ = cloud1080
    md, spp, N = scenes.CLOUD_MAXDEPTH, 1024, 8
    npix = 1920 * 1080
    rgb_sh = np.zeros(3 * npix)
    w_sh = np.zeros(npix)
    for k in range(N):
        lo, hi = shard_samples(spp, k, N)
        integ.ctx.film_clear()
        integ.ctx.render(lo, hi, 0, md)
        r, w = integ.film_sums()
        rgb_sh += r
        w_sh += w
    first_sh, ns_sh, L_sh, lam_sh, _ = integ.ctx.last_pass_samples(npix, 64)
    integ.ctx.film_clear()
    integ.ctx.render(0, spp, 0, md)
    rgb1, w1 = integ.film_sums()
    first_1, ns_1, L_1, lam_1, _ = integ.ctx.last_pass_samples(npix, 64)
    assert (first_sh, ns_sh) == (first_1, ns_1)
    assert np.array_equal(L_sh.view(np.uint32), L_1.view(np.uint32))
    assert np.array_equal(lam_sh.view(np.uint32), lam_1.view(np.uint32))
    assert np.allclose(w_sh, w1, rtol=1e-10, atol=0) and float(w1.min()) > 0
    assert np.allclose(rgb_sh, rgb1, rtol=1e-10, atol=1e-300)
    img = integ.image(rgb1, w1)
    assert np.all(np.isfinite(img)) and float(img.mean()) > 0
    print(f"C4 1080p x 1024 spp: {npix * spp / 1e9:.2f} G samples per film, shards == unsharded")


def test_c4_1080p_replay_subset(cloud1080):
    from acceleratedvolrenderer_amd import scenes
    from oracle import binding
    integ, density = cloud1080
    md = scenes.CLOUD_MAXDEPTH
    integ.ctx.film_clear()
    integ.ctx.render(992, 1008, 0, md)      # passes of 8 sample indices at 1080p (16M paths)
    host = scenes.s_cloud(density.cpu().numpy(), width=1920, height=1080, sampler="zsobol", spp=1024,
                          filter="gaussian")
    canon = binding.OracleRun(host, max_depth=md, seed=0, libm="canonical")
    exact, total = _replay_subset(integ, canon, 1000, 8, stride=4591)
    print(f"C4 1080p replay: {exact}/{total} samples bit-identical")
    assert exact == total


# ------------------------------------------------------------------------------------ C5
@pytest.fixture(scope="module")
def explosion():
    from acceleratedvolrenderer_amd import scenes
    return scenes.explosion_vdb(1024)


def test_c5_explosion_1024_spectral_replay_subset(explosion):
    from acceleratedvolrenderer_amd import VolPathIntegrator, scenes
    from oracle import binding
    dens, temp = explosion
    scene = scenes.s_explosion(dens, temp, width=1280, height=720, spp=4096, Lescale=0.5)
    integ = VolPathIntegrator(scene, maxdepth=10, spp=4096, device=0)
    integ.ctx.film_clear()
    integ.ctx.render(0, 8, 0, 10)
    bs, bw = integ.spectral_sums()
    rgb, w = integ.film_sums()
    assert np.all(np.isfinite(bs)) and float(bs.sum()) > 0 and np.all(np.isfinite(rgb))
    canon = binding.OracleRun(scene, max_depth=10, seed=0, libm="canonical")
    exact, total = _replay_subset(integ, canon, 0, 8, stride=7919)
    print(f"C5 explosion 1024^3 NanoVDB spectral 720p: {exact}/{total} samples bit-identical")
    assert exact == total
    integ.close()


def test_c5_rgb_explosion_1024_spectral_majorant_and_replay_subset():
    from acceleratedvolrenderer_amd import VolPathIntegrator, scenes
    from oracle import binding
    n = 1024
    grids = scenes.rgb_explosion_grids(n, device=0)
    scene = scenes.s_rgb_explosion(*grids, spp=4096)
    md = scenes.CLOUD_MAXDEPTH
    integ = VolPathIntegrator(scene, maxdepth=md, spp=4096, device=0)
    integ.ctx.film_clear()
    integ.ctx.render(64, 72, 0, md)
    bs, bw = integ.spectral_sums()
    rgb, w = integ.film_sums()
    assert np.all(np.isfinite(bs)) and float(bs.sum()) > 0 and np.all(np.isfinite(rgb))
    maj = integ.ctx.majorant(16 ** 3)
    host = [g.cpu().numpy() for g in grids]
    del grids
    hscene = scenes.s_rgb_explosion(*host, spp=4096)
    canon = binding.OracleRun(hscene, max_depth=md, seed=0, libm="canonical")
    assert maj.view(np.uint32).tolist() == canon.majorant.view(np.uint32).tolist()
    exact, total = _replay_subset(integ, canon, 64, 8, stride=7919)
    print(f"C5 RGB-coefficient explosion 1024^3 spectral 720p: majorant bit-exact, {exact}/{total} samples "
          f"bit-identical, film sum {float(bs.sum()):.4e}")
    assert exact == total
    integ.close()


def _blackbody_norm(lam_nm, T):
    """BlackbodySpectrum(T)(lambda) (util/spectrum.h:69-80, 500-520) in f64."""
    c, h, kb = 299792458.0, 6.62606957e-34, 1.3806488e-23

    def B(l_nm):
        l = l_nm * 1e-9
        return (2 * h * c * c) / (l ** 5 * (np.exp((h * c) / (l * kb * T)) - 1))
    return B(lam_nm) / B(2.8977721e-3 / T * 1e9)


def test_c5_scale_emission_only_absorber_line_integral():
    """NanoVDB density block of ones (index [256, 768)^3 as 8^3 tiles) inside a temperature
    grid of constant T over the whole 1024^3 extent (tiles): along +z through the block's
    interior the density profile integrates to D = 512 voxels (index-space trilinear ramps
    of half a voxel each side, inside the bounds), and with sigma_s = 0 the VolPath emission
    estimator has E[L(lambda)] = Lescale B_T(lambda) (1 - exp(-sigma_a D))."""
    from acceleratedvolrenderer_amd import VolPathIntegrator
    from acceleratedvolrenderer_amd.scene import NanoVDBMedium, OrthographicCamera, RGBFilm, Scene
    from acceleratedvolrenderer_amd.vdb import NanoVDBGrid
    n, T, sa, les = 1024, 2200.0, 2.0, 0.75
    m = np.eye(4)
    m[0, 0] = m[1, 1] = m[2, 2] = 1.0 / n
    r = np.arange(256, 768, 128)
    bz, by, bx = np.meshgrid(r, r, r, indexing="ij")
    org = np.stack([bx.ravel(), by.ravel(), bz.ravel()], 1)
    dens = NanoVDBGrid(np.zeros((0, 3), np.int32), np.zeros((0, 8, 8, 8), np.float32), 0.0, org,
                       np.full(len(org), 128), np.ones(len(org), np.float32), [256, 256, 256, 767, 767, 767], m)
    r = np.arange(0, n, 256)
    bz, by, bx = np.meshgrid(r, r, r, indexing="ij")
    org = np.stack([bx.ravel(), by.ravel(), bz.ravel()], 1)
    temp = NanoVDBGrid(np.zeros((0, 3), np.int32), np.zeros((0, 8, 8, 8), np.float32), 0.0, org,
                       np.full(len(org), 256), np.full(len(org), T, np.float32), [0, 0, 0, n - 1, n - 1, n - 1], m)
    med = NanoVDBMedium(dens, temperature=temp, sigma_a=sa, sigma_s=0.0, Lescale=les)
    W = H = 256
    cam = OrthographicCamera(pos=(0.5, 0.5, -1.0), look=(0.5, 0.5, 0.0), up=(0.0, 1.0, 0.0),
                             screenwindow=(-0.2, 0.2, -0.2, 0.2))
    scene = Scene(cam, RGBFilm(W, H), med, [])
    spp = 16
    integ = VolPathIntegrator(scene, maxdepth=5, spp=spp, device=0)
    integ.render()
    _, ns, L, lam, _ = integ.ctx.last_pass_samples(W * H, spp)
    L = L.astype(np.float64)
    lam = lam.astype(np.float64)
    ratio = L / (les * _blackbody_norm(lam, T))
    want = 1 - np.exp(-sa * 512.0 / n)
    # each sample's four ratios are one estimate (shared path); MC noise from their spread
    per = ratio.mean(axis=1)
    tol = 4 * per.std() / np.sqrt(per.size) + 2e-3 * want   # + FastExp / float Blackbody slack
    print(f"C5-scale emission absorber: E[L/Le] {per.mean():.6f} vs 1 - exp(-tau) {want:.6f} (tol {tol:.2e})")
    assert abs(per.mean() - want) < tol
    integ.close()

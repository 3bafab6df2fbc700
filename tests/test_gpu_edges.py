"""GPU edge cases: degenerate films and sample ranges, ragged launches, path-length limits,
empty and single-voxel media, argument errors — each against the CPU oracle (per-sample
replay with the canonical transcendentals, as tests/test_gpu_parity.py) where it renders.
The reference's own tests do not cover these shapes; they pin the boundary's
behaviour: the oracle is the pbrt restatement, so a match means pbrt's result."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    torch.cuda.init()


def _replay(scene, maxdepth, spp, kernel):
    from acceleratedvolrenderer_amd import VolPathIntegrator
    from oracle import binding
    integ = VolPathIntegrator(scene, device=0, maxdepth=maxdepth, spp=spp, kernel=kernel)
    rgb, w = integ.render()
    f = scene.film
    npix = f.width * f.height
    _, _, L, lam, _ = integ.ctx.last_pass_samples(npix, spp)
    canon = binding.OracleRun(scene, max_depth=maxdepth, seed=0, libm="canonical")
    exact = 0
    for s in range(spp):
        for pix in range(npix):
            Lo, lo, _, _ = canon.pixel_sample(pix % f.width, pix // f.width, s)
            g = s * npix + pix
            exact += int(np.array_equal(L[g].view(np.uint32), Lo.view(np.uint32)) and
                         np.array_equal(lam[g].view(np.uint32), lo.view(np.uint32)))
    rgb_o, w_o = canon.render(0, spp, nthreads=4)
    return integ, exact / (spp * npix), rgb, w, rgb_o, w_o


def _scene(W, H, density, variant="scatter"):
    from acceleratedvolrenderer_amd import scenes
    return scenes.s_uniform(n=density.shape[0], width=W, height=H, variant=variant, density=density)


@pytest.mark.parametrize("kernel", ["persistent", "wavefront"])
@pytest.mark.parametrize("W,H,spp", [(1, 1, 1), (7, 3, 5), (65, 1, 3)], ids=["1x1", "ragged7x3", "row65"])
def test_degenerate_and_ragged_films(kernel, W, H, spp):
    dens = (0.2 + np.random.default_rng(W * 31 + H).random((6, 6, 6), dtype=np.float32)).astype(np.float32)
    integ, frac, rgb, w, rgb_o, w_o = _replay(_scene(W, H, dens), 6, spp, kernel)
    assert frac == 1.0
    assert np.array_equal(w, w_o) and np.array_equal(rgb, rgb_o)
    integ.close()


@pytest.mark.parametrize("kernel", ["persistent", "wavefront"])
@pytest.mark.parametrize("maxdepth", [0, 1, 1000])
def test_path_length_limits(kernel, maxdepth):
    """maxdepth 0: no scattering contributes beyond direct emission / escape; 1000: the
    furnace-like long paths (integrators.cpp:1042-1045 depth test)."""
    dens = np.full((4, 4, 4), 2.0, np.float32)
    integ, frac, rgb, w, rgb_o, w_o = _replay(_scene(8, 6, dens), maxdepth, 4, kernel)
    assert frac == 1.0
    assert np.array_equal(rgb, rgb_o)
    integ.close()


@pytest.mark.parametrize("kernel", ["persistent", "wavefront"])
@pytest.mark.parametrize("case", ["empty", "single_voxel", "half_empty"])
def test_empty_and_tiny_media(kernel, case):
    """All-zero density (every majorant cell zero: the zero-sigma_maj segment skip,
    media.h:760-768), a 1x1x1 grid, and a grid whose upper half is empty."""
    if case == "empty":
        dens = np.zeros((5, 5, 5), np.float32)
    elif case == "single_voxel":
        dens = np.full((1, 1, 1), 1.5, np.float32)
    else:
        dens = np.random.default_rng(3).random((8, 8, 8), dtype=np.float32)
        dens[4:] = 0
    integ, frac, rgb, w, rgb_o, w_o = _replay(_scene(9, 7, dens), 5, 4, kernel)
    assert frac == 1.0
    assert np.array_equal(rgb, rgb_o)
    if case == "empty":
        assert integ.stats()["medium_lookups"] == 0
    integ.close()


def test_empty_sample_range_and_argument_errors():
    from acceleratedvolrenderer_amd import VolPathIntegrator
    dens = np.ones((4, 4, 4), np.float32)
    integ = VolPathIntegrator(_scene(5, 4, dens), device=0, maxdepth=3, spp=2)
    integ.ctx.film_clear()
    integ.ctx.render(3, 3, 0, 3)          # empty range: no-op
    rgb, w = integ.film_sums()
    assert not rgb.any() and not w.any()
    with pytest.raises(RuntimeError, match="sample range"):
        integ.ctx.render(4, 2, 0, 3)
    with pytest.raises(RuntimeError, match="sample range"):
        integ.ctx.render(0, 1, 0, -1)
    integ.close()


@pytest.mark.parametrize("kernel", ["persistent", "wavefront"])
def test_zsobol_64bit_indices_replay_and_range_is_checked(kernel):
    """ZSobol indices past 2^32 (Morton(pixel) << log2(spp) | index: 4096 spp on a film
    whose rounded-up resolution is 2048 = 34 bits, config C5's regime) replay the oracle's
    64-bit GetSampleIndex / SobolSample bit for bit, with and without the pixel table;
    beyond SobolSample's 2^52 index range (sobolmatrices.h:16) the render fails instead of
    aliasing."""
    from acceleratedvolrenderer_amd import VolPathIntegrator, ZSobolSampler
    from acceleratedvolrenderer_amd.scene import Scene
    from oracle import binding
    dens = (0.3 + np.random.default_rng(4).random((6, 6, 6), dtype=np.float32)).astype(np.float32)
    base = _scene(1100, 3, dens)
    scene = Scene(base.camera, base.film, base.medium, base.lights, sampler=ZSobolSampler(1 << 12))
    canon = binding.OracleRun(scene, max_depth=5, seed=0, libm="canonical")
    for dims in (256, 0):
        integ = VolPathIntegrator(scene, device=0, maxdepth=5, spp=4096, kernel=kernel)
        integ.ctx.set_sampler_table(dims)
        integ.ctx.film_clear()
        integ.ctx.render(4090, 4096, 0, 5)
        npix = 1100 * 3
        first, ns, L, lam, _ = integ.ctx.last_pass_samples(npix, 6)
        assert (first, ns) == (4090, 6)
        exact = 0
        for s in range(ns):
            for pix in range(0, npix, 7):
                Lo, lo, _, _ = canon.pixel_sample(pix % 1100, pix // 1100, first + s)
                g = s * npix + pix
                exact += int(np.array_equal(L[g].view(np.uint32), Lo.view(np.uint32)) and
                             np.array_equal(lam[g].view(np.uint32), lo.view(np.uint32)))
        total = ns * len(range(0, npix, 7))
        print(f"zsobol 64-bit ({kernel}, table {dims}): {exact}/{total} bit-identical")
        assert exact == total
        integ.close()
    big = Scene(base.camera, _scene(40000, 1, dens).film, base.medium, base.lights, sampler=ZSobolSampler(1 << 21))
    integ = VolPathIntegrator(big, device=0, maxdepth=1, spp=1, kernel=kernel)
    with pytest.raises(RuntimeError, match="2\\^52"):
        integ.ctx.render(0, 1, 0, 1)
    integ.close()
    # a film whose rounded-up resolution exceeds 65536: Morton(pixel) needs more than the 32
    # bits of the pixel-digit table and of zsobol_upper, so the render is refused
    wide = Scene(base.camera, _scene(70000, 1, dens).film, base.medium, base.lights, sampler=ZSobolSampler(1))
    integ = VolPathIntegrator(wide, device=0, maxdepth=1, spp=1, kernel=kernel)
    with pytest.raises(RuntimeError, match="65536"):
        integ.ctx.render(0, 1, 0, 1)
    integ.close()


@pytest.mark.parametrize("kernel", ["persistent", "wavefront"])
def test_readback_is_ordered_after_an_asynchronous_render(kernel):
    """avr_render only enqueues on the context's (non-blocking) stream; the per-sample
    readback must still see the finished pass (it drains the stream first)."""
    from acceleratedvolrenderer_amd import VolPathIntegrator, scenes
    from oracle import binding
    dens = binding.cloud_grid(16)
    scene = scenes.s_cloud(dens, width=40, height=24)
    integ = VolPathIntegrator(scene, device=0, maxdepth=scenes.CLOUD_MAXDEPTH, spp=8, kernel=kernel)
    integ.ctx.render(8, 16, 0, scenes.CLOUD_MAXDEPTH)        # no sync before the readback
    _, _, L, _, _ = integ.ctx.last_pass_samples(40 * 24, 8)
    canon = binding.OracleRun(scene, max_depth=scenes.CLOUD_MAXDEPTH, seed=0, libm="canonical")
    same = sum(np.array_equal(L[s * 960 + p].view(np.uint32),
                              canon.pixel_sample(p % 40, p // 40, 8 + s)[0].view(np.uint32))
               for s in range(8) for p in range(0, 960, 7))
    assert same == 8 * len(range(0, 960, 7))
    integ.close()


def test_film_reduce_rccl_single_gpu():
    """avr_film_reduce_rccl with one context (the 1-GPU box): the root film is its own sum;
    a second context on the same device is refused (one context per GPU)."""
    from acceleratedvolrenderer_amd import VolPathIntegrator, capi
    dens = np.random.default_rng(4).random((6, 6, 6), dtype=np.float32)
    a = VolPathIntegrator(_scene(12, 8, dens), device=0, maxdepth=4, spp=4)
    b = VolPathIntegrator(_scene(12, 8, dens), device=0, maxdepth=4, spp=4)
    rgb, w = a.render()
    capi.film_reduce_rccl([a.ctx], root=0)
    rgb2, w2 = a.film_sums()
    assert np.array_equal(rgb, rgb2) and np.array_equal(w, w2)
    with pytest.raises(RuntimeError, match="one context per GPU"):
        capi.film_reduce_rccl([a.ctx, b.ctx], root=0)
    with pytest.raises(RuntimeError, match="context list"):
        capi.film_reduce_rccl([a.ctx], root=1)
    a.close()
    b.close()


def test_volpathcustom_maxdepth_override_renders_the_override_depth():
    """a21: Integrator::Create("volpathcustom") with pbrt's --maxdepth (src/graph/
    volpath_custom.cpp:736-749) renders exactly what maxdepth=<override> renders; the
    scene file's maxdepth is ignored. Bit-identical films, and different from the file's."""
    from acceleratedvolrenderer_amd import VolPathIntegrator
    dens = np.full((4, 4, 4), 2.0, np.float32)
    scene = _scene(8, 6, dens)
    a = VolPathIntegrator.create("volpathcustom", {"maxdepth": 50, "pixelsamples": 8}, scene, device=0,
                                 maxdepth_override=2)
    assert a.maxdepth == 2
    rgb_a, w_a = a.render()
    b = VolPathIntegrator(scene, maxdepth=2, spp=8, device=0)
    rgb_b, w_b = b.render()
    c = VolPathIntegrator.create("volpath", {"maxdepth": 50, "pixelsamples": 8}, scene, device=0,
                                 maxdepth_override=2)
    rgb_c, _ = c.render()
    assert np.array_equal(rgb_a, rgb_b) and np.array_equal(w_a, w_b)
    assert not np.array_equal(rgb_a, rgb_c)
    for x in (a, b, c):
        x.close()


def test_wavefront_ray_binning_changes_order_not_results():
    """N1 ray binning (avr_set_ray_binning): the medium and shadow queues are counting-sorted
    by (majorant cell, octant) before each launch; every path's arithmetic is unchanged, so the
    film and the work counters are identical to the unsorted wavefront run (and to k_paths)."""
    from acceleratedvolrenderer_amd import VolPathIntegrator, scenes
    from oracle import binding
    dens = binding.cloud_grid(32)
    scene = scenes.s_cloud(dens, width=48, height=27)
    runs = []
    for kernel, binning in (("wavefront", 0), ("wavefront", 1), ("persistent", 0)):
        integ = VolPathIntegrator(scene, maxdepth=scenes.CLOUD_MAXDEPTH, spp=8, seed=0, device=0, kernel=kernel)
        integ.ctx.set_ray_binning(binning)
        rgb, w = integ.render()
        st = integ.stats()
        runs.append((rgb, w, st))
        integ.close()
    (r0, w0, s0), (r1, w1, s1), (r2, w2, _) = runs
    assert np.array_equal(r0, r1) and np.array_equal(w0, w1)
    assert np.array_equal(r0, r2) and np.array_equal(w0, w2)
    for k in ("medium_lookups", "shadow_lookups", "shadow_items", "medium_items_in"):
        assert s0[k] == s1[k], k
    assert s1["ms_binning"] > 0 and s0["ms_binning"] == 0


def test_nanovdb_medium_from_nvdb_file_renders_identically(tmp_path):
    """f1: a NanoVDBMedium read back from an .nvdb file (NanoVDBMedium::Create's readGrid,
    media.cpp:487-509) renders bit-identically to the tree it was written from."""
    from acceleratedvolrenderer_amd import VolPathIntegrator, scenes
    from acceleratedvolrenderer_amd.vdb import NanoVDBGrid
    from oracle import binding
    dens = binding.cloud_grid(32)
    g = scenes.vdb_grid(dens)
    p = tmp_path / "cloud.nvdb"
    g.write_nvdb(p)
    r = NanoVDBGrid.read_nvdb(p)
    films = []
    for grid in (g, r):
        scene = scenes.s_cloud_vdb(grid, width=40, height=24)
        integ = VolPathIntegrator(scene, maxdepth=scenes.CLOUD_MAXDEPTH, spp=4, seed=0, device=0)
        films.append(integ.render())
        integ.close()
    assert np.array_equal(films[0][0], films[1][0]) and np.array_equal(films[0][1], films[1][1])


@pytest.mark.parametrize("mres", [None, 21, 70])
def test_nanovdb_majorant_occupancy_level_changes_nothing(mres):
    """The coarse occupancy level of NanoVDB's majorant in LDS (avr_set_majorant_occupancy):
    majorant-0 cells read a trailing zero instead of their own 0 — the films and work counters
    equal the run without the level and the wavefront kernels' run. Resolutions: pbrt's 64^3,
    an odd 21^3 (pairs straddle rows, a ragged last word) and 70^3 (more cells than the LDS
    level holds: no level)."""
    from acceleratedvolrenderer_amd import VolPathIntegrator, scenes
    from oracle import binding
    dens = binding.cloud_grid(32)
    g = scenes.vdb_grid(dens)
    runs = []
    for kernel, occ in (("persistent", 1), ("persistent", 0), ("wavefront", 1)):
        scene = scenes.s_cloud_vdb(g, width=40, height=24)
        if mres:
            scene.medium.majorant_res = (mres,) * 3
        integ = VolPathIntegrator(scene, maxdepth=scenes.CLOUD_MAXDEPTH, spp=4, seed=0, device=0, kernel=kernel)
        integ.ctx.set_majorant_occupancy(occ)
        rgb, w = integ.render()
        runs.append((rgb, w, integ.stats()))
        integ.close()
    (r0, w0, s0), (r1, w1, s1), (r2, w2, _) = runs
    assert np.array_equal(r0, r1) and np.array_equal(w0, w1)
    assert np.array_equal(r0, r2) and np.array_equal(w0, w2)
    for k in ("medium_lookups", "shadow_lookups", "medium_dda_steps"):
        assert s0[k] == s1[k], k


def test_density_fetch_kernel_and_lookup_trace():
    """The standalone density fetch (avr_density_fetch) is SampledGrid::Lookup bit for bit (oracle
    grid_lookup), in both grid layouts; the wavefront lookup trace records one point per
    density fetch the kernels' work counters report."""
    from acceleratedvolrenderer_amd import VolPathIntegrator, scenes
    from oracle import binding
    dens = binding.cloud_grid(24)
    for layout in ("fat", "linear", "brick"):
        scene = scenes.s_cloud(dens, width=40, height=24)
        integ = VolPathIntegrator(scene, maxdepth=scenes.CLOUD_MAXDEPTH, spp=4, seed=0, device=0, kernel="wavefront",
                                  grid_layout=layout)
        cap = 1 << 20
        pts = torch.zeros((cap, 4), dtype=torch.float32, device="cuda:0")
        cnt = torch.zeros(1, dtype=torch.int64, device="cuda:0")
        integ.ctx.record_lookups(pts.data_ptr(), cap, cnt.data_ptr())
        integ.render()
        st = integ.stats()
        integ.ctx.record_lookups(0, 0, 0)
        n = int(cnt.item())
        assert n == st["medium_lookups"] + st["shadow_lookups"] and 0 < n <= cap
        out = torch.empty(n, dtype=torch.float32, device="cuda:0")
        ms = integ.ctx.density_fetch(pts.data_ptr(), n, out.data_ptr())
        assert ms > 0
        got = out.cpu().numpy()
        p = pts[:n].cpu().numpy()
        L = binding.lib()
        for i in range(0, n, max(1, n // 2000)):
            want = L.oracle_grid_lookup(binding.fp(dens), 24, 24, 24, float(p[i, 0]), float(p[i, 1]), float(p[i, 2]))
            assert np.float32(want).view(np.uint32) == got[i].view(np.uint32), (layout, i)
        integ.close()


@pytest.mark.parametrize("sampler", ["zsobol", "independent"])
def test_pixel_order_changes_order_not_results(sampler):
    """avr_set_pixel_order (N1: k_paths hands pixels to lanes sorted by the majorant cell of
    the camera ray's entry): the film and every sample are bit-identical to scanline order."""
    from acceleratedvolrenderer_amd import VolPathIntegrator, scenes
    from oracle import binding
    dens = binding.cloud_grid(24)
    scene = scenes.s_cloud(dens, width=40, height=24, sampler=sampler, spp=64, filter="gaussian")
    integ = VolPathIntegrator(scene, maxdepth=scenes.CLOUD_MAXDEPTH, spp=8, seed=0, device=0)
    rgb, w = integ.render()
    _, _, L, lam, pdf = integ.ctx.last_pass_samples(40 * 24, 8)
    wts = integ.ctx.last_pass_weights(40 * 24, 8)
    order = integ.entry_cell_order()
    assert sorted(order.tolist()) == list(range(40 * 24)) and order.tolist() != list(range(40 * 24))
    integ.ctx.set_pixel_order(order)
    rgb2, w2 = integ.render()
    _, _, L2, lam2, pdf2 = integ.ctx.last_pass_samples(40 * 24, 8)
    assert np.array_equal(rgb, rgb2) and np.array_equal(w, w2)
    for a, b in ((L, L2), (lam, lam2), (pdf, pdf2)):
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    assert np.array_equal(wts, integ.ctx.last_pass_weights(40 * 24, 8))
    with pytest.raises(RuntimeError):
        integ.ctx.set_pixel_order(np.zeros(40 * 24, np.int32))   # not a permutation
    integ.ctx.set_pixel_order(None)
    rgb3, _ = integ.render()
    assert np.array_equal(rgb, rgb3)
    integ.close()


@pytest.mark.parametrize("kernel", ["persistent", "wavefront"])
def test_film_nan_inf_guard_with_overflowing_radiance(kernel):
    """The NaN / Inf guard before RGBFilm::AddSample (integrators.cpp:272-282): a sample whose
    L.y(lambda) overflows is dropped (L = 0). An emissive medium whose Lescale spans 1e26..1e38
    along x puts samples below k_film's finite-y bound (no divisions) and between the bound and
    FLT_MAX (the exact guard evaluates y and keeps or drops them; sensor RGB components may
    overflow to inf in kept samples, as in pbrt): the GPU film must equal the canonical
    oracle's, sample for sample and sum for sum (inf included)."""
    from acceleratedvolrenderer_amd import scenes
    from acceleratedvolrenderer_amd.scene import GridMedium
    n, W, H, spp = 8, 24, 16, 4
    dens = (0.5 + np.random.default_rng(11).random((n, n, n), dtype=np.float32)).astype(np.float32)
    scene = _scene(W, H, dens, variant="emissive")
    x = np.linspace(0.0, 1.0, n)
    les = np.broadcast_to((10.0 ** (26.0 + 12.0 * x)).astype(np.float32), (n, n, n)).copy()
    m = scene.medium
    scene.medium = GridMedium(dens, sigma_a=0.6, sigma_s=1.5, g=-0.2, Le=(0.5 + np.linspace(0, 1, 471) ** 2)
                              .astype(np.float32), Lescale=les)
    del m
    integ, frac, rgb, w, rgb_o, w_o = _replay(scene, 4, spp, kernel)
    _, _, L, _, _ = integ.ctx.last_pass_samples(W * H, spp)
    big = np.max(np.abs(L), axis=1)
    print(f"{kernel}: {int(np.sum(big < 1e30))} samples < 1e30, {int(np.sum((big >= 1e30) & np.isfinite(big)))} "
          f"in [1e30, FLT_MAX], {int(np.sum(~np.isfinite(big)))} non-finite; replay {frac:.4f}")
    assert np.sum(big < 1e30) > 0 and np.sum((big >= 1e33) & np.isfinite(big)) > 0
    assert not np.isfinite(rgb_o).all(), "some kept samples overflow a sensor RGB component"
    assert frac == 1.0
    assert np.array_equal(w, w_o) and np.array_equal(rgb, rgb_o, equal_nan=True)
    integ.close()


def test_pass_tables_built_ahead_change_nothing():
    """avr_set_pass_table_ahead: the next pass's ZSobol pass table built on the side stream while
    this pass runs. Films bit-identical with it on and off for per-pass calls in order (every
    pass after the first uses the table built ahead), out of order and pbrt's doubling waves
    (the keys differ: those passes build in front of their camera stage), and one call of six
    passes (max_paths), which also equals the in-order per-pass calls; calls with a stride of 2
    passes (a rank of a sample shard: the table ahead follows the stride)."""
    from acceleratedvolrenderer_amd import VolPathIntegrator, scenes
    from oracle import binding
    dens = binding.cloud_grid(24)
    W, H, S = 40, 24, 8

    def run(ahead, seq, max_paths=0):
        scene = scenes.s_cloud(dens, width=W, height=H, sampler="zsobol", spp=64, filter="gaussian")
        integ = VolPathIntegrator(scene, maxdepth=scenes.CLOUD_MAXDEPTH, spp=64, seed=0, device=0,
                                  max_paths=max_paths)
        integ.ctx.set_pass_table_ahead(ahead)
        integ.ctx.film_clear()
        for b, e in seq:
            integ.ctx.render(b, e, 0, scenes.CLOUD_MAXDEPTH)
        out = integ.film_sums()
        integ.close()
        return out

    def same(a, b):
        return np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])

    in_order = [(k * S, (k + 1) * S) for k in range(6)]
    strided = [(k * 2 * S, k * 2 * S + S) for k in range(4)]   # a rank of a 2-way sample shard
    seqs = [in_order, [(16, 24), (0, 8), (8, 16), (32, 40), (24, 32)], [(0, 1), (1, 2), (2, 4), (4, 8), (8, 16), (16, 32)],
            strided]
    per_pass = []
    for seq in seqs:
        a, b = run(1, seq), run(0, seq)
        assert same(a, b), seq
        assert a[1].sum() > 0
        per_pass.append(a)
    one_a, one_b = run(1, [(0, 6 * S)], max_paths=S * W * H), run(0, [(0, 6 * S)], max_paths=S * W * H)
    assert same(one_a, one_b)
    assert same(one_a, per_pass[0])

"""The synthetic inputs of BASELINE.md §2 (the disney-cloud assets are not available offline).

S-uniform  (config C2): GridMedium n^3 of 1.0 on [0,1]^3, orthographic camera looking down +z
           at the z=0 face through a screen window equal to that face, 512x512.
           variants: "absorber" (sigma_a=1, sigma_s=0, uniform infinite light Le=1 -> analytic
           Beer-Lambert), "furnace" (sigma_a=0, sigma_s=4, uniform infinite Le=1, maxdepth 1000
           -> L = Le), "scatter" (sigma_a=0.5, sigma_s=2, distant light + sky), "chromatic"
           (wavelength-dependent sigma_a/sigma_s ramps, distant light + sky), "emissive" /
           "emissive_chromatic" (gray / chromatic sigma, Le with a spatially varying Lescale).
S-cloud    (metric input): GridMedium n^3 filled with CloudMedium::Density (media.h:496-520,
           density 1, wispiness 1, frequency 5) at voxel centres; sigma_a=0, sigma_s=1,
           scale 4 (albedo 1), g 0.877, distant light + dim sky, perspective 1280x720, maxdepth 100.
S-sphere   (SURVEY §8f row 3, medium interfaces) S-uniform's medium and variants bounded by an
           interface sphere (a shape with no material, MediumInterface inside = the medium),
           centre and radius in world space; by default inscribed in the [0,1]^3 grid box.
S-vdb      NanoVDBMedium over a sparse copy of a dense grid (index i at world i / n, so the
           world bbox of an n^3 grid is [0, 1]^3), S-uniform's camera and light variants.
"""
import numpy as np

from . import spectra
from .scene import (GridMedium, DistantLight, UniformInfiniteLight, OrthographicCamera, PerspectiveCamera, RGBFilm,
                    Scene, BoxFilter, GaussianFilter, IndependentSampler, ZSobolSampler, NanoVDBMedium)
from .vdb import NanoVDBGrid

CLOUD_G = 0.877
CLOUD_MAXDEPTH = 100


def s_uniform(n=256, width=512, height=512, variant="absorber", density=None):
    if density is None:
        density = np.ones((n, n, n), np.float32)
    if variant == "absorber":
        med = GridMedium(density, sigma_a=1.0, sigma_s=0.0, g=0.0)
        lights = [UniformInfiniteLight(L=1.0, scale=float(spectra.spectrum_to_photometric(spectra.constant(1.0))))]
    elif variant == "furnace":
        med = GridMedium(density, sigma_a=0.0, sigma_s=4.0, g=0.0)
        lights = [UniformInfiniteLight(L=1.0, scale=float(spectra.spectrum_to_photometric(spectra.constant(1.0))))]
    elif variant == "scatter":
        med = GridMedium(density, sigma_a=0.5, sigma_s=2.0, g=0.3)
        lights = [DistantLight(from_=(-1.0, 1.0, -1.0), to=(0.0, 0.0, 0.0), scale=2.0),
                  UniformInfiniteLight(scale=0.25)]
    elif variant in ("chromatic", "emissive", "emissive_chromatic"):
        # sigma tables that vary over 360..830 nm exercise the 4-wavelength (non-gray) path
        ramp = np.linspace(0.0, 1.0, spectra.N, dtype=np.float32)
        chrom = variant != "emissive"
        sa = (0.2 + 1.0 * ramp).astype(np.float32) if chrom else 0.6
        ss = (2.5 - 2.0 * ramp).astype(np.float32) if chrom else 1.5
        le = les = None
        if variant != "chromatic":
            le = (0.5 + ramp * ramp).astype(np.float32)
            d = np.asarray(density) if not hasattr(density, "data_ptr") else None
            shape = d.shape if d is not None else tuple(int(x) for x in density.shape)
            z, y, x = np.meshgrid(*(np.linspace(0.0, 1.0, k, dtype=np.float32) for k in shape), indexing="ij")
            les = (2.0 * x * (1.0 - y) + 0.25 * z).astype(np.float32)
        med = GridMedium(density, sigma_a=sa, sigma_s=ss, g=-0.2, Le=le, Lescale=les)
        lights = [DistantLight(from_=(1.0, 1.0, -1.0), to=(0.0, 0.0, 0.0), scale=1.5),
                  UniformInfiniteLight(scale=0.2)]
    else:
        raise ValueError(variant)
    cam = OrthographicCamera(pos=(0.5, 0.5, -1.0), look=(0.5, 0.5, 0.0), up=(0.0, 1.0, 0.0),
                             screenwindow=(-0.5, 0.5, -0.5, 0.5))
    film = RGBFilm(width, height)
    return Scene(cam, film, med, lights)


def s_sphere(n=32, width=64, height=64, variant="scatter", density=None, center=(0.5, 0.5, 0.5), radius=0.45,
             camera="orthographic"):
    """S-uniform's scene with the medium bounded by an interface sphere instead of its box."""
    base = s_uniform(n=n, width=width, height=height, variant=variant, density=density)
    cam = base.camera
    if camera == "perspective":
        cam = PerspectiveCamera(fov=50.0, pos=(0.9, 0.7, -1.1), look=(0.5, 0.5, 0.5), up=(0.0, 1.0, 0.0))
    return Scene(cam, base.film, base.medium, base.lights, sampler=base.sampler,
                 interface_sphere=(tuple(float(v) for v in center), float(radius)))


def box_mesh(p0, p1, rotate_deg=0.0):
    """A closed box triangle mesh (pbrt `Shape "trianglemesh"`) from p0 to p1, optionally rotated
    about the y axis through its centre: (vertices (8, 3), triangles (12, 3))."""
    p0, p1 = np.asarray(p0, np.float64), np.asarray(p1, np.float64)
    v = np.array([[x, y, z] for z in (p0[2], p1[2]) for y in (p0[1], p1[1]) for x in (p0[0], p1[0])])
    if rotate_deg:
        c = (p0 + p1) / 2
        a = np.radians(rotate_deg)
        r = np.array([[np.cos(a), 0, np.sin(a)], [0, 1, 0], [-np.sin(a), 0, np.cos(a)]])
        v = (v - c) @ r.T + c
    t = np.array([[0, 2, 1], [1, 2, 3], [4, 5, 6], [5, 7, 6], [0, 1, 4], [1, 5, 4], [2, 6, 3], [3, 6, 7],
                  [0, 4, 2], [2, 4, 6], [1, 3, 5], [3, 7, 5]])
    return v, t


def s_mesh_interface(n=32, width=64, height=64, variant="scatter", density=None, mesh=None, camera="orthographic"):
    """S-uniform's medium bounded by a convex triangle-mesh interface (default: a box rotated by
    30 degrees inside the grid box)."""
    base = s_uniform(n=n, width=width, height=height, variant=variant, density=density)
    if mesh is None:
        mesh = box_mesh((0.2, 0.15, 0.2), (0.8, 0.85, 0.8), rotate_deg=30.0)
    cam = base.camera
    if camera == "perspective":
        cam = PerspectiveCamera(fov=50.0, pos=(0.9, 0.7, -1.1), look=(0.5, 0.5, 0.5), up=(0.0, 1.0, 0.0))
    return Scene(cam, base.film, base.medium, base.lights, sampler=base.sampler, interface_mesh=mesh)


def vdb_grid(density, index_to_world=None, index_min=(0, 0, 0), background=0.0):
    """Sparse NanoVDB-style copy of a dense (nz, ny, nx) grid; default map: index i at world
    i / n per axis. A torch tensor (e.g. a device-generated grid) is classified where it lives."""
    d = density if hasattr(density, "data_ptr") else np.asarray(density, np.float32)
    if index_to_world is None:
        index_to_world = np.eye(4)
        index_to_world[0, 0], index_to_world[1, 1], index_to_world[2, 2] = (1.0 / d.shape[2], 1.0 / d.shape[1],
                                                                            1.0 / d.shape[0])
    return NanoVDBGrid.from_dense(d, index_min=index_min, index_to_world=index_to_world, background=background)


def s_vdb(density, width=64, height=64, variant="scatter", temperature=None, index_to_world=None, **medium):
    """NanoVDBMedium scene: `density` dense (nz, ny, nx) or a NanoVDBGrid; `temperature`
    likewise (optional). variants as S-uniform's ("absorber", "furnace", "scatter")."""
    grid = density if isinstance(density, NanoVDBGrid) else vdb_grid(density, index_to_world)
    tgrid = None
    if temperature is not None:
        tgrid = temperature if isinstance(temperature, NanoVDBGrid) else vdb_grid(temperature, index_to_world)
    base = s_uniform(n=1, width=width, height=height, variant=variant)
    kw = {"absorber": dict(sigma_a=1.0, sigma_s=0.0), "furnace": dict(sigma_a=0.0, sigma_s=4.0),
          "scatter": dict(sigma_a=0.5, sigma_s=2.0, g=0.3)}[variant]
    kw.update(medium)
    med = NanoVDBMedium(grid, temperature=tgrid, **kw)
    return Scene(base.camera, base.film, med, base.lights)


def cloud_medium(density):
    return GridMedium(density, sigma_a=0.0, sigma_s=1.0, scale=4.0, g=CLOUD_G)


def s_cloud(density, width=1280, height=720, fov=45.0, sampler="independent", spp=16, filter="box"):
    """sampler "zsobol" / filter "gaussian" are pbrt's defaults (scene.cpp:93-94) and
    BASELINE.md §2's S-cloud configuration; "independent" / "box" replay-friendly ones."""
    med = cloud_medium(density)
    # key light from upper right behind the cloud (silver lining with g = 0.877) plus a dim sky
    lights = [DistantLight(from_=(0.7, 1.0, 0.6), to=(0.0, 0.0, 0.0), scale=3.0), UniformInfiniteLight(scale=0.15)]
    # framed so the 16:9 view is filled by the [0,1]^3 medium box
    cam = PerspectiveCamera(fov=fov, pos=(0.5, 0.42, -0.75), look=(0.5, 0.38, 0.5), up=(0.0, 1.0, 0.0))
    film = RGBFilm(width, height, filter=GaussianFilter() if filter == "gaussian" else BoxFilter())
    smp = ZSobolSampler(spp) if sampler == "zsobol" else IndependentSampler(spp)
    return Scene(cam, film, med, lights, sampler=smp)


def cloud_vdb_medium(grid):
    """The S-cloud medium as a NanoVDBMedium (the disney-cloud's medium type, C3/C4): same
    sigma (sigma_a 0, sigma_s 1 x scale 4) and g over a sparse tree of the cloud density."""
    return NanoVDBMedium(grid, sigma_a=0.0, sigma_s=1.0, scale=4.0, g=CLOUD_G)


def s_cloud_vdb(density, width=1280, height=720, fov=45.0, sampler="independent", spp=16, filter="box"):
    """S-cloud framing and lights over a NanoVDBMedium built from a dense (n, n, n) host
    density (index i at world i / n) or a NanoVDBGrid."""
    grid = density if isinstance(density, NanoVDBGrid) else vdb_grid(density)
    base = s_cloud(np.zeros((1, 1, 1), np.float32), width, height, fov, sampler, spp, filter)
    return Scene(base.camera, base.film, cloud_vdb_medium(grid), base.lights, sampler=base.sampler)


def explosion_vdb(n=1024, radius=0.36, t_max=3000.0, seed=7):
    """Synthetic stand-in for BASELINE config C5's emissive explosion (1024^3 NanoVDB; the
    asset is absent): density and temperature NanoVDBGrids over an n^3 index extent (index i
    at world i / n), leaves only inside a sphere of `radius` (world units) around the centre.
    Radial profiles with a deterministic per-leaf perturbation:
      density     = clamp(1.2 (1 - r/R) + 0.15 w, 0, 1)
      temperature = t_max (1 - r/R)^2 (1 + 0.1 w)   (K, > 100 K only well inside)
    where w in [-1, 1) is hashed from the leaf origin. Built leaf-vectorised on the host:
    (4/3) pi (R n / 8)^3 leaves (~390k, 0.8 GB per grid at n = 1024)."""
    nb = n // 8
    R = radius * n
    c = n / 2.0
    bz, by, bx = np.meshgrid(np.arange(nb), np.arange(nb), np.arange(nb), indexing="ij")
    org = np.stack([bx.ravel(), by.ravel(), bz.ravel()], 1).astype(np.int64) * 8
    centre = org + 4.0
    keep = np.sqrt(((centre - c) ** 2).sum(1)) < R + 8.0
    org = org[keep]
    del bx, by, bz, centre
    h = (org[:, 0] * 73856093) ^ (org[:, 1] * 19349663) ^ (org[:, 2] * 83492791) ^ seed
    w = ((h % 2000) / 1000.0 - 1.0).astype(np.float32)[:, None, None, None]
    l = np.arange(8, dtype=np.float32)
    # leaf values x-major [x][y][z]
    lx, ly, lz = np.meshgrid(l, l, l, indexing="ij")
    dens = np.empty((len(org), 8, 8, 8), np.float32)
    temp = np.empty((len(org), 8, 8, 8), np.float32)
    step = 65536
    for i in range(0, len(org), step):
        o = org[i:i + step].astype(np.float32)
        dx = o[:, 0, None, None, None] + lx - np.float32(c)
        dy = o[:, 1, None, None, None] + ly - np.float32(c)
        dz = o[:, 2, None, None, None] + lz - np.float32(c)
        q = np.maximum(np.float32(0), np.float32(1) - np.sqrt(dx * dx + dy * dy + dz * dz) / np.float32(R))
        ww = w[i:i + step]
        dens[i:i + step] = np.clip(np.float32(1.2) * q + np.float32(0.15) * ww * (q > 0), 0, 1)
        temp[i:i + step] = np.float32(t_max) * q * q * (np.float32(1) + np.float32(0.1) * ww)
    m = np.eye(4)
    m[0, 0] = m[1, 1] = m[2, 2] = 1.0 / n
    bb = np.array([0, 0, 0, n - 1, n - 1, n - 1], np.int32)
    org32 = org.astype(np.int32)
    return (NanoVDBGrid(org32, dens, 0.0, index_bbox=bb, index_to_world=m),
            NanoVDBGrid(org32, temp, 0.0, index_bbox=bb, index_to_world=m))


def s_explosion(density, temperature, width=1280, height=720, sampler="zsobol", spp=256, nbuckets=16,
                Lescale=1.0, **medium):
    """C5 stand-in scene: an emissive NanoVDBMedium (density + temperature grids) seen by a
    perspective camera on a SpectralFilm (C5 is spectral), a dim sky for scattered light."""
    from .scene import SpectralFilm
    med = NanoVDBMedium(density, temperature=temperature, sigma_a=medium.pop("sigma_a", 1.0),
                        sigma_s=medium.pop("sigma_s", 1.0), scale=medium.pop("scale", 4.0),
                        g=medium.pop("g", 0.2), Lescale=Lescale, **medium)
    cam = PerspectiveCamera(fov=45.0, pos=(0.5, 0.5, -0.9), look=(0.5, 0.5, 0.5), up=(0.0, 1.0, 0.0))
    film = SpectralFilm(width, height, nbuckets=nbuckets, filter=GaussianFilter())
    smp = ZSobolSampler(spp) if sampler == "zsobol" else IndependentSampler(spp)
    return Scene(cam, film, med, [UniformInfiniteLight(scale=0.05)], sampler=smp)


def rgb_explosion_grids(n=1024, device=0):
    """The synthetic RGB-coefficient explosion (BASELINE config C5's "emissive RGB-coefficient
    explosion volume", asset absent) generated on the device by k_rgb_explosion: three
    float32 (n, n, n, 4) tensors of {c0, c1, c2, scale} — sigma_a, sigma_s (RGBUnboundedSpectrum)
    and Le (RGBIlluminantSpectrum) — 16 B per voxel per field (48 GiB at n = 1024)."""
    import torch
    from . import capi
    grids = [torch.empty((n, n, n, 4), dtype=torch.float32, device=f"cuda:{device}") for _ in range(3)]
    ctx = capi.Context(device)
    try:
        slab = n * n * 32
        for first in range(0, n ** 3, slab):
            cnt = min(slab, n ** 3 - first)
            ctx.generate_rgb_explosion(*(t.data_ptr() + 16 * first for t in grids), n, first, cnt)
        ctx.sync()
    finally:
        ctx.close()
    return grids


def s_rgb_explosion(sigma_a, sigma_s, Le, width=1280, height=720, sampler="zsobol", spp=4096, nbuckets=16,
                    filter="gaussian"):
    """C5 as an RGBGridMedium: the coefficient grids of rgb_explosion_grids (device tensors, or
    their host copies for the oracle) on the unit cube, g 0.2, seen like s_explosion on a
    SpectralFilm (C5 is spectral; nbuckets 0 = RGBFilm) with a dim sky."""
    from .scene import SpectralFilm, RGBGridMedium
    med = RGBGridMedium(sigma_a_coeffs=sigma_a, sigma_s_coeffs=sigma_s, Le_coeffs=Le, scale=1.0, g=0.2, Lescale=1.0)
    cam = PerspectiveCamera(fov=45.0, pos=(0.5, 0.5, -0.9), look=(0.5, 0.5, 0.5), up=(0.0, 1.0, 0.0))
    filt = GaussianFilter() if filter == "gaussian" else BoxFilter()
    film = SpectralFilm(width, height, nbuckets=nbuckets, filter=filt) if nbuckets else RGBFilm(width, height, filter=filt)
    smp = ZSobolSampler(spp) if sampler == "zsobol" else IndependentSampler(spp)
    return Scene(cam, film, med, [UniformInfiniteLight(scale=0.05)], sampler=smp)

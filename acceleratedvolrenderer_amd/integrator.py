"""VolPathIntegrator on MI355X — the host-side mirror of pbrt-v4's integrator plugin.

pbrt: `Integrator::Create("volpath" | "volpathcustom", ...)` (cpu/integrators.cpp:3658-3709,
src/graph/volpath_custom.cpp:736-749) builds a VolPathIntegrator(maxdepth=5, lightsampler="bvh")
whose Render() walks pixel samples (integrators.cpp:72-232). Here Render() drives the
HIP wavefront through the C-ABI (include/avr.h). Parameter names and defaults follow
pbrt: maxdepth 5, IndependentSampler seed 0 (pbrt's `--seed`), `--maxdepth` override as
in the fork's volpathcustom (volpath_custom.cpp:740-741).

Multi-GPU (one process per GPU, torch.distributed over RCCL/xGMI): the sample range is
split across ranks (rank k renders sample indices [k*spp/N, (k+1)*spp/N) of every pixel,
samplers.h:457-460 indexes by (pixel, sampleIndex), so the union equals the 1-GPU run
up to fp64 summation order), and the fp64 film sums are reduced once with a SUM.
"""
import time

import numpy as np

from . import capi, imageio
from .imgtool import channel_average
from .scene import film_rgb, GBufferFilm, gbuffer_image

INTEGRATOR_NAMES = ("volpath", "volpathcustom", "volpath_mi355x")


def shard_samples(spp, rank, world_size):
    """Sample-index range [lo, hi) of `rank` — contiguous, load-balanced split."""
    lo = (spp * rank) // world_size
    hi = (spp * (rank + 1)) // world_size
    return lo, hi


def film_buffer_size(npix, nbuckets=0):
    """Doubles of the exported film: rgb (3), weight (1) and, for a SpectralFilm, 2 x nbuckets per pixel."""
    return (4 + 2 * int(nbuckets)) * int(npix)


def reduce_film(buf, npix, nbuckets, rank, group=None):
    """The one exchange step of the multi-GPU path: SUM-reduce of the packed fp64 film
    (avr_film_export_device layout) to rank 0 over the process group (RCCL on GPUs, gloo in
    the CPU tests). Rank 0 gets the unpacked sums, other ranks None."""
    import torch.distributed as dist
    dist.reduce(buf, dst=0, op=dist.ReduceOp.SUM, group=group)
    if rank != 0:
        return None
    host = buf.cpu().numpy()
    out = (host[:3 * npix].copy(), host[3 * npix:4 * npix].copy())
    if nbuckets:
        k = npix * nbuckets
        out += (host[4 * npix:4 * npix + k].reshape(npix, nbuckets).copy(),
                host[4 * npix + k:4 * npix + 2 * k].reshape(npix, nbuckets).copy())
    return out


# avr_set_grid_layout: pbrt's linear SampledGrid, the fat footprint copy (8x), 8^3 apron bricks (1.42x)
GRID_LAYOUTS = {"linear": 0, "fat": 1, "brick": 2}
GRID_LAYOUT_NAMES = {v: k for k, v in GRID_LAYOUTS.items()}

class VolPathIntegrator:
    def __init__(self, scene, maxdepth=5, spp=16, seed=0, device=0, max_paths=0, lightsampler="bvh",
                 regularize=False, name="volpath", kernel="persistent", grid_layout="fat", mode="replay"):
        if name not in INTEGRATOR_NAMES:
            raise ValueError(f"unknown integrator {name!r}")
        if lightsampler not in ("bvh", "uniform", "power"):
            raise ValueError(f"{lightsampler}: unknown light sampling strategy")
        # With only infinite lights "bvh" and "uniform" pick uniformly with pmf 1/N
        # (lightsamplers.h:266-277, 35-50); "power" draws from an alias table over the lights'
        # Phi (PowerLightSampler, lightsamplers.cpp:76-96; avr_light_sampler)
        self.lightsampler = lightsampler
        self.scene = scene
        self.maxdepth = int(maxdepth)
        self.spp = int(spp)
        self.seed = int(seed)
        self.device = int(device)
        self.ctx = capi.Context(device, max_paths)
        if kernel not in ("persistent", "wavefront"):
            raise ValueError("kernel must be 'persistent' or 'wavefront'")
        self.ctx.set_kernel_mode(0 if kernel == "persistent" else 1)
        if grid_layout not in GRID_LAYOUTS:
            raise ValueError(f"grid_layout must be one of {sorted(GRID_LAYOUTS)}")
        self.ctx.set_grid_layout(GRID_LAYOUTS[grid_layout])
        if mode not in ("replay", "fast"):
            raise ValueError("mode must be 'replay' (per-sample parity) or 'fast' (statistical parity)")
        self.mode = mode
        self.ctx.set_render_mode(mode)
        self.ctx.set_light_sampler(1 if lightsampler == "power" else 0)
        self.ctx.set_scene(scene)

    @staticmethod
    def create_params(name, params, maxdepth_override=None):
        """Constructor arguments of Integrator::Create(name, parameters) for the volumetric
        integrators (cpu/integrators.cpp:3658-3709). "volpath": maxdepth from the scene file
        (default 5), lightsampler, regularize (VolPathIntegrator::Create,
        integrators.cpp:1408-1418); the command-line --maxdepth does not reach it. The fork's
        "volpathcustom" (src/graph/volpath_custom.cpp:736-749) takes the --maxdepth option
        whenever it is given (a std::optional: 0 counts) over the file's value;
        "volpath_mi355x" (this library's registration) behaves like it.
        pixelsamples and seed are the sampler's. Unknown names raise as pbrt's ErrorExit."""
        if name not in INTEGRATOR_NAMES:
            raise ValueError(f"{name}: integrator type unknown.")
        maxdepth = int(params.get("maxdepth", 5))
        if maxdepth_override is not None and name != "volpath":
            maxdepth = int(maxdepth_override)
        return dict(maxdepth=maxdepth, spp=int(params.get("pixelsamples", 16)), seed=int(params.get("seed", 0)),
                    lightsampler=params.get("lightsampler", "bvh"), regularize=bool(params.get("regularize", False)),
                    name=name)

    @classmethod
    def create(cls, name, params, scene, device=0, maxdepth_override=None, **kw):
        """Integrator::Create-style factory from a pbrt ParameterDictionary-like dict."""
        return cls(scene, device=device, **cls.create_params(name, params, maxdepth_override), **kw)

    def tune_majorant(self, candidates=(1, 2, 4, 8, 16), probe=(0, 64)):
        """The fast mode's tuned majorant: time one probe render of sample
        indices [probe[0], probe[1]) per candidate majorant resolution (r^3) on the device and
        keep the fastest (64 indices, a full pass at 720p: with 4 or 16 the launch's drain and
        the camera stage and film, which the majorant does not change, hid the difference, and
        1^3 and 2^3 swapped between runs — 2^3 renders 4 % slower at 64 indices per pass) (avr_tune_majorant; the film is left as it was). Any conservative
        majorant gives the same estimator in expectation; only pbrt's own resolution (16^3
        grids, 64^3 NanoVDB) replays pbrt's sample streams. Returns (chosen, {r: probe ms})."""
        cands = [(int(r),) * 3 for r in candidates]
        chosen, ms = self.ctx.tune_majorant(cands, probe[0], probe[1], self.seed, self.maxdepth)
        return chosen, {c[0]: float(t) for c, t in zip(cands, ms)}

    def entry_cell_order(self):
        """A pixel order for avr_set_pixel_order (the north star's "sorted ray
        packets"): pixels sorted by the majorant cell where the ray through the pixel centre
        enters the medium's bounds (pixels whose ray misses them last), scanline order within a
        cell. Host arithmetic in f64 (an ordering heuristic, not a sample)."""
        sc = self.scene
        f = sc.film
        y, x = np.mgrid[0:f.height, 0:f.width]
        pr = np.stack([x.ravel() + 0.5, y.ravel() + 0.5, np.zeros(x.size), np.ones(x.size)], 1)
        pc = pr @ np.asarray(sc.camera_from_raster, np.float64).T
        pc = pc[:, :3] / pc[:, 3:4]
        if int(sc.camera.type_id) == 0:    # orthographic: origin on the film plane, along +z
            o_c, d_c = pc, np.tile([0.0, 0.0, 1.0], (len(pc), 1))
        else:
            o_c, d_c = np.zeros_like(pc), pc / np.linalg.norm(pc, axis=1, keepdims=True)
        rfc = np.asarray(sc.render_from_camera, np.float64)
        mfr = np.asarray(sc.medium_from_render, np.float64)
        m = mfr @ rfc
        o = o_c @ m[:3, :3].T + m[:3, 3]
        d = d_c @ m[:3, :3].T
        b = np.asarray(sc.medium.bounds, np.float64)
        with np.errstate(divide="ignore", invalid="ignore"):
            t0 = (b[:3] - o) / d
            t1 = (b[3:] - o) / d
        tn = np.nanmax(np.minimum(t0, t1), axis=1)
        tf = np.nanmin(np.maximum(t0, t1), axis=1)
        hit = (tf >= np.maximum(tn, 0)) & np.isfinite(tn)
        p = o + d * np.maximum(tn, 0)[:, None]
        res = np.asarray(sc.medium.majorant_res, np.int64)
        c = np.clip(((p - b[:3]) / (b[3:] - b[:3]) * res).astype(np.int64), 0, res - 1)
        key = np.where(hit, (c[:, 2] * res[1] + c[:, 1]) * res[0] + c[:, 0], res.prod())
        return np.argsort(key, kind="stable").astype(np.int32)

    def render(self, spp_begin=0, spp_end=None, clear=True):
        """Render sample indices [spp_begin, spp_end); returns (rgb_sum, w_sum) fp64."""
        if spp_end is None:
            spp_end = self.spp
        if clear:
            self.ctx.film_clear()
        self.ctx.render(spp_begin, spp_end, self.seed, self.maxdepth)
        return self.film_sums()

    def film_sums(self):
        f = self.scene.film
        return self.ctx.film_read(f.width * f.height)

    def spectral_sums(self):
        """SpectralFilm Pixel::bucketSums / weightSums, (W*H, nbuckets) fp64 each."""
        f = self.scene.film
        if not getattr(f, "nbuckets", 0):
            raise ValueError("the scene's film is not a SpectralFilm")
        return self.ctx.film_read_spectral(f.width * f.height, f.nbuckets)

    def spectral_image(self, fp16=True):
        """SpectralFilm::GetImage: (H, W, 3 + nbuckets), channels film.channel_names()."""
        from .scene import spectral_image
        rgb, w = self.film_sums()
        bs, bw = self.spectral_sums()
        return spectral_image(self.scene.film, rgb, w, bs, bw, fp16=fp16)

    def image(self, rgb_sum=None, w_sum=None):
        if rgb_sum is None:
            rgb_sum, w_sum = self.film_sums()
        return film_rgb(self.scene.film, rgb_sum, w_sum)

    def stats(self):
        return self.ctx.stats()

    def get_image(self, rgb_sum=None, w_sum=None, fp16=True):
        """RGBFilm::GetImage (film.cpp:533-565): GetPixelRGB per pixel, and for the fp16
        image ("savefp16", default true) the 65504 clamp and the half rounding."""
        img = self.image(rgb_sum, w_sum)
        if fp16:
            img = np.minimum(img, np.float32(65504)).astype(np.float16).astype(np.float32)
        return img

    def write_image(self, path, rgb_sum=None, w_sum=None, spp=None, render_time=None, mse=None, fp16=True):
        """RGBFilm::WriteImage -> Image::Write: EXR (pbrt's attributes, ZIP) or PFM by extension.
        SpectralFilm (film.cpp:955-1028): EXR only, R G B + S0.<lambda>nm channels and the
        spectral layout strings."""
        f = self.scene.film
        if getattr(f, "nbuckets", 0):
            if not str(path).lower().endswith(".exr"):
                raise ValueError(f"{path}: EXR is the only output format supported by the SpectralFilm.")
            img = self.spectral_image(fp16)
            if fp16:
                img = img.astype(np.float16).astype(np.float32)
            imageio.write_exr(path, img, channels=f.channel_names(), half=fp16,
                              samples_per_pixel=spp if spp is not None else self.spp, render_time_seconds=render_time,
                              mse=mse, strings={"spectralLayoutVersion": "1.0", "emissiveUnits": "W.m^-2.sr^-1"})
            return img
        if isinstance(f, GBufferFilm):
            if rgb_sum is None:
                rgb_sum, w_sum = self.film_sums()
            img = gbuffer_image(f, rgb_sum, w_sum, fp16)
            if fp16:
                img = img.astype(np.float16).astype(np.float32)
            imageio.write_exr(path, img, channels=f.channel_names(), half=fp16,
                              samples_per_pixel=spp if spp is not None else self.spp, render_time_seconds=render_time,
                              mse=mse)
            return img
        img = self.get_image(rgb_sum, w_sum, fp16)
        if str(path).lower().endswith(".pfm"):
            imageio.write_pfm(path, img)
        else:
            imageio.write_exr(path, img, half=fp16, samples_per_pixel=spp if spp is not None else self.spp,
                              render_time_seconds=render_time, mse=mse)
        return img

    def render_waves(self, mse_reference=None, mse_out=None, metric="MSE"):
        """ImageTileIntegrator::Render's wave loop (integrators.cpp:166-232): waves of
        1, 1, 2, 4, ... 64 sample indices; with an MSE reference image every wave is one
        sample and after each the film's (fp16) image is compared with the reference on the
        device, written as pbrt's "spp, mse" lines (integrators.cpp:209-219) to `mse_out`.
        Returns (rgb_sum, w_sum, [(spp, error), ...])."""
        f = self.scene.film
        if mse_reference is not None:
            ref = np.asarray(mse_reference, np.float32)
            if ref.shape != (f.height, f.width, 3):
                raise ValueError(f"reference image must be {(f.height, f.width, 3)}")
            self.ctx.film_set_reference(ref, f.output_from_sensor, fp16=True)
        self.ctx.film_clear()
        log = []
        wave_start, wave_end, next_wave = 0, 1, 1
        out = open(mse_out, "w") if mse_out else None
        t0 = time.time()
        try:
            while wave_start < self.spp:
                self.ctx.render(wave_start, wave_end, self.seed, self.maxdepth)
                wave_start = wave_end
                wave_end = min(self.spp, wave_end + next_wave)
                if mse_reference is None:
                    next_wave = min(2 * next_wave, 64)
                else:
                    v = self.ctx.film_metric(metric)
                    err = float(channel_average(v[0] if metric == "ME" else v))
                    log.append((wave_start, err))
                    if out:
                        out.write(f"{wave_start}, {err:.9g}\n")
                        out.flush()
        finally:
            if out:
                out.close()
        self.last_render_seconds = time.time() - t0
        rgb, w = self.film_sums()
        return rgb, w, log

    def render_distributed(self, rank, world_size, group=None):
        """Render this rank's sample shard and SUM-reduce the fp64 film to rank 0 (RCCL).

        Returns (rgb_sum, w_sum) on rank 0 — (rgb_sum, w_sum, bucket_sums, weight_sums) for a
        SpectralFilm — and None elsewhere.
        """
        import torch

        lo, hi = shard_samples(self.spp, rank, world_size)
        self.ctx.film_clear()
        if hi > lo:
            self.ctx.render(lo, hi, self.seed, self.maxdepth)
        f = self.scene.film
        nb = int(getattr(f, "nbuckets", 0))
        buf = torch.empty(film_buffer_size(f.width * f.height, nb), dtype=torch.float64, device=f"cuda:{self.device}")
        self.ctx.film_export_device(buf.data_ptr())
        return reduce_film(buf, f.width * f.height, nb, rank, group)

    def close(self):
        self.ctx.close()

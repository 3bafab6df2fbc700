"""Scene description for the volumetric path: the subset of pbrt-v4 scene objects
the MI355X integrator consumes, with pbrt's parameter names and defaults.

    GridMedium            media.h:265-352, GridMedium::Create media.cpp:249-330
    DistantLight          lights.h:244-305, DistantLight::Create lights.cpp:246-276
    UniformInfiniteLight  lights.cpp:950-972, creation lights.cpp:1529-1566
    Orthographic/PerspectiveCamera  cameras.h:245-273, cameras.cpp:284-306, 404-427, 365-400, 490-520
    RGBFilm + PixelSensor film.h:95-100, 232-316; film.cpp:212-250, 484-497, 567-585
    CameraTransform       cameras.cpp:27-57 (default rendering space: CameraWorld)

The medium's box `[p0, p1]` doubles as the scene's only geometry: an "interface"
boundary (no BSDF; rays cross it without scattering, interaction.cpp:91-97).
See DESIGN.md "Scene model" for why that is exact for VolPath's sampling.
"""
import math

import numpy as np

from . import spectra
from . import transform as xf


class GridMedium:
    """pbrt "uniformgrid" medium (GridMedium::Create, media.cpp:249-330).

    density: float32 array shaped (nz, ny, nx) (x fastest, containers.h:834), or a
    device tensor with `.data_ptr()` (kept alive by the caller) plus `shape`.
    """

    def __init__(self, density, p0=(0.0, 0.0, 0.0), p1=(1.0, 1.0, 1.0), world_from_medium=None, sigma_a=None,
                 sigma_s=None, scale=1.0, g=0.0, Le=None, Lescale=None, majorant_res=(16, 16, 16), temperature=None,
                 temperaturescale=1.0, temperatureoffset=0.0):
        if hasattr(density, "data_ptr"):
            check_device_grid(density, "density", 3)
            self.device_density = density
            self.density = None
            nz, ny, nx = (int(s) for s in density.shape)
        else:
            d = np.ascontiguousarray(np.asarray(density, np.float32))
            if d.ndim != 3:
                raise ValueError("density must be (nz, ny, nx)")
            self.device_density = None
            self.density = d
            nz, ny, nx = d.shape
        self.nx, self.ny, self.nz = nx, ny, nz
        self.p0 = np.asarray(p0, np.float32)
        self.p1 = np.asarray(p1, np.float32)
        self.world_from_medium = np.eye(4) if world_from_medium is None else np.asarray(world_from_medium, np.float64)
        self.g = np.float32(g)
        # DenselySampledSpectrum(sigma).Scale(sigmaScale) (media.cpp:229-231), defaults 1 (media.cpp:313-320)
        self.sigma_a = spectra.scaled(spectra.as_table(sigma_a, 1.0), scale)
        self.sigma_s = spectra.scaled(spectra.as_table(sigma_s, 1.0), scale)
        # Le / LeScale (media.cpp:283-305)
        le_norm = np.float32(1.0)
        if Le is None or float(np.max(spectra.as_table(Le, 0.0))) == 0.0:
            self.Le = None
        else:
            self.Le = spectra.as_table(Le, 0.0)
            le_norm = np.float32(1.0) / spectra.spectrum_to_photometric(self.Le)
        if Lescale is None:
            self.Lescale = np.array([[[le_norm]]], np.float32)
        else:
            ls = np.asarray(Lescale, np.float32)
            if ls.shape != (nz, ny, nx):
                raise ValueError("Lescale must match the density grid shape")
            self.Lescale = (ls * le_norm).astype(np.float32)
        self.majorant_res = tuple(int(r) for r in majorant_res)
        # temperature grid (media.cpp:255-266, 321-326): blackbody emission, exclusive with Le
        self.temperature = None
        if temperature is not None:
            if self.Le is not None:
                raise ValueError('Both "Le" and "temperature" values were provided.')
            t = np.ascontiguousarray(np.asarray(temperature, np.float32))
            if t.shape != (nz, ny, nx):
                raise ValueError("temperature must match the density grid shape")
            self.temperature = t
        self.temperature_scale = np.float32(temperaturescale)
        self.temperature_offset = np.float32(temperatureoffset)

    type_id = 0

    @property
    def bounds(self):
        return np.concatenate([self.p0, self.p1]).astype(np.float32)


class _AnalyticMedium:
    """Shared surface of the media without a density grid (the C-ABI and the oracle see a
    1^3 grid of 1.0 and a 1^3 majorant; the kernels never read them)."""
    device_density = None
    nx = ny = nz = 1
    majorant_res = (1, 1, 1)

    def _box(self, p0, p1, world_from_medium):
        self.p0 = np.asarray(p0, np.float32)
        self.p1 = np.asarray(p1, np.float32)
        self.world_from_medium = np.eye(4) if world_from_medium is None else np.asarray(world_from_medium, np.float64)
        self.density = np.ones((1, 1, 1), np.float32)
        self.Lescale = np.ones((1, 1, 1), np.float32)

    @property
    def bounds(self):
        return np.concatenate([self.p0, self.p1]).astype(np.float32)


class HomogeneousMedium(_AnalyticMedium):
    """pbrt "homogeneous" medium (HomogeneousMedium::Create, media.cpp:166-200): sigma_a,
    sigma_s (default 1) x scale, g, Le (illuminant) x Lescale / photometric(Le). pbrt's
    medium is unbounded; here it fills the interface box [p0, p1] (its majorant segment is
    the box crossing, as the box's interface surfaces would bound it in pbrt)."""
    type_id = 1

    def __init__(self, p0=(0.0, 0.0, 0.0), p1=(1.0, 1.0, 1.0), world_from_medium=None, sigma_a=None, sigma_s=None,
                 scale=1.0, g=0.0, Le=None, Lescale=1.0):
        self._box(p0, p1, world_from_medium)
        self.g = np.float32(g)
        self.sigma_a = spectra.scaled(spectra.as_table(sigma_a, 1.0), scale)
        self.sigma_s = spectra.scaled(spectra.as_table(sigma_s, 1.0), scale)
        if Le is None or float(np.max(spectra.as_table(Le, 0.0))) == 0.0:
            self.Le = None
        else:
            le = spectra.as_table(Le, 0.0)
            self.Le = spectra.scaled(le, np.float32(np.float32(Lescale) / spectra.spectrum_to_photometric(le)))


class CloudMedium(_AnalyticMedium):
    """pbrt "cloud" medium (CloudMedium::Create, media.cpp:463-484): procedural Perlin
    density (density 1, wispiness 1, frequency 5), sigma_a / sigma_s default 1 (no scale
    parameter in pbrt), g, bounds p0/p1."""
    type_id = 2

    def __init__(self, p0=(0.0, 0.0, 0.0), p1=(1.0, 1.0, 1.0), world_from_medium=None, sigma_a=None, sigma_s=None,
                 g=0.0, density=1.0, wispiness=1.0, frequency=5.0):
        self._box(p0, p1, world_from_medium)
        self.g = np.float32(g)
        self.sigma_a = spectra.as_table(sigma_a, 1.0)
        self.sigma_s = spectra.as_table(sigma_s, 1.0)
        self.Le = None
        self.cloud = (np.float32(density), np.float32(wispiness), np.float32(frequency))


class NanoVDBMedium:
    """pbrt "nanovdb" medium (NanoVDBMedium::Create, media.cpp:618-665; ctor 511-616):
    `density` and optional `temperature` are NanoVDBGrid trees (vdb.py) in place of the
    "filename" / "gridname" / "temperaturename" file read. sigma_a / sigma_s default 1,
    x "scale"; "g"; "Lescale" (default 1); "temperatureoffset" (falls back to
    "temperaturecutoff", default 0); "temperaturescale" (default 1). Bounds = the density
    grid's world bbox union the temperature grid's; 64^3 majorant."""
    type_id = 3
    device_density = None
    nx = ny = nz = 1
    majorant_res = (64, 64, 64)
    temperature = None   # (GridMedium's dense temperature grid; this medium's is temperature_grid)

    def __init__(self, density, temperature=None, world_from_medium=None, sigma_a=None, sigma_s=None, scale=1.0,
                 g=0.0, Lescale=1.0, temperatureoffset=None, temperaturecutoff=0.0, temperaturescale=1.0):
        self.grid = density
        self.temperature_grid = temperature
        p0, p1 = density.world_bbox()
        if temperature is not None:
            t0, t1 = temperature.world_bbox()
            p0, p1 = np.minimum(p0, t0), np.maximum(p1, t1)
        self.p0, self.p1 = p0.astype(np.float32), p1.astype(np.float32)
        self.world_from_medium = np.eye(4) if world_from_medium is None else np.asarray(world_from_medium, np.float64)
        self.g = np.float32(g)
        self.sigma_a = spectra.scaled(spectra.as_table(sigma_a, 1.0), scale)
        self.sigma_s = spectra.scaled(spectra.as_table(sigma_s, 1.0), scale)
        self.Le = None
        self.Lescale_value = np.float32(Lescale)
        self.temperature_offset = np.float32(temperaturecutoff if temperatureoffset is None else temperatureoffset)
        self.temperature_scale = np.float32(temperaturescale)
        self.density = None
        self.Lescale = np.ones((1, 1, 1), np.float32)

    @property
    def bounds(self):
        return np.concatenate([self.p0, self.p1]).astype(np.float32)


def check_device_grid(t, name, ndim):
    """A grid handed to the device entry points as a tensor: float32 (the kernels read f32 /
    float4 elements, so a narrower dtype would be read past its end), contiguous, on a GPU."""
    if str(getattr(t, "dtype", "")) != "torch.float32":
        raise ValueError(f"{name} tensor must be float32 (got {getattr(t, 'dtype', None)})")
    if t.dim() != ndim or not t.is_contiguous():
        raise ValueError(f"{name} tensor must be contiguous with {ndim} dimensions")
    if getattr(t.device, "type", None) != "cuda":
        raise ValueError(f"{name} tensor must live on a GPU (got {t.device}); pass a numpy array for host data")


class RGBGridMedium:
    """pbrt "rgbgrid" medium (RGBGridMedium::Create, media.cpp:380-453): per-voxel RGB
    "sigma_a" / "sigma_s" (RGBUnboundedSpectrum) and "Le" (RGBIlluminantSpectrum) arrays
    shaped (nz, ny, nx, 3), converted with `rgb_table` (rgbspectrum.RGBToSpectrumTable of
    the colour space, sRGB by default); or the converted {c0, c1, c2, scale} arrays
    (nz, ny, nx, 4) directly as sigma_a_coeffs / sigma_s_coeffs / Le_coeffs. "p0"/"p1"
    bounds, "scale" (sigmaScale), "g", "Lescale" (default 1). `illuminant`: the colour
    space's illuminant table (default D65 = sRGB's). Coefficient arrays may be device tensors
    (torch, float32 (nz, ny, nx, 4) on the context's GPU): they are then used in place
    (avr_medium_rgbgrid_device) and `on_device` is True."""
    type_id = 4
    on_device = False
    device_density = None
    majorant_res = (16, 16, 16)
    temperature = None
    Le = None

    def __init__(self, sigma_a=None, sigma_s=None, Le=None, p0=(0.0, 0.0, 0.0), p1=(1.0, 1.0, 1.0),
                 world_from_medium=None, scale=1.0, g=0.0, Lescale=1.0, rgb_table=None, illuminant=None,
                 sigma_a_coeffs=None, sigma_s_coeffs=None, Le_coeffs=None):
        def conv(rgb, coeffs, name):
            if coeffs is not None and hasattr(coeffs, "data_ptr"):
                if tuple(coeffs.shape[3:]) != (4,) or coeffs.dim() != 4:
                    raise ValueError(f"{name}_coeffs must be a contiguous (nz, ny, nx, 4) tensor")
                check_device_grid(coeffs, f"{name}_coeffs", 4)
                self.on_device = True
                return coeffs
            if coeffs is not None:
                c = np.ascontiguousarray(np.asarray(coeffs, np.float32))
                if c.ndim != 4 or c.shape[3] != 4:
                    raise ValueError(f"{name}_coeffs must be (nz, ny, nx, 4)")
                return c
            if rgb is None:
                return None
            v = np.asarray(rgb, np.float32)
            if v.ndim != 4 or v.shape[3] != 3:
                raise ValueError(f"{name} must be (nz, ny, nx, 3) RGB")
            if rgb_table is None:
                raise ValueError(f"{name} given as RGB needs rgb_table (rgbspectrum.RGBToSpectrumTable)")
            return np.ascontiguousarray(rgb_table.spectrum_coeffs(v))

        self.rgb_sigma_a = conv(sigma_a, sigma_a_coeffs, "sigma_a")
        self.rgb_sigma_s = conv(sigma_s, sigma_s_coeffs, "sigma_s")
        self.rgb_Le = conv(Le, Le_coeffs, "Le")
        given = [x for x in (self.rgb_sigma_a, self.rgb_sigma_s, self.rgb_Le) if x is not None]
        if self.on_device:
            # the device entry point takes device pointers for every grid: no host arrays mixed in
            if not all(hasattr(x, "data_ptr") for x in given):
                raise ValueError("RGB grids given as device tensors must all be device tensors (got a host array too)")
            if len({(x.device.type, x.device.index) for x in given}) != 1:
                raise ValueError("RGB grids given as device tensors must all live on the same GPU")
        if self.rgb_sigma_a is None and self.rgb_sigma_s is None:
            raise ValueError('RGB grid requires "sigma_a" and/or "sigma_s" parameter values.')
        if self.rgb_Le is not None and self.rgb_sigma_a is None:
            raise ValueError('RGB grid requires "sigma_a" if "Le" value provided.')
        grids = [x for x in (self.rgb_sigma_a, self.rgb_sigma_s, self.rgb_Le) if x is not None]
        if any(x.shape != grids[0].shape for x in grids):
            raise ValueError("sigma_a, sigma_s and Le must have the same number of samples")
        self.nz, self.ny, self.nx = grids[0].shape[:3]
        self.p0 = np.asarray(p0, np.float32)
        self.p1 = np.asarray(p1, np.float32)
        self.world_from_medium = np.eye(4) if world_from_medium is None else np.asarray(world_from_medium, np.float64)
        self.g = np.float32(g)
        self.sigma_scale = np.float32(scale)
        self.Le_scale = np.float32(Lescale)
        self.illuminant = (spectra.TABLES["D65"] if illuminant is None else spectra.as_table(illuminant, 0.0)).astype(np.float32)
        # SampleRay's sigma_t = 1 (media.h:417) through the shared tables
        self.sigma_a = np.ones(spectra.N, np.float32)
        self.sigma_s = np.zeros(spectra.N, np.float32)
        self.density = None
        self.Lescale = np.ones((1, 1, 1), np.float32)

    @property
    def bounds(self):
        return np.concatenate([self.p0, self.p1]).astype(np.float32)


class DistantLight:
    """DistantLight::Create (lights.cpp:246-276). L defaults to the color space illuminant."""
    type_id = 0

    def __init__(self, from_=(0.0, 0.0, 0.0), to=(0.0, 0.0, 1.0), L=None, scale=1.0, illuminance=None,
                 world_from_light=None):
        self.L = spectra.TABLES["D65"].copy() if L is None else spectra.as_table(L, 1.0)
        sc = np.float32(scale) / spectra.spectrum_to_photometric(self.L)
        if illuminance is not None and illuminance > 0:
            sc = np.float32(sc * np.float32(illuminance))
        self.scale = np.float32(sc)
        w = np.asarray(from_, np.float64) - np.asarray(to, np.float64)
        self.w_light = w / np.linalg.norm(w)
        self.world_from_light = np.eye(4) if world_from_light is None else np.asarray(world_from_light, np.float64)

    def render_direction(self, render_from_world):
        """Normalize(renderFromLight(Vector3f(0, 0, 1))) (lights.h:287)."""
        v = (render_from_world @ self.world_from_light)[:3, :3] @ self.w_light
        return (v / np.linalg.norm(v)).astype(np.float32)


class UniformInfiniteLight:
    """"infinite" light with constant L (lights.cpp:1529-1566); scale /= SpectrumToPhotometric."""
    type_id = 1

    def __init__(self, L=None, scale=1.0):
        self.L = spectra.TABLES["D65"].copy() if L is None else spectra.as_table(L, 1.0)
        self.scale = np.float32(np.float32(scale) / spectra.spectrum_to_photometric(self.L))

    def render_direction(self, render_from_world):
        return np.zeros(3, np.float32)


class ImageInfiniteLight:
    """"infinite" light with "filename" (ImageInfiniteLight, lights.h:552-640; Create
    lights.cpp:1568-1660): a square equal-area octahedral RGB map. `image` is an (res, res, 3)
    array or `filename` an EXR/PFM; "scale" / SpectrumToPhotometric(illuminant) and the
    optional "illuminance" normalisation as Create computes them. The per-pixel
    RGBIlluminantSpectrum conversion needs the colour space's `rgb_table`
    (rgbspectrum.RGBToSpectrumTable; sRGB by default with the D65 illuminant)."""
    type_id = 2

    def __init__(self, image=None, filename=None, scale=1.0, illuminance=None, world_from_light=None,
                 rgb_table=None, illuminant=None):
        if (image is None) == (filename is None):
            raise ValueError("give exactly one of image / filename")
        if filename is not None:
            from . import imageio
            image = imageio.read_rgb(filename)
        img = np.ascontiguousarray(np.asarray(image, np.float32)[:, :, :3])
        if img.ndim != 3 or img.shape[0] != img.shape[1]:
            raise ValueError("image resolution is non-square: not an equal-area environment map")
        if not np.all(np.isfinite(img)):
            raise ValueError("image has infinite or NaN pixel values and so is not suitable as a light")
        if rgb_table is None:
            raise ValueError("ImageInfiniteLight needs rgb_table (rgbspectrum.RGBToSpectrumTable)")
        self.res = img.shape[0]
        self.image = img
        self.illuminant = (spectra.TABLES["D65"] if illuminant is None else spectra.as_table(illuminant, 0.0)
                           ).astype(np.float32)
        sc = np.float32(np.float32(scale) / spectra.spectrum_to_photometric(self.illuminant))
        if illuminance is not None and illuminance > 0:
            sc = np.float32(sc * np.float32(illuminance) / np.float32(self._illuminance(img)))
        self.scale = sc
        self.L = np.zeros(spectra.N, np.float32)
        self.world_from_light = np.eye(4) if world_from_light is None else np.asarray(world_from_light, np.float64)
        # ImageLe: RGBIlluminantSpectrum(cs, ClampZero(rgb)) per pixel (lights.h:620-627)
        self.coeffs = np.ascontiguousarray(rgb_table.spectrum_coeffs(np.maximum(img, np.float32(0))))
        # Image::GetSamplingDistribution (util/image.h:451-470): ImageChannelValues::Average
        # (float sum in channel order / 3) times dxdA = 1
        avg = ((np.float32(0) + img[:, :, 0]) + img[:, :, 1]) + img[:, :, 2]
        self.distribution = np.ascontiguousarray((avg / np.float32(3)).astype(np.float32))

    @staticmethod
    def _illuminance(img):
        """Upper-hemisphere illuminance of the map (lights.cpp:1621-1641) with the colour
        space's LuminanceVector (row Y of XYZFromRGB); accumulated in f64."""
        res = img.shape[0]
        lum = np.linalg.inv(spectra.TABLES["srgb_rgb_from_xyz"].astype(np.float64))[1]
        total = 0.0
        for y in range(res):
            v = (y + 0.5) / res
            for x in range(res):
                u = (x + 0.5) / res
                uu, vv = 2 * u - 1, 2 * v - 1
                up, vp = abs(uu), abs(vv)
                sd = 1 - (up + vp)
                r = 1 - abs(sd)
                phi = (1 if r == 0 else (vp - up) / r + 1) * math.pi / 4
                z = math.copysign(1 - r * r, sd)
                if z <= 0:
                    continue
                total += float(np.dot(img[y, x].astype(np.float64), lum)) * z
        return total * 2 * math.pi / (res * res)

    def render_direction(self, render_from_world):
        return np.zeros(3, np.float32)


class _ProjectiveCamera:
    type_id = -1

    def __init__(self, pos=(0, 0, 0), look=(0, 0, 1), up=(0, 1, 0), screenwindow=None, frameaspectratio=None,
                 camera_from_world=None):
        self.camera_from_world = (xf.look_at(pos, look, up) if camera_from_world is None
                                  else np.asarray(camera_from_world, np.float64))
        self.screenwindow = screenwindow
        self.frameaspectratio = frameaspectratio

    def _screen(self, xres, yres):
        frame = self.frameaspectratio if self.frameaspectratio is not None else xres / yres
        if frame > 1:
            s = [-frame, frame, -1.0, 1.0]
        else:
            s = [-1.0, 1.0, -1.0 / frame, 1.0 / frame]
        if self.screenwindow is not None:
            s = list(self.screenwindow)
        return s

    def camera_from_raster(self, xres, yres):
        """ProjectiveCamera ctor (cameras.h:254-273)."""
        x0, x1, y0, y1 = self._screen(xres, yres)
        ndc_from_screen = xf.scale(1 / (x1 - x0), 1 / (y1 - y0), 1) @ xf.translate([-x0, -y1, 0])
        raster_from_ndc = xf.scale(xres, -yres, 1)
        screen_from_raster = np.linalg.inv(raster_from_ndc @ ndc_from_screen)
        return np.linalg.inv(self.screen_from_camera()) @ screen_from_raster

    def world_from_camera(self):
        return np.linalg.inv(self.camera_from_world)


class OrthographicCamera(_ProjectiveCamera):
    """OrthographicCamera (cameras.h:280-300): screenFromCamera = Orthographic(0, 1)."""
    type_id = 0

    def screen_from_camera(self):
        return xf.orthographic(0.0, 1.0)


class PerspectiveCamera(_ProjectiveCamera):
    """PerspectiveCamera (cameras.h:340-350): screenFromCamera = Perspective(fov, 1e-2, 1000)."""
    type_id = 1

    def __init__(self, fov=90.0, **kw):
        super().__init__(**kw)
        self.fov = float(fov)

    def screen_from_camera(self):
        return xf.perspective(self.fov, 1e-2, 1000.0)


class BoxFilter:
    """BoxFilter (filters.h:48-77; Create filters.cpp: radius default 0.5)."""
    type_id = 0

    def __init__(self, radius=(0.5, 0.5)):
        self.radius = np.asarray(radius, np.float32)
        self.sigma = np.float32(0)


class GaussianFilter:
    """GaussianFilter (filters.h:80-118; Create filters.cpp: radius 1.5, sigma 0.5) — pbrt's
    default filter (scene.cpp:94). Sampled through FilterSampler's tabulated distribution;
    samples carry weight f/pdf."""
    type_id = 1

    def __init__(self, radius=(1.5, 1.5), sigma=0.5):
        self.radius = np.asarray(radius, np.float32)
        self.sigma = np.float32(sigma)
        if not (self.radius > 0).all() or int(32 * self.radius[0]) < 1 or int(32 * self.radius[1]) < 1:
            raise ValueError("gaussian filter radius too small")
        if int(32 * self.radius[0]) > 128 or int(32 * self.radius[1]) > 128:
            raise ValueError("gaussian filter radius above 4 is not supported")


class IndependentSampler:
    """IndependentSampler (samplers.h:442-476): PCG32 stream per (pixel, sampleIndex)."""
    type_id = 0

    def __init__(self, pixelsamples=16, seed=None):
        self.pixelsamples = int(pixelsamples)
        self.seed = seed


class ZSobolSampler:
    """ZSobolSampler (samplers.h:225-330) with FastOwen randomisation — pbrt's default
    sampler (scene.cpp:93). pixelsamples should be a power of two (Warning otherwise)."""
    type_id = 1

    def __init__(self, pixelsamples=16, seed=None, randomization="fastowen"):
        if randomization != "fastowen":
            raise NotImplementedError("only the default FastOwen randomisation is implemented")
        self.pixelsamples = int(pixelsamples)
        self.seed = seed


class RGBFilm:
    """RGBFilm (film.h:232-316) with the cie1931 PixelSensor (film.cpp:212-250) and a box
    (default here) or Gaussian pixel filter."""

    def __init__(self, xresolution=1280, yresolution=720, filter_radius=(0.5, 0.5), iso=100.0, exposure_time=1.0,
                 maxcomponentvalue=math.inf, filter=None):
        self.width = int(xresolution)
        self.height = int(yresolution)
        self.filter = filter if filter is not None else BoxFilter(filter_radius)
        self.filter_radius = self.filter.radius
        self.imaging_ratio = np.float32(np.float32(exposure_time) * np.float32(iso) / np.float32(100))
        self.max_component_value = np.float32(maxcomponentvalue)
        self.sensor = spectra.sensor_cie1931()
        # outputRGBFromSensorRGB = colorSpace->RGBFromXYZ * XYZFromSensorRGB (film.cpp:496), cie1931: I
        self.output_from_sensor = spectra.TABLES["srgb_rgb_from_xyz"].astype(np.float32)


class SpectralFilm(RGBFilm):
    """SpectralFilm (film.h:401-530, film.cpp:849-1066): the RGB sums of RGBFilm plus
    `nbuckets` (default 16) per-pixel spectral buckets over [lambdamin, lambdamax] (default
    360-830 nm); wavelengths sampled uniformly (SampledWavelengths::SampleUniform). Here the
    range must lie within 360-830 nm (the densely sampled tables' domain)."""
    nbuckets_default = 16

    def __init__(self, xresolution=1280, yresolution=720, nbuckets=16, lambdamin=360.0, lambdamax=830.0, **kw):
        super().__init__(xresolution, yresolution, **kw)
        if int(nbuckets) < 1:
            raise ValueError("nbuckets must be positive")
        if not (360.0 <= float(lambdamin) < float(lambdamax) <= 830.0):
            raise ValueError("SpectralFilm wavelength range must lie within 360..830 nm")
        self.nbuckets = int(nbuckets)
        self.lambdamin = np.float32(lambdamin)
        self.lambdamax = np.float32(lambdamax)

    def bucket_centers(self):
        """Channel wavelengths of GetImage: Lerp((i + 0.5) / nBuckets, min, max) (film.cpp:969)."""
        t = ((np.arange(self.nbuckets, dtype=np.float32) + np.float32(0.5)) / np.float32(self.nbuckets)).astype(
            np.float32)
        return ((np.float32(1) - t) * self.lambdamin + t * self.lambdamax).astype(np.float32)

    def channel_names(self):
        """R, G, B, then S0.<lambda>nm with ',' for '.' (film.cpp:963-973)."""
        return ["R", "G", "B"] + ["S0." + ("%.3fnm" % float(l)).replace(".", ",") for l in self.bucket_centers()]


class GBufferFilm(RGBFilm):
    """GBufferFilm (film.h:319-400, film.cpp:588-800). Its geometric channels (albedo, P,
    dzdx/dzdy, N, Ns, uv) and the RGB variance estimators are fed only by a VisibleSurface,
    which VolPathIntegrator::Li sets at the first intersection whose material has a BSDF
    (cpu/integrators.cpp:1124-1151); the medium boundaries this path renders are interface
    shapes (no BSDF), so those channels stay at their zero initial values and the radiance
    part is RGBFilm's (same AddSample sums: the device film is shared)."""
    CHANNELS = ["R", "G", "B", "Albedo.R", "Albedo.G", "Albedo.B", "P.X", "P.Y", "P.Z", "dzdx", "dzdy", "N.X",
                "N.Y", "N.Z", "Ns.X", "Ns.Y", "Ns.Z", "u", "v", "Variance.R", "Variance.G", "Variance.B",
                "RelativeVariance.R", "RelativeVariance.G", "RelativeVariance.B"]

    def channel_names(self):
        return list(self.CHANNELS)


def gbuffer_image(film, rgb_sum, w_sum, fp16=True):
    """GBufferFilm::GetImage (film.cpp:688-800), no splats and no visible surfaces:
    (H, W, 25) float32 in GBufferFilm.CHANNELS order."""
    rgb = film_rgb(film, rgb_sum, w_sum)
    if fp16:
        rgb = np.minimum(rgb, np.float32(65504))
    out = np.zeros((film.height, film.width, len(GBufferFilm.CHANNELS)), np.float32)
    out[:, :, :3] = rgb
    return out


def spectral_image(film, rgb_sum, w_sum, bucket_sums, weight_sums, fp16=True):
    """SpectralFilm::GetImage (film.cpp:961-1028), no splats: (H, W, 3 + nbuckets) float32."""
    rgb = film_rgb(film, rgb_sum, w_sum)
    if fp16:
        rgb = np.minimum(rgb, np.float32(65504))
    bs = np.asarray(bucket_sums, np.float64).reshape(film.height, film.width, film.nbuckets)
    bw = np.asarray(weight_sums, np.float64).reshape(film.height, film.width, film.nbuckets)
    with np.errstate(divide="ignore", invalid="ignore"):
        c = np.where(bw > 0, (bs / np.where(bw > 0, bw, 1)).astype(np.float32), np.float32(0))
    if fp16:
        c = np.minimum(c, np.float32(65504))
    return np.concatenate([rgb, c.astype(np.float32)], axis=2)


def convex_mesh_planes(vertices, triangles):
    """Outward face planes {nx, ny, nz, h} (inside: n.p <= h) of a closed convex triangle mesh,
    coplanar faces merged; f64."""
    v = np.asarray(vertices, np.float64).reshape(-1, 3)
    t = np.asarray(triangles, np.int64).reshape(-1, 3)
    c = v.mean(axis=0)
    out = []
    for a, b, d in t:
        n = np.cross(v[b] - v[a], v[d] - v[a])
        ln = np.linalg.norm(n)
        if ln == 0:
            continue
        n = n / ln
        h = float(n @ v[a])
        if n @ c > h:
            n, h = -n, -h
        if not any(np.allclose(n, q[:3], atol=1e-9) and abs(h - q[3]) < 1e-9 for q in out):
            out.append(np.array([*n, h]))
    if len(out) < 4:
        raise ValueError("interface mesh must be a closed convex polyhedron")
    planes = np.array(out)
    if np.any(v @ planes[:, :3].T > planes[:, 3] + 1e-6 * (1 + np.abs(planes[:, 3]))):
        raise ValueError("interface mesh is not convex")
    return planes


def _bounding_sphere_radius(pmin, pmax):
    """Bounds3::BoundingSphere (vecmath.h:1335-1338) in float32."""
    pmin = pmin.astype(np.float32)
    pmax = pmax.astype(np.float32)
    center = ((pmin + pmax) / np.float32(2)).astype(np.float32)
    inside = bool(np.all(center >= pmin) and np.all(center <= pmax))
    if not inside:
        return np.float32(0)
    d = (pmax - center).astype(np.float32)
    return np.float32(np.sqrt(np.float32(np.float32(d[0] * d[0] + d[1] * d[1]) + d[2] * d[2])))


class Scene:
    """Resolved render-space scene (CameraWorld rendering space, cameras.cpp:35-41)."""

    def __init__(self, camera, film, medium, lights, sampler=None, interface_sphere=None, interface_mesh=None):
        """interface_sphere: None (the medium's bounds box is its interface shape) or
        (world-space centre, radius) of a sphere without material whose MediumInterface holds
        the medium inside (pbrt's `AttributeBegin MediumInterface "cloud" "" Shape "sphere"`).
        interface_mesh: (vertices, triangles) of a closed CONVEX triangle mesh in world space
        (e.g. pbrt's `Shape "trianglemesh"` cube around a medium) bounding the medium instead."""
        self.camera, self.film, self.medium, self.lights = camera, film, medium, list(lights)
        self.interface_sphere = interface_sphere
        self.sampler = sampler if sampler is not None else IndependentSampler()
        if len(self.lights) > 8:
            raise ValueError("at most 8 lights")
        wfc = camera.world_from_camera()
        cam_pos = wfc @ np.array([0, 0, 0, 1.0])
        self.render_from_world = xf.translate(-cam_pos[:3])
        self.render_from_camera = xf.f32(self.render_from_world @ wfc)
        self.camera_from_raster = xf.f32(camera.camera_from_raster(film.width, film.height))
        rfm = self.render_from_world @ medium.world_from_medium
        self.render_from_medium = xf.f32(rfm)
        self.medium_from_render = xf.f32(np.linalg.inv(rfm))
        # scene bounds = render-space bounds of the interface box (the only shape)
        c = np.array([[x, y, z, 1.0] for x in (medium.p0[0], medium.p1[0]) for y in (medium.p0[1], medium.p1[1])
                      for z in (medium.p0[2], medium.p1[2])])
        rc = (rfm @ c.T).T[:, :3]
        self.scene_radius = _bounding_sphere_radius(rc.min(axis=0), rc.max(axis=0))
        self.interface_sphere_render = None
        self.interface_planes_render = None
        if interface_mesh is not None:
            verts, tris = interface_mesh
            pw = convex_mesh_planes(verts, tris)
            off = np.asarray(self.render_from_world, np.float64)[:3, 3]   # CameraWorld: a translation
            pr = pw.copy()
            pr[:, 3] = pw[:, 3] + pw[:, :3] @ off
            self.interface_planes_render = pr.astype(np.float32)
            vr = np.asarray(verts, np.float64) + off
            self.scene_radius = _bounding_sphere_radius(vr.min(axis=0), vr.max(axis=0))
        if interface_sphere is not None:
            cw, r = interface_sphere
            if not float(r) > 0:
                raise ValueError("interface sphere radius must be > 0")
            cr = (self.render_from_world @ np.array([*map(float, cw), 1.0]))[:3].astype(np.float32)
            self.interface_sphere_render = np.array([*cr, np.float32(r)], np.float32)
            # the sphere is then the scene's only shape: Sphere::Bounds (shapes.cpp) -> sceneRadius
            lo = cr.astype(np.float64) - float(r)
            hi = cr.astype(np.float64) + float(r)
            self.scene_radius = _bounding_sphere_radius(lo, hi)
        self.light_types = np.array([l.type_id for l in self.lights], np.int32)
        self.light_w = np.stack([l.render_direction(self.render_from_world) for l in self.lights]).astype(
            np.float32) if self.lights else np.zeros((0, 3), np.float32)
        self.light_L = np.stack([l.L for l in self.lights]).astype(np.float32) if self.lights else np.zeros(
            (0, spectra.N), np.float32)
        self.light_scale = np.array([l.scale for l in self.lights], np.float32)
        # image lights: renderFromLight and its inverse (ImageInfiniteLight's transform)
        self.light_rfl = [xf.f32(self.render_from_world @ l.world_from_light) if l.type_id == 2 else None
                          for l in self.lights]
        self.light_lfr = [xf.f32(np.linalg.inv(self.render_from_world @ l.world_from_light)) if l.type_id == 2
                          else None for l in self.lights]


def film_rgb(film, rgb_sum, w_sum):
    """RGBFilm::GetPixelRGB (film.h:258-274) in float32, no splats: returns (H, W, 3)."""
    rgb = np.asarray(rgb_sum, np.float64).reshape(-1, 3).astype(np.float32)
    w = np.asarray(w_sum, np.float64).reshape(-1).astype(np.float32)
    nz = w != 0
    rgb[nz] = (rgb[nz] / w[nz, None]).astype(np.float32)
    m = film.output_from_sensor.astype(np.float32)
    out = np.empty_like(rgb)
    for r in range(3):
        out[:, r] = ((m[r, 0] * rgb[:, 0] + m[r, 1] * rgb[:, 1]).astype(np.float32) + m[r, 2] * rgb[:, 2]).astype(
            np.float32)
    return out.reshape(film.height, film.width, 3)

"""acceleratedvolrenderer_amd — MI355X-native volumetric path integrator.

A from-scratch HIP/gfx950 implementation of the hot path of tsvdh/AcceleratedVolRenderer
(a pbrt-v4 fork): pbrt's null-scattering VolPathIntegrator — delta-tracking free-flight
sampling, ratio-tracking transmittance, majorant-grid DDA over GridMedium, wavefront
queues with wave64 ballot compaction, RGBFilm accumulation — behind the C-ABI in
include/avr.h. See DESIGN.md.
"""
from . import spectra, transform
from .scene import (GridMedium, DistantLight, UniformInfiniteLight, ImageInfiniteLight, OrthographicCamera, PerspectiveCamera, RGBFilm, SpectralFilm, spectral_image, GBufferFilm, gbuffer_image,
                    Scene, film_rgb, HomogeneousMedium, CloudMedium, NanoVDBMedium, RGBGridMedium, BoxFilter, GaussianFilter,
                    IndependentSampler, ZSobolSampler)
from .vdb import NanoVDBGrid
from .rgbspectrum import RGBToSpectrumTable
from .integrator import VolPathIntegrator, shard_samples, INTEGRATOR_NAMES
from . import capi
from . import scenes

__all__ = ["spectra", "transform", "GridMedium", "DistantLight", "UniformInfiniteLight", "OrthographicCamera",
           "PerspectiveCamera", "RGBFilm", "Scene", "film_rgb", "VolPathIntegrator", "shard_samples",
           "INTEGRATOR_NAMES", "capi", "scenes", "HomogeneousMedium", "CloudMedium", "NanoVDBMedium", "NanoVDBGrid", "RGBGridMedium", "RGBToSpectrumTable",
           "SpectralFilm", "spectral_image", "GBufferFilm", "gbuffer_image", "ImageInfiniteLight", "BoxFilter", "GaussianFilter", "IndependentSampler", "ZSobolSampler"]

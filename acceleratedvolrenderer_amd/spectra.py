"""Spectral tables and DenselySampledSpectrum helpers (host side).

Mirrors pbrt-v4 `DenselySampledSpectrum` (util/spectrum.h:374-420): a spectrum is a
471-entry float32 table over 360..830 nm, sampled at `lround(lambda) - 360`.
Tables (data/spectra_f32.bin) were dumped from the reference's own spectrum.cpp /
colorspace.cpp by oracle/ref/gen_golden.py: CIE 1931 x̄ȳz̄, the sRGB illuminant (D65)
as RGBColorSpace::illuminant holds it, sRGB RGBFromXYZ and the D65 photometric scale.
"""
import os

import numpy as np

LAMBDA_MIN, LAMBDA_MAX = 360, 830
N = LAMBDA_MAX - LAMBDA_MIN + 1  # 471
CIE_Y_INTEGRAL = np.float32(106.856895)  # util/spectrum.h:38

_DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "spectra_f32.bin")


def _load():
    raw = np.fromfile(_DATA, dtype="<f4")
    expected = 4 * N + 9 + 2
    if raw.size != expected:
        raise RuntimeError(f"{_DATA}: expected {expected} floats, found {raw.size}")
    t = {
        "X": raw[0:N].copy(),
        "Y": raw[N:2 * N].copy(),
        "Z": raw[2 * N:3 * N].copy(),
        "D65": raw[3 * N:4 * N].copy(),
        "srgb_rgb_from_xyz": raw[4 * N:4 * N + 9].reshape(3, 3).copy(),
        "d65_scale": np.float32(raw[4 * N + 9]),
    }
    return t


TABLES = _load()


def constant(c):
    """ConstantSpectrum(c) densely sampled (spectrum.h:354-372)."""
    return np.full(N, np.float32(c), dtype=np.float32)


def as_table(s, default=1.0):
    """Accept None (-> constant `default`), a scalar (ConstantSpectrum) or a 471 table."""
    if s is None:
        return constant(default)
    a = np.asarray(s, dtype=np.float32)
    if a.ndim == 0:
        return constant(float(a))
    if a.shape != (N,):
        raise ValueError(f"spectrum table must have {N} entries (360..830 nm), got {a.shape}")
    return a.copy()


def scaled(table, s):
    """DenselySampledSpectrum::Scale — per-entry float32 multiply (spectrum.h:410-413)."""
    return (np.asarray(table, np.float32) * np.float32(s)).astype(np.float32)


def inner_product_y(table):
    """InnerProduct(&Spectra::Y(), s) with pbrt's float accumulation order (spectrum.cpp)."""
    acc = np.float32(0.0)
    y = TABLES["Y"]
    t = np.asarray(table, np.float32)
    for i in range(N):
        acc = np.float32(acc + np.float32(y[i] * t[i]))
    return acc


def spectrum_to_photometric(table):
    """SpectrumToPhotometric (spectrum.cpp:37-47) for a densely sampled, non-RGB spectrum."""
    return inner_product_y(table)


def blackbody(T):
    """BlackbodySpectrum(T) densely sampled (spectrum.h:500-530), normalised to peak 1."""
    lam = np.arange(LAMBDA_MIN, LAMBDA_MAX + 1, dtype=np.float64)

    def bb(l_nm):
        c, h, kb = 299792458.0, 6.62606957e-34, 1.3806488e-23
        l = l_nm * 1e-9
        return (2 * h * c * c) / (l ** 5 * (np.exp((h * c) / (l * kb * T)) - 1))

    lambda_max = 2.8977721e-3 / T
    return (bb(lam) / bb(lambda_max * 1e9)).astype(np.float32)


def sensor_cie1931():
    """cie1931 PixelSensor response (film.h:220-231): r̄ḡb̄ = X, Y, Z; XYZFromSensorRGB = I."""
    return np.stack([TABLES["X"], TABLES["Y"], TABLES["Z"]]).astype(np.float32)

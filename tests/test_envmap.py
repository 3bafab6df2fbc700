"""ImageInfiniteLight pieces (lights.h:552-640) against the reference's own functions
(tests/golden/ref_vectors.json: EqualAreaSquareToSphere / EqualAreaSphereToSquare,
RemapPixelCoords(OctahedralSphere), PiecewiseConstant2D Sample/PDF), the host-compiled
device header (csrc/avr_envmap.h) against the oracle's canonical mode, and the oracle's
image-light estimator on a known answer (a constant map is a uniform light: furnace)."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from oracle import binding

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
F = ctypes.POINTER(ctypes.c_float)


def _u(bits):
    return np.array(bits, np.uint32).view(np.float32)


def _bits(a):
    return np.asarray(a, np.float32).view(np.uint32).tolist()


def test_equal_area_mapping_matches_reference(golden):
    L = binding.lib()
    binding.set_libm("platform")
    out = np.zeros(3, np.float32)
    for row in golden["equal_area"]:
        u, v = _u(row[:2])
        L.oracle_equal_area_square_to_sphere(float(u), float(v), out.ctypes.data_as(F))
        assert _bits(out) == row[2:5], row
        q = np.zeros(2, np.float32)
        L.oracle_equal_area_sphere_to_square(*map(float, out), q.ctypes.data_as(F))
        assert _bits(q) == row[5:7], row
    for row in golden["equal_area_dirs"]:
        d = _u(row[:3])
        q = np.zeros(2, np.float32)
        L.oracle_equal_area_sphere_to_square(*map(float, d), q.ctypes.data_as(F))
        assert _bits(q) == row[3:5], row


def test_octahedral_wrap_matches_reference(golden):
    L = binding.lib()
    out = (ctypes.c_int * 2)()
    for res, x, y, xr, yr in golden["octahedral_wrap"]:
        L.oracle_remap_octahedral(x, y, res, out)
        assert (out[0], out[1]) == (xr, yr), (res, x, y)


def test_piecewise_constant_2d_matches_reference(golden):
    func = _u(golden["pc2d_func"])
    rows = golden["pc2d_sample"]
    u = np.array([_u(r[:2]) for r in rows], np.float32)
    out = np.zeros((len(rows), 4), np.float32)
    binding.lib().oracle_pc2d(func.ctypes.data_as(F), 7, 5, len(rows), u.ctypes.data_as(F), out.ctypes.data_as(F))
    assert [_bits(o) for o in out] == [r[2:] for r in rows]


@pytest.fixture(scope="module")
def hdr(tmp_path_factory):
    d = tmp_path_factory.mktemp("env")
    src = d / "shim.cpp"
    src.write_text(
        "#define AVR_HD inline\n"
        f'#include "{ROOT}/acceleratedvolrenderer_amd/csrc/avr_envmap.h"\n'
        'extern "C" {\n'
        "void s2s(int n, const float *uv, float *out) { for (int i = 0; i < n; ++i)\n"
        "  avr::env::square_to_sphere(uv[2 * i], uv[2 * i + 1], out + 3 * i, out + 3 * i + 1, out + 3 * i + 2); }\n"
        "void s2q(int n, const float *d, float *out) { for (int i = 0; i < n; ++i)\n"
        "  avr::env::sphere_to_square(d[3 * i], d[3 * i + 1], d[3 * i + 2], out + 2 * i, out + 2 * i + 1); }\n"
        "int pix(float u, float v, int res) { return avr::env::octahedral_pixel(u, v, res); }\n"
        "}\n")
    so = d / "shim.so"
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-shared", "-fPIC", str(src), "-o", str(so)])
    L = ctypes.CDLL(str(so))
    L.pix.argtypes = [ctypes.c_float, ctypes.c_float, ctypes.c_int]
    return L


def test_device_header_equals_oracle_canonical(hdr, golden):
    rng = np.random.default_rng(3)
    uv = np.concatenate([rng.random((4000, 2)), [[0, 0], [1, 1], [0.5, 0.5], [1, 0], [0, 1]]]).astype(np.float32)
    dev = np.zeros((len(uv), 3), np.float32)
    hdr.s2s(len(uv), uv.ctypes.data_as(F), dev.ctypes.data_as(F))
    binding.set_libm("canonical")
    L = binding.lib()
    ora = np.zeros((len(uv), 3), np.float32)
    for i, (u, v) in enumerate(uv):
        L.oracle_equal_area_square_to_sphere(float(u), float(v), ora[i].ctypes.data_as(F))
    binding.set_libm("platform")
    assert _bits(dev) == _bits(ora)
    d = rng.normal(size=(4000, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    d = d.astype(np.float32)
    q = np.zeros((len(d), 2), np.float32)
    hdr.s2q(len(d), d.ctypes.data_as(F), q.ctypes.data_as(F))
    qo = np.zeros((len(d), 2), np.float32)
    for i, v in enumerate(d):
        L.oracle_equal_area_sphere_to_square(*map(float, v), qo[i].ctypes.data_as(F))
    assert _bits(q) == _bits(qo)
    out = (ctypes.c_int * 2)()
    for res, x, y, xr, yr in golden["octahedral_wrap"]:
        if 0 <= x <= res and 0 <= y <= res:   # reachable from uv in [0, 1]
            assert hdr.pix(x / res, y / res, res) == yr * res + xr


def test_oracle_image_light_furnace(srgb_table):
    """A constant grey map (rgb 0.5: RGBIlluminantSpectrum = 0.5 x D65) around an albedo-1 grey
    medium: every path ends escaping, so E[L(lambda)] = Le(lambda) = 0.5 D65(lambda) x scale.
    NEE through the (uniform, compensated) map distribution and escapes are MIS-combined, so
    the identity holds in expectation, checked per wavelength-normalised sample mean."""
    from acceleratedvolrenderer_amd import scenes, spectra, ImageInfiniteLight
    from acceleratedvolrenderer_amd.scene import Scene
    base = scenes.s_uniform(n=4, width=8, height=8, variant="furnace")
    img = np.full((16, 16, 3), 0.5, np.float32)
    light = ImageInfiniteLight(image=img, rgb_table=srgb_table)
    assert np.all(light.coeffs[..., :3] == 0) or np.all(light.coeffs[..., 2] == 0)   # grey: rsp = 1/2
    scene = Scene(base.camera, base.film, base.medium, [light])
    run = binding.OracleRun(scene, max_depth=1000, seed=0)
    d65 = spectra.TABLES["D65"]
    ratios = []
    for px in range(8):
        for py in range(8):
            for smp in range(16):
                L, lam, _, _ = run.pixel_sample(px, py, smp)
                le = np.float32(0.5) * d65[np.floor(lam + 0.5).astype(int) - 360] * light.scale
                ratios.append(L / le)
    r = np.array(ratios)
    assert np.all(np.isfinite(r))
    m, sd = float(r.mean()), float(r.std() / np.sqrt(r.size))
    assert abs(m - 1) < 5 * sd + 1e-3, (m, sd)


def test_srgb_subset_fixture_converts_the_envmap_like_the_full_table(srgb_table):
    """tests/golden/srgb_table_subset.npz (what the GPU image-light test loads on the box,
    where the reference sources are absent) gives the same coefficients as the full table
    generated by the reference's rgb2spec_opt, for the test's environment map."""
    import os
    import sys
    from acceleratedvolrenderer_amd import RGBToSpectrumTable
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "tests", "golden"))
    from make_srgb_subset import envmap_image
    sub = RGBToSpectrumTable.load(os.path.join(root, "tests", "golden", "srgb_table_subset.npz"))
    img = envmap_image()
    assert np.array_equal(sub.spectrum_coeffs(img).view(np.uint32), srgb_table.spectrum_coeffs(img).view(np.uint32))

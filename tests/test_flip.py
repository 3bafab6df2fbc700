"""FLIP (src/ext/flip/flip.cpp, `imgtool diff --metric FLIP`) against the reference's own FLIP:
tests/golden/flip_vectors.npz holds error maps produced by the unmodified flip.cpp built into
oracle/_ref/flip_ref (generator: oracle/ref/gen_flip_golden.py). The device pipeline
(csrc/avr_flip.h, shared with the k_flip_* kernels), compiled for the host, reproduces them bit
for bit (same libm, same tap order); the GPU path is checked in test_gpu_parity.py."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
F = ctypes.POINTER(ctypes.c_float)
CASES = ("smooth_noise", "edges_ppd20", "identical")


@pytest.fixture(scope="module")
def golden_flip():
    return np.load(os.path.join(ROOT, "tests", "golden", "flip_vectors.npz"))


@pytest.fixture(scope="module")
def hdr(tmp_path_factory):
    d = tmp_path_factory.mktemp("flip")
    src = d / "shim.cpp"
    src.write_text(
        "#define AVR_HD inline\n"
        f'#include "{ROOT}/acceleratedvolrenderer_amd/csrc/avr_flip.h"\n'
        "using namespace avr::flip;\n"
        'extern "C" void run(const float *t, const float *r, int w, int h, float ppd, float *out) {\n'
        "  if (!(ppd > 0)) ppd = ppd_default();\n"
        "  std::vector<float> sf, ef, pf; int rs = spatial_filter(ppd, sf); int rd = detection_filter(ppd, false, ef);\n"
        "  detection_filter(ppd, true, pf); float cmax = max_distance();\n"
        "  std::vector<F4> yT(w * h), yR(w * h);\n"
        "  for (int i = 0; i < w * h; ++i) { yT[i] = prep_pixel(t[3*i], t[3*i+1], t[3*i+2]); yR[i] = prep_pixel(r[3*i], r[3*i+1], r[3*i+2]); }\n"
        "  for (int y = 0; y < h; ++y) for (int x = 0; x < w; ++x)\n"
        "    out[y * w + x] = error_at(yT.data(), yR.data(), w, h, x, y, sf.data(), rs, ef.data(), pf.data(), rd, cmax);\n"
        "}\n")
    so = d / "shim.so"
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-shared", "-fPIC", str(src), "-o", str(so)])
    L = ctypes.CDLL(str(so))
    L.run.argtypes = [F, F, ctypes.c_int, ctypes.c_int, ctypes.c_float, F]
    return L


@pytest.mark.parametrize("case", CASES)
def test_flip_header_matches_reference(hdr, golden_flip, case):
    t = np.ascontiguousarray(golden_flip[case + "_test"], np.float32)
    r = np.ascontiguousarray(golden_flip[case + "_ref"], np.float32)
    want = golden_flip[case + "_flip"]
    out = np.zeros(want.shape, np.float32)
    hdr.run(t.ctypes.data_as(F), r.ctypes.data_as(F), t.shape[1], t.shape[0], float(golden_flip[case + "_ppd"]),
            out.ctypes.data_as(F))
    assert out.view(np.uint32).tolist() == want.view(np.uint32).tolist()


def test_flip_header_matches_reference_binary_on_random_images(hdr, tmp_path):
    """When oracle/_ref/flip_ref was built here: random images and ppds beyond the fixtures."""
    exe = os.path.join(ROOT, "oracle", "_ref", "flip_ref")
    if not os.path.exists(exe):
        pytest.skip("oracle/_ref/flip_ref not built")
    rng = np.random.default_rng(11)
    for k, (h, w, ppd) in enumerate([(17, 23, 0.0), (9, 31, 35.5), (40, 12, 12.0)]):
        t = rng.random((h, w, 3)).astype(np.float32)
        r = np.clip(t + rng.normal(0, 0.1, t.shape), 0, 1).astype(np.float32)
        t.tofile(tmp_path / "t.f32")
        r.tofile(tmp_path / "r.f32")
        subprocess.check_call([exe, str(tmp_path / "t.f32"), str(tmp_path / "r.f32"), str(w), str(h), repr(ppd),
                               str(tmp_path / "o.f32")])
        want = np.fromfile(tmp_path / "o.f32", np.float32).reshape(h, w)
        out = np.zeros((h, w), np.float32)
        hdr.run(t.ctypes.data_as(F), r.ctypes.data_as(F), w, h, ppd, out.ctypes.data_as(F))
        assert out.view(np.uint32).tolist() == want.view(np.uint32).tolist(), k

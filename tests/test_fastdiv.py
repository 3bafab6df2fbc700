"""FastDiv (avr_numerics.h): the camera stage's and k_paths' index splits (sample index ->
(slot, sample), pixel -> (x, y)) divide by a multiply and a shift; floor(n / d) must be exact
for every n < 2^31 and every divisor the host can pass (pass pixel counts, film widths)."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def lib(tmp_path_factory):
    d = tmp_path_factory.mktemp("fdiv")
    src = d / "shim.cpp"
    src.write_text(
        "#define AVR_HD inline\n"
        "#include <cstdint>\n"
        f'#include "{ROOT}/acceleratedvolrenderer_amd/csrc/avr_fastdiv.h"\n'
        'extern "C" long long check(unsigned d, int n, const int *v) {\n'
        "  avr::FastDiv f = avr::fastdiv_make(d); long long bad = 0;\n"
        "  for (int i = 0; i < n; ++i) { int q = avr::fdiv(v[i], f);\n"
        "    bad += q != v[i] / (int)d || avr::fmod_(v[i], q, f) != v[i] % (int)d; }\n"
        "  return bad; }\n")
    so = d / "shim.so"
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-shared", "-fPIC",
                           "-I" + os.path.join(ROOT, "include"), str(src), "-o", str(so)])
    L = ctypes.CDLL(str(so))
    L.check.restype = ctypes.c_longlong
    L.check.argtypes = [ctypes.c_uint, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
    return L


def test_fastdiv_exact(lib):
    rng = np.random.default_rng(11)
    divisors = [1, 2, 3, 5, 7, 24, 33, 64, 100, 1280, 1920, 3840, 921600, 2073600, 2 ** 20 + 1, 2 ** 30,
                2 ** 31 - 1] + [int(x) for x in rng.integers(1, 2 ** 31 - 1, 40)]
    for d in divisors:
        v = np.concatenate([np.arange(0, 4096), rng.integers(0, 2 ** 31 - 1, 20000),
                            np.array([2 ** 31 - 1, 2 ** 31 - 2]),
                            # around every multiple of d near the top of the range and near 0
                            (np.arange(1, 64) * d)[np.arange(1, 64) * d < 2 ** 31 - 1],
                            ((2 ** 31 - 1) // d * d - np.arange(0, 3))]).astype(np.int64)
        v = np.concatenate([v, v - 1, v + 1])
        v = v[(v >= 0) & (v < 2 ** 31)].astype(np.int32)
        v = np.ascontiguousarray(v)
        assert lib.check(d, len(v), v.ctypes.data_as(ctypes.POINTER(ctypes.c_int))) == 0, d

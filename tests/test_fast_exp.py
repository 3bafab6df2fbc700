"""The walk's reject factor (avr_numerics.h fast_exp_m40, k_paths' gray replay walk) equals pbrt's
FastExp (util/math.h:450-471, restated as fast_exp) bit for bit for every x in (-40, 0]: there the
exponent stays inside [-58, 0] and FastExp's two range checks cannot fire."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def lib(tmp_path_factory):
    d = tmp_path_factory.mktemp("fexp")
    src = d / "shim.cpp"
    src.write_text(
        f'#include "{ROOT}/acceleratedvolrenderer_amd/csrc/avr_numerics.h"\n'
        'extern "C" long long check(long long n, const float *x) {\n'
        "  long long bad = 0;\n"
        "  for (long long i = 0; i < n; ++i) bad += avr::f2u(avr::fast_exp_m40(x[i])) != avr::f2u(avr::fast_exp(x[i]));\n"
        "  return bad; }\n")
    so = d / "shim.so"
    # the device header host-compiled: HIP's headers in host-only mode give __host__ __device__
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-shared", "-fPIC", "-D__HIP_PLATFORM_AMD__",
                           "-I/opt/rocm/include", "-I" + os.path.join(ROOT, "include"), str(src), "-o", str(so)])
    L = ctypes.CDLL(str(so))
    L.check.restype = ctypes.c_longlong
    L.check.argtypes = [ctypes.c_longlong, ctypes.POINTER(ctypes.c_float)]
    return L


def test_fast_exp_m40_equals_fast_exp(lib):
    # every float in (-40, 0] with a stride, every 89th float in (-1e-3, 0], the integer and
    # half-integer points of x log2(e), and the ends
    lo = np.float32(-40).view(np.uint32)
    allbits = np.arange(np.uint32(0x80000000), lo, 97, dtype=np.uint64).astype(np.uint32)
    small = np.arange(np.uint32(0x80000000), np.float32(-1e-3).view(np.uint32), 89, dtype=np.uint64).astype(np.uint32)
    k = np.arange(0, 58 * 4 + 1) / 4.0
    edges = (-k / np.log2(np.e)).astype(np.float32)
    edges = np.concatenate([edges, np.nextafter(edges, np.float32(0)), np.nextafter(edges, np.float32(-41))])
    x = np.concatenate([allbits.view(np.float32), small.view(np.float32), edges,
                        np.array([0.0, -0.0, np.nextafter(np.float32(-40), np.float32(0))], np.float32)])
    x = np.ascontiguousarray(x[(x > -40) & (x <= 0)], np.float32)
    assert len(x) > 10 ** 7
    assert lib.check(len(x), x.ctypes.data_as(ctypes.POINTER(ctypes.c_float))) == 0

"""The canonical transcendental convention (acceleratedvolrenderer_amd/csrc/avr_canon.h,
restated in the oracle's "canonical" libm mode):
  * it is the correctly rounded float on the input ranges the path produces (compared with
    the f64 libm result rounded once, itself correctly rounded in practice);
  * the device header, compiled for the host, and the oracle restatement agree bit for bit
    (the GPU parity tests then pin the device build to the oracle)."""
import ctypes
import math
import os
import subprocess

import numpy as np
import pytest

from oracle import binding as ob

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
F = ctypes.c_float
FP = ctypes.POINTER(ctypes.c_float)


def _oracle():
    L = ob.lib()
    for n in ("oracle_canon_log", "oracle_canon_atanh", "oracle_canon_cosh"):
        getattr(L, n).restype = F
        getattr(L, n).argtypes = [F]
    L.oracle_canon_sincos.argtypes = [F, FP, FP]
    return L


@pytest.fixture(scope="module")
def header_lib(tmp_path_factory):
    d = tmp_path_factory.mktemp("canon")
    src = d / "shim.cpp"
    src.write_text(
        "#include <cmath>\n#define AVR_HD inline\n"
        f'#include "{ROOT}/acceleratedvolrenderer_amd/csrc/avr_canon.h"\n'
        'extern "C" {\n'
        "float h_log(float x) { return avr::canon::log_f(x); }\n"
        "float h_atanh(float x) { return avr::canon::atanh_f(x); }\n"
        "float h_cosh(float x) { return avr::canon::cosh_f(x); }\n"
        "void h_sincos(float x, float *s, float *c) { avr::canon::sincos_f(x, s, c); }\n}\n")
    so = d / "shim.so"
    subprocess.check_call(["g++", "-O2", "-ffp-contract=off", "-shared", "-fPIC", str(src), "-o", str(so)])
    L = ctypes.CDLL(str(so))
    for n in ("h_log", "h_atanh", "h_cosh"):
        getattr(L, n).restype = F
        getattr(L, n).argtypes = [F]
    L.h_sincos.argtypes = [F, FP, FP]
    return L


def _inputs(n=40000):
    u = np.random.default_rng(11).random(n, dtype=np.float32)
    return {
        "log": (np.float32(1) - u).astype(np.float32),                                   # 1 - u
        "atanh": (np.float32(0.85691062) - np.float32(1.82750197) * u).astype(np.float32),
        "cosh": (np.float32(0.0072) * (np.float32(470) * u - np.float32(178))).astype(np.float32),
        "sincos": (np.float32(2 * math.pi) * u).astype(np.float32),                       # 2 pi u
    }


def _sincos(fn, x):
    s, c = F(), F()
    fn(float(x), ctypes.byref(s), ctypes.byref(c))
    return np.float32(s.value), np.float32(c.value)


def test_canonical_is_correctly_rounded_on_path_ranges():
    L = _oracle()
    xs = _inputs()
    ref = {"log": math.log, "atanh": math.atanh, "cosh": math.cosh}
    for name in ("log", "atanh", "cosh"):
        fn = getattr(L, f"oracle_canon_{name}")
        bad = sum(np.float32(fn(float(x))).view(np.uint32) != np.float32(ref[name](float(x))).view(np.uint32)
                  for x in xs[name])
        assert bad <= len(xs[name]) * 1e-5, (name, bad)
    bad = 0
    for x in xs["sincos"]:
        s, c = _sincos(L.oracle_canon_sincos, x)
        bad += s != np.float32(math.sin(float(x))) or c != np.float32(math.cos(float(x)))
    assert bad <= len(xs["sincos"]) * 1e-5


def test_canonical_special_values():
    L = _oracle()
    assert L.oracle_canon_log(1.0) == 0.0
    assert L.oracle_canon_log(0.0) == -np.inf
    assert math.isnan(L.oracle_canon_log(-1.0))
    assert L.oracle_canon_atanh(0.0) == 0.0
    assert L.oracle_canon_cosh(0.0) == 1.0
    assert _sincos(L.oracle_canon_sincos, 0.0) == (0.0, 1.0)


def test_device_header_matches_oracle_restatement_bit_for_bit(header_lib):
    L = _oracle()
    xs = _inputs(20000)
    for name in ("log", "atanh", "cosh"):
        a, b = getattr(L, f"oracle_canon_{name}"), getattr(header_lib, f"h_{name}")
        for x in xs[name]:
            assert np.float32(a(float(x))).view(np.uint32) == np.float32(b(float(x))).view(np.uint32), (name, x)
    for x in xs["sincos"]:
        assert _sincos(L.oracle_canon_sincos, x) == _sincos(header_lib.h_sincos, x), x

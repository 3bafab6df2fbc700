"""The compiled C caller of include/avr.h (tests/capi_smoke.c) on an MI355X: the boundary
as pbrt's C++ adapter would use it, without Python in between."""
import os
import subprocess

import pytest

from acceleratedvolrenderer_amd import capi

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_c_caller_renders_beer_lambert(tmp_path):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    capi.load()
    exe = tmp_path / "capi_smoke"
    libdir = os.path.dirname(capi.LIB_PATH)
    subprocess.check_call(["gcc", "-std=c99", "-O2", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "capi_smoke.c"), "-o", str(exe), "-L", libdir, "-lavr_hip",
                           "-Wl,-rpath," + libdir, "-lm"])
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Beer-Lambert" in r.stdout

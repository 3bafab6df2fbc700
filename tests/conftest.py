import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "ref_vectors.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def srgb_table():
    """sRGB RGBToSpectrumTable as the reference's own cmd/rgb2spec_opt generates it
    (oracle/ref/Makefile builds the tool from the reference source into oracle/_ref and runs
    it). Skips where neither the generated table nor the reference sources are present."""
    import subprocess
    path = os.path.join(ROOT, "oracle", "_ref", "srgb_table.inc")
    if not os.path.exists(path):
        if not os.path.isdir("/root/reference/src/pbrt"):
            pytest.skip("sRGB table not generated and reference sources absent")
        subprocess.check_call(["make", "-s", "../_ref/srgb_table.inc"], cwd=os.path.join(ROOT, "oracle", "ref"))
    from acceleratedvolrenderer_amd.rgbspectrum import RGBToSpectrumTable
    cache = os.path.join(ROOT, "oracle", "_ref", "srgb_table.npz")
    if os.path.exists(cache) and os.path.getmtime(cache) >= os.path.getmtime(path):
        return RGBToSpectrumTable.load(cache)
    t = RGBToSpectrumTable.load(path)
    t.save(cache)
    return t

"""EXR / PFM film files (imageio.py) against EXR files pbrt itself wrote (OpenEXR is an
empty submodule here, so the files the reference holds are the fixtures:
tests/golden/exr/ holds two small ones copied from it; the larger ones are read in place
when /root/reference is present).

The ZIP transform is pinned exactly: for every chunk of a pbrt-written file, our encoder's
pre-deflate bytes (even/odd byte split + delta predictor) of the decoded scanlines equal
zlib.decompress of pbrt's chunk."""
import glob
import os
import struct
import zlib

import numpy as np
import pytest

from acceleratedvolrenderer_amd import imageio as io

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = sorted(glob.glob(os.path.join(HERE, "golden", "exr", "*.exr")))
REF = [f for f in ("/root/reference/disney-cloud-720p.exr", "/root/reference/results/ref1.exr")
       if os.path.exists(f)]


def _chunks(path):
    b = open(path, "rb").read()
    img, names, hdr = io.read_exr(path)
    p = 8   # walk the attribute header to the offset table
    while b[p] != 0:
        e = b.index(b"\0", p)
        e2 = b.index(b"\0", e + 1)
        size = struct.unpack("<i", b[e2 + 1:e2 + 5])[0]
        p = e2 + 5 + size
    p += 1
    h = img.shape[0]
    lines = 16 if hdr["compression"] == io.ZIP else 1
    n = (h + lines - 1) // lines
    offs = struct.unpack(f"<{n}Q", b[p:p + 8 * n])
    for off in offs:
        y, size = struct.unpack("<ii", b[off:off + 8])
        yield y - hdr["dataWindow"][1], b[off + 8:off + 8 + size], img, names, hdr


@pytest.mark.parametrize("path", FIX + REF, ids=os.path.basename)
def test_zip_transform_matches_openexr(path):
    checked = stored = 0
    for y0, data, img, names, hdr in _chunks(path):
        if hdr["compression"] != io.ZIP:
            continue
        w = img.shape[1]
        n = min(16, img.shape[0] - y0)
        dt = {1: "<f2", 2: "<f4"}
        types = [t for _, t, _, _ in hdr["channels"]]
        raw = b"".join(img[y, :, c].astype(dt[types[c]]).tobytes() for y in range(y0, y0 + n)
                       for c in range(len(names)))
        if len(data) >= len(raw):       # OpenEXR stores a chunk raw when deflate does not shrink it
            assert data == raw
            stored += 1
            continue
        assert zlib.decompress(io._zip_encode(raw)) == zlib.decompress(data)
        checked += 1
    assert checked + stored > 0


@pytest.mark.parametrize("path", FIX + REF, ids=os.path.basename)
def test_read_pbrt_files(path):
    img, names, hdr = io.read_exr(path)
    assert set("RGB") <= set(names)
    assert np.isfinite(img).all() and img.min() >= 0
    dw = hdr["dataWindow"]
    assert img.shape[:2] == (dw[3] - dw[1] + 1, dw[2] - dw[0] + 1)


def test_cube_metadata():
    img, names, hdr = io.read_exr(os.path.join(HERE, "golden", "exr", "cube.exr"))
    assert hdr["samplesPerPixel"] == 128 and hdr["dataWindow"] == (300, 200, 300, 200)
    assert hdr["displayWindow"] == (0, 0, 639, 479) and hdr["worldToCamera"].shape == (4, 4)


@pytest.mark.parametrize("half", [True, False])
@pytest.mark.parametrize("comp", [io.NONE, io.ZIPS, io.ZIP])
def test_write_read_roundtrip(tmp_path, half, comp):
    rng = np.random.default_rng(0)
    img = (rng.random((37, 53, 3)) * 3).astype(np.float32)
    img[0, 0] = 70000.0                       # fp16 output clamps to 65504 (film.cpp:543-551)
    p = tmp_path / "a.exr"
    io.write_exr(p, img, half=half, compression=comp, samples_per_pixel=64, render_time_seconds=1.5, mse=0.25,
                 world_to_camera=np.eye(4), strings={"renderer": "avr"}, data_window=(10, 20, 62, 56),
                 display_window=(0, 0, 99, 99))
    got = io.read_rgb(p)
    want = np.minimum(img, 65504).astype(np.float16).astype(np.float32) if half else img
    assert np.array_equal(got, want)
    _, names, hdr = io.read_exr(p)
    assert names == ["B", "G", "R"] and hdr["samplesPerPixel"] == 64 and hdr["MSE"] == np.float32(0.25)
    assert hdr["renderer"] == "avr" and hdr["dataWindow"] == (10, 20, 62, 56) and hdr["compression"] == comp


def test_pfm_roundtrip(tmp_path):
    img = np.random.default_rng(1).random((9, 14, 3)).astype(np.float32)
    io.write_pfm(tmp_path / "a.pfm", img)
    assert open(tmp_path / "a.pfm", "rb").read(3) == b"PF\n"
    assert np.array_equal(io.read_pfm(tmp_path / "a.pfm"), img)


def test_imgtool_metrics_restate_image_cpp():
    """Image::ME/MAE/MSE/MRSE (util/image.cpp:543-678) written out as pbrt's loops."""
    from acceleratedvolrenderer_amd import imgtool
    rng = np.random.default_rng(2)
    a = (rng.random((6, 5, 3)) * 2).astype(np.float32)
    r = (rng.random((6, 5, 3)) * 2).astype(np.float32)
    a[1, 2, 0] = np.inf
    for name in ("MAE", "MSE", "MRSE"):
        sums = [0.0, 0.0, 0.0]
        for y in range(6):
            for x in range(5):
                for c in range(3):
                    d = float(a[y, x, c]) - float(r[y, x, c])
                    t = abs(d) if name == "MAE" else (d * d if name == "MSE" else d * d / (float(r[y, x, c]) + 0.01) ** 2)
                    if np.isinf(t):
                        continue
                    sums[c] += t
        want = np.array([s / float(np.float32(5) * np.float32(6)) for s in sums], np.float32)
        assert np.array_equal(imgtool.metric(a, r, name), want), name
    ae, pe, ne = imgtool.metric(a, r, "ME")
    assert np.all(ae >= 0) and np.all(pe >= 0) and np.all(ne <= 0)
    assert np.allclose(ae, pe - ne, rtol=1e-6)


def test_imgtool_cli_on_pbrt_files(tmp_path, capsys):
    from acceleratedvolrenderer_amd import imgtool
    f = os.path.join(HERE, "golden", "exr", "bdpt_d01_s00_t03.exr")
    img = io.read_rgb(f)
    noisy = img + np.float32(0.5)
    io.write_exr(tmp_path / "n.exr", noisy, half=False)
    assert imgtool.main(["diff", "--reference", f, str(tmp_path / "n.exr"), "--metric", "MSE"]) == 1
    out = capsys.readouterr().out
    assert "MSE = 0.250000" in out
    io.write_exr(tmp_path / "e_0.exr", noisy, half=False)
    io.write_exr(tmp_path / "e_1.exr", noisy, half=False)
    assert imgtool.main(["error", "--reference", f, str(tmp_path / "e_*.exr")]) == 0
    assert "MSE estimate = 0.5" in capsys.readouterr().out

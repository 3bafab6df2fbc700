"""Generate tests/golden/srgb_table_subset.npz: the entries of pbrt's sRGB
RGBToSpectrumTable (as the reference's own cmd/rgb2spec_opt generates it: oracle/ref/Makefile
-> oracle/_ref/srgb_table.inc) that the GPU image-light test's environment map touches,
every other coefficient zero. The GPU box has no reference sources, so the GPU test reads
this fixture; the conversion of that image through it is asserted identical to the full
table's here, before the file is written.

usage: python tests/golden/make_srgb_subset.py   (needs oracle/_ref/srgb_table.inc)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from acceleratedvolrenderer_amd.rgbspectrum import RGBToSpectrumTable  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "srgb_table_subset.npz")


def envmap_image(res=32):
    """The environment map of tests/test_gpu_parity.py::test_image_infinite_light_replay."""
    y, x = np.mgrid[0:res, 0:res] / res
    img = np.stack([0.3 + 0.5 * x, 0.2 + 0.6 * y, 0.4 + 0.3 * x * y], 2).astype(np.float32)
    img[5:8, 20:23] = [30, 25, 18]
    return img


def touched(table, rgb):
    """Table cells RGBToSpectrumTable::operator() reads for the spectrum_coeffs of rgb."""
    v = np.maximum(np.asarray(rgb, np.float32).reshape(-1, 3), np.float32(0))
    m = v.max(axis=1)
    scale = (np.float32(2) * m).astype(np.float32)
    q = np.where(scale[:, None] != 0, v / np.where(scale == 0, np.float32(1), scale)[:, None], np.float32(0))
    q = np.maximum(q.astype(np.float32), np.float32(0))
    r, g, b = q[:, 0], q[:, 1], q[:, 2]
    c = q[~((r == g) & (g == b))]
    maxc = np.where(c[:, 0] > c[:, 1], np.where(c[:, 0] > c[:, 2], 0, 2), np.where(c[:, 1] > c[:, 2], 1, 2))
    ar = np.arange(len(c))
    z = c[ar, maxc]
    res = table.res
    x = (c[ar, (maxc + 1) % 3] * np.float32(res - 1)) / z
    y = (c[ar, (maxc + 2) % 3] * np.float32(res - 1)) / z
    xi = np.minimum(x.astype(np.int32), res - 2)
    yi = np.minimum(y.astype(np.int32), res - 2)
    zi = np.clip(np.searchsorted(table.z_nodes, z, side="left") - 1, 0, res - 2)
    mask = np.zeros(table.coeffs.shape[:4], bool)
    for oz in (0, 1):
        for oy in (0, 1):
            for ox in (0, 1):
                mask[maxc, zi + oz, yi + oy, xi + ox] = True
    return mask


def main():
    src = os.path.join(ROOT, "oracle", "_ref", "srgb_table.inc")
    full = RGBToSpectrumTable.load(src)
    img = envmap_image()
    mask = touched(full, img)
    sub = RGBToSpectrumTable(full.z_nodes, np.where(mask[..., None], full.coeffs, np.float32(0)))
    a, b = full.spectrum_coeffs(img), sub.spectrum_coeffs(img)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), "subset table changes the conversion"
    np.savez_compressed(OUT, z_nodes=sub.z_nodes, coeffs=sub.coeffs)
    print(f"{OUT}: {int(mask.sum())} of {mask.size} cells kept, {os.path.getsize(OUT)} bytes")


if __name__ == "__main__":
    main()

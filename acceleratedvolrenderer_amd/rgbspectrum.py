"""RGB -> spectrum for RGBGridMedium's grids (host side of the C-ABI).

pbrt converts each voxel's RGB once at scene creation (RGBGridMedium::Create,
media.cpp:431-450): RGBUnboundedSpectrum / RGBIlluminantSpectrum (spectrum.cpp:236-247) take
m = max(r, g, b), scale = 2m and the sigmoid-polynomial coefficients
RGBColorSpace::ToRGBCoeffs(rgb / scale) = RGBToSpectrumTable::operator() (color.cpp:31-68),
a trilinear lookup in a 3 x 64^3 coefficient table that pbrt's build generates with
cmd/rgb2spec_opt. The device receives {c0, c1, c2, scale} per voxel and evaluates the
sigmoid itself (csrc/avr_kernels.hip rsp_eval).

The table is data, not code: `RGBToSpectrumTable.load(path)` reads rgb2spec_opt's output
file (`rgbspectrum_srgb.cpp` in a pbrt build tree) or a `.npz` saved by `save`. All
arithmetic below is float32 in pbrt's operation order (no fused operations).
"""
import re

import numpy as np

_F = np.float32


class RGBToSpectrumTable:
    res = 64

    def __init__(self, z_nodes, coeffs):
        self.z_nodes = np.ascontiguousarray(z_nodes, np.float32).reshape(self.res)
        self.coeffs = np.ascontiguousarray(coeffs, np.float32).reshape(3, self.res, self.res, self.res, 3)

    @classmethod
    def load(cls, path):
        path = str(path)
        if path.endswith(".npz"):
            z = np.load(path, allow_pickle=False)
            return cls(z["z_nodes"], z["coeffs"])
        with open(path) as f:
            text = f.read()

        def numbers(marker, count):
            start = text.index("=", text.index(marker)) + 1
            body = re.sub(r"[{},;]", " ", text[start:])
            vals = np.array(body.split(None, count)[:count], np.float64).astype(np.float32)
            if len(vals) != count:
                raise ValueError(f"{path}: expected {count} values after {marker}")
            return vals

        n = cls.res
        return cls(numbers("ToSpectrumTable_Scale", n), numbers("ToSpectrumTable_Data", 3 * n * n * n * 3))

    def save(self, path):
        np.savez(path, z_nodes=self.z_nodes, coeffs=self.coeffs)

    def __call__(self, rgb):
        """RGBToSpectrumTable::operator() for rgb (n, 3) in [0, 1]: (n, 3) c0, c1, c2."""
        rgb = np.asarray(rgb, np.float32).reshape(-1, 3)
        n = len(rgb)
        out = np.zeros((n, 3), np.float32)
        r, g, b = rgb[:, 0], rgb[:, 1], rgb[:, 2]
        uni = (r == g) & (g == b)
        with np.errstate(divide="ignore", invalid="ignore"):
            ru = r[uni]
            out[uni, 2] = (ru - _F(.5)) / np.sqrt(ru * (_F(1) - ru))
        idx = np.nonzero(~uni)[0]
        if len(idx) == 0:
            return out
        c = rgb[idx]
        maxc = np.where(c[:, 0] > c[:, 1], np.where(c[:, 0] > c[:, 2], 0, 2), np.where(c[:, 1] > c[:, 2], 1, 2))
        ar = np.arange(len(idx))
        z = c[ar, maxc]
        x = (c[ar, (maxc + 1) % 3] * _F(self.res - 1)) / z
        y = (c[ar, (maxc + 2) % 3] * _F(self.res - 1)) / z
        xi = np.minimum(x.astype(np.int32), self.res - 2)
        yi = np.minimum(y.astype(np.int32), self.res - 2)
        # FindInterval(res, zNodes[i] < z): the last node below z, clamped to [0, res - 2]
        zi = np.clip(np.searchsorted(self.z_nodes, z, side="left") - 1, 0, self.res - 2)
        dx = x - xi.astype(np.float32)
        dy = y - yi.astype(np.float32)
        dz = (z - self.z_nodes[zi]) / (self.z_nodes[zi + 1] - self.z_nodes[zi])

        def lerp(t, a, b):
            return (_F(1) - t) * a + t * b

        T = self.coeffs
        for i in range(3):
            co = lambda ox, oy, oz: T[maxc, zi + oz, yi + oy, xi + ox, i]
            out[idx, i] = lerp(dz, lerp(dy, lerp(dx, co(0, 0, 0), co(1, 0, 0)), lerp(dx, co(0, 1, 0), co(1, 1, 0))),
                               lerp(dy, lerp(dx, co(0, 0, 1), co(1, 0, 1)), lerp(dx, co(0, 1, 1), co(1, 1, 1))))
        return out

    def spectrum_coeffs(self, rgb):
        """RGBUnboundedSpectrum / RGBIlluminantSpectrum(cs, rgb) for rgb (..., 3):
        (..., 4) float32 {c0, c1, c2, scale} (the two share the conversion; the
        illuminant is applied when the spectrum is sampled)."""
        rgb = np.asarray(rgb, np.float32)
        shape = rgb.shape[:-1]
        v = rgb.reshape(-1, 3)
        m = np.max(v, axis=1)
        scale = (_F(2) * m).astype(np.float32)
        with np.errstate(divide="ignore", invalid="ignore"):
            q = np.where(scale[:, None] != 0, v / np.where(scale == 0, _F(1), scale)[:, None], _F(0))
        q = np.maximum(q.astype(np.float32), _F(0))   # ClampZero (colorspace.cpp:43-46)
        out = np.empty((len(v), 4), np.float32)
        out[:, :3] = self(q)
        out[:, 3] = scale
        return out.reshape(shape + (4,))

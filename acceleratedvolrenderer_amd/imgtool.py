"""imgtool's image comparison (cmd/imgtool.cpp `diff` 1049-1238, `error` 921-1047) and the
Image metrics behind it (util/image.cpp:543-678): ME (absolute / positive / negative mean
error, the fork's addition), MAE, MSE, MRSE. Sums are f64 in pbrt's order (rows, then
pixels, per channel) and divided by Float(xres) * Float(yres); infinite terms are skipped.

    python -m acceleratedvolrenderer_amd.imgtool diff --reference ref.exr img.exr [--metric MSE]
    python -m acceleratedvolrenderer_amd.imgtool error --reference ref.exr "img_*.exr" [--metric MRSE]

FLIP (`--metric FLIP`, src/ext/flip) runs on the GPU through the C-ABI (avr_flip): images are
clamped to [0, 1] first and the error is the mean of the FLIP map, as imgtool.cpp:1181-1209.
"""
import argparse
import glob
import sys

import numpy as np

from . import imageio

METRICS = ("ME", "MAE", "MSE", "MRSE", "FLIP")


def _seq_sum(v):
    """Sequential f64 sum (pbrt's loop order): the last element of the running sum."""
    v = np.asarray(v, np.float64).reshape(-1)
    return float(np.cumsum(v)[-1]) if len(v) else 0.0


def _terms(image, reference, metric):
    a = np.asarray(image, np.float32).astype(np.float64)
    r = np.asarray(reference, np.float32).astype(np.float64)
    if a.shape != r.shape:
        raise ValueError(f"resolution mismatch {a.shape} vs {r.shape}")
    d = a - r
    if metric == "MAE":
        t = np.abs(d)
    elif metric == "MSE":
        t = d * d
    elif metric == "MRSE":   # Sqr(v - vref) / Sqr(vref + 0.01): vref float + 0.01 double
        q = r + 0.01
        with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
            t = (d * d) / (q * q)
    else:
        t = d
    return t


def metric(image, reference, metric="MSE"):
    """Image::MAE / MSE / MRSE: per-channel values (float32), or for "ME" the tuple
    (absolute, positive, negative) of per-channel values."""
    if metric not in METRICS:
        raise ValueError(f"{metric}: --metric must be one of {METRICS}")
    t = _terms(image, reference, metric)
    h, w, nc = t.shape
    npix = np.float32(np.float32(w) * np.float32(h))
    if metric != "ME":
        out = np.empty(nc, np.float32)
        for c in range(nc):
            v = t[:, :, c].reshape(-1)
            out[c] = np.float32(_seq_sum(np.where(np.isinf(v), 0.0, v)) / float(npix))
        return out
    res = []
    for sel in (np.abs, lambda v: np.where(v > 0, v, 0.0), lambda v: np.where(v > 0, 0.0, v)):
        out = np.empty(nc, np.float32)
        for c in range(nc):
            v = t[:, :, c].reshape(-1)
            v = np.where(np.isinf(v), 0.0, v)
            out[c] = np.float32(np.float32(_seq_sum(sel(v))) / npix)
        res.append(out)
    return tuple(res)


def channel_average(values):
    """ImageChannelValues::Average: float sum in order, divided by the count."""
    s = np.float32(0)
    for v in np.asarray(values, np.float32):
        s = np.float32(s + v)
    return np.float32(s / np.float32(len(values)))


def average(image):
    """Image::Average(...).Average(): per-channel f64 mean (stored as float), then their mean."""
    a = np.asarray(image, np.float32)
    h, w, nc = a.shape
    return channel_average([np.float32(_seq_sum(a[:, :, c]) / (w * h)) for c in range(nc)])


def flip_map(image, reference, ppd=0.0, device=0):
    """FLIP error map on the GPU (capi.Context.flip); both images clamped to [0, 1] first."""
    from . import capi
    ctx = capi.Context(device)
    try:
        return ctx.flip(np.clip(np.asarray(image, np.float32), 0, 1), np.clip(np.asarray(reference, np.float32), 0, 1),
                        ppd)
    finally:
        ctx.close()


def flip_error(image, reference, ppd=0.0, device=0):
    """imgtool diff --metric FLIP's value: float sum of the map in row order / (xres * yres)."""
    m = flip_map(image, reference, ppd, device)
    s = np.float32(0)
    for v in m.reshape(-1):
        s = np.float32(s + v)
    return np.float32(s / np.float32(m.shape[0] * m.shape[1]))


def diff(image, reference, metric_name="MSE"):
    """imgtool diff on two (H, W, C) images: infinite values clamped to 0 first. Returns a
    dict with the averages, the delta %, and the metric (ME: AE / PE / NE)."""
    img = np.where(np.isinf(image), 0, image).astype(np.float32)
    ref = np.where(np.isinf(reference), 0, reference).astype(np.float32)
    ia, ra = average(img), average(ref)
    out = {"image_average": float(ia), "reference_average": float(ra),
           "delta_percent": float(np.float32(100) * (ia - ra) / ra) if ra != 0 else float("nan")}
    if metric_name == "FLIP":
        out["FLIP"] = float(flip_error(img, ref))
        return out
    m = metric(img, ref, metric_name)
    if metric_name == "ME":
        out.update(AE=float(channel_average(m[0])), PE=float(channel_average(m[1])), NE=float(channel_average(m[2])))
    else:
        out[metric_name] = float(channel_average(m))
    return out


def error_estimate(images, reference, metric_name="MSE"):
    """imgtool error: the metric of each image against the reference, summed and divided
    by (n - 1) as imgtool.cpp:1039 does."""
    if metric_name not in ("MSE", "MRSE", "MAE"):
        raise ValueError("--metric must be MAE, MSE or MRSE")
    total = 0.0
    for im in images:
        total += float(channel_average(metric(im, reference, metric_name)))
    return total / (len(images) - 1) if len(images) > 1 else float("nan")


def main(argv=None):
    ap = argparse.ArgumentParser(prog="imgtool")
    sub = ap.add_subparsers(dest="cmd", required=True)
    d = sub.add_parser("diff")
    d.add_argument("image")
    d.add_argument("--reference", required=True)
    d.add_argument("--metric", default="MSE", choices=METRICS)
    d.add_argument("--channels", default="R,G,B")
    e = sub.add_parser("error")
    e.add_argument("images")
    e.add_argument("--reference", required=True)
    e.add_argument("--metric", default="MSE", choices=("MAE", "MSE", "MRSE"))
    a = ap.parse_args(argv)
    ref = imageio.read_rgb(a.reference)
    if a.cmd == "diff":
        r = diff(imageio.read_rgb(a.image), ref, a.metric)
        if a.metric == "ME":
            print(f"Images differ:\n\t{a.image} {a.reference}\n\tavg = {r['image_average']:f} / "
                  f"{r['reference_average']:f} ({r['delta_percent']:f}% delta), AE = {r['AE']:f}; "
                  f"PE = {r['PE']:f}; NE = {r['NE']:f}")
        else:
            print(f"Images differ:\n\t{a.image} {a.reference}\n\tavg = {r['image_average']:f} / "
                  f"{r['reference_average']:f} ({r['delta_percent']:f}% delta), {a.metric} = {r[a.metric]:f}")
        return 1
    files = sorted(glob.glob(a.images))
    if not files:
        print(f"{a.images}: no matching filenames!", file=sys.stderr)
        return 1
    est = error_estimate([imageio.read_rgb(f) for f in files], ref, a.metric)
    print(f"{a.metric} estimate = {est:.9g}")
    return 0


if __name__ == "__main__":
    sys.exit(main())

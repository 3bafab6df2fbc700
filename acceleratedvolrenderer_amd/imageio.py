"""Film images on disk: OpenEXR (scanline, NONE / ZIPS / ZIP, half or float channels) and PFM.

pbrt writes its film with OpenEXR (RGBFilm::WriteImage -> GetImage -> Image::WriteEXR,
film.cpp:527-565, util/image.cpp:1212-1290): channels R, G, B as half (RGBFilm "savefp16",
default true; values clamped to 65504) or float, ZIP compression (the Imf::Header default),
INCREASING_Y, attributes renderTimeSeconds, worldToCamera, worldToNDC, samplesPerPixel, MSE,
string metadata, and chromaticities when the colour space is not sRGB. OpenEXR is an empty
submodule of the reference; this module implements the published file layout directly
(magic, attribute header, chunk offset table, per-chunk scanlines with channels in
alphabetical order; ZIP = byte split into even/odd halves + delta predictor + zlib) and is
checked against the EXR files pbrt wrote that the reference holds (tests/test_imageio.py).
PFM: Image::WritePFM (util/image.cpp:1795-1850), rows bottom to top, scale -1 (little endian).
"""
import struct
import zlib

import numpy as np

MAGIC = 20000630
NONE, RLE, ZIPS, ZIP = 0, 1, 2, 3
_LINES = {NONE: 1, ZIPS: 1, ZIP: 16}
_HALF, _FLOAT, _UINT = 1, 2, 0
_DT = {_HALF: np.dtype("<f2"), _FLOAT: np.dtype("<f4"), _UINT: np.dtype("<u4")}


def _zip_encode(raw):
    b = np.frombuffer(raw, np.uint8)
    t = np.concatenate([b[0::2], b[1::2]])
    d = t.copy()
    d[1:] = (t[1:].astype(np.int32) - t[:-1].astype(np.int32) + 128 + 256).astype(np.uint8)
    return zlib.compress(d.tobytes())


def _zip_decode(data, raw_size):
    t = np.frombuffer(zlib.decompress(data), np.uint8)
    if len(t) != raw_size:
        raise ValueError("EXR ZIP chunk: bad uncompressed size")
    t = np.cumsum(t.astype(np.int64) - 128) + 128 if len(t) else t   # t[i] = t[i-1] + d[i] - 128
    t = (t & 0xff).astype(np.uint8)
    half = (len(t) + 1) // 2
    out = np.empty(len(t), np.uint8)
    out[0::2] = t[:half]
    out[1::2] = t[half:]
    return out.tobytes()


def _attr(name, typ, payload):
    return name.encode() + b"\0" + typ.encode() + b"\0" + struct.pack("<i", len(payload)) + payload


def write_exr(path, image, channels=("R", "G", "B"), half=True, compression=ZIP, samples_per_pixel=None,
              render_time_seconds=None, mse=None, world_to_camera=None, world_to_ndc=None, strings=None,
              chromaticities=None, data_window=None, display_window=None):
    """Write image (H, W, C) float as a scanline EXR in pbrt's layout.

    half: RGBFilm's fp16 output (values above 65504 clamp to 65504 as GetImage does).
    data_window / display_window: (xmin, ymin, xmax, ymax) inclusive; default the image."""
    img = np.asarray(image, np.float32)
    if img.ndim == 2:
        img = img[:, :, None]
    h, w, nc = img.shape
    if len(channels) != nc:
        raise ValueError("one channel name per image channel")
    if compression not in _LINES:
        raise ValueError("compression must be NONE, ZIPS or ZIP")
    if half:
        img = np.minimum(img, np.float32(65504))
    ptype = _HALF if half else _FLOAT
    order = sorted(range(nc), key=lambda c: channels[c])   # OpenEXR keeps channels sorted by name
    dw = tuple(data_window) if data_window is not None else (0, 0, w - 1, h - 1)
    if dw[2] - dw[0] + 1 != w or dw[3] - dw[1] + 1 != h:
        raise ValueError("data window does not match the image")
    disp = tuple(display_window) if display_window is not None else dw
    attrs = {}
    chl = b"".join(channels[c].encode() + b"\0" + struct.pack("<iB3xii", ptype, 0, 1, 1) for c in order) + b"\0"
    attrs["channels"] = ("chlist", chl)
    attrs["compression"] = ("compression", struct.pack("<B", compression))
    attrs["dataWindow"] = ("box2i", struct.pack("<4i", *dw))
    attrs["displayWindow"] = ("box2i", struct.pack("<4i", *disp))
    attrs["lineOrder"] = ("lineOrder", struct.pack("<B", 0))
    attrs["pixelAspectRatio"] = ("float", struct.pack("<f", 1.0))
    attrs["screenWindowCenter"] = ("v2f", struct.pack("<2f", 0.0, 0.0))
    attrs["screenWindowWidth"] = ("float", struct.pack("<f", 1.0))
    if render_time_seconds is not None:
        attrs["renderTimeSeconds"] = ("float", struct.pack("<f", float(render_time_seconds)))
    if world_to_camera is not None:
        attrs["worldToCamera"] = ("m44f", np.asarray(world_to_camera, "<f4").reshape(16).tobytes())
    if world_to_ndc is not None:
        attrs["worldToNDC"] = ("m44f", np.asarray(world_to_ndc, "<f4").reshape(16).tobytes())
    if samples_per_pixel is not None:
        attrs["samplesPerPixel"] = ("int", struct.pack("<i", int(samples_per_pixel)))
    if mse is not None:
        attrs["MSE"] = ("float", struct.pack("<f", float(mse)))
    for k, v in (strings or {}).items():
        attrs[k] = ("string", v.encode())
    if chromaticities is not None:
        attrs["chromaticities"] = ("chromaticities", struct.pack("<8f", *[float(v) for v in chromaticities]))
    long_names = any(len(k) > 31 for k in attrs) or any(len(c) > 31 for c in channels)
    header = struct.pack("<ii", MAGIC, 2 | (0x400 if long_names else 0))
    header += b"".join(_attr(k, *attrs[k]) for k in sorted(attrs)) + b"\0"
    lines = _LINES[compression]
    nchunks = (h + lines - 1) // lines
    dt = _DT[ptype]
    planes = [np.ascontiguousarray(img[:, :, c]).astype(dt) for c in order]
    chunks = []
    for k in range(nchunks):
        y0, y1 = k * lines, min(h, (k + 1) * lines)
        raw = b"".join(p[y].tobytes() for y in range(y0, y1) for p in planes)
        data = raw
        if compression != NONE:
            z = _zip_encode(raw)
            if len(z) < len(raw):
                data = z
        chunks.append(struct.pack("<ii", dw[1] + y0, len(data)) + data)
    offset = len(header) + 8 * nchunks
    table = []
    for c in chunks:
        table.append(offset)
        offset += len(c)
    with open(path, "wb") as f:
        f.write(header + struct.pack(f"<{nchunks}Q", *table) + b"".join(chunks))


def _parse_attr(typ, v):
    if typ == "int":
        return struct.unpack("<i", v)[0]
    if typ == "float":
        return struct.unpack("<f", v)[0]
    if typ == "box2i":
        return struct.unpack("<4i", v)
    if typ in ("compression", "lineOrder"):
        return v[0]
    if typ == "v2f":
        return struct.unpack("<2f", v)
    if typ == "m44f":
        return np.frombuffer(v, "<f4").reshape(4, 4).copy()
    if typ == "chromaticities":
        return struct.unpack("<8f", v)
    if typ == "string":
        return v.decode(errors="replace")
    if typ == "chlist":
        out, q = [], 0
        while v[q] != 0:
            e = v.index(b"\0", q)
            name = v[q:e].decode()
            ptype, _, xs, ys = struct.unpack("<iB3xii", v[e + 1:e + 17])
            out.append((name, ptype, xs, ys))
            q = e + 17
        return out
    return v


def read_exr(path):
    """Read a single-part scanline EXR (NONE / ZIPS / ZIP): returns (image (H, W, C) float32,
    channel names in file order, header dict)."""
    with open(path, "rb") as f:
        b = f.read()
    magic, version = struct.unpack("<ii", b[:8])
    if magic != MAGIC:
        raise ValueError(f"{path}: not an OpenEXR file")
    if version & 0x200 or version & 0x1000:
        raise ValueError(f"{path}: tiled / multi-part EXR not supported")
    p, hdr = 8, {}
    while b[p] != 0:
        e = b.index(b"\0", p)
        name = b[p:e].decode()
        e2 = b.index(b"\0", e + 1)
        typ = b[e + 1:e2].decode()
        size = struct.unpack("<i", b[e2 + 1:e2 + 5])[0]
        hdr[name] = _parse_attr(typ, b[e2 + 5:e2 + 5 + size])
        p = e2 + 5 + size
    p += 1
    comp = hdr["compression"]
    if comp not in _LINES:
        raise ValueError(f"{path}: compression {comp} not supported (NONE, ZIPS, ZIP)")
    xmin, ymin, xmax, ymax = hdr["dataWindow"]
    w, h = xmax - xmin + 1, ymax - ymin + 1
    chans = hdr["channels"]
    if any(xs != 1 or ys != 1 for _, _, xs, ys in chans):
        raise ValueError(f"{path}: subsampled channels not supported")
    lines = _LINES[comp]
    nchunks = (h + lines - 1) // lines
    offsets = struct.unpack(f"<{nchunks}Q", b[p:p + 8 * nchunks])
    img = np.zeros((h, w, len(chans)), np.float32)
    line_bytes = sum(_DT[t].itemsize for _, t, _, _ in chans) * w
    for off in offsets:
        y, size = struct.unpack("<ii", b[off:off + 8])
        data = b[off + 8:off + 8 + size]
        y0 = y - ymin
        n = min(lines, h - y0)
        raw_size = line_bytes * n
        raw = data if size >= raw_size or comp == NONE else _zip_decode(data, raw_size)
        q = 0
        for yy in range(y0, y0 + n):
            for c, (_, t, _, _) in enumerate(chans):
                nb = _DT[t].itemsize * w
                img[yy, :, c] = np.frombuffer(raw[q:q + nb], _DT[t]).astype(np.float32)
                q += nb
    return img, [c[0] for c in chans], hdr


def read_rgb(path):
    """(H, W, 3) float32 R, G, B of an EXR or PFM file."""
    if str(path).lower().endswith(".pfm"):
        return read_pfm(path)
    img, names, _ = read_exr(path)
    return np.stack([img[:, :, names.index(c)] for c in ("R", "G", "B")], axis=2)


def write_pfm(path, image):
    img = np.asarray(image, np.float32)
    h, w = img.shape[:2]
    with open(path, "wb") as f:
        f.write(b"PF\n%d %d\n%f\n" % (w, h, -1.0))
        f.write(np.ascontiguousarray(img[::-1, :, :3], "<f4").tobytes())


def read_pfm(path):
    with open(path, "rb") as f:
        kind = f.readline().strip()
        w, h = (int(v) for v in f.readline().split())
        scale = float(f.readline())
        nc = 3 if kind == b"PF" else 1
        data = np.frombuffer(f.read(w * h * nc * 4), "<f4" if scale < 0 else ">f4").reshape(h, w, nc)
    img = data[::-1].astype(np.float32) * np.float32(abs(scale))
    return np.repeat(img, 3, axis=2) if nc == 1 else img

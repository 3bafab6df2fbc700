"""`.nvdb` files: NanoVDB's serialized FloatGrid.

pbrt's NanoVDBMedium::Create reads the grid with NanoVDB's `io::readGrid` (media.cpp:487-509;
cmd/nanovdb2pbrt.cpp reads the same files). NanoVDB (openvdb @ 414bed84, feature/nanovdb) is
an un-vendored submodule, so this module restates the published, uncompressed file layout
(nanovdb/util/IO.h + nanovdb/NanoVDB.h, version 32.3) and maps the tree onto `NanoVDBGrid`,
the form the C-ABI's `avr_vdb_grid` takes. PARITY UNPINNED: neither the NanoVDB sources nor
an `.nvdb` asset exist offline, so the reader is checked by round trips through the writer
below (tests/test_nvdb.py) and by rendering a round-tripped grid, not against NanoVDB itself.

File   := Header(16) { MetaData(176) name[nameSize] GridBuffer[fileSize] } x gridCount
Header := magic u64 "NanoVDB0" | version u32 (major<<21|minor<<10|patch) | gridCount u16 | codec u16
          (0 = NONE, 1 = ZIP: the GridBuffer is stored as u64 compressedBytes + one zlib stream
          of it, io::Internal::write/read in nanovdb/util/IO.h; 2 = BLOSC is refused — no blosc
          library here)
GridBuffer := GridData(672) TreeData(64) Root Upper* Lower* Leaf*
  GridData: magic, checksum, version, flags, gridIndex, gridCount, gridSize, name[256],
            Map {matF[9] invMatF[9] vecF[3] taperF, matD[9] invMatD[9] vecD[3] taperD},
            worldBBox (2 x Vec3d), voxelSize Vec3d, gridClass, gridType, blind metadata
  TreeData: nodeOffset[4] (leaf, lower, upper, root; bytes from TreeData), nodeCount[3],
            tileCount[3], voxelCount
  Root:     indexBBox (2 x Coord), tableSize, background, min, max, avg, stddev | Tile[tableSize]
            Tile {key u64, child i64 (bytes from the root, 0 = tile), state u32, value f32} (32 B)
  Upper (32^3 of 128^3 children) / Lower (16^3 of 8^3 leaves): bbox, flags, valueMask,
            childMask, min, max, avg, stddev | table[] of {value f32 | child i64 (bytes from
            the node)}, slot n = ((x & M) >> c) << 2L | ((y & M) >> c) << L | ((z & M) >> c)
  Leaf:     bboxMin Coord, bboxDif u8[3], flags u8, valueMask u64[8], min, max, avg, stddev |
            values f32[512] at ((x & 7) << 6) | ((y & 7) << 3) | (z & 7)
Every node starts on a 32-byte boundary (NANOVDB_DATA_ALIGNMENT).
"""
import struct
import zlib

import numpy as np

from .vdb import NanoVDBGrid

MAGIC = 0x304244566F6E614E          # "NanoVDB0" little endian
VERSION = (32 << 21) | (3 << 10) | 3
GRID_TYPE_FLOAT = 1
GRID_CLASS_FOG_VOLUME = 2
CODEC_NONE = 0
CODEC_ZIP = 1
CODEC_BLOSC = 2
CODECS = {"none": CODEC_NONE, "zip": CODEC_ZIP}

GRID_DATA = 672
TREE_DATA = 64
ROOT_HDR = 64
ROOT_TILE = 32
LEAF_HDR = 96
LEAF_SIZE = LEAF_HDR + 512 * 4
LEAF_DTYPE = np.dtype([("bmin", "<i4", 3), ("dif", "u1", 3), ("flags", "u1"), ("mask", "u1", 64),
                       ("stats", "<f4", 4), ("values", "<f4", 512)])
assert LEAF_DTYPE.itemsize == LEAF_SIZE


def _align(n, a=32):
    return (n + a - 1) // a * a


class _Level:
    """An internal node level: LOG2DIM and the log2 edge of its children (in voxels)."""

    def __init__(self, log2dim, child_total):
        self.log2dim, self.child_total = log2dim, child_total
        self.total = log2dim + child_total
        self.slots = 1 << (3 * log2dim)
        mask_bytes = self.slots // 8
        self.hdr = _align(24 + 8 + 2 * mask_bytes + 16)
        self.size = self.hdr + 8 * self.slots
        self.mask_bytes = mask_bytes

    def slot(self, ijk):
        m = (1 << self.total) - 1
        x, y, z = ((int(v) & m) >> self.child_total for v in ijk)
        return (x << (2 * self.log2dim)) | (y << self.log2dim) | z


UPPER = _Level(5, 7)    # 32^3 children of 128^3 voxels
LOWER = _Level(4, 3)    # 16^3 leaves of 8^3 voxels


def root_key(ijk):
    """RootNode::CoordToKey (32-bit coordinates, upper nodes of 4096^3 voxels)."""
    x, y, z = (int(np.uint32(np.int64(v) & 0xFFFFFFFF)) >> 12 for v in ijk)
    return z | (y << 21) | (x << 42)


def _set_bit(mask, n):
    mask[n >> 3] |= np.uint8(1 << (n & 7))


def _bit(mask, n):
    return (int(mask[n >> 3]) >> (n & 7)) & 1


def _split_tiles(grid):
    """The grid's tiles as NanoVDB's tile levels: 4096 (root), 128 (upper), 8 (lower) edges."""
    out = []
    for o, s, v in zip(grid.tile_origins, grid.tile_sizes, grid.tile_values):
        s = int(s)
        if s in (8, 128, 4096) and np.all(np.asarray(o) % s == 0):
            out.append((tuple(int(c) for c in o), s, np.float32(v)))
            continue
        for dz in range(0, s, 8):
            for dy in range(0, s, 8):
                for dx in range(0, s, 8):
                    out.append(((int(o[0]) + dx, int(o[1]) + dy, int(o[2]) + dz), 8, np.float32(v)))
    return out


def grid_buffer(grid, name="density"):
    """Serialize a NanoVDBGrid as one NanoVDB FloatGrid buffer (bytes)."""
    bg = np.float32(grid.background)
    leaves = [tuple(int(c) for c in o) for o in grid.leaf_origins]
    tiles = _split_tiles(grid)
    # node sets: upper origins (multiples of 4096) and lower origins (multiples of 128)
    up_of = lambda p: tuple((c >> 12) << 12 for c in p)
    lo_of = lambda p: tuple((c >> 7) << 7 for c in p)
    uppers, lowers = {}, {}
    for p in leaves:
        uppers.setdefault(up_of(p), None)
        lowers.setdefault(lo_of(p), None)
    for p, s, _ in tiles:
        if s == 8:
            uppers.setdefault(up_of(p), None)
            lowers.setdefault(lo_of(p), None)
        elif s == 128:
            uppers.setdefault(up_of(p), None)
    root_tiles = [(p, v) for p, s, v in tiles if s == 4096]
    up_list = sorted(uppers, key=root_key)
    lo_list = sorted(lowers, key=lambda p: (root_key(p), UPPER.slot(p)))
    up_index = {p: i for i, p in enumerate(up_list)}
    lo_index = {p: i for i, p in enumerate(lo_list)}
    n_root = len(up_list) + len(root_tiles)
    root_size = _align(ROOT_HDR + ROOT_TILE * n_root)
    off_root = GRID_DATA + TREE_DATA
    off_up = off_root + root_size
    off_lo = off_up + UPPER.size * len(up_list)
    off_leaf = off_lo + LOWER.size * len(lo_list)
    total = off_leaf + LEAF_SIZE * len(leaves)
    buf = bytearray(total)

    # ---- leaves (one structured array: bbox of the active voxels, value mask, stats, values)
    lvals = np.asarray(grid.leaf_values, np.float32).reshape(-1, 512)
    if len(leaves):
        active = lvals != bg
        lin = np.arange(512)
        coords = np.stack([lin >> 6, (lin >> 3) & 7, lin & 7], 1)          # (512, 3) x, y, z
        big = np.where(active[:, :, None], coords[None], 8).min(axis=1)
        small = np.where(active[:, :, None], coords[None], -1).max(axis=1)
        none = ~active.any(axis=1)
        big[none] = 0
        small[none] = 0
        rec = np.zeros(len(leaves), LEAF_DTYPE)
        rec["bmin"] = grid.leaf_origins + big
        rec["dif"] = (small - big).astype(np.uint8)
        rec["mask"] = np.packbits(active, axis=1, bitorder="little")
        rec["stats"] = np.stack([lvals.min(1), lvals.max(1), lvals.mean(1), lvals.std(1)], 1)
        rec["values"] = lvals
        buf[off_leaf:off_leaf + LEAF_SIZE * len(leaves)] = rec.tobytes()
        vmin_l, vmax_l = float(lvals.min()), float(lvals.max())
    else:
        vmin_l = vmax_l = float(bg)

    def write_internal(level, o, origin, entries):
        """entries: slot -> ("child", byte offset of the child) or ("tile", value, active)."""
        vmask = np.zeros(level.mask_bytes, np.uint8)
        cmask = np.zeros(level.mask_bytes, np.uint8)
        table = np.zeros(level.slots, np.int64)
        tview = table.view(np.float32).reshape(level.slots, 2)
        tview[:, 0] = bg
        for n, e in entries.items():
            if e[0] == "child":
                _set_bit(cmask, n)
                table[n] = e[1] - o
            else:
                tview[n, 0] = e[1]
                tview[n, 1] = 0.0
                if e[2]:
                    _set_bit(vmask, n)
        edge = 1 << level.total
        struct.pack_into("<6i", buf, o, *origin, *(c + edge - 1 for c in origin))
        struct.pack_into("<Q", buf, o + 24, 0)
        buf[o + 32:o + 32 + level.mask_bytes] = vmask.tobytes()
        buf[o + 32 + level.mask_bytes:o + 32 + 2 * level.mask_bytes] = cmask.tobytes()
        struct.pack_into("<4f", buf, o + 32 + 2 * level.mask_bytes, 0.0, 0.0, 0.0, 0.0)
        buf[o + level.hdr:o + level.size] = table.astype("<i8").tobytes()

    lo_entries = {p: {} for p in lo_list}
    for k, p in enumerate(leaves):
        lo_entries[lo_of(p)][LOWER.slot(p)] = ("child", off_leaf + k * LEAF_SIZE)
    up_entries = {p: {} for p in up_list}
    for p, s, v in tiles:
        if s == 8:
            lo_entries[lo_of(p)][LOWER.slot(p)] = ("tile", v, bool(v != bg))
        elif s == 128:
            up_entries[up_of(p)][UPPER.slot(p)] = ("tile", v, bool(v != bg))
    for i, p in enumerate(lo_list):
        o = off_lo + i * LOWER.size
        write_internal(LOWER, o, p, lo_entries[p])
        up_entries[up_of(p)][UPPER.slot(p)] = ("child", o)
    for i, p in enumerate(up_list):
        write_internal(UPPER, off_up + i * UPPER.size, p, up_entries[p])

    # ---- root: index bbox, background, stats; tiles sorted by key
    bb = [int(c) for c in grid.index_bbox]
    vmin = min([vmin_l] + [float(t[2]) for t in tiles] + [float(bg)])
    vmax = max([vmax_l] + [float(t[2]) for t in tiles] + [float(bg)])
    struct.pack_into("<6iI5f", buf, off_root, *bb, n_root, float(bg), vmin, vmax, 0.0, 0.0)
    rt = [(root_key(p), off_up + up_index[p] * UPPER.size - off_root, 0, float(bg)) for p in up_list]
    rt += [(root_key(p), 0, int(v != bg), float(v)) for p, v in root_tiles]
    for k, (key, child, state, val) in enumerate(sorted(rt)):
        struct.pack_into("<QqIf", buf, off_root + ROOT_HDR + k * ROOT_TILE, key, child, state, val)

    # ---- tree and grid headers
    struct.pack_into("<4Q3I3IQ", buf, GRID_DATA, off_leaf - GRID_DATA, off_lo - GRID_DATA, off_up - GRID_DATA,
                     off_root - GRID_DATA, len(leaves), len(lo_list), len(up_list),
                     sum(1 for t in tiles if t[1] == 8), sum(1 for t in tiles if t[1] == 128), len(root_tiles),
                     int(np.count_nonzero(lvals != bg)))
    m = np.asarray(grid.index_to_world, np.float64)
    inv = np.asarray(grid.world_to_index, np.float64)
    nm = name.encode()[:255]
    struct.pack_into("<QQIIIIQ", buf, 0, MAGIC, 0, VERSION, 0, 0, 1, total)
    buf[40:40 + len(nm)] = nm
    mo = 296
    struct.pack_into("<9f9f3ff", buf, mo, *m[:, :3].ravel().astype(np.float32).tolist(),
                     *inv.ravel().astype(np.float32).tolist(), *m[:, 3].astype(np.float32).tolist(), 1.0)
    struct.pack_into("<9d9d3dd", buf, mo + 88, *m[:, :3].ravel().tolist(), *inv.ravel().tolist(), *m[:, 3].tolist(), 1.0)
    lo, hi = grid.world_bbox()
    struct.pack_into("<6d", buf, 560, *[float(v) for v in lo], *[float(v) for v in hi])
    struct.pack_into("<3d", buf, 608, *[float(np.linalg.norm(m[:, k])) for k in range(3)])
    struct.pack_into("<IIqI", buf, 632, GRID_CLASS_FOG_VOLUME, GRID_TYPE_FLOAT, 0, 0)
    return bytes(buf)


def write_nvdb(path, grids, codec="none"):
    """Write {name: NanoVDBGrid} (or [(name, grid)]) as an .nvdb file, uncompressed (codec
    "none") or ZIP-coded ("zip": each grid buffer as u64 compressed size + zlib stream, as
    NanoVDB's io::Internal::write does with NANOVDB_USE_ZIP)."""
    if codec not in CODECS:
        raise ValueError(f"codec {codec!r}: one of {sorted(CODECS)} (BLOSC is not available)")
    cid = CODECS[codec]
    items = list(grids.items()) if isinstance(grids, dict) else list(grids)
    with open(path, "wb") as f:
        f.write(struct.pack("<QIHH", MAGIC, VERSION, len(items), cid))
        for name, g in items:
            gb = grid_buffer(g, name)
            if cid == CODEC_ZIP:
                z = zlib.compress(gb)
                stored = struct.pack("<Q", len(z)) + z
            else:
                stored = gb
            nm = name.encode() + b"\0"
            lo, hi = g.world_bbox()
            vc = int(np.count_nonzero(np.asarray(g.leaf_values) != g.background))
            f.write(struct.pack("<QQQQII6d6i3dI4I3IHHI", len(gb), len(stored), 0, vc, GRID_TYPE_FLOAT,
                                GRID_CLASS_FOG_VOLUME, *[float(v) for v in lo], *[float(v) for v in hi],
                                *[int(c) for c in g.index_bbox], 1.0, 1.0, 1.0, len(nm),
                                *_node_counts(gb), 0, 0, 0, cid, 0, VERSION))
            f.write(nm)
            f.write(stored)


def _node_counts(gb):
    return list(struct.unpack_from("<3I", gb, GRID_DATA + 32)) + [1]


def list_grids(path):
    """[(name, grid type, codec, fileSize)] of an .nvdb file."""
    return [(n, t, c, s) for n, t, c, s, _ in _segments(path)]


def _segments(path):
    with open(path, "rb") as f:
        head = f.read(16)
        if len(head) < 16:
            raise ValueError(f"{path}: not a NanoVDB file (too short)")
        magic, version, count, codec = struct.unpack("<QIHH", head)
        if magic != MAGIC:
            raise ValueError(f"{path}: bad NanoVDB magic number {magic:#x}")
        if (version >> 21) != 32:
            raise ValueError(f"{path}: NanoVDB major version {version >> 21} (this reader restates 32)")
        out = []
        for _ in range(count):
            md = f.read(176)
            if len(md) < 176:
                raise ValueError(f"{path}: truncated grid metadata")
            grid_size, file_size = struct.unpack_from("<QQ", md, 0)
            gtype = struct.unpack_from("<I", md, 32)[0]
            name_size = struct.unpack_from("<I", md, 136)[0]
            gcodec = struct.unpack_from("<H", md, 176 - 8)[0]
            name = f.read(name_size).rstrip(b"\0").decode(errors="replace")
            pos = f.tell()
            f.seek(file_size, 1)
            out.append((name, gtype, gcodec if gcodec else codec, file_size, (pos, grid_size, file_size)))
        return out


def read_nvdb(path, name=None):
    """NanoVDB io::readGrid(path[, name]) for an uncompressed or ZIP-coded FloatGrid ->
    NanoVDBGrid (the first grid when name is None, as NanoVDBMedium::Create's readGrid does)."""
    segs = _segments(path)
    if not segs:
        raise ValueError(f"{path}: no grids")
    pick = segs[0] if name is None else next((s for s in segs if s[0] == name), None)
    if pick is None:
        raise ValueError(f"{path}: no grid named {name!r} (grids: {[s[0] for s in segs]})")
    gname, gtype, codec, fsize, (pos, gsize, stored) = pick
    if codec not in (CODEC_NONE, CODEC_ZIP):
        raise ValueError(f"{path}: grid {gname!r} uses codec {codec} (BLOSC); only uncompressed and ZIP grids are read")
    if gtype != GRID_TYPE_FLOAT:
        raise ValueError(f"{path}: grid {gname!r} has type {gtype}, NanoVDBMedium needs a FloatGrid")
    with open(path, "rb") as f:
        f.seek(pos)
        raw = f.read(stored if codec == CODEC_ZIP else gsize)
    if codec == CODEC_ZIP:
        # io::Internal::read: u64 residual, then uncompress(residual bytes) into gridSize bytes
        if len(raw) < 8:
            raise ValueError(f"{path}: grid {gname!r}: truncated ZIP stream")
        n = struct.unpack_from("<Q", raw, 0)[0]
        if 8 + n > len(raw):
            raise ValueError(f"{path}: grid {gname!r}: ZIP stream of {n} bytes exceeds the stored {len(raw) - 8}")
        try:
            buf = zlib.decompress(raw[8:8 + n])
        except zlib.error as e:
            raise ValueError(f"{path}: grid {gname!r}: bad ZIP stream ({e})") from None
        if len(buf) != gsize:
            raise ValueError(f"{path}: grid {gname!r}: ZIP stream holds {len(buf)} bytes, gridSize is {gsize}")
    else:
        buf = raw
    if len(buf) < gsize:
        raise ValueError(f"{path}: grid {gname!r}: truncated grid buffer")
    return parse_grid_buffer(buf)


def parse_grid_buffer(buf):
    mv = memoryview(buf)
    magic, _, version = struct.unpack_from("<QQI", mv, 0)
    if magic != MAGIC:
        raise ValueError("grid buffer: bad magic number")
    gclass, gtype = struct.unpack_from("<II", mv, 632)
    if gtype != GRID_TYPE_FLOAT:
        raise ValueError(f"grid buffer: grid type {gtype}, expected Float")
    matD = np.array(struct.unpack_from("<9d", mv, 296 + 88)).reshape(3, 3)
    vecD = np.array(struct.unpack_from("<3d", mv, 296 + 88 + 144))
    m = np.concatenate([matD, vecD[:, None]], axis=1)
    off = struct.unpack_from("<4Q", mv, GRID_DATA)
    root = GRID_DATA + off[3]
    bb = struct.unpack_from("<6i", mv, root)
    table_size = struct.unpack_from("<I", mv, root + 24)[0]
    bg = np.float32(struct.unpack_from("<f", mv, root + 28)[0])
    leaf_off, tiles = [], []

    def walk_internal(level, o, child_fn):
        vmask = np.frombuffer(mv, np.uint8, level.mask_bytes, o + 32)
        cmask = np.frombuffer(mv, np.uint8, level.mask_bytes, o + 32 + level.mask_bytes)
        table = np.frombuffer(mv, "<i8", level.slots, o + level.hdr)
        origin = np.array(struct.unpack_from("<3i", mv, o))
        cbits = np.unpackbits(cmask, bitorder="little").astype(bool)
        vbits = np.unpackbits(vmask, bitorder="little").astype(bool)
        vals = table.view(np.float32).reshape(-1, 2)[:, 0]
        edge = 1 << level.child_total
        L = level.log2dim
        for n in np.nonzero(cbits)[0]:
            child_fn(o + int(table[n]))
        for n in np.nonzero(~cbits & (vbits | (vals != bg)))[0]:
            x, y, z = (int(n) >> (2 * L)) & ((1 << L) - 1), (int(n) >> L) & ((1 << L) - 1), int(n) & ((1 << L) - 1)
            tiles.append((origin + np.array([x, y, z]) * edge, edge, vals[n]))

    for k in range(table_size):
        key, child, state, val = struct.unpack_from("<QqIf", mv, root + ROOT_HDR + k * ROOT_TILE)
        if child:
            walk_internal(UPPER, root + child, lambda lo: walk_internal(LOWER, lo, leaf_off.append))
        elif state or np.float32(val) != bg:
            x, y, z = (key >> 42) & 0x1FFFFF, (key >> 21) & 0x1FFFFF, key & 0x1FFFFF
            c = [np.int32(np.uint32(v << 12)) for v in (x, y, z)]
            tiles.append((np.array(c), 4096, np.float32(val)))
    # leaves are one contiguous array (TreeData::mNodeOffset[0], mNodeCount[0]); the tree walk
    # gives the ones reachable from the root
    leaf0 = GRID_DATA + off[0]
    n_all = struct.unpack_from("<I", mv, GRID_DATA + 32)[0]
    rel = np.asarray(leaf_off, np.int64) - leaf0
    if len(rel) and (np.any(rel % LEAF_SIZE) or rel.min() < 0 or rel.max() >= LEAF_SIZE * n_all):
        raise ValueError("grid buffer: leaf outside the leaf array")
    arr = np.frombuffer(mv, LEAF_DTYPE, n_all, leaf0)[rel // LEAF_SIZE]
    # the leaf's origin: bboxMin rounded down to the leaf grid
    origins = ((arr["bmin"] >> 3) << 3).astype(np.int32)
    values = np.ascontiguousarray(arr["values"], np.float32)
    if tiles:
        to = np.array([t[0] for t in tiles], np.int32)
        ts = np.array([t[1] for t in tiles], np.int32)
        tv = np.array([t[2] for t in tiles], np.float32)
    else:
        to, ts, tv = None, None, None
    return NanoVDBGrid(origins, values.reshape(-1, 8, 8, 8), bg, to, ts, tv, index_bbox=bb, index_to_world=m)

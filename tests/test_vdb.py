"""NanoVDBMedium's sparse grids (media.h:602-685, media.cpp:511-616) on the CPU.

NanoVDB (openvdb @ 414bed84, feature/nanovdb) is an empty submodule of the reference and
no reference test or asset exercises NanoVDBMedium: PARITY UNPINNED. What is checked:
  * the host container (vdb.NanoVDBGrid) and the oracle's tree restatement return the
    dense values they were built from (leaves, tiles, background, negative origins);
  * SURVEY.md §8f's self-consistency: a dense grid read as GridMedium (SampledGrid,
    voxel centres at (i + 0.5) / n) and as a NanoVDB grid whose map puts index i at world
    (i + 0.5) / n sample the same trilinear density (to float rounding of the two maps);
  * the 64^3 majorant bounds every sampled density in its cell (conservative);
  * the device header (csrc/avr_vdb.h, host-compiled) equals the oracle bit for bit;
  * cmd/nanovdb2pbrt.cpp's dense dump (to_grid_medium).
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from acceleratedvolrenderer_amd import NanoVDBGrid, NanoVDBMedium
from oracle import binding

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _dense(seed=1, shape=(13, 11, 9)):
    rng = np.random.default_rng(seed)
    d = rng.random(shape).astype(np.float32)
    d[:3] = 0.0
    return d


def _rotated_map(n):
    """index -> world: scale 1/n, rotation about y by 20 degrees, translation."""
    c, s = np.cos(np.radians(20)), np.sin(np.radians(20))
    m = np.eye(4)
    m[:3, :3] = np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]]) @ np.diag([1.0 / n, 1.3 / n, 0.8 / n])
    m[:3, 3] = [0.1, -0.05, 0.2]
    return m


def test_from_dense_values_tiles_and_roundtrip(tmp_path):
    d = _dense()
    d[8:, 0:8, 0:8] = 0.0
    d[8:13, 0:8, 0:8] = 0.0
    g = NanoVDBGrid.from_dense(d, index_min=(-3, 2, 5), voxel_size=0.1, origin=(0.2, -0.1, 0.05))
    # a block-aligned constant region becomes a tile
    e = np.zeros((16, 16, 16), np.float32)
    e[8:16, 0:8, 8:16] = 0.75
    e[0, 0, 0] = 0.25
    gt = NanoVDBGrid.from_dense(e, index_min=(-8, 0, 8))
    assert len(gt.tile_values) == 1 and gt.tile_values[0] == np.float32(0.75)
    assert len(gt.leaf_origins) == 1
    rng = np.random.default_rng(2)
    for grid, dense, mn in ((g, d, (-3, 2, 5)), (gt, e, (-8, 0, 8))):
        tree = binding.VdbTree(grid)
        pts = rng.integers(-20, 30, (3000, 3))
        rel = pts - np.asarray(mn)
        inside = np.all((rel >= 0) & (rel < np.asarray(dense.shape)[::-1]), axis=1)
        want = np.zeros(len(pts), np.float32)
        want[inside] = dense[rel[inside, 2], rel[inside, 1], rel[inside, 0]]
        assert np.array_equal(grid.values(pts), want)
        assert np.array_equal(np.array([tree.value(*p) for p in pts], np.float32), want)
    # active bbox: voxels != background
    act = np.argwhere(d != 0)
    assert g.index_bbox.tolist() == (act.min(0)[::-1] + (-3, 2, 5)).tolist() + (act.max(0)[::-1] + (-3, 2, 5)).tolist()
    g.save(tmp_path / "g.npz")
    h = NanoVDBGrid.load(tmp_path / "g.npz")
    pts = rng.integers(-20, 30, (500, 3))
    assert np.array_equal(h.values(pts), g.values(pts))
    assert h.index_bbox.tolist() == g.index_bbox.tolist()


@pytest.mark.parametrize("case", ["offset", "aligned", "background", "notiles"])
def test_from_dense_torch_equals_numpy(case):
    """The torch block classification (used for device-generated 1024^3 grids: bench.py's
    NanoVDB leg, the full-size NanoVDB replay test) builds exactly the tree of the numpy one."""
    torch = pytest.importorskip("torch")
    d = _dense(3, (24, 16, 21))
    d[8:16, 0:8, 0:8] = 0.5       # constant blocks -> tiles (where block-aligned)
    d[16:24, 8:16, 8:16] = 0.0
    kw = {"offset": dict(index_min=(-3, 2, 5)), "aligned": dict(index_min=(8, -16, 0)),
          "background": dict(index_min=(1, 1, 1), background=0.5), "notiles": dict(tiles=False)}[case]
    a = NanoVDBGrid.from_dense(d, **kw)
    b = NanoVDBGrid.from_dense(torch.from_numpy(d), **kw)
    ka = np.lexsort(a.leaf_origins.T[::-1])
    kb = np.lexsort(b.leaf_origins.T[::-1])
    assert np.array_equal(a.leaf_origins[ka], b.leaf_origins[kb])
    assert np.array_equal(a.leaf_values[ka].view(np.uint32), b.leaf_values[kb].view(np.uint32))
    ta, tb = np.lexsort(a.tile_origins.T[::-1]), np.lexsort(b.tile_origins.T[::-1])
    assert np.array_equal(a.tile_origins[ta], b.tile_origins[tb])
    assert np.array_equal(a.tile_values[ta], b.tile_values[tb]) and np.array_equal(a.tile_sizes, b.tile_sizes)
    assert a.index_bbox.tolist() == b.index_bbox.tolist() and a.background == b.background
    assert np.array_equal(a.index_to_world, b.index_to_world)
    if case == "aligned":   # scenes.vdb_grid takes the tensor as it is (bench.py's NanoVDB leg)
        from acceleratedvolrenderer_amd import scenes
        c, e = scenes.vdb_grid(torch.from_numpy(d)), scenes.vdb_grid(d)
        assert np.array_equal(c.leaf_values, e.leaf_values) and np.array_equal(c.index_to_world, e.index_to_world)


def test_world_bbox_python_equals_oracle():
    g = NanoVDBGrid.from_dense(_dense(), index_min=(1, -4, 0), index_to_world=_rotated_map(9))
    t = NanoVDBGrid.from_dense(_dense(3, (5, 5, 5)) * 3000, index_min=(20, 0, 0), index_to_world=_rotated_map(9))
    tree, ttree = binding.VdbTree(g), binding.VdbTree(t)
    assert np.array_equal(binding.vdb_bounds(tree), np.concatenate(g.world_bbox()))
    med = NanoVDBMedium(g, temperature=t)
    assert np.array_equal(binding.vdb_bounds(tree, ttree), med.bounds)
    assert np.all(med.bounds[3:] >= np.concatenate(t.world_bbox())[3:])


def test_nanovdb_matches_gridmedium_sampling():
    """Same dense data as SampledGrid (GridMedium) and as a NanoVDB grid mapped so that
    index i sits at world (i + 0.5) / n: trilinear densities agree to float rounding."""
    n = 12
    d = (0.2 + np.random.default_rng(4).random((n, n, n))).astype(np.float32)
    m = np.eye(4)
    m[:3, :3] /= n
    m[:3, 3] = 0.5 / n
    g = NanoVDBGrid.from_dense(d, index_to_world=m)
    tree = binding.VdbTree(g)
    p = np.random.default_rng(5).random((4000, 3)).astype(np.float32)
    vdb = tree.sample_world(p)
    L = binding.lib()
    grid = np.array([L.oracle_grid_lookup(binding.fp(d), n, n, n, *map(float, q)) for q in p], np.float32)
    assert np.max(np.abs(vdb - grid)) < 2e-5


def test_majorant_is_conservative():
    g = NanoVDBGrid.from_dense(_dense(6, (20, 17, 23)), index_min=(-5, 3, 1), index_to_world=_rotated_map(20))
    tree = binding.VdbTree(g)
    b = binding.vdb_bounds(tree)
    res = 8
    maj = binding.vdb_majorant(tree, b, (res, res, res))
    rng = np.random.default_rng(7)
    p = (b[:3] + rng.random((20000, 3)) * (b[3:] - b[:3])).astype(np.float32)
    dens = tree.sample_world(p)
    cell = np.clip(((p - b[:3]) / (b[3:] - b[:3]) * res).astype(int), 0, res - 1)
    mv = maj[cell[:, 0] + res * (cell[:, 1] + res * cell[:, 2])]
    assert np.all(dens <= mv)
    assert dens.max() > 0.5   # the sample actually hits the grid


def test_to_grid_medium_is_nanovdb2pbrt_dump():
    d = _dense(8, (9, 10, 11))
    g = NanoVDBGrid.from_dense(d, index_min=(2, 3, 4), voxel_size=0.5)
    vals, p0, p1 = g.to_grid_medium()
    b = g.index_bbox
    assert vals.shape == (b[5] - b[2] + 2, b[4] - b[1] + 2, b[3] - b[0] + 2)
    # [min, max + 1] inclusive: the last plane is past the active voxels (background here)
    assert np.all(vals[-1] == 0) and np.all(vals[:, -1] == 0) and np.all(vals[:, :, -1] == 0)
    z0 = b[2] - 4
    assert np.array_equal(vals[:-1, :-1, :-1], d[z0:z0 + vals.shape[0] - 1, b[1] - 3:b[4] - 2, b[0] - 2:b[3] - 1])
    assert np.allclose(p0, 0.5 * b[:3]) and np.allclose(p1, 0.5 * (b[3:] + 1))


def _slots(grid):
    """The device's block-slot layout (avr_capi.hip upload_vdb), built here for the
    host-compiled header test."""
    boxes = [(o, 8) for o in grid.leaf_origins] + list(zip(grid.tile_origins, grid.tile_sizes))
    lo = np.min([o for o, _ in boxes], axis=0)
    hi = np.max([o + s for o, s in boxes], axis=0)
    nb = (hi - lo) // 8
    slot = np.full((nb[2], nb[1], nb[0]), np.iinfo(np.int32).min, np.int32)
    for t, (o, s) in enumerate(zip(grid.tile_origins, grid.tile_sizes)):
        b = (o - lo) // 8
        slot[b[2]:b[2] + s // 8, b[1]:b[1] + s // 8, b[0]:b[0] + s // 8] = -(t + 1)
    for i, o in enumerate(grid.leaf_origins):
        b = (o - lo) // 8
        slot[b[2], b[1], b[0]] = i
    return slot, lo, nb


@pytest.fixture(scope="module")
def hdr(tmp_path_factory):
    d = tmp_path_factory.mktemp("vdb")
    src = d / "shim.cpp"
    src.write_text(
        "#define AVR_HD inline\n"
        f'#include "{ROOT}/acceleratedvolrenderer_amd/csrc/avr_vdb.h"\n'
        "using namespace avr::vdb;\n"
        'extern "C" void sample(const int *slot, const float *leaves, const float *tiles, const int *o, const int *nb,\n'
        "                       float bg, const float *inv, const float *vec, int n, const float *p, float *out) {\n"
        "  Grid g{slot, leaves, tiles, o[0], o[1], o[2], nb[0], nb[1], nb[2], bg};\n"
        "  for (int k = 0; k < 9; ++k) g.inv[k] = inv[k];\n"
        "  for (int k = 0; k < 3; ++k) g.vec[k] = vec[k];\n"
        "  for (int i = 0; i < n; ++i) out[i] = sample_world(g, p[3 * i], p[3 * i + 1], p[3 * i + 2]);\n"
        "}\n"
        # the apron layout the kernels sample, built on the host exactly as upload_vdb +
        # k_vdb_apron build it on the device
        'extern "C" long long sample_apron(const int *slot, const float *leaves, const float *tiles, int ntiles,\n'
        "                       const int *o, const int *nb, float bg, const float *inv, const float *vec, int n,\n"
        "                       const float *p, float *out, float *vals, int fat) {\n"
        "  Grid g{slot, leaves, tiles, o[0], o[1], o[2], nb[0], nb[1], nb[2], bg};\n"
        "  std::vector<int> aslot; std::vector<long long> list;\n"
        "  build_apron_slots(slot, nb[0], nb[1], nb[2], tiles, ntiles, bg, aslot, list);\n"
        "  std::vector<float> consts(tiles, tiles + ntiles); consts.push_back(bg);\n"
        "  std::vector<float> blocks(list.size() * kApronVals);\n"
        "  for (std::size_t i = 0; i < list.size(); ++i) {\n"
        "    const long long e = list[i];\n"
        "    const int ex = e % (nb[0] + 1), ey = (e / (nb[0] + 1)) % (nb[1] + 1), ez = e / ((nb[0] + 1) * (nb[1] + 1));\n"
        "    for (int k = 0; k < kApronVals; ++k) blocks[i * kApronVals + k] = apron_value(g, ex, ey, ez, k);\n"
        "  }\n"
        "  Apron a{aslot.data(), blocks.data(), consts.data(), o[0], o[1], o[2], nb[0], nb[1], nb[2], bg};\n"
        "  for (int k = 0; k < 9; ++k) a.inv[k] = inv[k];\n"
        "  for (int k = 0; k < 3; ++k) a.vec[k] = vec[k];\n"
        "  std::vector<float> fatv(fat ? list.size() * 512 * 8 : 0);\n"
        "  for (long long e = 0; e < (long long)fatv.size() / 8; ++e) apron_fat_entry(blocks.data(), e >> 9, (int)(e & 511), &fatv[8 * e]);\n"
        "  a.fat = fat ? fatv.data() : nullptr;\n"
        "  for (int i = 0; i < n; ++i) out[i] = sample_world(a, p[3 * i], p[3 * i + 1], p[3 * i + 2]);\n"
        "  // getValue over the extent +-10 voxels from the apron layout\n"
        "  long long q = 0;\n"
        "  for (int z = o[2] - 10; z < o[2] + 8 * nb[2] + 10; ++z)\n"
        "    for (int y = o[1] - 10; y < o[1] + 8 * nb[1] + 10; ++y)\n"
        "      for (int x = o[0] - 10; x < o[0] + 8 * nb[0] + 10; ++x) vals[q++] = get_value(a, x, y, z) - get_value(g, x, y, z);\n"
        "  return (long long)list.size();\n"
        "}\n")
    so = d / "shim.so"
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-shared", "-fPIC", str(src), "-o", str(so)])
    return ctypes.CDLL(str(so))


def test_device_header_equals_oracle(hdr):
    e = _dense(9, (21, 19, 26))
    e[0:8, 0:8, 0:8] = 0.6                      # block-aligned constant: a tile
    g = NanoVDBGrid.from_dense(e, index_min=(-8, 0, -16), index_to_world=_rotated_map(20), background=0.0)
    assert len(g.tile_values) >= 1
    slot, lo, nb = _slots(g)
    tree = binding.VdbTree(g)
    b = binding.vdb_bounds(tree)
    rng = np.random.default_rng(11)
    p = (b[:3] - 0.05 + rng.random((20000, 3)) * (b[3:] - b[:3] + 0.1)).astype(np.float32)
    out = np.zeros(len(p), np.float32)
    I = ctypes.POINTER(ctypes.c_int)
    F = ctypes.POINTER(ctypes.c_float)
    arr = lambda a, t: np.ascontiguousarray(a).ctypes.data_as(t)
    inv = g.world_to_index.astype(np.float32).reshape(-1)
    vec = g.index_to_world[:, 3].astype(np.float32)
    lo32, nb32 = lo.astype(np.int32), nb.astype(np.int32)
    tiles = g.tile_values if len(g.tile_values) else np.zeros(1, np.float32)
    hdr.sample(arr(slot, I), arr(g.leaf_values, F), arr(tiles, F), arr(lo32, I), arr(nb32, I),
               ctypes.c_float(float(g.background)), arr(inv, F), arr(vec, F), len(p), arr(p, F), arr(out, F))
    want = tree.sample_world(p)
    assert out.view(np.uint32).tolist() == want.view(np.uint32).tolist()


@pytest.mark.parametrize("fat", [0, 1])
@pytest.mark.parametrize("case", ["tiles", "two_tiles", "single_leaf"])
def test_apron_layout_equals_oracle(hdr, case, fat):
    """The apron layout (one slot + one 9^3 block per lookup; fat: + one 32-B tap entry per
    base voxel) samples the same bits as the oracle's tree, and its getValue equals the base
    layout's everywhere around the extent."""
    if case == "tiles":
        e = _dense(9, (21, 19, 26))
        e[0:8, 0:8, 0:8] = 0.6
        g = NanoVDBGrid.from_dense(e, index_min=(-8, 0, -16), index_to_world=_rotated_map(20), background=0.0)
    elif case == "two_tiles":   # neighbouring tiles of different values, a background hole, bg != 0
        e = np.full((24, 16, 16), 0.25, np.float32)
        e[0:8, 0:8, 0:8] = 0.6
        e[8:16, 0:8, 8:16] = 0.9
        e[16:24, 8:16, 0:8] = 0.0
        e[3, 12, 5] = 1.5
        g = NanoVDBGrid.from_dense(e, index_min=(8, -8, 0), background=0.25)
    else:
        e = np.zeros((3, 3, 3), np.float32)
        e[1, 1, 1] = 2.0
        g = NanoVDBGrid.from_dense(e, index_min=(7, 7, 7), voxel_size=0.5, background=0.0)
    slot, lo, nb = _slots(g)
    tree = binding.VdbTree(g)
    b = binding.vdb_bounds(tree)
    rng = np.random.default_rng(12)
    p = (b[:3] - 0.3 + rng.random((20000, 3)) * (b[3:] - b[:3] + 0.6)).astype(np.float32)
    out = np.zeros(len(p), np.float32)
    I = ctypes.POINTER(ctypes.c_int)
    F = ctypes.POINTER(ctypes.c_float)
    arr = lambda a, t: np.ascontiguousarray(a).ctypes.data_as(t)
    inv = g.world_to_index.astype(np.float32).reshape(-1)
    vec = g.index_to_world[:, 3].astype(np.float32)
    lo32, nb32 = lo.astype(np.int32), nb.astype(np.int32)
    tiles = g.tile_values if len(g.tile_values) else np.zeros(1, np.float32)
    nvals = int(np.prod(8 * nb + 20))
    vals = np.full(nvals, np.nan, np.float32)
    hdr.sample_apron.restype = ctypes.c_longlong
    nblk = hdr.sample_apron(arr(slot, I), arr(g.leaf_values, F), arr(tiles, F), len(g.tile_values), arr(lo32, I),
                            arr(nb32, I), ctypes.c_float(float(g.background)), arr(inv, F), arr(vec, F), len(p),
                            arr(p, F), arr(out, F), arr(vals, F), fat)
    assert nblk >= len(g.leaf_origins)
    want = tree.sample_world(p)
    assert out.view(np.uint32).tolist() == want.view(np.uint32).tolist()
    assert np.all(vals == 0)


def test_oracle_vdb_absorber_known_answer():
    """sigma_s = 0, sigma_a = 1, an n^3 block of ones with index i at world i / n: along z
    the trilinear density is 1 on [0, (n-1)/n] and ramps to 0 on the last voxel, so
    L = exp(-(1 - 0.5/n)) for interior pixels (delta-tracking absorption: 0/1 per sample)."""
    from acceleratedvolrenderer_amd import scenes
    n, W, H, spp = 8, 16, 16, 256
    scene = scenes.s_vdb(np.ones((n, n, n), np.float32), W, H, variant="absorber")
    assert np.array_equal(scene.medium.bounds, np.array([0, 0, 0, 1, 1, 1], np.float32))
    run = binding.OracleRun(scene, max_depth=5, seed=0)
    rgb, w = run.render(0, spp, nthreads=8)
    # per-sample L through pixel_sample on interior pixels (x, y index in [1, n-2])
    Ls = [run.pixel_sample(px, py, s)[0][0] for px in range(3, W - 3) for py in range(3, H - 3) for s in range(24)]
    want = np.exp(-(1 - 0.5 / n))
    m = float(np.mean(Ls))
    assert abs(m - want) < 4 * np.sqrt(want * (1 - want) / len(Ls)), (m, want)


def test_oracle_vdb_white_furnace():
    """Albedo-1 NanoVDB medium (with tiles and empty blocks) in a uniform infinite light:
    every escaping path carries exactly L = Le = 1."""
    from acceleratedvolrenderer_amd import scenes
    d = np.zeros((16, 16, 16), np.float32)
    d[8:16, 8:16, 0:8] = 0.9                     # a tile
    d[2:8, 2:8, 2:14] += np.random.default_rng(0).random((6, 6, 12)).astype(np.float32)
    scene = scenes.s_vdb(d, 12, 12, variant="furnace")
    assert len(scene.medium.grid.tile_values) >= 1
    run = binding.OracleRun(scene, max_depth=1000, seed=0)
    Ls = np.array([run.pixel_sample(px, py, s)[0] for px in range(12) for py in range(12) for s in range(4)])
    assert np.all(Ls == 1.0)


def test_oracle_tree_unaligned_tile():
    """The oracle's tree takes tiles as given (oracle_vdb_create): an 8^3 tile whose origin is
    not 8-aligned covers exactly its own box, not the hash block its origin falls in."""
    from types import SimpleNamespace
    g = SimpleNamespace(leaf_origins=np.zeros((0, 3), np.int32), leaf_values=np.zeros((0, 8, 8, 8), np.float32),
                        tile_origins=np.array([[3, -5, 12], [16, 16, 16]], np.int32), tile_sizes=np.array([8, 8], np.int32),
                        tile_values=np.array([0.5, 0.75], np.float32), background=np.float32(0.125),
                        index_bbox=np.array([3, -5, 12, 23, 23, 23], np.int32), index_to_world=np.eye(4)[:3],
                        world_to_index=np.eye(3))
    tree = binding.VdbTree(g)
    for x in range(-2, 28):
        for y in range(-8, 26, 3):
            for z in range(8, 26, 2):
                inside = [3 <= x < 11 and -5 <= y < 3 and 12 <= z < 20, 16 <= x < 24 and 16 <= y < 24 and 16 <= z < 24]
                want = 0.5 if inside[0] else (0.75 if inside[1] else 0.125)
                assert tree.value(x, y, z) == np.float32(want), (x, y, z)

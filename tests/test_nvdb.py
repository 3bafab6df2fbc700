"""f1 `.nvdb` files (NanoVDBMedium::Create's readGrid, media.cpp:487-509): the uncompressed
NanoVDB FloatGrid layout restated in acceleratedvolrenderer_amd/nvdb.py. PARITY UNPINNED
against NanoVDB itself (no source, no asset offline): these tests pin the reader to the
writer and both to the tree they serialize — values at every voxel (leaves, 8^3 / 128^3 /
4096^3 tiles, background, negative coordinates), the index bbox, the map, several grids per
file looked up by name — plus the error paths."""
import struct

import numpy as np
import pytest

from acceleratedvolrenderer_amd import nvdb
from acceleratedvolrenderer_amd.vdb import NanoVDBGrid


def _same_tree(a, b, probes):
    assert a.background == b.background
    assert np.array_equal(a.index_bbox, b.index_bbox)
    assert np.array_equal(a.index_to_world, b.index_to_world)
    assert np.allclose(a.world_to_index, b.world_to_index, rtol=0, atol=1e-15)
    assert np.array_equal(a.values(probes), b.values(probes))


def test_round_trip_dense_grid_with_tiles_and_negative_origins(tmp_path):
    rng = np.random.default_rng(3)
    d = np.zeros((40, 36, 30), np.float32)
    d[3:20, 5:30, 2:25] = rng.random((17, 25, 23), dtype=np.float32)
    d[24:40, 8:16, 8:24] = 0.75                       # constant blocks -> 8^3 tiles
    g = NanoVDBGrid.from_dense(d, index_min=(-16, 8, -72), voxel_size=0.02, origin=(0.1, -0.3, 2.0))
    assert len(g.tile_origins) > 0 and len(g.leaf_origins) > 0
    p = tmp_path / "grid.nvdb"
    nvdb.write_nvdb(p, {"density": g})
    assert nvdb.list_grids(p)[0][:3] == ("density", nvdb.GRID_TYPE_FLOAT, nvdb.CODEC_NONE)
    r = nvdb.read_nvdb(p)
    lo, hi = g.index_bbox[:3] - 9, g.index_bbox[3:] + 9
    probes = np.stack(np.meshgrid(*(np.arange(lo[k], hi[k] + 1, 3) for k in range(3)), indexing="ij"), -1).reshape(-1, 3)
    _same_tree(g, r, probes)
    assert np.array_equal(np.sort(g.leaf_origins.view("i4,i4,i4"), axis=0), np.sort(r.leaf_origins.view("i4,i4,i4"), axis=0))
    gw = g.world_bbox()
    rw = r.world_bbox()
    assert np.array_equal(gw[0], rw[0]) and np.array_equal(gw[1], rw[1])


@pytest.mark.parametrize("codec", ["none", "zip"])
def test_zip_codec_round_trip(tmp_path, codec):
    """ZIP-coded grids (NanoVDB io::Internal::write with NANOVDB_USE_ZIP: u64 compressed size +
    one zlib stream per grid buffer) read back to the same tree as the uncompressed file; a
    file mixing both is read grid by grid."""
    rng = np.random.default_rng(9)
    d = np.zeros((24, 24, 24), np.float32)
    d[4:20, 2:22, 6:18] = rng.random((16, 20, 12), dtype=np.float32)
    d[16:24, 16:24, 16:24] = 0.5
    g = NanoVDBGrid.from_dense(d, index_min=(-8, 16, 0), voxel_size=0.1)
    t = NanoVDBGrid.from_dense(np.full((8, 8, 8), 1200.0, np.float32), background=0.0)
    p = tmp_path / f"{codec}.nvdb"
    nvdb.write_nvdb(p, [("density", g), ("temperature", t)], codec=codec)
    segs = nvdb.list_grids(p)
    assert [s[2] for s in segs] == [nvdb.CODECS[codec]] * 2
    if codec == "zip":   # the stored segment is smaller than the grid buffer it holds
        plain = tmp_path / "plain.nvdb"
        nvdb.write_nvdb(plain, [("density", g), ("temperature", t)])
        assert segs[0][3] < nvdb.list_grids(plain)[0][3]
    r = nvdb.read_nvdb(p)
    lo, hi = g.index_bbox[:3] - 9, g.index_bbox[3:] + 9
    probes = np.stack(np.meshgrid(*(np.arange(lo[k], hi[k] + 1, 2) for k in range(3)), indexing="ij"), -1).reshape(-1, 3)
    _same_tree(g, r, probes)
    rt = nvdb.read_nvdb(p, "temperature")
    assert np.array_equal(rt.values([[3, 4, 5], [9, 0, 0]]), np.array([1200.0, 0.0], np.float32))


def test_upper_and_root_tiles_and_several_grids(tmp_path):
    leaf = np.arange(512, dtype=np.float32).reshape(8, 8, 8) / 512
    g = NanoVDBGrid(leaf_origins=[(0, 0, 0), (-8, 128, 4096)], leaf_values=[leaf, 1 - leaf], background=0.0,
                    tile_origins=[(128, 0, 0), (-4096, 0, 0), (256, 256, 256)], tile_sizes=[128, 4096, 16],
                    tile_values=[0.5, 0.25, 0.125])
    t = NanoVDBGrid.from_dense(np.full((8, 8, 8), 1500.0, np.float32), background=0.0)
    p = tmp_path / "two.nvdb"
    nvdb.write_nvdb(p, [("density", g), ("temperature", t)])
    assert [n for n, *_ in nvdb.list_grids(p)] == ["density", "temperature"]
    r = nvdb.read_nvdb(p, "density")
    probes = np.array([[1, 2, 3], [-3, 130, 4100], [130, 5, 7], [255, 127, 127], [-4000, 7, 4000],
                       [-4097, 0, 0], [260, 270, 271], [272, 256, 256], [9, 9, 9], [0, 0, 0]])
    _same_tree(g, r, probes)
    rt = nvdb.read_nvdb(p, "temperature")
    assert np.array_equal(rt.values([[3, 4, 5], [9, 0, 0]]), np.array([1500.0, 0.0], np.float32))


def test_reader_errors(tmp_path):
    g = NanoVDBGrid.from_dense(np.ones((8, 8, 8), np.float32), tiles=False)
    p = tmp_path / "g.nvdb"
    nvdb.write_nvdb(p, {"density": g})
    with pytest.raises(ValueError, match="no grid named"):
        nvdb.read_nvdb(p, "temperature")
    raw = bytearray(p.read_bytes())
    bad = tmp_path / "bad.nvdb"
    bad.write_bytes(b"\0" * 8 + bytes(raw[8:]))
    with pytest.raises(ValueError, match="magic"):
        nvdb.read_nvdb(bad)
    zipped = bytearray(raw)
    struct.pack_into("<H", zipped, 14, 1)          # file codec ZIP over an uncompressed buffer
    (tmp_path / "zip.nvdb").write_bytes(bytes(zipped))
    with pytest.raises(ValueError, match="ZIP"):
        nvdb.read_nvdb(tmp_path / "zip.nvdb")
    blosc = bytearray(raw)
    struct.pack_into("<H", blosc, 14, 2)           # file codec BLOSC: refused
    (tmp_path / "blosc.nvdb").write_bytes(bytes(blosc))
    with pytest.raises(ValueError, match="BLOSC"):
        nvdb.read_nvdb(tmp_path / "blosc.nvdb")
    with pytest.raises(ValueError, match="codec"):
        nvdb.write_nvdb(tmp_path / "x.nvdb", {"density": g}, codec="blosc")
    z = tmp_path / "z.nvdb"
    nvdb.write_nvdb(z, {"density": g}, codec="zip")
    zr = bytearray(z.read_bytes())
    (tmp_path / "ztrunc.nvdb").write_bytes(bytes(zr[:-10]))   # stream cut short
    with pytest.raises(ValueError):
        nvdb.read_nvdb(tmp_path / "ztrunc.nvdb")
    zc = bytearray(zr)
    zc[16 + 176 + len(b"density") + 1 + 8 + 4] ^= 0xFF        # corrupt the deflate stream
    (tmp_path / "zbad.nvdb").write_bytes(bytes(zc))
    with pytest.raises(ValueError, match="ZIP"):
        nvdb.read_nvdb(tmp_path / "zbad.nvdb")
    typed = bytearray(raw)
    struct.pack_into("<I", typed, 16 + 32, 2)      # MetaData gridType Double
    (tmp_path / "dbl.nvdb").write_bytes(bytes(typed))
    with pytest.raises(ValueError, match="FloatGrid"):
        nvdb.read_nvdb(tmp_path / "dbl.nvdb")
    (tmp_path / "short.nvdb").write_bytes(b"Nano")
    with pytest.raises(ValueError):
        nvdb.read_nvdb(tmp_path / "short.nvdb")


def test_nanovdb_medium_from_file_matches_in_memory_grid(tmp_path):
    """NanoVDBMedium built from the file samples the same densities as from the tree it was
    written from (oracle sampler, world space)."""
    from oracle import binding
    from acceleratedvolrenderer_amd import scenes
    rng = np.random.default_rng(5)
    d = rng.random((16, 16, 16), dtype=np.float32)
    g = scenes.vdb_grid(d)
    p = tmp_path / "m.nvdb"
    nvdb.write_nvdb(p, {"density": g})
    r = nvdb.read_nvdb(p)
    a, b = binding.VdbTree(g), binding.VdbTree(r)
    pts = rng.random((500, 3), dtype=np.float32)
    assert np.array_equal(a.sample_world(pts).view(np.uint32), b.sample_world(pts).view(np.uint32))

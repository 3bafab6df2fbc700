"""Lighting-graph precompute (src/graph).

CPU (not gpu):
  * the oracle's GetHits(sphere) and ComputeFinalLight against golden vectors the REAL
    reference produced (oracle/ref/graph_ref.cpp over pbrt's Sphere and the reference's
    vendored Eigen; tests/golden/graph_vectors.json): hit type and t0 bit-exact, t1 within
    4e-6 relative (the oracle takes both roots from one quadric solve, pbrt re-intersects from
    the spawned exit point), transport totals and stop iteration bit-exact;
  * the C++ FreeGraph assembly (avr_graph_*, host code in libavr_hip.so) against the
    pure-Python restatement oracle/graph_builder.py — bit-exact;
  * host ray-grid geometry (graph.MediumData.box_hits) against the oracle's box hits —
    bit-exact; disk point counts against the oracle's GetDiskPoints.
GPU (gpu): the HIP walks, light vector and bounce propagation against the oracle on the
same seeded inputs. Walks and light replay the oracle's sample streams with the canonical
transcendentals: >= 99.9 % of walks / vertices bit-identical; propagation
is bit-exact (ascending-column float sums, the oracle's and Eigen's order).
"""
import json
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def f(u32):
    return np.array(u32, dtype=np.uint32).view(np.float32)


@pytest.fixture(scope="module")
def graph_golden():
    with open(os.path.join(ROOT, "tests", "golden", "graph_vectors.json")) as fh:
        return json.load(fh)


def _csr(n, rows, cols, vals):
    o = np.lexsort((cols, rows))
    rows, cols, vals = np.asarray(rows)[o], np.asarray(cols, np.int32)[o], np.asarray(vals, np.float32)[o]
    rp = np.zeros(n + 1, np.int64)
    np.add.at(rp, rows + 1, 1)
    return np.cumsum(rp).astype(np.int32), cols, vals


# ---------------------------------------------------------------------------- CPU

def test_sphere_hits_match_reference(graph_golden):
    from oracle import binding
    types = {}
    for row in graph_golden["sphere_hits"]:
        v = f(row[:10])
        ty, t0, t1 = binding.graph_sphere_hits(v[0:3], v[3], v[4:7], v[7:10])
        types[row[10]] = types.get(row[10], 0) + 1
        assert ty == row[10]
        assert np.float32(t0).view(np.uint32) == row[11]
        if ty == 0:
            ref = f([row[12]])[0]
            assert abs(t1 - ref) <= 4e-6 * abs(ref)
    assert set(types) == {0, 2, 3}   # two hits, misses, inside


def test_transport_iteration_matches_reference_eigen(graph_golden):
    from oracle import binding
    for case in graph_golden["transport"]:
        n = case["n"]
        rp, col, val = _csr(n, case["rows"], case["cols"], f(case["vals"]))
        total, it = binding.graph_propagate(n, rp, col, val, f(case["light"]), case["bounces"])
        assert it == case["iterations"]
        assert total.view(np.uint32).tolist() == case["total"]
    assert any(c["iterations"] < c["bounces"] for c in graph_golden["transport"])   # NaN/Inf stop covered


def _synthetic_walks(rng, n_walks, max_depth, radius):
    """Clustered scatter points (merges, revisits, self-edges) and forced ends."""
    centers = rng.random((12, 3), dtype=np.float32)
    pts = np.zeros((n_walks, max_depth, 3), np.float32)
    counts = rng.integers(0, max_depth + 1, n_walks).astype(np.int32)
    for w in range(n_walks):
        for k in range(counts[w]):
            c = centers[rng.integers(0, len(centers))]
            pts[w, k] = c + (rng.random(3, dtype=np.float32) - 0.5) * np.float32(2.2 * radius)
    return pts, counts


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_graph_assembly_matches_restatement(seed):
    from acceleratedvolrenderer_amd import capi
    from oracle.graph_builder import OracleGraph
    rng = np.random.default_rng(seed)
    radius, max_depth = 0.04, 6
    pts, counts = _synthetic_walks(rng, 300, max_depth, radius)
    g = capi.Graph(radius)
    g.add_walks(pts, counts, max_depth)
    ref = OracleGraph(radius)
    ref.add_walks(pts, counts, max_depth)
    xyz, smp = g.vertices()
    assert len(xyz) == len(ref.xyz) > 12
    assert np.array_equal(xyz, np.array(ref.xyz, np.float32))
    assert smp.tolist() == ref.samples
    fr, to, es = g.edges()
    assert list(zip(fr.tolist(), to.tolist(), es.tolist())) == [(a, b, s) for (a, b), s in ref.edges.items()]
    assert any(a == b for a, b in ref.edges)   # self-edges (a walk staying in one vertex)
    rp, col, val = g.transport()
    T = np.zeros((len(xyz), len(xyz)), np.float32)
    for r in range(len(xyz)):
        assert np.all(np.diff(col[rp[r]:rp[r + 1]]) > 0)
        T[r, col[rp[r]:rp[r + 1]]] = val[rp[r]:rp[r + 1]]
    assert np.array_equal(T, ref.transport_dense())
    avg, cnt = g.in_node_path_length()
    assert cnt == ref.pl_count
    assert avg == pytest.approx(ref.pl_sum / ref.pl_count, rel=1e-6)


def test_graph_assembly_with_start_vertices_matches_restatement():
    """Reinforcement walks (TracePath's startingVertex, free_graph_builder.cpp:24-25): the
    start vertex heads the path, takes the first segment's sample and the first edge; out
    degrees and radius counts (CountInRadius, :229-236) against the restatement."""
    from acceleratedvolrenderer_amd import capi
    from oracle.graph_builder import OracleGraph
    rng = np.random.default_rng(7)
    radius, md = 0.04, 6
    pts, counts = _synthetic_walks(rng, 200, md, radius)
    g, ref = capi.Graph(radius), OracleGraph(radius)
    g.add_walks(pts, counts, md)
    ref.add_walks(pts, counts, md)
    nv = g.size()[0]
    p2, c2 = _synthetic_walks(rng, 150, md - 1, radius)
    padded = np.zeros((150, md, 3), np.float32)
    padded[:, :md - 1] = p2
    start = rng.integers(0, nv, 150).astype(np.int32)
    g.add_walks_from(padded, c2, md, start)
    for w in range(150):
        ref.add_walk(p2[w, :c2[w]], int(c2[w]) == md - 1, start=int(start[w]))
    xyz, smp = g.vertices()
    assert np.array_equal(xyz, np.array(ref.xyz, np.float32)) and smp.tolist() == ref.samples
    fr, to, es = g.edges()
    assert list(zip(fr.tolist(), to.tolist(), es.tolist())) == [(a, b, s) for (a, b), s in ref.edges.items()]
    assert g.out_degrees().tolist() == ref.out_degrees().tolist()
    ids = np.arange(len(xyz), dtype=np.int32)
    for r in (0.03, 0.1, 0.5):
        assert g.count_in_radius(ids, r).tolist() == [ref.count_in_radius(v, r) for v in ids]
    avg, cnt = g.in_node_path_length()
    assert cnt == ref.pl_count and avg == pytest.approx(ref.pl_sum / ref.pl_count, rel=1e-6)
    with pytest.raises(RuntimeError, match="start vertex"):
        g.add_walks_from(padded[:1], c2[:1], md, np.array([len(xyz) + 5], np.int32))


def test_graph_assembly_argument_errors():
    from acceleratedvolrenderer_amd import capi
    with pytest.raises(RuntimeError, match="radius"):
        capi.Graph(0.0)
    g = capi.Graph(0.1)
    with pytest.raises(RuntimeError, match="count out of range"):
        g.add_walks(np.zeros((1, 2, 3), np.float32), np.array([3], np.int32), 2)
    assert g.size() == (0, 0)


def _graph_scene(n=12, seed=5):
    from acceleratedvolrenderer_amd import scenes, GridMedium
    from acceleratedvolrenderer_amd.scene import Scene
    base = scenes.s_uniform(n=2, width=16, height=16, variant="scatter")
    dens = (0.2 + 0.8 * np.random.default_rng(seed).random((n, n, n), dtype=np.float32)).astype(np.float32)
    med = GridMedium(dens, sigma_a=0.4, sigma_s=6.0, g=0.5)
    return Scene(base.camera, base.film, med, base.lights)


def test_host_box_hits_match_oracle():
    from acceleratedvolrenderer_amd import graph
    from oracle import binding
    scene = _graph_scene()
    md = graph.MediumData(scene)
    run = binding.OracleRun(scene)
    rng = np.random.default_rng(4)
    kinds = set()
    for _ in range(400):
        o = (md.bounds_center + (rng.random(3, dtype=np.float32) - 0.5) * 3).astype(np.float32)
        d = (rng.random(3, dtype=np.float32) - 0.5).astype(np.float32)
        d = (d / np.float32(np.linalg.norm(d))).astype(np.float32)
        a = md.box_hits(o, d)
        b = run.graph_box_hits(o, d)
        kinds.add(a[0])
        assert a[0] == b[0]
        if a[0] != 2:
            assert np.float32(a[1]).view(np.uint32) == np.float32(b[1]).view(np.uint32)
        if a[0] == 0:
            assert np.float32(a[2]).view(np.uint32) == np.float32(b[2]).view(np.uint32)
    assert kinds == {0, 2, 3}


def test_disk_points_and_config():
    from acceleratedvolrenderer_amd import graph
    from oracle import binding
    for n in range(0, 7):
        assert graph.disk_points_size(n) == len(binding.graph_disk_points((0, 0, 0), 1.0, n, (1, 0, 0)))
    cfg = graph.Config.from_json({
        "graphBuilder": {"radiusModifier": 2.0, "maxDepth": 50, "dimensionSteps": 20, "iterationsPerStep": 4,
                         "renderSearchRange": {"active": False, "neighboursToUse": 5, "runInParallel": True}},
        "lightingCalculator": {"lightIterations": 10, "pointsOnRadiusLight": 3, "bounces": [5, 20],
                               "runInParallel": True}})
    s = graph.GraphSampling.for_config(cfg)
    assert s.samples_per_pixel == 16                      # RoundUpPow2(lightIterations)
    n_disk = graph.disk_points_size(3)
    assert s.resolution[0] == int(np.ceil(np.sqrt(20 * 20 * 4 * 50 * n_disk)))
    assert cfg.lighting_calculator.bounces == [5, 20]
    with pytest.raises(ValueError, match="light ray iteration"):
        graph.LightingCalculator(None, None, None, (0, 0, 1), s, graph.LightingCalculatorConfig(light_iterations=0))


# ---------------------------------------------------------------------------- GPU

torch = None


@pytest.fixture(scope="module")
def gpu_ctx():
    global torch
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from acceleratedvolrenderer_amd import capi
    scene = _graph_scene()
    ctx = capi.Context(0)
    ctx.set_scene(scene)
    yield scene, ctx
    ctx.close()


def _sampling(kind):
    from acceleratedvolrenderer_amd import graph
    return graph.GraphSampling(sampler=kind, seed=3, samples_per_pixel=16, resolution=(64, 64))


def _oracle_sampler(s):
    return (s.sampler, s.seed, s.samples_per_pixel, s.resolution[0], s.resolution[1])


def _builder(scene, ctx, kind, steps=8, iters=6, max_depth=12):
    from acceleratedvolrenderer_amd import graph
    cfg = graph.GraphBuilderConfig(radius_modifier=60.0, max_depth=max_depth, dimension_steps=steps,
                                   iterations_per_step=iters)
    md = graph.MediumData(scene)
    d = np.array([0.3, -0.5, 0.81], np.float32)
    d = (d / np.float32(np.linalg.norm(d))).astype(np.float32)
    return graph.FreeGraphBuilder(ctx, md, d, _sampling(kind), cfg)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", [0, 1], ids=["independent", "zsobol"])
def test_graph_walks_replay(gpu_ctx, kind):
    from oracle import binding
    scene, ctx = gpu_ctx
    b = _builder(scene, ctx, kind)
    o, d, t, idx = b.start_rays()
    assert len(o) > 20
    c = b.config
    pts, counts = ctx.graph_walks(b.sampling.struct(), o, d, t, idx, c.iterations_per_step, 0, c.max_depth)
    run = binding.OracleRun(scene, libm="canonical")
    pts_o, counts_o = run.graph_walks(o, d, t, idx, c.iterations_per_step, 0, b.sampling.resolution[0], c.max_depth,
                                      sampler=_oracle_sampler(b.sampling))
    same = np.array([counts[w] == counts_o[w] and np.array_equal(pts[w, :counts[w]], pts_o[w, :counts_o[w]])
                     for w in range(len(counts))])
    print(f"walks {len(counts)}, mean scatters {counts.mean():.2f}, forced {np.mean(counts == c.max_depth):.3f}, "
          f"bit-identical {same.mean():.5f}")
    assert counts.mean() > 1.0
    assert same.mean() == 1.0


@pytest.mark.gpu
@pytest.mark.parametrize("kind", [0, 1], ids=["independent", "zsobol"])
def test_graph_light_replay(gpu_ctx, kind):
    from acceleratedvolrenderer_amd import graph
    from oracle import binding
    scene, ctx = gpu_ctx
    md = graph.MediumData(scene)
    rng = np.random.default_rng(9)
    verts = (md.pmin + rng.random((150, 3), dtype=np.float32) * (md.pmax - md.pmin)).astype(np.float32)
    d = np.array([0.3, -0.5, 0.81], np.float32)
    d = (d / np.float32(np.linalg.norm(d))).astype(np.float32)
    s = _sampling(kind)
    radius = np.float32(0.05)
    light = ctx.graph_light(s.struct(), verts, d, radius, 2, 4, md.max_dist_to_center)
    run = binding.OracleRun(scene, libm="canonical")
    ref = run.graph_light(verts, d, radius, 2, 4, s.resolution[0], md.max_dist_to_center,
                          sampler=_oracle_sampler(s))
    same = np.mean(light.view(np.uint32) == ref.view(np.uint32))
    print(f"light: mean {light.mean():.4e}, bit-identical {same:.5f}, max rel {np.max(np.abs(light - ref) / np.maximum(ref, 1e-30)):.2e}")
    assert light.mean() > 0
    assert same == 1.0
    assert np.allclose(light, ref, rtol=1e-5, atol=0)


@pytest.mark.gpu
def test_graph_propagate_bit_exact(gpu_ctx, graph_golden):
    from oracle import binding
    _, ctx = gpu_ctx
    for case in graph_golden["transport"]:
        n = case["n"]
        rp, col, val = _csr(n, case["rows"], case["cols"], f(case["vals"]))
        total, it = ctx.graph_propagate(rp, col, val, f(case["light"]), case["bounces"])
        assert it == case["iterations"]
        assert total.view(np.uint32).tolist() == case["total"]
    # a larger random graph against the oracle restatement
    rng = np.random.default_rng(1)
    n = 20000
    rows = np.repeat(np.arange(n), 6)
    cols = rng.integers(0, n, len(rows))
    key = np.unique(rows.astype(np.int64) * n + cols)
    rows, cols = key // n, key % n
    vals = (rng.random(len(rows), dtype=np.float32) / np.float32(6.5)).astype(np.float32)
    rp, col, val = _csr(n, rows, cols, vals)
    light = rng.random(n, dtype=np.float32)
    total, it = ctx.graph_propagate(rp, col, val, light, 30)
    ref, it_o = binding.graph_propagate(n, rp, col, val, light, 30)
    assert it == it_o == 30
    assert np.array_equal(total.view(np.uint32), ref.view(np.uint32))


@pytest.mark.gpu
def test_graph_pipeline_end_to_end(gpu_ctx):
    """BuildGraph -> GetLightVector -> GetTransportMatrix -> ComputeFinalLight on the GPU
    against the oracle pipeline on the same walks (oracle walks merged by the Python
    restatement)."""
    from acceleratedvolrenderer_amd import graph
    from oracle import binding
    from oracle.graph_builder import OracleGraph
    scene, ctx = gpu_ctx
    b = _builder(scene, ctx, 0, steps=6, iters=4, max_depth=8)
    g = b.build_graph()
    assert g.num_vertices > 10
    lc = graph.LightingCalculator(ctx, g, b.md, b.in_dir, b.sampling,
                                  graph.LightingCalculatorConfig(light_iterations=4, points_on_radius_light=1,
                                                                 bounces=[6]))
    it = lc.compute_final_light()
    assert it == 6

    run = binding.OracleRun(scene, libm="canonical")
    o, d, t, idx = b.start_rays()
    c = b.config
    pts, counts = run.graph_walks(o, d, t, idx, c.iterations_per_step, 0, b.sampling.resolution[0], c.max_depth,
                                  sampler=_oracle_sampler(b.sampling))
    og = OracleGraph(b.radius)
    og.add_walks(pts, counts, c.max_depth)
    assert np.array_equal(g.points, np.array(og.xyz, np.float32))
    light = run.graph_light(g.points, b.in_dir, g.radius, 1, 4, b.sampling.resolution[0], b.md.max_dist_to_center,
                            sampler=_oracle_sampler(b.sampling))
    T = og.transport_dense()
    rows, cols = np.nonzero(T)
    rp, col, val = _csr(len(T), rows, cols, T[rows, cols])
    total, it_o = binding.graph_propagate(len(T), rp, col, val, light, 6)
    assert it_o == 6
    assert np.allclose(lc.light_scalar, total, rtol=1e-5)
    print(f"graph: {g.num_vertices} vertices, {len(g.edge_from)} edges, light total mean {total.mean():.4e}")


@pytest.mark.gpu
@pytest.mark.parametrize("kind", [0, 1], ids=["independent", "zsobol"])
def test_graph_reinforce_rays_replay(gpu_ctx, kind):
    """ReinforceSparseVertices' sphere rays (free_graph_builder.cpp:434-475) bit-exact."""
    from acceleratedvolrenderer_amd import graph
    from oracle import binding
    scene, ctx = gpu_ctx
    md = graph.MediumData(scene)
    rng = np.random.default_rng(5)
    pts = (md.pmin - 0.02 + rng.random((40, 3), dtype=np.float32) * (md.pmax - md.pmin + 0.04)).astype(np.float32)
    ids = rng.permutation(200)[:40].astype(np.int32)
    s = _sampling(kind)
    o, d, t, valid = ctx.graph_reinforce_rays(s.struct(), ids, pts, 0.03, 7, 2)
    ro, rd, rt, rv = binding.OracleRun(scene, libm="canonical").graph_reinforce_rays(
        ids, pts, 0.03, 7, 2, s.resolution[0], sampler=_oracle_sampler(s))
    assert np.array_equal(valid, rv) and valid.mean() > 0.5
    for a, b in ((o, ro), (d, rd), (t, rt)):
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.mark.gpu
def test_graph_build_with_reinforcement_end_to_end(gpu_ctx):
    """BuildGraph with edge and neighbour reinforcement active on the GPU against the oracle
    restatement of the same loop (oracle/graph_builder.reinforce): identical vertices,
    samples and edges."""
    from oracle import binding
    from oracle.graph_builder import OracleGraph, reinforce
    scene, ctx = gpu_ctx
    b = _builder(scene, ctx, 0, steps=5, iters=3, max_depth=6)
    ecfg = {"active": True, "unsatisfiedAllowedRatio": 0.3, "reinforcementRays": 4, "edgesForNotSparse": 3}
    ncfg = {"active": True, "unsatisfiedAllowedRatio": 0.3, "reinforcementRays": 3, "neighboursForNotSparse": 3,
            "neighbourRangeModifier": 2.0}
    b.config.edge_reinforcement, b.config.neighbour_reinforcement = ecfg, ncfg
    g = b.build_graph()
    run = binding.OracleRun(scene, libm="canonical")
    o, d, t, idx = b.start_rays()
    c = b.config
    smp = _oracle_sampler(b.sampling)
    pts, counts = run.graph_walks(o, d, t, idx, c.iterations_per_step, 0, b.sampling.resolution[0], c.max_depth,
                                  sampler=smp)
    og = OracleGraph(b.radius)
    og.add_walks(pts, counts, c.max_depth)
    n_before = len(og.xyz)
    cycles = reinforce(og, run, smp, b.radius, c.max_depth, ecfg, ncfg)
    print(f"reinforcement: {cycles} cycles, vertices {n_before} -> {len(og.xyz)}")
    assert cycles == b.reinforce_cycles >= 1
    assert np.array_equal(g.points, np.array(og.xyz, np.float32))
    assert g.samples.tolist() == og.samples
    assert list(zip(g.edge_from.tolist(), g.edge_to.tolist(), g.edge_samples.tolist())) == [
        (a, b_, s) for (a, b_), s in og.edges.items()]

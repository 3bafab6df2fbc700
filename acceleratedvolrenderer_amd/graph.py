"""Lighting-graph precompute — host mirror of the fork's src/graph tools.

The reference builds a "free graph" of scatter points in a medium lit by one distant light,
then solves light transport on it (cmd/graph_maker.cpp:70-160):

  FreeGraphBuilder::BuildGraph  (free/free_graph_builder.cpp:143-214) — a dimensionSteps²
      grid of rays along the light direction, `iterationsPerStep` delta-tracking walks each
      (TracePath, :19-141), scatter points merged into vertices of radius
      GetSameSpotRadius * radiusModifier (util.h:465-467);
  LightingCalculator            (lighting_calculator.cpp) — the initial light of every vertex
      by ratio tracking from a disk of rays (GetLightVector, :84-155), the transport matrix
      (GetTransportMatrix, :61-82) and the bounce iteration (ComputeFinalLight, :23-59).

Here the walks (k_graph_walks), the per-vertex transmittance estimates (k_graph_disk /
k_graph_tr / k_graph_average) and the sparse bounce iteration (k_graph_spmv) run on the GPU
through include/avr.h; the order-dependent vertex merge runs in C++ on the host
(avr_graph_add_walks). Names, parameters and error behaviour follow the reference. All
geometry is in the scene's render space; the medium's boundary primitive is its bounds box
(DESIGN.md §9).

ReinforceSparseVertices (:280-475) runs its rays and walks on the GPU and its sparse-vertex
checks on the host graph. Not mirrored: the graph's text file format.
"""
import json
import math

import numpy as np

from . import capi

f32 = np.float32


# ---------------------------------------------------------------------------
# Config (util.h:707-748 and its from_json readers :750-812)

class GraphBuilderConfig:
    def __init__(self, radius_modifier=1.0, max_depth=100, dimension_steps=10, iterations_per_step=10,
                 render_search_range=None, edge_reinforcement=None, neighbour_reinforcement=None):
        self.radius_modifier = float(radius_modifier)
        self.max_depth = int(max_depth)
        self.dimension_steps = int(dimension_steps)
        self.iterations_per_step = int(iterations_per_step)
        self.render_search_range = render_search_range or {"active": False, "neighboursToUse": 0}
        self.edge_reinforcement = edge_reinforcement or {"active": False}
        self.neighbour_reinforcement = neighbour_reinforcement or {"active": False}


class LightingCalculatorConfig:
    def __init__(self, light_iterations=16, points_on_radius_light=2, bounces=(10,)):
        self.light_iterations = int(light_iterations)
        self.points_on_radius_light = int(points_on_radius_light)
        self.bounces = [int(b) for b in bounces]


class Config:
    def __init__(self, graph_builder=None, lighting_calculator=None):
        self.graph_builder = graph_builder or GraphBuilderConfig()
        self.lighting_calculator = lighting_calculator or LightingCalculatorConfig()

    @classmethod
    def from_json(cls, text_or_dict):
        """The reference's graph config JSON (util.h:750-812 field names)."""
        j = json.loads(text_or_dict) if isinstance(text_or_dict, str) else text_or_dict
        gb, lc = j["graphBuilder"], j["lightingCalculator"]
        b = GraphBuilderConfig(gb["radiusModifier"], gb["maxDepth"], gb["dimensionSteps"], gb["iterationsPerStep"],
                               gb["renderSearchRange"], gb.get("edgeReinforcement"), gb.get("neighbourReinforcement"))
        c = LightingCalculatorConfig(lc["lightIterations"], lc["pointsOnRadiusLight"], lc["bounces"])
        return cls(b, c)


def disk_points_size(n):
    """util::GetDiskPointsSize (util.h:206-208): points of GetDiskPoints(radius 1)."""
    if n == 0:
        return 1
    step = f32(1) / f32(n + 1)
    k = 0
    for x in range(-n, n + 1):
        for y in range(-n, n + 1):
            # CoordinateSystem((1,0,0)) = (0,0,-1), (0,1,0): |p - c| = step * sqrt(x^2 + y^2)
            a, b = f32(f32(x) * step), f32(f32(y) * step)
            if f32(np.sqrt(f32(f32(a * a) + f32(b * b)))) <= f32(1):
                k += 1
    return k


def round_up_pow2(v):
    v = int(v)
    return 1 if v <= 1 else 1 << (v - 1).bit_length()


class GraphSampling:
    """The graph tools' sampler setup (graph_maker.cpp:84-104): pixelSamples =
    RoundUpPow2(lightIterations), a square sampling resolution large enough for one sample
    index per ray, the scene's sampler type and seed."""

    def __init__(self, sampler=0, seed=0, samples_per_pixel=16, resolution=(1024, 1024)):
        self.sampler, self.seed, self.samples_per_pixel = int(sampler), int(seed), int(samples_per_pixel)
        self.resolution = (int(resolution[0]), int(resolution[1]))

    @classmethod
    def for_config(cls, config, sampler=0, seed=0):
        gb, lc = config.graph_builder, config.lighting_calculator
        max_disk = disk_points_size(lc.points_on_radius_light)
        max_sphere = max(int(gb.edge_reinforcement.get("reinforcementRays", 0)),
                         int(gb.neighbour_reinforcement.get("reinforcementRays", 0)))
        max_rays_per_vertex = max(max_disk, max_sphere)
        max_vertices = gb.dimension_steps ** 2 * gb.iterations_per_step * gb.max_depth
        dim = int(math.ceil(math.sqrt(max_vertices * max_rays_per_vertex)))
        if dim > 2 ** 31 - 1:
            raise ValueError("Dimension size too big")
        return cls(sampler, seed, round_up_pow2(lc.light_iterations), (dim, dim))

    def struct(self):
        return capi.AvrGraphSampling(self.sampler, self.seed, self.samples_per_pixel, self.resolution[0],
                                     self.resolution[1], self.resolution[0])


# ---------------------------------------------------------------------------
# Medium geometry (util.h:45-91 PrimitiveData / MediumData, 419-503 GetHits / StartEndT)

def _gamma(n):
    eps = f32(np.finfo(np.float32).eps) * f32(0.5)
    return f32(f32(n) * eps) / f32(f32(1) - f32(f32(n) * eps))


def _xf_point(m, p):   # Transform::operator()(Point3f): left-to-right sums (affine)
    return np.array([f32(f32(f32(m[r, 0] * p[0]) + f32(m[r, 1] * p[1])) + f32(m[r, 2] * p[2])) + m[r, 3]
                     for r in range(3)], f32)


def _xf_vector(m, v):
    return np.array([f32(f32(f32(m[r, 0] * v[0]) + f32(m[r, 1] * v[1])) + f32(m[r, 2] * v[2])) for r in range(3)], f32)


def coordinate_system(v):
    """CoordinateSystem (vecmath.h:1007-1013) in float32."""
    v = np.asarray(v, f32)
    sign = f32(math.copysign(1.0, float(v[2])))
    a = f32(-1) / f32(sign + v[2])
    b = f32(f32(v[0] * v[1]) * a)
    x = np.array([f32(1) + f32(f32(sign * f32(v[0] * v[0])) * a), f32(sign * b), f32(-sign * v[0])], f32)
    y = np.array([b, f32(sign + f32(f32(v[1] * v[1]) * a)), f32(-v[1])], f32)
    return x, y


class MediumData:
    """util::MediumData / PrimitiveData (util.h:45-91): the medium's boundary box in render
    space, its center and maxDistToCenter = |Diagonal / 2|."""

    def __init__(self, scene):
        med = scene.medium
        self.scene = scene
        self.mfr = np.asarray(scene.medium_from_render, f32)
        b = np.asarray(med.bounds, f32)
        self.bmin, self.bmax = b[:3], b[3:]
        rfm = np.asarray(scene.render_from_medium, f32)
        corners = [_xf_point(rfm, np.array([x, y, z], f32)) for x in (b[0], b[3]) for y in (b[1], b[4])
                   for z in (b[2], b[5])]
        self.pmin = np.min(corners, axis=0).astype(f32)
        self.pmax = np.max(corners, axis=0).astype(f32)
        diag = (self.pmax - self.pmin).astype(f32)
        half = (diag / f32(2)).astype(f32)
        self.bounds_center = (self.pmin + half).astype(f32)
        self.max_dist_to_center = f32(np.sqrt(f32(f32(f32(half[0] * half[0]) + f32(half[1] * half[1])) +
                                                  f32(half[2] * half[2]))))

    def box_hits(self, o, d):
        """GetHits(primitive) in the model: (type, t0, t1); 0 OutsideTwoHits, 2 zero hits,
        3 InsideOneHit (t0 = exit). Bounds3::IntersectP (vecmath.h:1547-1571) in medium space."""
        om, dm = _xf_point(self.mfr, o), _xf_vector(self.mfr, d)
        t0, t1 = f32(0), f32(np.inf)
        s = f32(f32(1) + f32(f32(2) * _gamma(3)))
        with np.errstate(divide="ignore", invalid="ignore"):
            for i in range(3):
                inv = f32(f32(1) / dm[i])
                tn = f32(f32(self.bmin[i] - om[i]) * inv)
                tf = f32(f32(self.bmax[i] - om[i]) * inv)
                if tn > tf:
                    tn, tf = tf, tn
                tf = f32(tf * s)
                t0 = tn if tn > t0 else t0
                t1 = tf if tf < t1 else t1
                if t0 > t1:
                    return 2, f32(0), f32(0)
        if t0 > 0:
            return 0, t0, t1
        return 3, t1, f32(0)


def same_spot_radius(medium_data):
    """GetSameSpotRadius (util.h:465-467)."""
    return f32(f32(medium_data.max_dist_to_center * f32(2)) / f32(1000))


# ---------------------------------------------------------------------------

class FreeGraph:
    """The assembled graph: vertices (id = row), vertex samples, edges with samples, and
    the in-node path length average (Graph::inNodePathLengthAverager)."""

    def __init__(self, builder_handle, radius):
        self._g = builder_handle
        self.radius = f32(radius)
        self.points, self.samples = builder_handle.vertices()
        self.edge_from, self.edge_to, self.edge_samples = builder_handle.edges()
        self.in_node_path_length, self.in_node_path_count = builder_handle.in_node_path_length()
        self.search_range = None

    @property
    def num_vertices(self):
        return len(self.samples)

    def transport_csr(self):
        """GetTransportMatrix (lighting_calculator.cpp:61-82) as CSR."""
        return self._g.transport()


class FreeGraphBuilder:
    """FreeGraphBuilder (free/free_graph_builder.cpp): walks on the GPU, merge on the host."""

    def __init__(self, ctx, medium_data, in_direction, sampling, config, node_radius=None, sample_index_offset=0):
        self.ctx = ctx
        self.md = medium_data
        self.in_dir = np.asarray(in_direction, f32)
        self.sampling = sampling
        self.config = config
        r = node_radius if node_radius is not None else f32(same_spot_radius(medium_data) * f32(config.radius_modifier))
        self.radius = f32(r)
        self.sample_index_offset = int(sample_index_offset)

    def start_rays(self):
        """BuildGraph's ray grid (:143-199): origins, directions, first-segment tMax (the
        medium exit after SkipIntersection) and the first sampling index per ray."""
        c = self.config
        md = self.md
        d = self.in_dir
        xv, yv = coordinate_system(d)
        origin = (md.bounds_center - (d * md.max_dist_to_center) * f32(2)).astype(f32)
        origin = (origin - ((xv + yv).astype(f32) * md.max_dist_to_center)).astype(f32)
        step = f32(f32(md.max_dist_to_center * f32(2)) / f32(c.dimension_steps + 1))
        xv, yv = (xv * step).astype(f32), (yv * step).astype(f32)
        o, t, idx = [], [], []
        for x in range(1, c.dimension_steps + 1):
            for y in range(1, c.dimension_steps + 1):
                p = ((origin + (xv * f32(x)).astype(f32)).astype(f32) + (yv * f32(y)).astype(f32)).astype(f32)
                ty, t0, t1 = md.box_hits(p, d)
                if ty == 2:
                    continue
                if ty == 0:
                    p = (p + (d * t0).astype(f32)).astype(f32)     # SkipIntersection (no offset)
                    t_exit = f32(t1 - t0)
                else:
                    t_exit = t0
                o.append(p)
                t.append(t_exit)
                idx.append(((y - 1) + (x - 1) * c.dimension_steps) * c.iterations_per_step)
        n = len(o)
        return (np.array(o, f32).reshape(n, 3), np.tile(d, (n, 1)).astype(f32), np.array(t, f32),
                np.array(idx, np.int64))

    def build_graph(self):
        c = self.config
        o, d, t, idx = self.start_rays()
        pts, counts = self.ctx.graph_walks(self.sampling.struct(), o, d, t, idx, c.iterations_per_step,
                                           self.sample_index_offset, c.max_depth)
        g = capi.Graph(self.radius)
        g.add_walks(pts, counts, c.max_depth)
        self.reinforce_cycles = self.reinforce_sparse_vertices(g)
        graph = FreeGraph(g, self.radius)
        if c.render_search_range.get("active"):
            graph.search_range = compute_search_ranges(graph.points, int(c.render_search_range["neighboursToUse"]))
        return graph


    def _reinforce(self, g, ids, cfg, cycle):
        """ReinforceSparseVertices(graph, sparseVertices, ...) (:434-475): every listed
        vertex's sphere rays in one device call, their walks in a second (the rays never
        depend on the graph), merged in vertex then point order as the reference's loop."""
        if not len(ids):
            return
        md = self.config.max_depth
        k = int(cfg["reinforcementRays"])
        ids = np.asarray(ids, np.int32)
        xyz, _ = g.vertices()
        smp = self.sampling.struct()
        o, d, t, valid = self.ctx.graph_reinforce_rays(smp, ids, xyz[ids], self.radius, k, cycle)
        sel = valid.ravel() != 0
        if not sel.any():
            return
        index0 = (ids.astype(np.int64)[:, None] * k + np.arange(k)[None, :]).ravel()[sel]
        pts, counts = self.ctx.graph_walks(smp, o.reshape(-1, 3)[sel], d.reshape(-1, 3)[sel], t.ravel()[sel], index0,
                                           1, cycle, md - 1, skip_dims=2)
        padded = np.zeros((len(counts), md, 3), np.float32)   # avr_graph_add_walks_from: stride max_depth
        padded[:, :md - 1] = pts[:, :md - 1]
        g.add_walks_from(padded, counts, md, np.repeat(ids, k)[sel])

    def reinforce_sparse_vertices(self, g):
        """FreeGraphBuilder::ReinforceSparseVertices (free_graph_builder.cpp:280-432): until the
        fraction of initial vertices with fewer than `edgesForNotSparse` out-edges (and / or
        fewer than `neighboursForNotSparse` vertices within radius x neighbourRangeModifier)
        drops below `unsatisfiedAllowedRatio`, walks from `reinforcementRays` random points in
        each sparse vertex's sphere are added, one sampler cycle per round. The sparse lists are
        re-checked after every pass (the reference skips the re-check when quiet, :392-408,
        which never terminates). Returns the cycles run."""
        c = self.config
        ec, nc = c.edge_reinforcement, c.neighbour_reinforcement
        ea, na = bool(ec.get("active")), bool(nc.get("active"))
        if not (ea or na):
            return 0
        if c.max_depth == 1:
            raise ValueError("Unable to reinforce with max depth of 1")
        n0 = g.size()[0]
        initial = np.arange(n0, dtype=np.int32)
        r_sq = f32(self.radius * self.radius)
        n_radius = f32(f32(np.sqrt(r_sq)) * f32(nc.get("neighbourRangeModifier", 1.0)))
        state = {"e": initial, "n": initial}

        def check_e():
            deg = g.out_degrees()
            state["e"] = state["e"][deg[state["e"]] < int(ec["edgesForNotSparse"])]
            return len(state["e"]) / n0 < float(ec["unsatisfiedAllowedRatio"])

        def check_n():
            cnt = g.count_in_radius(state["n"], n_radius)
            state["n"] = state["n"][cnt < int(nc["neighboursForNotSparse"])]
            return len(state["n"]) / n0 < float(nc["unsatisfiedAllowedRatio"])

        sat_e = check_e() if ea else True
        sat_n = check_n() if na else True
        cycle = 0
        while not (sat_e and sat_n):
            if cycle >= self.max_reinforce_cycles:
                raise RuntimeError(f"graph reinforcement not satisfied after {cycle} cycles")
            if ea and not sat_e:
                self._reinforce(g, state["e"], ec, cycle)
                sat_e = check_e()
            if na and not sat_n:
                self._reinforce(g, state["n"], nc, cycle)
                sat_n = check_n()
            cycle += 1
        return cycle

    max_reinforce_cycles = 64


def compute_search_ranges(points, n_closest):
    """FreeGraphBuilder::ComputeSearchRanges (:486-548): the average distance to the
    n closest other vertices, averaged again over the vertex and those neighbours."""
    n = len(points)
    if n_closest > n:
        raise ValueError("Graph does not contain enough vertices")
    from scipy.spatial import cKDTree
    tree = cKDTree(points.astype(np.float64))
    dist, nb = tree.query(points.astype(np.float64), k=min(n, n_closest + 1))
    dist, nb = np.atleast_2d(dist)[:, 1:], np.atleast_2d(nb)[:, 1:]
    avg = dist.mean(axis=1).astype(f32) if n_closest > 0 else np.zeros(n, f32)
    return ((avg + avg[nb].sum(axis=1)) / (1 + nb.shape[1])).astype(f32)


class LightingCalculator:
    """LightingCalculator (lighting_calculator.cpp): light vector and bounce propagation
    on the GPU."""

    def __init__(self, ctx, graph, medium_data, in_direction, sampling, config):
        if config.light_iterations <= 0:
            raise ValueError("Must have at least one light ray iteration")
        self.ctx, self.graph, self.md = ctx, graph, medium_data
        self.in_dir = np.asarray(in_direction, f32)
        self.sampling, self.config = sampling, config
        self.light_scalar = None

    def get_light_vector(self):
        c = self.config
        return self.ctx.graph_light(self.sampling.struct(), self.graph.points, self.in_dir, self.graph.radius,
                                    c.points_on_radius_light, c.light_iterations, self.md.max_dist_to_center)

    def get_transport_matrix(self):
        return self.graph.transport_csr()

    def compute_final_light(self, bounces_index=0, light=None, transport=None):
        """Returns the bounces completed; sets light_scalar (VertexData.lightScalar)."""
        light = self.get_light_vector() if light is None else light
        rp, col, val = self.get_transport_matrix() if transport is None else transport
        total, it = self.ctx.graph_propagate(rp, col, val, light, self.config.bounces[bounces_index])
        self.light_scalar = total
        return it

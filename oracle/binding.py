"""ctypes binding of the CPU oracle (oracle/volpath_oracle.cpp) — TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module, and only as the checker / CPU baseline; the product never does.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "volpath_oracle.cpp")
LIB = os.path.join(HERE, "_build", "liboracle.so")

c_float_p = ctypes.POINTER(ctypes.c_float)
c_double_p = ctypes.POINTER(ctypes.c_double)
c_u32_p = ctypes.POINTER(ctypes.c_uint32)


def build(force=False):
    """g++ -O2 -ffp-contract=off (pbrt's CMakeLists.txt:134-137 float semantics)."""
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    if not force and os.path.exists(LIB) and os.path.getmtime(LIB) >= os.path.getmtime(SRC):
        return LIB
    cmd = ["g++", "-std=c++17", "-O2", "-ffp-contract=off", "-fPIC", "-shared", "-Wall", SRC, "-o", LIB,
           "-lpthread"]
    subprocess.check_call(cmd)
    return LIB


class OracleScene(ctypes.Structure):
    _fields_ = [
        ("density", c_float_p), ("nx", ctypes.c_int), ("ny", ctypes.c_int), ("nz", ctypes.c_int),
        ("bounds", ctypes.c_float * 6),
        ("render_from_medium", ctypes.c_float * 16),
        ("medium_from_render", ctypes.c_float * 16),
        ("sigma_a", c_float_p), ("sigma_s", c_float_p),
        ("g", ctypes.c_float),
        ("emissive", ctypes.c_int),
        ("Le", c_float_p),
        ("Lescale", c_float_p), ("lnx", ctypes.c_int), ("lny", ctypes.c_int), ("lnz", ctypes.c_int),
        ("majorant", c_float_p), ("mres", ctypes.c_int * 3),
        ("nlights", ctypes.c_int),
        ("light_type", ctypes.c_int * 8),
        ("light_w", (ctypes.c_float * 3) * 8),
        ("light_L", c_float_p * 8),
        ("light_scale", ctypes.c_float * 8),
        ("scene_radius", ctypes.c_float),
        ("camera_type", ctypes.c_int),
        ("camera_from_raster", ctypes.c_float * 16),
        ("render_from_camera", ctypes.c_float * 16),
        ("width", ctypes.c_int), ("height", ctypes.c_int),
        ("filter_radius", ctypes.c_float * 2),
        ("sensor_xyz", c_float_p),
        ("imaging_ratio", ctypes.c_float),
        ("output_from_sensor", ctypes.c_float * 9),
        ("max_component_value", ctypes.c_float),
        ("max_depth", ctypes.c_int),
        ("seed", ctypes.c_int),
        ("sampler_type", ctypes.c_int),
        ("samples_per_pixel", ctypes.c_int),
        ("filter_type", ctypes.c_int),
        ("filter_sigma", ctypes.c_float),
        ("medium_type", ctypes.c_int),
        ("cloud", ctypes.c_float * 3),
        ("temperature", c_float_p),
        ("temperature_scale", ctypes.c_float),
        ("temperature_offset", ctypes.c_float),
        ("vdb", ctypes.c_void_p),
        ("vdb_temperature", ctypes.c_void_p),
        ("vdb_lescale", ctypes.c_float),
        ("rgb_sigma_a", c_float_p), ("rgb_sigma_s", c_float_p), ("rgb_Le", c_float_p),
        ("rgb_illuminant", c_float_p),
        ("rgb_sigma_scale", ctypes.c_float), ("rgb_Le_scale", ctypes.c_float),
        ("light_img", c_float_p * 8), ("light_res", ctypes.c_int * 8), ("light_dist", c_float_p * 8),
        ("light_rfl", (ctypes.c_float * 9) * 8), ("light_lfr", (ctypes.c_float * 9) * 8),
        ("light_illuminant", c_float_p),
        ("film_nbuckets", ctypes.c_int), ("film_lambda_min", ctypes.c_float), ("film_lambda_max", ctypes.c_float),
        ("boundary", ctypes.c_int), ("sphere", ctypes.c_float * 4), ("n_planes", ctypes.c_int), ("planes", c_float_p),
        ("light_sampler", ctypes.c_int),
    ]


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = ctypes.CDLL(build())
        L = _lib
        L.oracle_pixel_sample.restype = ctypes.c_int
        L.oracle_pixel_sample.argtypes = [ctypes.POINTER(OracleScene), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          c_float_p, c_float_p, c_float_p, c_float_p]
        L.oracle_zsobol.argtypes = [ctypes.c_int] * 7 + [ctypes.c_char_p, c_float_p]
        L.oracle_sobol_fastowen.restype = ctypes.c_float
        L.oracle_sobol_fastowen.argtypes = [ctypes.c_ulonglong, ctypes.c_int, ctypes.c_uint]
        L.oracle_sobol_plain.restype = ctypes.c_float
        L.oracle_sobol_plain.argtypes = [ctypes.c_ulonglong, ctypes.c_int]
        L.oracle_gaussian_filter_sample.argtypes = [ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_int,
                                                    c_float_p, c_float_p]
        L.oracle_render.restype = ctypes.c_longlong
        L.oracle_render.argtypes = [ctypes.POINTER(OracleScene), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    c_double_p, c_double_p]
        L.oracle_render_list.restype = ctypes.c_longlong
        L.oracle_render_list.argtypes = [ctypes.POINTER(OracleScene), ctypes.POINTER(ctypes.c_int), ctypes.c_int,
                                         ctypes.c_int, ctypes.c_int, ctypes.c_int, c_double_p, c_double_p]
        L.oracle_film_resolve.argtypes = [ctypes.POINTER(OracleScene), c_double_p, c_double_p, c_float_p]
        L.oracle_transmittance.argtypes = [ctypes.POINTER(OracleScene), ctypes.c_int, c_float_p, c_float_p,
                                           ctypes.c_float, c_float_p]
        L.oracle_dda_segments.restype = ctypes.c_int
        L.oracle_dda_segments.argtypes = [ctypes.POINTER(OracleScene), c_float_p, c_float_p, ctypes.c_float,
                                          ctypes.c_float, ctypes.c_int, c_float_p]
        L.oracle_build_majorant.argtypes = [c_float_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                            ctypes.c_int, ctypes.c_int, c_float_p]
        L.oracle_rng.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int, c_u32_p, ctypes.c_int64, c_u32_p,
                                 ctypes.c_int]
        L.oracle_rng_uniform.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int, ctypes.c_int, c_float_p]
        L.oracle_rng_single.argtypes = [ctypes.c_uint64, ctypes.c_int, c_u32_p]
        for name, args in (("oracle_hash_float", [ctypes.c_float]),
                           ("oracle_hash_pixel_seed", [ctypes.c_int, ctypes.c_int, ctypes.c_int]),
                           ("oracle_hash_point3f", [ctypes.c_float, ctypes.c_float, ctypes.c_float]),
                           ("oracle_mixbits", [ctypes.c_uint64])):
            getattr(L, name).restype = ctypes.c_uint64
            getattr(L, name).argtypes = args
        for name, args in (("oracle_fastexp", [ctypes.c_float]),
                           ("oracle_sample_exponential", [ctypes.c_float, ctypes.c_float]),
                           ("oracle_hg_eval", [ctypes.c_float, ctypes.c_float]),
                           ("oracle_grid_lookup", [c_float_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                   ctypes.c_float, ctypes.c_float, ctypes.c_float]),
                           ("oracle_grid_maxvalue", [c_float_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                     c_float_p]),
                           ("oracle_noise", [ctypes.c_float, ctypes.c_float, ctypes.c_float, c_float_p]),
                           ("oracle_blackbody", [ctypes.c_float, ctypes.c_float]),
                           ("oracle_cloud_density", [ctypes.c_float] * 6)):
            getattr(L, name).restype = ctypes.c_float
            getattr(L, name).argtypes = args
        L.oracle_sample_discrete3.restype = ctypes.c_int
        L.oracle_sample_discrete3.argtypes = [c_float_p, ctypes.c_float]
        L.oracle_sample_visible.argtypes = [ctypes.c_float, c_float_p, c_float_p]
        L.oracle_sample_uniform.argtypes = [ctypes.c_float, ctypes.c_float, ctypes.c_float, c_float_p, c_float_p]
        L.oracle_render_spectral.restype = ctypes.c_longlong
        L.oracle_render_spectral.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int] + [
            ctypes.POINTER(ctypes.c_double)] * 4
        L.oracle_hg_sample.argtypes = [c_float_p, ctypes.c_float, ctypes.c_float, ctypes.c_float, c_float_p,
                                       c_float_p]
        L.oracle_intersectp.restype = ctypes.c_int
        L.oracle_intersectp.argtypes = [c_float_p, c_float_p, c_float_p, ctypes.c_float, c_float_p]
        L.oracle_transform_ray.argtypes = [c_float_p, c_float_p, c_float_p, c_float_p, ctypes.c_int, c_float_p]
        L.oracle_independent_sampler.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                 ctypes.c_int, ctypes.c_int, c_float_p]
        L.oracle_cloud_grid.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, c_float_p]
        L.oracle_set_libm.argtypes = [ctypes.c_int]
        L.oracle_transmittance4.argtypes = [ctypes.POINTER(OracleScene), ctypes.c_int, c_float_p, c_float_p,
                                            c_float_p, c_float_p]
        L.oracle_get_libm.restype = ctypes.c_int
        c_int_p = ctypes.POINTER(ctypes.c_int)
        L.oracle_vdb_create.restype = ctypes.c_void_p
        L.oracle_vdb_create.argtypes = [ctypes.c_int, c_int_p, c_float_p, ctypes.c_int, c_int_p, c_int_p, c_float_p,
                                        ctypes.c_float, c_int_p, c_double_p, c_double_p]
        L.oracle_vdb_free.argtypes = [ctypes.c_void_p]
        L.oracle_equal_area_square_to_sphere.argtypes = [ctypes.c_float, ctypes.c_float, c_float_p]
        L.oracle_equal_area_sphere_to_square.argtypes = [ctypes.c_float] * 3 + [c_float_p]
        L.oracle_remap_octahedral.argtypes = [ctypes.c_int] * 3 + [c_int_p]
        L.oracle_pc2d.argtypes = [c_float_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_float_p, c_float_p]
        for name in ("oracle_rsp_eval", "oracle_rsp_max"):
            getattr(L, name).restype = ctypes.c_float
        L.oracle_rsp_eval.argtypes = [ctypes.c_float] * 4
        L.oracle_rsp_max.argtypes = [ctypes.c_float] * 3
        L.oracle_rgb_majorant.argtypes = [c_float_p, c_float_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_float, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_float_p]
        L.oracle_vdb_value.restype = ctypes.c_float
        L.oracle_vdb_value.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.oracle_vdb_sample_world.restype = ctypes.c_float
        L.oracle_vdb_sample_world.argtypes = [ctypes.c_void_p, ctypes.c_float, ctypes.c_float, ctypes.c_float]
        L.oracle_vdb_bounds.argtypes = [ctypes.c_void_p, ctypes.c_void_p, c_float_p]
        L.oracle_vdb_majorant.argtypes = [ctypes.c_void_p, c_float_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          c_float_p]
        c_ll_p = ctypes.POINTER(ctypes.c_longlong)
        L.oracle_graph_light.argtypes = [ctypes.POINTER(OracleScene), ctypes.c_int, c_float_p, c_float_p,
                                         ctypes.c_float, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                         c_float_p]
        L.oracle_graph_walks.argtypes = [ctypes.POINTER(OracleScene), ctypes.c_int, c_float_p, c_float_p, c_float_p,
                                         c_ll_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         c_float_p, c_int_p]
        L.oracle_graph_reinforce_rays.argtypes = [ctypes.POINTER(OracleScene), ctypes.c_int, c_int_p, c_float_p,
                                                  ctypes.c_float, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_float_p,
                                                  c_float_p, c_float_p, c_int_p]
        L.oracle_graph_propagate.restype = ctypes.c_int
        L.oracle_graph_propagate.argtypes = [ctypes.c_int, c_int_p, c_int_p, c_float_p, c_float_p, ctypes.c_int,
                                             c_float_p]
        L.oracle_graph_sphere_hits.restype = ctypes.c_int
        L.oracle_graph_sphere_hits.argtypes = [ctypes.c_float] * 4 + [c_float_p, c_float_p, c_float_p]
        L.oracle_graph_box_hits.restype = ctypes.c_int
        L.oracle_graph_box_hits.argtypes = [ctypes.POINTER(OracleScene), c_float_p, c_float_p, c_float_p]
        L.oracle_graph_disk_points.restype = ctypes.c_int
        L.oracle_graph_disk_points.argtypes = [c_float_p, ctypes.c_float, ctypes.c_int, c_float_p, c_float_p,
                                               ctypes.c_int]
    return _lib


# ---------------------------------------------------------------------------
# Lighting graph (src/graph) — oracle_graph_* in volpath_oracle.cpp

def _ip(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int))


def graph_sphere_hits(c, r, o, d):
    """(type, t0, t1) of the model's GetHits(sphere) — 0 OutsideTwoHits, 2 zero, 3 InsideOneHit."""
    t = np.zeros(2, np.float32)
    o = np.ascontiguousarray(o, np.float32)
    d = np.ascontiguousarray(d, np.float32)
    ty = lib().oracle_graph_sphere_hits(float(c[0]), float(c[1]), float(c[2]), float(r), fp(o), fp(d), fp(t))
    return ty, t[0], t[1]


def graph_disk_points(center, radius, n, direction):
    cap = (2 * n + 1) ** 2
    out = np.zeros((cap, 3), np.float32)
    c = np.ascontiguousarray(center, np.float32)
    d = np.ascontiguousarray(direction, np.float32)
    k = lib().oracle_graph_disk_points(fp(c), float(radius), int(n), fp(d), fp(out), cap)
    return out[:k]


def graph_propagate(n, rowptr, col, val, light, bounces):
    """ComputeFinalLight restated: (total light, iterations completed)."""
    rowptr = np.ascontiguousarray(rowptr, np.int32)
    col = np.ascontiguousarray(col, np.int32)
    val = np.ascontiguousarray(val, np.float32)
    light = np.ascontiguousarray(light, np.float32)
    total = np.zeros(n, np.float32)
    it = lib().oracle_graph_propagate(int(n), _ip(rowptr), _ip(col), fp(val), fp(light), int(bounces), fp(total))
    return total, it


LIBM_MODES = {"platform": 0, "canonical": 1}


def set_libm(mode):
    """'platform': pbrt's float libm calls as built on this host (pinned by the goldens);
    'canonical': correctly rounded transcendentals, the HIP path's convention."""
    lib().oracle_set_libm(LIBM_MODES[mode])


def fp(a):
    return a.ctypes.data_as(c_float_p)


def build_majorant(density, res=(16, 16, 16)):
    d = np.ascontiguousarray(density, np.float32)
    nz, ny, nx = d.shape
    out = np.empty(res[0] * res[1] * res[2], np.float32)
    lib().oracle_build_majorant(fp(d), nx, ny, nz, res[0], res[1], res[2], fp(out))
    return out


def cloud_grid(n, z0=0, z1=None):
    z1 = n if z1 is None else z1
    out = np.empty((z1 - z0, n, n), np.float32)
    lib().oracle_cloud_grid(n, z0, z1, fp(out))
    return out


class VdbTree:
    """The oracle's NanoVDB tree restatement built from a vdb.NanoVDBGrid."""

    def __init__(self, grid):
        ip = lambda a: np.ascontiguousarray(a, np.int32).ctypes.data_as(ctypes.POINTER(ctypes.c_int))
        self._keep = [np.ascontiguousarray(a) for a in (grid.leaf_origins, grid.leaf_values, grid.tile_origins,
                                                          grid.tile_sizes, grid.tile_values, grid.index_bbox,
                                                          grid.index_to_world, grid.world_to_index)]
        lo, lv, to, ts, tv, bb, m, mi = self._keep
        self.h = lib().oracle_vdb_create(len(lo), ip(lo), fp(lv.astype(np.float32)), len(tv), ip(to), ip(ts),
                                         fp(tv.astype(np.float32)), float(grid.background), ip(bb),
                                         m.astype(np.float64).ctypes.data_as(c_double_p),
                                         mi.astype(np.float64).ctypes.data_as(c_double_p))

    def value(self, x, y, z):
        return lib().oracle_vdb_value(self.h, int(x), int(y), int(z))

    def sample_world(self, p):
        return np.array([lib().oracle_vdb_sample_world(self.h, *map(float, q)) for q in np.asarray(p, np.float32)],
                        np.float32)

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.oracle_vdb_free(self.h)
            self.h = None


def rgb_majorant(med):
    """RGBGridMedium's 16^3 majorant (media.cpp:364-377) for a scene.RGBGridMedium."""
    a = np.ascontiguousarray(med.rgb_sigma_a, np.float32) if med.rgb_sigma_a is not None else None
    s = np.ascontiguousarray(med.rgb_sigma_s, np.float32) if med.rgb_sigma_s is not None else None
    res = med.majorant_res
    out = np.zeros(res[0] * res[1] * res[2], np.float32)
    lib().oracle_rgb_majorant(fp(a) if a is not None else None, fp(s) if s is not None else None, med.nx, med.ny,
                              med.nz, float(med.sigma_scale), res[0], res[1], res[2], fp(out))
    return out


def vdb_bounds(dtree, ttree=None):
    out = np.zeros(6, np.float32)
    lib().oracle_vdb_bounds(dtree.h, ttree.h if ttree is not None else None, fp(out))
    return out


def vdb_majorant(dtree, bounds, res=(64, 64, 64)):
    b = np.ascontiguousarray(bounds, np.float32)
    out = np.zeros(res[0] * res[1] * res[2], np.float32)
    lib().oracle_vdb_majorant(dtree.h, fp(b), res[0], res[1], res[2], fp(out))
    return out


class OracleRun:
    """Holds an OracleScene and the numpy buffers it points into."""

    def __init__(self, scene, max_depth=5, seed=0, libm="platform", lightsampler="bvh"):
        if libm not in LIBM_MODES:
            raise ValueError(f"libm must be one of {sorted(LIBM_MODES)}")
        if lightsampler not in ("bvh", "uniform", "power"):
            raise ValueError(f"{lightsampler}: unknown light sampling strategy")
        self.libm = libm
        med = scene.medium
        is_vdb = int(getattr(med, "type_id", 0)) == 3
        is_rgb = int(getattr(med, "type_id", 0)) == 4
        if med.density is None and not (is_vdb or is_rgb):
            raise ValueError("oracle needs a host density grid")
        s = OracleScene()
        keep = []

        def arr(a):
            a = np.ascontiguousarray(np.asarray(a, np.float32))
            keep.append(a)
            return fp(a)

        s.density = arr(med.density if med.density is not None else np.zeros((1, 1, 1), np.float32))
        s.nx, s.ny, s.nz = med.nx, med.ny, med.nz
        s.bounds[:] = [float(v) for v in med.bounds]
        s.render_from_medium[:] = [float(v) for v in scene.render_from_medium.reshape(-1)]
        s.medium_from_render[:] = [float(v) for v in scene.medium_from_render.reshape(-1)]
        s.sigma_a = arr(med.sigma_a)
        s.sigma_s = arr(med.sigma_s)
        s.g = float(med.g)
        s.emissive = 1 if (med.Le is not None and float(np.max(med.Le)) > 0) else 0
        s.Le = arr(med.Le if med.Le is not None else np.zeros(471, np.float32))
        ls = np.ascontiguousarray(med.Lescale, np.float32)
        s.Lescale = arr(ls)
        s.lnz, s.lny, s.lnx = ls.shape
        if is_vdb:
            self.vdb = VdbTree(med.grid)
            self.vdb_temperature = VdbTree(med.temperature_grid) if med.temperature_grid is not None else None
            self.bounds = vdb_bounds(self.vdb, self.vdb_temperature)
            s.bounds[:] = [float(v) for v in self.bounds]
            s.vdb = self.vdb.h
            s.vdb_temperature = self.vdb_temperature.h if self.vdb_temperature is not None else None
            s.vdb_lescale = float(med.Lescale_value)
            s.temperature_scale = float(med.temperature_scale)
            s.temperature_offset = float(med.temperature_offset)
            self.majorant = vdb_majorant(self.vdb, self.bounds, med.majorant_res)
        elif is_rgb:
            opt = lambda g: arr(g.reshape(-1)) if g is not None else None
            s.rgb_sigma_a, s.rgb_sigma_s, s.rgb_Le = opt(med.rgb_sigma_a), opt(med.rgb_sigma_s), opt(med.rgb_Le)
            s.rgb_illuminant = arr(med.illuminant)
            s.rgb_sigma_scale = float(med.sigma_scale)
            s.rgb_Le_scale = float(med.Le_scale)
            self.majorant = rgb_majorant(med)
        else:
            self.majorant = build_majorant(med.density, med.majorant_res)
        s.majorant = arr(self.majorant)
        s.mres[:] = list(med.majorant_res)
        s.medium_type = int(getattr(med, "type_id", 0))
        temp = getattr(med, "temperature", None)
        if temp is not None:
            s.temperature = arr(temp)
            s.temperature_scale = float(med.temperature_scale)
            s.temperature_offset = float(med.temperature_offset)
            s.emissive = 1
        if s.medium_type == 2:
            s.cloud[:] = [float(v) for v in med.cloud]
        s.nlights = len(scene.lights)
        for i in range(s.nlights):
            s.light_type[i] = int(scene.light_types[i])
            for k in range(3):
                s.light_w[i][k] = float(scene.light_w[i][k])
            s.light_L[i] = arr(scene.light_L[i])
            s.light_scale[i] = float(scene.light_scale[i])
            lt = scene.lights[i]
            if lt.type_id == 2:
                s.light_img[i] = arr(lt.coeffs.reshape(-1))
                s.light_res[i] = int(lt.res)
                s.light_dist[i] = arr(lt.distribution.reshape(-1))
                s.light_rfl[i][:] = [float(v) for v in scene.light_rfl[i][:3, :3].reshape(-1)]
                s.light_lfr[i][:] = [float(v) for v in scene.light_lfr[i][:3, :3].reshape(-1)]
                s.light_illuminant = arr(lt.illuminant)
        s.scene_radius = float(scene.scene_radius)
        s.light_sampler = 1 if lightsampler == "power" else 0
        s.camera_type = int(scene.camera.type_id)
        s.camera_from_raster[:] = [float(v) for v in scene.camera_from_raster.reshape(-1)]
        s.render_from_camera[:] = [float(v) for v in scene.render_from_camera.reshape(-1)]
        f = scene.film
        s.width, s.height = f.width, f.height
        s.filter_radius[:] = [float(v) for v in f.filter_radius]
        s.sensor_xyz = arr(f.sensor.reshape(-1))
        s.imaging_ratio = float(f.imaging_ratio)
        s.output_from_sensor[:] = [float(v) for v in f.output_from_sensor.reshape(-1)]
        s.max_component_value = float(f.max_component_value)
        s.film_nbuckets = int(getattr(f, "nbuckets", 0))
        s.film_lambda_min = float(getattr(f, "lambdamin", 360.0))
        s.film_lambda_max = float(getattr(f, "lambdamax", 830.0))
        sph = getattr(scene, "interface_sphere_render", None)
        s.boundary = 1 if sph is not None else 0
        if sph is not None:
            s.sphere[:] = [float(v) for v in sph]
        planes = getattr(scene, "interface_planes_render", None)
        if planes is not None:
            s.boundary = 2
            s.n_planes = len(planes)
            s.planes = arr(np.ascontiguousarray(planes, np.float32).reshape(-1))
        s.max_depth = int(max_depth)
        s.seed = int(seed)
        smp = scene.sampler
        s.sampler_type = int(smp.type_id)
        s.samples_per_pixel = int(smp.pixelsamples)
        s.filter_type = int(f.filter.type_id)
        s.filter_sigma = float(f.filter.sigma)
        self.s = s
        self.keep = keep
        self.scene = scene

    def pixel_sample(self, px, py, sample_index, with_weight=False):
        L = np.zeros(4, np.float32)
        lam = np.zeros(4, np.float32)
        pdf = np.zeros(4, np.float32)
        w = np.zeros(1, np.float32)
        set_libm(self.libm)
        n = lib().oracle_pixel_sample(ctypes.byref(self.s), px, py, sample_index, fp(L), fp(lam), fp(pdf), fp(w))
        if with_weight:
            return L, lam, pdf, n, w[0]
        return L, lam, pdf, n

    def render(self, spp0, spp1, nthreads=1):
        f = self.scene.film
        npix = f.width * f.height
        rgb = np.zeros(3 * npix, np.float64)
        w = np.zeros(npix, np.float64)
        set_libm(self.libm)
        events = lib().oracle_render(ctypes.byref(self.s), spp0, spp1, nthreads, rgb.ctypes.data_as(c_double_p),
                                     w.ctypes.data_as(c_double_p))
        self.last_events = events
        return rgb, w

    def render_spectral(self, spp0, spp1, nthreads=1):
        """SpectralFilm render: (rgb_sum, w_sum, bucket_sums, weight_sums), buckets (W*H, nb)."""
        f = self.scene.film
        npix, nb = f.width * f.height, int(self.s.film_nbuckets)
        if nb <= 0:
            raise ValueError("scene film is not a SpectralFilm")
        rgb = np.zeros(3 * npix, np.float64)
        w = np.zeros(npix, np.float64)
        bs = np.zeros(npix * nb, np.float64)
        bw = np.zeros(npix * nb, np.float64)
        set_libm(self.libm)
        dp = lambda a: a.ctypes.data_as(c_double_p)
        self.last_events = lib().oracle_render_spectral(ctypes.byref(self.s), spp0, spp1, nthreads, dp(rgb), dp(w),
                                                        dp(bs), dp(bw))
        return rgb, w, bs.reshape(npix, nb), bw.reshape(npix, nb)

    def render_list(self, pixels, spp0, spp1, nthreads=1):
        pixels = np.ascontiguousarray(pixels, np.int32)
        rgb = np.zeros(3 * len(pixels), np.float64)
        w = np.zeros(len(pixels), np.float64)
        set_libm(self.libm)
        events = lib().oracle_render_list(ctypes.byref(self.s), pixels.ctypes.data_as(ctypes.POINTER(ctypes.c_int)),
                                          len(pixels), spp0, spp1, nthreads, rgb.ctypes.data_as(c_double_p),
                                          w.ctypes.data_as(c_double_p))
        return rgb, w, events

    def transmittance(self, p0, p1, lambda_u=0.5):
        p0 = np.ascontiguousarray(p0, np.float32)
        p1 = np.ascontiguousarray(p1, np.float32)
        out = np.zeros(len(p0), np.float32)
        set_libm(self.libm)
        lib().oracle_transmittance(ctypes.byref(self.s), len(p0), fp(p0), fp(p1), lambda_u, fp(out))
        return out

    def graph_light(self, verts, in_dir, radius, points_on_radius, iterations, res_x, max_dist_to_center,
                    sampler=None):
        """LightingCalculator::GetLightVector (per-vertex light, Inv4Pi applied).
        sampler = (type, seed, spp, width, height) of the scene sampler, default: the scene's."""
        verts = np.ascontiguousarray(verts, np.float32)
        d = np.ascontiguousarray(in_dir, np.float32)
        out = np.zeros(len(verts), np.float32)
        set_libm(self.libm)
        with self._graph_sampler(sampler) as s:
            lib().oracle_graph_light(ctypes.byref(s), len(verts), fp(verts), fp(d), float(radius),
                                     int(points_on_radius), int(iterations), int(res_x), float(max_dist_to_center),
                                     fp(out))
        return out

    def graph_reinforce_rays(self, ids, points, radius, n_rays, cycle, res_x, sampler=None):
        """ReinforceSparseVertices' rays: (o, d (n, n_rays, 3), t_first, valid (n, n_rays))."""
        ids = np.ascontiguousarray(ids, np.int32)
        pts = np.ascontiguousarray(points, np.float32)
        n, k = len(ids), int(n_rays)
        o = np.zeros((n, k, 3), np.float32)
        d = np.zeros((n, k, 3), np.float32)
        t = np.zeros((n, k), np.float32)
        valid = np.zeros((n, k), np.int32)
        set_libm(self.libm)
        with self._graph_sampler(sampler) as s:
            lib().oracle_graph_reinforce_rays(ctypes.byref(s), n, _ip(ids), fp(pts), float(radius), k, int(cycle),
                                              int(res_x), fp(o), fp(d), fp(t), _ip(valid))
        return o, d, t, valid

    def graph_walks(self, o, d, t_first, index0, iterations, sample_index, res_x, max_depth, sampler=None,
                    skip_dims=0):
        """FreeGraphBuilder::TracePath walks: (points[nrays*iterations, max_depth, 3], counts)."""
        o = np.ascontiguousarray(o, np.float32)
        d = np.ascontiguousarray(d, np.float32)
        t_first = np.ascontiguousarray(t_first, np.float32)
        index0 = np.ascontiguousarray(index0, np.int64)
        n = len(o) * int(iterations)
        pts = np.zeros((n, max(1, int(max_depth)), 3), np.float32)
        counts = np.zeros(n, np.int32)
        set_libm(self.libm)
        with self._graph_sampler(sampler) as s:
            lib().oracle_graph_walks(ctypes.byref(s), len(o), fp(o), fp(d), fp(t_first),
                                     index0.ctypes.data_as(ctypes.POINTER(ctypes.c_longlong)), int(iterations),
                                     int(sample_index), int(skip_dims), int(res_x), int(max_depth), fp(pts),
                                     _ip(counts))
        return pts, counts

    def graph_box_hits(self, o, d):
        t = np.zeros(2, np.float32)
        ty = lib().oracle_graph_box_hits(ctypes.byref(self.s), fp(np.ascontiguousarray(o, np.float32)),
                                         fp(np.ascontiguousarray(d, np.float32)), fp(t))
        return ty, t[0], t[1]

    def _graph_sampler(self, sampler):
        import contextlib

        @contextlib.contextmanager
        def ctx():
            s = self.s
            saved = (s.sampler_type, s.seed, s.samples_per_pixel, s.width, s.height)
            if sampler is not None:
                s.sampler_type, s.seed, s.samples_per_pixel, s.width, s.height = [int(v) for v in sampler]
            try:
                yield s
            finally:
                s.sampler_type, s.seed, s.samples_per_pixel, s.width, s.height = saved
        return ctx()

    def transmittance4(self, p0, p1, lam):
        """Integrator::Tr at explicit wavelengths: (n, 4)."""
        p0 = np.ascontiguousarray(p0, np.float32)
        p1 = np.ascontiguousarray(p1, np.float32)
        lam = np.ascontiguousarray(lam, np.float32)
        out = np.zeros((len(p0), 4), np.float32)
        set_libm(self.libm)
        lib().oracle_transmittance4(ctypes.byref(self.s), len(p0), fp(p0), fp(p1), fp(lam), fp(out))
        return out

    def dda_segments(self, o, d, tmax=np.inf, lambda_u=0.5, max_segs=256):
        o = np.ascontiguousarray(o, np.float32)
        d = np.ascontiguousarray(d, np.float32)
        out = np.zeros(3 * max_segs, np.float32)
        set_libm(self.libm)
        n = lib().oracle_dda_segments(ctypes.byref(self.s), fp(o), fp(d), float(tmax), lambda_u, max_segs, fp(out))
        return out[:3 * n].reshape(n, 3)


def zsobol_stream(spp, resx, resy, px, py, sample_index, seed, pattern):
    """ZSobolSampler outputs for a pattern of '1' (Get1D) / '2' (Get2D) calls."""
    n = sum(1 if c == "1" else 2 for c in pattern)
    out = np.zeros(n, np.float32)
    lib().oracle_zsobol(spp, resx, resy, px, py, sample_index, seed, pattern.encode(), fp(out))
    return out


def gaussian_filter_samples(rx, ry, sigma, u):
    """GaussianFilter::Sample for u (n x 2): rows (p.x, p.y, weight)."""
    u = np.ascontiguousarray(u, np.float32)
    out = np.zeros((len(u), 3), np.float32)
    lib().oracle_gaussian_filter_sample(rx, ry, sigma, len(u), fp(u), fp(out))
    return out

"""ctypes binding of the C-ABI in include/avr.h (libavr_hip.so, built in-tree).

This is the same binding a pbrt-side Python tool (or the ctypes stub in
INTEGRATION.md) would use. There is no fallback: if the HIP library is missing or
fails to load, importing the product raises.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# AVR_LIB overrides the library path (A/B experiments with variant builds); default in-tree.
LIB_PATH = os.environ.get("AVR_LIB", os.path.join(_HERE, "libavr_hip.so"))

c_float_p = ctypes.POINTER(ctypes.c_float)
c_double_p = ctypes.POINTER(ctypes.c_double)
c_int_p = ctypes.POINTER(ctypes.c_int)


class AvrStats(ctypes.Structure):
    _fields_ = [
        ("medium_lookups", ctypes.c_ulonglong),
        ("medium_items_in", ctypes.c_ulonglong),
        ("medium_items_out", ctypes.c_ulonglong),
        ("shadow_lookups", ctypes.c_ulonglong),
        ("shadow_items", ctypes.c_ulonglong),
        ("medium_dda_steps", ctypes.c_ulonglong),
        ("shadow_dda_steps", ctypes.c_ulonglong),
        ("medium_launches", ctypes.c_ulonglong),
        ("loop_iterations", ctypes.c_ulonglong),
        ("active_lane_iterations", ctypes.c_ulonglong),
        ("ms_camera", ctypes.c_double),
        ("ms_medium", ctypes.c_double),
        ("ms_shadow", ctypes.c_double),
        ("ms_film", ctypes.c_double),
        ("ms_total", ctypes.c_double),
        ("ms_setup", ctypes.c_double),
        ("ms_binning", ctypes.c_double),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class AvrGraphSampling(ctypes.Structure):
    """avr_graph_sampling (include/avr.h): the graph tools' sampler setup."""
    _fields_ = [("sampler", ctypes.c_int), ("seed", ctypes.c_int), ("samples_per_pixel", ctypes.c_int),
                ("film_width", ctypes.c_int), ("film_height", ctypes.c_int), ("resolution_x", ctypes.c_int)]


class AvrVdbGrid(ctypes.Structure):
    """avr_vdb_grid (include/avr.h): one NanoVDB FloatGrid's tree."""
    _fields_ = [
        ("n_leaves", ctypes.c_int),
        ("leaf_origin", c_int_p),
        ("leaf_values", c_float_p),
        ("n_tiles", ctypes.c_int),
        ("tile_origin", c_int_p),
        ("tile_size", c_int_p),
        ("tile_value", c_float_p),
        ("background", ctypes.c_float),
        ("index_bbox", ctypes.c_int * 6),
        ("index_to_world", ctypes.c_double * 12),
        ("world_to_index", ctypes.c_double * 9),
    ]

    @classmethod
    def of(cls, grid):
        """Struct view of a vdb.NanoVDBGrid (the grid's arrays must outlive the call)."""
        g = cls()
        ip = lambda a: a.ctypes.data_as(c_int_p) if a.size else None
        g.n_leaves = len(grid.leaf_origins)
        g.leaf_origin = ip(grid.leaf_origins)
        g.leaf_values = grid.leaf_values.ctypes.data_as(c_float_p) if grid.leaf_values.size else None
        g.n_tiles = len(grid.tile_values)
        g.tile_origin = ip(grid.tile_origins)
        g.tile_size = ip(grid.tile_sizes)
        g.tile_value = grid.tile_values.ctypes.data_as(c_float_p) if grid.tile_values.size else None
        g.background = float(grid.background)
        g.index_bbox[:] = [int(v) for v in grid.index_bbox]
        g.index_to_world[:] = [float(v) for v in grid.index_to_world.reshape(-1)]
        g.world_to_index[:] = [float(v) for v in grid.world_to_index.reshape(-1)]
        return g


# name -> (restype, argtypes); every symbol include/avr.h declares
SIGNATURES = {
    "avr_last_error": (ctypes.c_char_p, []),
    "avr_context_create": (ctypes.c_int, [ctypes.c_int, ctypes.c_longlong, ctypes.POINTER(ctypes.c_void_p)]),
    "avr_context_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "avr_set_stream": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "avr_set_kernel_mode": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "avr_set_render_mode": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "avr_record_lookups": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p]),
    "avr_density_fetch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_longlong, c_float_p, c_float_p]),
    "avr_set_ray_binning": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "avr_set_majorant_occupancy": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "avr_set_pass_table_ahead": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "avr_set_majorant_res": (ctypes.c_int, [ctypes.c_void_p, c_int_p]),
    "avr_medium_boundary_sphere": (ctypes.c_int, [ctypes.c_void_p, c_float_p, ctypes.c_float]),
    "avr_medium_boundary_convex": (ctypes.c_int, [ctypes.c_void_p, c_float_p, ctypes.c_int]),
    "avr_tune_majorant": (ctypes.c_int, [ctypes.c_void_p, c_int_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int, ctypes.c_int, c_int_p, c_float_p]),
    "avr_tune_walk": (ctypes.c_int, [ctypes.c_void_p, c_int_p, ctypes.c_int, c_int_p, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_int, ctypes.c_int, c_int_p, c_float_p]),
    "avr_set_refill_min": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "avr_light_sampler": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "avr_set_dda_budget": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "avr_set_grid_layout": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "avr_grid_layout_active": (ctypes.c_int, [ctypes.c_void_p]),
    "avr_medium_grid": (ctypes.c_int, [ctypes.c_void_p, c_float_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       c_float_p, c_float_p, c_float_p, c_float_p, c_float_p, ctypes.c_float,
                                       c_float_p, c_float_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_int_p]),
    "avr_medium_grid_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                              ctypes.c_int, c_float_p, c_float_p, c_float_p, c_float_p, c_float_p,
                                              ctypes.c_float, c_float_p, c_float_p, ctypes.c_int, ctypes.c_int,
                                              ctypes.c_int, c_int_p]),
    "avr_generate_cloud": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong,
                                          ctypes.c_longlong, ctypes.c_float, ctypes.c_float, ctypes.c_float]),
    "avr_generate_rgb_explosion": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                  ctypes.c_int, ctypes.c_longlong, ctypes.c_longlong]),
    "avr_medium_rgbgrid_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                 c_float_p, c_float_p, c_float_p, ctypes.c_void_p, ctypes.c_void_p,
                                                 ctypes.c_float, ctypes.c_float, ctypes.c_void_p, c_float_p,
                                                 ctypes.c_float]),
    "avr_read_majorant": (ctypes.c_int, [ctypes.c_void_p, c_float_p]),
    "avr_lights": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, c_int_p, c_float_p, c_float_p, c_float_p,
                                  ctypes.c_float]),
    "avr_camera": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, c_float_p, c_float_p]),
    "avr_light_image": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, c_float_p, c_float_p, c_float_p,
                                       c_float_p, c_float_p]),
    "avr_flip": (ctypes.c_int, [ctypes.c_void_p, c_float_p, c_float_p, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                c_float_p]),
    "avr_film_image_device": (ctypes.c_int, [ctypes.c_void_p, c_float_p, ctypes.c_int, ctypes.c_void_p]),
    "avr_film_set_reference": (ctypes.c_int, [ctypes.c_void_p, c_float_p, c_float_p, ctypes.c_int]),
    "avr_film_metric": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, c_float_p]),
    "avr_last_pass_weights": (ctypes.c_int, [ctypes.c_void_p, c_float_p, ctypes.c_longlong]),
    "avr_last_kernel": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int]),
    "avr_transmittance": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_longlong, c_float_p, c_float_p, c_float_p,
                                         c_float_p]),
    "avr_transmittance_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p,
                                                ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "avr_medium_temperature": (ctypes.c_int, [ctypes.c_void_p, c_float_p, ctypes.c_float, ctypes.c_float]),
    "avr_medium_homogeneous": (ctypes.c_int, [ctypes.c_void_p, c_float_p, c_float_p, c_float_p, c_float_p,
                                              c_float_p, ctypes.c_float, c_float_p]),
    "avr_medium_cloud": (ctypes.c_int, [ctypes.c_void_p, c_float_p, c_float_p, c_float_p, c_float_p, c_float_p,
                                        ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float]),
    "avr_medium_nanovdb": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(AvrVdbGrid), ctypes.POINTER(AvrVdbGrid),
                                          c_float_p, c_float_p, c_float_p, c_float_p, ctypes.c_float, ctypes.c_float,
                                          ctypes.c_float, ctypes.c_float]),
    "avr_medium_bounds": (ctypes.c_int, [ctypes.c_void_p, c_float_p]),
    "avr_medium_rgbgrid": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_float_p,
                                          c_float_p, c_float_p, c_float_p, c_float_p, ctypes.c_float, ctypes.c_float,
                                          c_float_p, c_float_p, ctypes.c_float]),
    "avr_set_filter": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, c_float_p, ctypes.c_float]),
    "avr_set_sampler": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]),
    "avr_set_sampler_table": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "avr_set_sampler_pass_table": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "avr_set_pixel_order": (ctypes.c_int, [ctypes.c_void_p, c_int_p, ctypes.c_longlong]),
    "avr_film": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, c_float_p, c_float_p, ctypes.c_float,
                                ctypes.c_float]),
    "avr_film_clear": (ctypes.c_int, [ctypes.c_void_p]),
    "avr_render": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "avr_sync": (ctypes.c_int, [ctypes.c_void_p]),
    "avr_get_stats": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(AvrStats)]),
    "avr_reset_stats": (ctypes.c_int, [ctypes.c_void_p]),
    "avr_film_read": (ctypes.c_int, [ctypes.c_void_p, c_double_p, c_double_p]),
    "avr_film_spectral": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_float]),
    "avr_film_read_spectral": (ctypes.c_int, [ctypes.c_void_p, c_double_p, c_double_p]),
    "avr_film_spectral_device_ptrs": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p),
                                                     ctypes.POINTER(ctypes.c_void_p)]),
    "avr_film_device_ptrs": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p),
                                            ctypes.POINTER(ctypes.c_void_p)]),
    "avr_film_export_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "avr_film_reduce_rccl": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_int]),
    "avr_last_pass_samples": (ctypes.c_int, [ctypes.c_void_p, c_float_p, c_float_p, c_float_p, ctypes.c_longlong,
                                             c_int_p, c_int_p]),
    "avr_graph_walks": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(AvrGraphSampling), ctypes.c_longlong, c_float_p,
                                       c_float_p, c_float_p, ctypes.POINTER(ctypes.c_longlong), ctypes.c_int,
                                       ctypes.c_int, ctypes.c_int, c_float_p, c_int_p]),
    "avr_graph_walks_from": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(AvrGraphSampling), ctypes.c_longlong,
                                            c_float_p, c_float_p, c_float_p, ctypes.POINTER(ctypes.c_longlong),
                                            ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_float_p, c_int_p]),
    "avr_graph_reinforce_rays": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(AvrGraphSampling), ctypes.c_int,
                                                c_int_p, c_float_p, ctypes.c_float, ctypes.c_int, ctypes.c_int,
                                                c_float_p, c_float_p, c_float_p, c_int_p]),
    "avr_graph_add_walks_from": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int, c_float_p, c_int_p,
                                                c_int_p]),
    "avr_graph_out_degrees": (ctypes.c_int, [ctypes.c_void_p, c_int_p]),
    "avr_graph_count_in_radius": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, c_int_p, ctypes.c_float, c_int_p]),
    "avr_graph_light": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(AvrGraphSampling), ctypes.c_int, c_float_p,
                                       c_float_p, ctypes.c_float, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                       c_float_p]),
    "avr_graph_propagate": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, c_int_p, c_int_p, c_float_p, c_float_p,
                                           ctypes.c_int, c_float_p, c_int_p]),
    "avr_graph_propagate_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong, ctypes.c_void_p,
                                                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                                  ctypes.c_void_p, c_int_p]),
    "avr_graph_create": (ctypes.c_int, [ctypes.c_float, ctypes.POINTER(ctypes.c_void_p)]),
    "avr_graph_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "avr_graph_add_walks": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int, c_float_p, c_int_p]),
    "avr_graph_size": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_longlong),
                                      ctypes.POINTER(ctypes.c_longlong)]),
    "avr_graph_vertices": (ctypes.c_int, [ctypes.c_void_p, c_float_p, c_int_p]),
    "avr_graph_edges": (ctypes.c_int, [ctypes.c_void_p, c_int_p, c_int_p, c_int_p]),
    "avr_graph_transport": (ctypes.c_int, [ctypes.c_void_p, c_int_p, c_int_p, c_float_p]),
    "avr_graph_in_node_path_length": (ctypes.c_int, [ctypes.c_void_p, c_float_p,
                                                     ctypes.POINTER(ctypes.c_longlong)]),
}

_lib = None


def load():
    """Load libavr_hip.so (no GPU is touched). Raises if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} not built: run __graft_entry__.build() (hipcc --offload-arch=gfx950)")
    lib = ctypes.CDLL(LIB_PATH)
    # a variant library named by AVR_LIB (A/B runs against older builds) may lack the newest
    # entry points (calling one then raises AttributeError); the in-tree library must export
    # every one, so a stale build fails here, at load, naming what is missing
    variant = os.path.abspath(LIB_PATH) != os.path.join(_HERE, "libavr_hip.so")
    missing = []
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name, None)
        if fn is None:
            missing.append(name)
            continue
        fn.restype = res
        fn.argtypes = args
    if missing and not variant:
        raise RuntimeError(f"{LIB_PATH} is stale: it lacks {', '.join(missing)} — rebuild it (__graft_entry__.build())")
    _lib = lib
    return lib


def _fp(a):
    return a.ctypes.data_as(c_float_p) if a is not None else None


def _check(rc):
    if rc != 0:
        raise RuntimeError(f"avr error {rc}: {_lib.avr_last_error().decode()}")


class Context:
    """One HIP device context of the integrator (avr_context_create)."""

    def __init__(self, device=0, max_paths=0):
        self.lib = load()
        h = ctypes.c_void_p()
        _check(self.lib.avr_context_create(int(device), int(max_paths), ctypes.byref(h)))
        self.h = h
        self.device = int(device)
        self._keep = []

    def close(self):
        if self.h:
            self.lib.avr_context_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_render_mode(self, mode):
        """0 / "replay": canonical math, per-sample parity with the CPU oracle; 1 / "fast":
        hardware transcendentals, statistical parity (avr_set_render_mode)."""
        m = {"replay": 0, "fast": 1}.get(mode, mode)
        _check(self.lib.avr_set_render_mode(self.h, int(m)))

    def set_majorant_res(self, res):
        r = np.asarray(res, np.int32).reshape(3)
        _check(self.lib.avr_set_majorant_res(self.h, r.ctypes.data_as(c_int_p)))

    def tune_majorant(self, candidates, spp_begin, spp_end, seed, max_depth):
        """avr_tune_majorant: returns (chosen (x, y, z), per-candidate probe ms)."""
        cand = np.ascontiguousarray(np.asarray(candidates, np.int32).reshape(-1, 3))
        chosen = np.zeros(3, np.int32)
        ms = np.zeros(len(cand), np.float32)
        _check(self.lib.avr_tune_majorant(self.h, cand.ctypes.data_as(c_int_p), len(cand), int(spp_begin),
                                          int(spp_end), int(seed), int(max_depth), chosen.ctypes.data_as(c_int_p),
                                          ms.ctypes.data_as(c_float_p)))
        return tuple(int(v) for v in chosen), ms

    def tune_walk(self, refill, dda, spp_begin, spp_end, seed, max_depth):
        """avr_tune_walk: returns ((refill, dda) chosen, probe ms as a len(refill) x len(dda) array)."""
        r = np.ascontiguousarray(np.asarray(refill, np.int32).ravel())
        d = np.ascontiguousarray(np.asarray(dda, np.int32).ravel())
        chosen = np.zeros(2, np.int32)
        ms = np.zeros(len(r) * len(d), np.float32)
        _check(self.lib.avr_tune_walk(self.h, r.ctypes.data_as(c_int_p), len(r), d.ctypes.data_as(c_int_p), len(d),
                                      int(spp_begin), int(spp_end), int(seed), int(max_depth),
                                      chosen.ctypes.data_as(c_int_p), ms.ctypes.data_as(c_float_p)))
        return (int(chosen[0]), int(chosen[1])), ms.reshape(len(r), len(d))

    def set_ray_binning(self, on):
        _check(self.lib.avr_set_ray_binning(self.h, 1 if on else 0))

    def set_majorant_occupancy(self, on):
        _check(self.lib.avr_set_majorant_occupancy(self.h, 1 if on else 0))

    def set_pass_table_ahead(self, on):
        _check(self.lib.avr_set_pass_table_ahead(self.h, 1 if on else 0))

    def record_lookups(self, d_points, cap, d_count):
        """Trace the wavefront kernels' density fetches into device buffers (0 / None stops)."""
        _check(self.lib.avr_record_lookups(self.h, ctypes.c_void_p(d_points or None), int(cap),
                                           ctypes.c_void_p(d_count or None)))

    def density_fetch(self, d_points, n, d_out):
        """avr_density_fetch on device buffers; returns the kernel time in ms."""
        ms = ctypes.c_float(0.0)
        _check(self.lib.avr_density_fetch(self.h, ctypes.c_void_p(d_points), int(n),
                                          ctypes.cast(ctypes.c_void_p(d_out), c_float_p), ctypes.byref(ms)))
        return float(ms.value)

    def set_kernel_mode(self, mode):
        """0 = persistent megakernel (default), 1 = wavefront queues."""
        _check(self.lib.avr_set_kernel_mode(self.h, int(mode)))

    def set_grid_layout(self, layout):
        """1 = fat footprint copy (default), 0 = pbrt's linear layout only; applies to the next set_scene."""
        _check(self.lib.avr_set_grid_layout(self.h, int(layout)))

    def grid_layout_active(self):
        return int(self.lib.avr_grid_layout_active(self.h))

    def set_dda_budget(self, cells):
        _check(self.lib.avr_set_dda_budget(self.h, int(cells)))

    def set_light_sampler(self, kind):
        """0: "bvh" / "uniform" (identical for infinite lights); 1: "power" (avr_light_sampler)."""
        _check(self.lib.avr_light_sampler(self.h, int(kind)))

    def set_refill_min(self, lanes):
        _check(self.lib.avr_set_refill_min(self.h, int(lanes)))

    def set_sampler_table(self, dims):
        """ZSobol pixel-table dimensions (0 = compute every digit per call)."""
        _check(self.lib.avr_set_sampler_table(self.h, int(dims)))

    def set_sampler_pass_table(self, dims):
        """ZSobol per-pass table dimensions (avr_set_sampler_pass_table; 0 = off, default 96)."""
        _check(self.lib.avr_set_sampler_pass_table(self.h, int(dims)))

    def set_pixel_order(self, order):
        """avr_set_pixel_order: the persistent kernel's pixel order (a permutation of the film's
        row-major pixel ids), or None for scanline order."""
        if order is None:
            _check(self.lib.avr_set_pixel_order(self.h, None, 0))
            return
        o = np.ascontiguousarray(np.asarray(order, np.int32).reshape(-1))
        _check(self.lib.avr_set_pixel_order(self.h, o.ctypes.data_as(c_int_p), len(o)))

    def set_stream(self, stream_ptr):
        _check(self.lib.avr_set_stream(self.h, ctypes.c_void_p(stream_ptr)))

    def _check_device(self, tensors):
        """Device grids must live on this context's GPU (the kernels dereference them there)."""
        for t in tensors:
            if t is not None and hasattr(t, "data_ptr") and t.device.index != self.device:
                raise ValueError(f"grid tensor on {t.device}, but the context runs on cuda:{self.device}")

    def set_scene(self, scene):
        med = scene.medium
        self._check_device([getattr(med, "device_density", None)] +
                           ([med.rgb_sigma_a, med.rgb_sigma_s, med.rgb_Le] if getattr(med, "type_id", 0) == 4 else []))
        mres = np.asarray(med.majorant_res, np.int32)
        f32 = lambda a: np.ascontiguousarray(np.asarray(a, np.float32))
        args = [f32(med.bounds), f32(scene.render_from_medium), f32(scene.medium_from_render), f32(med.sigma_a),
                f32(med.sigma_s)]
        Le = f32(med.Le) if med.Le is not None else None
        ls = f32(med.Lescale)
        self._keep = args + [Le, ls, mres]
        if getattr(med, "type_id", 0) == 1:
            _check(self.lib.avr_medium_homogeneous(self.h, _fp(args[0]), _fp(args[1]), _fp(args[2]), _fp(args[3]),
                                                   _fp(args[4]), float(med.g), _fp(Le)))
        elif getattr(med, "type_id", 0) == 4 and getattr(med, "on_device", False):
            ill = f32(med.illuminant)
            self._keep += [ill]
            ptr = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None
            _check(self.lib.avr_medium_rgbgrid_device(
                self.h, med.nx, med.ny, med.nz, _fp(args[0]), _fp(args[1]), _fp(args[2]), ptr(med.rgb_sigma_a),
                ptr(med.rgb_sigma_s), float(med.sigma_scale), float(med.g), ptr(med.rgb_Le), _fp(ill),
                float(med.Le_scale)))
        elif getattr(med, "type_id", 0) == 4:
            grids = [f32(g) if g is not None else None for g in (med.rgb_sigma_a, med.rgb_sigma_s, med.rgb_Le)]
            ill = f32(med.illuminant)
            self._keep += grids + [ill]
            _check(self.lib.avr_medium_rgbgrid(self.h, med.nx, med.ny, med.nz, _fp(args[0]), _fp(args[1]),
                                               _fp(args[2]), _fp(grids[0]), _fp(grids[1]), float(med.sigma_scale),
                                               float(med.g), _fp(grids[2]), _fp(ill), float(med.Le_scale)))
        elif getattr(med, "type_id", 0) == 3:
            dg = AvrVdbGrid.of(med.grid)
            tg = AvrVdbGrid.of(med.temperature_grid) if med.temperature_grid is not None else None
            _check(self.lib.avr_medium_nanovdb(self.h, ctypes.byref(dg), ctypes.byref(tg) if tg is not None else None,
                                               _fp(args[1]), _fp(args[2]), _fp(args[3]), _fp(args[4]), float(med.g),
                                               float(med.Lescale_value), float(med.temperature_offset),
                                               float(med.temperature_scale)))
        elif getattr(med, "type_id", 0) == 2:
            _check(self.lib.avr_medium_cloud(self.h, _fp(args[0]), _fp(args[1]), _fp(args[2]), _fp(args[3]),
                                             _fp(args[4]), float(med.g), *[float(v) for v in med.cloud]))
        elif med.device_density is not None:
            _check(self.lib.avr_medium_grid_device(
                self.h, ctypes.c_void_p(med.device_density.data_ptr()), med.nx, med.ny, med.nz, _fp(args[0]),
                _fp(args[1]), _fp(args[2]), _fp(args[3]), _fp(args[4]), float(med.g), _fp(Le), _fp(ls),
                ls.shape[2], ls.shape[1], ls.shape[0], mres.ctypes.data_as(c_int_p)))
        else:
            _check(self.lib.avr_medium_grid(
                self.h, _fp(med.density), med.nx, med.ny, med.nz, _fp(args[0]), _fp(args[1]), _fp(args[2]),
                _fp(args[3]), _fp(args[4]), float(med.g), _fp(Le), _fp(ls), ls.shape[2], ls.shape[1], ls.shape[0],
                mres.ctypes.data_as(c_int_p)))
        sph = getattr(scene, "interface_sphere_render", None)
        if sph is not None:
            c3 = f32(sph[:3])
            self._keep.append(c3)
            _check(self.lib.avr_medium_boundary_sphere(self.h, _fp(c3), float(sph[3])))
        planes = getattr(scene, "interface_planes_render", None)
        if planes is not None:
            pl = f32(planes.reshape(-1))
            self._keep.append(pl)
            _check(self.lib.avr_medium_boundary_convex(self.h, _fp(pl), len(planes)))
        temp = getattr(med, "temperature", None)
        if temp is not None:
            self._keep.append(temp)
            _check(self.lib.avr_medium_temperature(self.h, _fp(temp), float(med.temperature_scale),
                                                   float(med.temperature_offset)))
        types = np.ascontiguousarray(scene.light_types, np.int32)
        w = f32(scene.light_w.reshape(-1))
        L = f32(scene.light_L.reshape(-1))
        sc = f32(scene.light_scale)
        _check(self.lib.avr_lights(self.h, len(scene.lights), types.ctypes.data_as(c_int_p), _fp(w), _fp(L), _fp(sc),
                                   float(scene.scene_radius)))
        for i, light in enumerate(scene.lights):
            if light.type_id == 2:
                arrs = [f32(light.coeffs), f32(light.distribution), f32(light.illuminant), f32(scene.light_rfl[i]),
                        f32(scene.light_lfr[i])]
                self._keep += arrs
                _check(self.lib.avr_light_image(self.h, i, int(light.res), *[_fp(a) for a in arrs]))
        _check(self.lib.avr_camera(self.h, int(scene.camera.type_id), _fp(f32(scene.camera_from_raster)),
                                   _fp(f32(scene.render_from_camera))))
        film = scene.film
        _check(self.lib.avr_film(self.h, film.width, film.height, _fp(f32(film.filter_radius)), _fp(f32(film.sensor)),
                                 float(film.imaging_ratio), float(film.max_component_value)))
        if getattr(film, "nbuckets", 0):
            _check(self.lib.avr_film_spectral(self.h, int(film.nbuckets), float(film.lambdamin),
                                              float(film.lambdamax)))
        flt = film.filter
        _check(self.lib.avr_set_filter(self.h, int(flt.type_id), _fp(f32(flt.radius)), float(flt.sigma)))
        _check(self.lib.avr_set_sampler(self.h, int(scene.sampler.type_id), int(scene.sampler.pixelsamples)))

    def generate_cloud(self, d_out_ptr, n, first, count, density=1.0, wispiness=1.0, frequency=5.0):
        _check(self.lib.avr_generate_cloud(self.h, ctypes.c_void_p(d_out_ptr), int(n), int(first), int(count),
                                           float(density), float(wispiness), float(frequency)))

    def generate_rgb_explosion(self, d_sa_ptr, d_ss_ptr, d_le_ptr, n, first, count):
        """k_rgb_explosion into three float4 device arrays (pointers at element `first`)."""
        _check(self.lib.avr_generate_rgb_explosion(self.h, ctypes.c_void_p(d_sa_ptr), ctypes.c_void_p(d_ss_ptr),
                                                   ctypes.c_void_p(d_le_ptr), int(n), int(first), int(count)))

    def medium_bounds(self):
        out = np.zeros(6, np.float32)
        _check(self.lib.avr_medium_bounds(self.h, _fp(out)))
        return out

    def majorant(self, n):
        out = np.empty(n, np.float32)
        _check(self.lib.avr_read_majorant(self.h, _fp(out)))
        return out

    def film_clear(self):
        _check(self.lib.avr_film_clear(self.h))

    def render(self, spp_begin, spp_end, seed, max_depth):
        _check(self.lib.avr_render(self.h, int(spp_begin), int(spp_end), int(seed), int(max_depth)))

    def sync(self):
        _check(self.lib.avr_sync(self.h))

    def reset_stats(self):
        _check(self.lib.avr_reset_stats(self.h))

    def stats(self):
        """Counters and kernel times accumulated since creation or reset_stats()."""
        s = AvrStats()
        _check(self.lib.avr_get_stats(self.h, ctypes.byref(s)))
        return s.as_dict()

    def film_read_spectral(self, npix, nbuckets):
        """SpectralFilm bucket sums: (bucket_sums, weight_sums), each (npix, nbuckets) fp64."""
        bs = np.zeros(npix * nbuckets, np.float64)
        bw = np.zeros(npix * nbuckets, np.float64)
        _check(self.lib.avr_film_read_spectral(self.h, bs.ctypes.data_as(c_double_p), bw.ctypes.data_as(c_double_p)))
        return bs.reshape(npix, nbuckets), bw.reshape(npix, nbuckets)

    def film_read(self, npix):
        rgb = np.zeros(3 * npix, np.float64)
        w = np.zeros(npix, np.float64)
        _check(self.lib.avr_film_read(self.h, rgb.ctypes.data_as(c_double_p), w.ctypes.data_as(c_double_p)))
        return rgb, w

    def last_pass_samples(self, npix, max_samples):
        n = npix * max_samples
        L = np.zeros((n, 4), np.float32)
        lam = np.zeros((n, 4), np.float32)
        pdf = np.zeros((n, 4), np.float32)
        first, ns = ctypes.c_int(), ctypes.c_int()
        _check(self.lib.avr_last_pass_samples(self.h, _fp(L), _fp(lam), _fp(pdf), n, ctypes.byref(first),
                                              ctypes.byref(ns)))
        m = npix * ns.value
        return first.value, ns.value, L[:m], lam[:m], pdf[:m]

    def last_kernel(self):
        """Template arguments of the last k_paths instantiation rendered ("k_paths<...>")."""
        buf = ctypes.create_string_buffer(64)
        _check(self.lib.avr_last_kernel(self.h, buf, 64))
        return buf.value.decode()

    def last_pass_weights(self, npix, max_samples):
        w = np.zeros(npix * max_samples, np.float32)
        _check(self.lib.avr_last_pass_weights(self.h, _fp(w), len(w)))
        return w

    def transmittance(self, p0, p1, lam):
        """Integrator::Tr for n queries: p0, p1 (n, 3) render-space points, lam (n, 4) nm."""
        p0 = np.ascontiguousarray(p0, np.float32)
        p1 = np.ascontiguousarray(p1, np.float32)
        lam = np.ascontiguousarray(lam, np.float32)
        out = np.zeros((len(p0), 4), np.float32)
        _check(self.lib.avr_transmittance(self.h, len(p0), _fp(p0), _fp(p1), _fp(lam), _fp(out)))
        return out

    # ---- lighting graph (src/graph) ----
    def graph_walks(self, sampling, o, d, t_first, index0, iterations, sample_index, max_depth, skip_dims=0):
        """FreeGraphBuilder::TracePath walks: (points (n_rays*iterations, max_depth, 3), counts)."""
        o = np.ascontiguousarray(o, np.float32).reshape(-1, 3)
        d = np.ascontiguousarray(d, np.float32).reshape(-1, 3)
        t_first = np.ascontiguousarray(t_first, np.float32)
        index0 = np.ascontiguousarray(index0, np.int64)
        n = len(o) * int(iterations)
        pts = np.zeros((n, max(1, int(max_depth)), 3), np.float32)
        counts = np.zeros(n, np.int32)
        _check(self.lib.avr_graph_walks_from(self.h, ctypes.byref(sampling), len(o), _fp(o), _fp(d), _fp(t_first),
                                             index0.ctypes.data_as(ctypes.POINTER(ctypes.c_longlong)),
                                             int(iterations), int(sample_index), int(skip_dims), int(max_depth),
                                             _fp(pts), counts.ctypes.data_as(c_int_p)))
        return pts, counts

    def graph_reinforce_rays(self, sampling, ids, points, radius, n_rays, cycle):
        """ReinforceSparseVertices' rays: (o, d (n, n_rays, 3), t_first, valid (n, n_rays))."""
        ids = np.ascontiguousarray(ids, np.int32)
        pts = np.ascontiguousarray(points, np.float32).reshape(-1, 3)
        n, k = len(ids), int(n_rays)
        o = np.zeros((n, k, 3), np.float32)
        d = np.zeros((n, k, 3), np.float32)
        t = np.zeros((n, k), np.float32)
        valid = np.zeros((n, k), np.int32)
        _check(self.lib.avr_graph_reinforce_rays(self.h, ctypes.byref(sampling), n, ids.ctypes.data_as(c_int_p),
                                                 _fp(pts), float(radius), k, int(cycle), _fp(o), _fp(d), _fp(t),
                                                 valid.ctypes.data_as(c_int_p)))
        return o, d, t, valid

    def graph_light(self, sampling, vertices, in_dir, radius, points_on_radius, iterations, max_dist_to_center):
        """LightingCalculator::GetLightVector: per-vertex light (Inv4Pi applied)."""
        v = np.ascontiguousarray(vertices, np.float32).reshape(-1, 3)
        dr = np.ascontiguousarray(in_dir, np.float32)
        out = np.zeros(len(v), np.float32)
        _check(self.lib.avr_graph_light(self.h, ctypes.byref(sampling), len(v), _fp(v), _fp(dr), float(radius),
                                        int(points_on_radius), int(iterations), float(max_dist_to_center),
                                        _fp(out)))
        return out

    def graph_propagate(self, row_ptr, col, val, light, bounces):
        """LightingCalculator::ComputeFinalLight: (total light, bounces completed)."""
        row_ptr = np.ascontiguousarray(row_ptr, np.int32)
        col = np.ascontiguousarray(col, np.int32)
        val = np.ascontiguousarray(val, np.float32)
        light = np.ascontiguousarray(light, np.float32)
        total = np.zeros(len(light), np.float32)
        it = ctypes.c_int(0)
        _check(self.lib.avr_graph_propagate(self.h, len(light), row_ptr.ctypes.data_as(c_int_p),
                                            col.ctypes.data_as(c_int_p), _fp(val), _fp(light), int(bounces),
                                            _fp(total), ctypes.byref(it)))
        return total, it.value

    def film_export_device(self, d_dst_ptr):
        _check(self.lib.avr_film_export_device(self.h, ctypes.c_void_p(d_dst_ptr)))

    METRICS = {"MSE": 0, "MAE": 1, "MRSE": 2, "ME": 3}

    def flip(self, test_rgb, reference_rgb, ppd=0.0):
        """FLIP error map (H, W) of two (H, W, 3) sRGB-encoded images (ComputeFLIPError)."""
        t = np.ascontiguousarray(test_rgb, np.float32)
        r = np.ascontiguousarray(reference_rgb, np.float32)
        if t.shape != r.shape or t.ndim != 3 or t.shape[2] != 3:
            raise ValueError("FLIP needs two (H, W, 3) images of the same resolution")
        out = np.zeros(t.shape[:2], np.float32)
        _check(self.lib.avr_flip(self.h, _fp(t), _fp(r), t.shape[1], t.shape[0], float(ppd), _fp(out)))
        return out

    def film_image_device(self, d_out_ptr, output_from_sensor, fp16=True):
        m = np.ascontiguousarray(output_from_sensor, np.float32).reshape(9)
        _check(self.lib.avr_film_image_device(self.h, _fp(m), 1 if fp16 else 0, ctypes.c_void_p(d_out_ptr)))

    def film_set_reference(self, reference_rgb, output_from_sensor, fp16=True):
        ref = np.ascontiguousarray(reference_rgb, np.float32)
        m = np.ascontiguousarray(output_from_sensor, np.float32).reshape(9)
        _check(self.lib.avr_film_set_reference(self.h, _fp(ref), _fp(m), 1 if fp16 else 0))

    def film_metric(self, metric="MSE"):
        """Per-channel metric of the film's image against the reference (ME: (3, 3) rows
        absolute / positive / negative)."""
        out = np.zeros(9, np.float32)
        _check(self.lib.avr_film_metric(self.h, self.METRICS[metric], _fp(out)))
        return out.reshape(3, 3) if metric == "ME" else out[:3].copy()

    def film_device_ptrs(self):
        a, b = ctypes.c_void_p(), ctypes.c_void_p()
        _check(self.lib.avr_film_device_ptrs(self.h, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value


class Graph:
    """Host FreeGraph assembly (avr_graph_*): walks merged in order, transport CSR."""

    def __init__(self, vertex_radius):
        self.lib = load()
        h = ctypes.c_void_p()
        _check(self.lib.avr_graph_create(float(vertex_radius), ctypes.byref(h)))
        self.h = h
        self.radius = float(vertex_radius)

    def close(self):
        if self.h:
            self.lib.avr_graph_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def add_walks(self, points, counts, max_depth):
        points = np.ascontiguousarray(points, np.float32)
        counts = np.ascontiguousarray(counts, np.int32)
        _check(self.lib.avr_graph_add_walks(self.h, len(counts), int(max_depth), _fp(points),
                                            counts.ctypes.data_as(c_int_p)))

    def add_walks_from(self, points, counts, max_depth, start_vertex):
        points = np.ascontiguousarray(points, np.float32)
        counts = np.ascontiguousarray(counts, np.int32)
        sv = np.ascontiguousarray(start_vertex, np.int32)
        _check(self.lib.avr_graph_add_walks_from(self.h, len(counts), int(max_depth), _fp(points),
                                                 counts.ctypes.data_as(c_int_p), sv.ctypes.data_as(c_int_p)))

    def out_degrees(self):
        nv, _ = self.size()
        out = np.zeros(nv, np.int32)
        _check(self.lib.avr_graph_out_degrees(self.h, out.ctypes.data_as(c_int_p)))
        return out

    def count_in_radius(self, ids, radius):
        ids = np.ascontiguousarray(ids, np.int32)
        out = np.zeros(len(ids), np.int32)
        _check(self.lib.avr_graph_count_in_radius(self.h, len(ids), ids.ctypes.data_as(c_int_p), float(radius),
                                                  out.ctypes.data_as(c_int_p)))
        return out

    def size(self):
        nv, ne = ctypes.c_longlong(), ctypes.c_longlong()
        _check(self.lib.avr_graph_size(self.h, ctypes.byref(nv), ctypes.byref(ne)))
        return nv.value, ne.value

    def vertices(self):
        nv, _ = self.size()
        xyz = np.zeros((nv, 3), np.float32)
        smp = np.zeros(nv, np.int32)
        _check(self.lib.avr_graph_vertices(self.h, _fp(xyz), smp.ctypes.data_as(c_int_p)))
        return xyz, smp

    def edges(self):
        _, ne = self.size()
        f, t, s = (np.zeros(ne, np.int32) for _ in range(3))
        _check(self.lib.avr_graph_edges(self.h, f.ctypes.data_as(c_int_p), t.ctypes.data_as(c_int_p),
                                        s.ctypes.data_as(c_int_p)))
        return f, t, s

    def transport(self):
        nv, ne = self.size()
        rp = np.zeros(nv + 1, np.int32)
        col = np.zeros(ne, np.int32)
        val = np.zeros(ne, np.float32)
        _check(self.lib.avr_graph_transport(self.h, rp.ctypes.data_as(c_int_p), col.ctypes.data_as(c_int_p),
                                            _fp(val)))
        return rp, col, val

    def in_node_path_length(self):
        a, n = ctypes.c_float(), ctypes.c_longlong()
        _check(self.lib.avr_graph_in_node_path_length(self.h, ctypes.byref(a), ctypes.byref(n)))
        return a.value, n.value


def film_reduce_rccl(contexts, root=0):
    """avr_film_reduce_rccl: SUM the films of `contexts` (one per GPU) into contexts[root]."""
    lib = load()
    arr = (ctypes.c_void_p * len(contexts))(*[c.h.value if hasattr(c.h, "value") else c.h for c in contexts])
    _check(lib.avr_film_reduce_rccl(arr, len(contexts), int(root)))

"""Benchmark: Msamples/s of the MI355X volumetric path integrator on the BASELINE.json
metric workload ("disney-cloud 720p" -> synthetic S-cloud-1024):
GridMedium 1024^3 f32 (4 GiB) filled on device with CloudMedium::Density, perspective
1280x720, VolPath maxdepth 100, ZSobol sampler + Gaussian filter (pbrt's defaults).

A step = one render pass of --spp-per-step sample indices over every pixel (the hot path:
camera rays -> delta tracking -> ratio-tracked shadow rays -> film). Each rank renders
its own disjoint sample indices (weak scaling); the fp64 film is SUM-reduced over RCCL
once at the end of the timed region (T_render ends at the film reduce).

`--gpus N` without a launcher starts N rank processes itself (torch.distributed.run as a
child, acceleratedvolrenderer_amd/launch.py); under a launcher WORLD_SIZE must equal N.

Prints ONE JSON line (rank 0) with
  * roofline: k_paths (the fused delta-tracking / ratio-tracking / density-fetch kernel),
    algorithmic HBM bytes per launch / its HIP-event time on the context stream, against the
    HBM peak; `traffic` (memory-side reads priced by request size + WRITE_SIZE) and the
    `limiter` block come from rocprofv3 PMC passes that this script runs as child processes
    on the same configuration (N=1, --pmc auto); the fast-mode and NanoVDB legs carry the
    same roofline block (NanoVDB's 64^3 majorant reads, served by L2, reported apart);
  * cpu_baseline: the oracle restatement (`port`) on a bounded sample of the same
    workload, on every host core this process may use (affinity and cgroup quota).
"""
import argparse
import csv
import glob
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
HBM_ACHIEVABLE_GBPS = 6300.0   # MI355X_MICROARCH.md: ~6.3 TB/s achievable streaming
HBM_REQUEST_BYTES = 128  # gfx950 memory-side read request of a 32-B random gather (TCC_EA0_RDREQ_128B:
                         # profiles/r06_fetch_size_calibration.json)
VALU_SIMDS = 1024       # 256 CUs x 4 SIMDs; a wave64 VALU op issues in 2 cycles (MI355X_MICROARCH.md)
# SURVEY.md §8d algorithmic bytes: 32 B per trilinear lookup (8 taps x 4 B) and 132 B per
# work item read / written (ray 24, tMax 4, lambda+pdf 32, beta/r_u/r_l 48, RNG 16, pixel/depth 8).
BYTES_PER_LOOKUP = 32
BYTES_PER_ITEM = 132
# k_paths' own per-unit bytes (DESIGN.md §4 "Algorithmic bytes"): it writes ONE 16-B record per
# sample (L; k_film takes the rest from the camera stage) and reads the camera stage's record of
# every path it starts: cam0..cam3 (4 x 16 B; ZSobol's first light-pick draw rides in cam1.w) +
# the 16-B PCG32 state (independent sampler)
BYTES_PER_SAMPLE_RECORD = 16
BYTES_CAMERA_RECORD_READ = {"zsobol": 64, "independent": 80}
# ZSobol pixel-table reads (one 4-B entry per draw): 5 draws per phase event in k_paths (phase
# 2D, the next segment's three 1D, the next light pick); 6 per camera-stage quad of 4 samples
ZSOBOL_TABLE_BYTES_PER_DRAW = 4
ZSOBOL_PASS_BYTES_PER_DRAW = 8   # the per-pass table's entries (avr_set_sampler_pass_table)
ZSOBOL_DRAWS_PER_PHASE = 5
ZSOBOL_CAMERA_DRAWS = 6
# the camera stage writes cam0, cam1, cam2, cam3 (4 x 16 B), the 4-B filter weight and, for the
# independent sampler, cam5 (16 B PCG32 state); the wavelength pdfs (cam4 until round 5) are
# evaluated by k_film from the wavelengths (AVR_FILM_PDF)
BYTES_CAMERA_WRITE = {"zsobol": 68, "independent": 84}
RGB_CPU_MAX_RES = 512   # the rgb-explosion CPU baseline copies its 3 grids to the host (6 GiB at 512^3)


def lookup_bytes(medium, emissive=False, rgb_fields=2):
    """SURVEY §8(d) algorithmic bytes of ONE density lookup of k_paths by medium kind: a trilinear
    lookup is 8 f32 taps = 32 B (GridMedium; NanoVDB likewise, plus the same again for the
    temperature grid of an emissive medium); RGBGridMedium 8 taps x 16 B {c0, c1, c2, scale} per
    field (sigma_a, sigma_s, and Le when emissive)."""
    if medium == "rgb":
        return 8 * 16 * (rgb_fields + (1 if emissive else 0))
    if medium == "nanovdb":
        return BYTES_PER_LOOKUP * (2 if emissive else 1)
    return BYTES_PER_LOOKUP


# NanoVDB's apron layout reads one 4-B slot index per grid lookup before the 32-B stencil entry:
# a cost of this implementation's sparse layout, not a §8(d) algorithmic byte
VDB_SLOT_BYTES = 4
# §8(d): "4 B per majorant DDA step (counted as 0 HBM if LDS-staged; report it separately)": the
# 16^3 majorants are in LDS; NanoVDB's 64^3 one (1 MiB) is read through L2 — reported apart
# (`l2_majorant`), never in an HBM fraction
BYTES_PER_MAJORANT_STEP = 4
# where `traffic` comes from: the memory-side reads by request size (TCC_EA0_RDREQ_32B/64B/128B)
# + WRITE_SIZE; FETCH_SIZE tallies 128-B requests at 64 B on gfx950 (MI355X_MICROARCH.md §HBM)
# and its x2 rule holds only for all-128-B streaming — calibrated on k_density_fetch over known
# byte counts in profiles/r06_fetch_size_calibration.json (tools/fetch_calibrate.py)
FETCH_CALIBRATION = "profiles/r06_fetch_size_calibration.json"


def kpaths_bytes(agg, sampler, medium="grid", emissive=False, zsobol_table=True, pass_table=False,
                 majorant_in_lds=True):
    """k_paths' HBM bytes over the stats `agg` (counters summed over its launches), split as SURVEY
    §8(d) prices them. Algorithmic: 32 B per trilinear lookup (delta + ratio tracking) and the
    per-work-item state k_paths moves through HBM — its 16-B sample record and the camera record
    it reads per path (BYTES_CAMERA_RECORD_READ: 64 B ZSobol / 80 B independent). Implementation
    (reported apart, not in `frac`): the ZSobol table entries of the phase draws (they replace
    register arithmetic pbrt does in samplers.h:225-330), NanoVDB's 4-B apron slot per lookup and
    — where the majorant is NOT staged in LDS (NanoVDB's 64^3 grid, 1 MiB, served by the XCD's L2)
    — §8(d)'s 4 B per majorant DDA step (`l2_majorant_steps`: L2, not HBM, bytes).
    Returns (algorithmic total, parts, implementation parts)."""
    # delta tracking evaluates emission (Le grid / temperature) at its lookups; shadow rays never
    lk = agg["medium_lookups"] * lookup_bytes(medium, emissive) + agg["shadow_lookups"] * lookup_bytes(medium, False)
    parts = {
        "density_lookups": lk,
        "sample_records_written": BYTES_PER_SAMPLE_RECORD * agg["medium_items_in"],
        "camera_records_read": BYTES_CAMERA_RECORD_READ[sampler] * agg["medium_items_in"],
    }
    impl = {
        "zsobol_table_reads": ((ZSOBOL_PASS_BYTES_PER_DRAW if pass_table else ZSOBOL_TABLE_BYTES_PER_DRAW) *
                               ZSOBOL_DRAWS_PER_PHASE * agg["medium_items_out"]
                               if sampler == "zsobol" and (zsobol_table or pass_table) else 0),
        "vdb_slot_reads": (VDB_SLOT_BYTES * (agg["medium_lookups"] * (2 if emissive else 1) + agg["shadow_lookups"])
                           if medium == "nanovdb" else 0),
        "l2_majorant_steps": 0 if majorant_in_lds else BYTES_PER_MAJORANT_STEP * agg["medium_dda_steps"],
    }
    return sum(parts.values()), parts, impl


def roofline_block(agg, launches, sampler, medium, emissive, zsobol_table, pass_table):
    """The §8(d) numbers of one k_paths configuration from its stats: per-launch algorithmic HBM
    bytes over the average HIP-event launch time, and the density-fetch share the north star
    prices (`density_fetch`: lookup bytes only); NanoVDB's L2-served majorant reads apart
    (`l2_majorant`)."""
    alg, parts, impl = kpaths_bytes(agg, sampler, medium, emissive, zsobol_table, pass_table,
                                    majorant_in_lds=medium != "nanovdb")
    ms = agg["ms_medium"] / launches
    s = ms / 1e3
    lk = parts["density_lookups"] / launches
    l2m = impl["l2_majorant_steps"] / launches
    return {
        "achieved": round(alg / launches / s / 1e9, 2) if s > 0 else 0.0,
        "peak": HBM_PEAK_GBPS, "unit": "GB/s",
        "frac": round(alg / launches / s / 1e9 / HBM_PEAK_GBPS, 5) if s > 0 else 0.0,
        "bytes_per_launch": alg / launches,
        "bytes_parts_per_launch": {k: v / launches for k, v in parts.items()},
        "implementation_bytes_per_launch": {k: v / launches for k, v in impl.items()},
        "avg_launch_ms": ms,
        "density_fetch": {"bytes_per_launch": lk, "GBps": round(lk / s / 1e9, 2) if s > 0 else 0.0,
                          "frac": round(lk / s / 1e9 / HBM_PEAK_GBPS, 5) if s > 0 else 0.0,
                          "basis": "32 B per trilinear lookup (SURVEY §8d) x lookups per launch / avg launch time"},
        "l2_majorant": ({"bytes_per_launch": l2m, "GBps": round(l2m / s / 1e9, 2) if s > 0 else 0.0,
                         "basis": "4 B per majorant DDA step (SURVEY §8d, reported separately): the 64^3 majorant "
                                  "(1 MiB) is served by the XCD's L2, not HBM; not in `frac`"} if l2m else None),
        "lookups_per_launch": (agg["medium_lookups"] + agg["shadow_lookups"]) / launches,
        "samples_per_launch": agg["medium_items_in"] / launches,
    }


def camera_bytes(samples, sampler, zsobol_table=True, pass_dims=0, pixels=0, launches=1):
    """The camera stage's algorithmic bytes for `samples` samples: its records
    (BYTES_CAMERA_WRITE: 68 / 84 B per sample) + the ZSobol table entries (6 draws per quad of 4 samples of one pixel) + with the
    pass table, its per-pass build (an 8-B entry written and a 4-B pixel-table entry read per
    pixel and dimension, once per launch)."""
    b = BYTES_CAMERA_WRITE[sampler] * samples
    if sampler == "zsobol" and (zsobol_table or pass_dims):
        b += (ZSOBOL_PASS_BYTES_PER_DRAW if pass_dims else ZSOBOL_TABLE_BYTES_PER_DRAW) * ZSOBOL_CAMERA_DRAWS * samples // 4
    if sampler == "zsobol" and pass_dims:
        b += launches * pixels * pass_dims * (ZSOBOL_PASS_BYTES_PER_DRAW + (ZSOBOL_TABLE_BYTES_PER_DRAW if zsobol_table else 0))
    return b


def kernel_targs(name):
    """The template arguments of a k_paths kernel name as a tuple of strings: from the demangled
    form ('void avr::k_paths<false, true, 3, 0, false, false>(avr::Params)', avr_last_kernel's
    'k_paths<...>') or the Itanium-mangled one ('_ZN3avr7k_pathsILb0ELb1ELi3ELi0ELb0ELb0EEEv...')."""
    m = re.search(r"k_paths<([^>]*)>", name)
    if m:
        return tuple(a.strip() for a in m.group(1).split(","))
    m = re.search(r"7k_pathsI((?:L[bi]\d+E)+)E", name)
    if m:
        out = []
        for kind, val in re.findall(r"L([bi])(\d+)E", m.group(1)):
            out.append(("true" if val == "1" else "false") if kind == "b" else val)
        return tuple(out)
    return None


# rocprofv3 passes (one run each; at most 8 SQ, 4 TCC (FETCH_SIZE 3, WRITE_SIZE 2), 2 GRBM)
RDREQ_SIZES = ("TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum")
PMC_PASSES = (("size", RDREQ_SIZES), ("fetch", ("FETCH_SIZE",)), ("write", ("WRITE_SIZE",)),
              ("tcc", ("TCC_HIT_sum", "TCC_MISS_sum")),
              ("sq", ("SQ_INSTS_VALU", "SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY",
                      "SQ_WAVES", "GRBM_GUI_ACTIVE")))


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=4)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--res", type=int, default=1024, help="density grid resolution (n^3)")
    p.add_argument("--width", type=int, default=1280)
    p.add_argument("--height", type=int, default=720)
    p.add_argument("--spp-per-step", type=int, default=64,
                   help="sample indices per pass (one step); 64 x 720p = 59M samples: k_paths' 16-B records and the "
                        "camera stage's 68 B per sample (ZSobol), 4.9 GB")
    p.add_argument("--max-paths", type=int, default=0)
    p.add_argument("--pixelsamples", type=int, default=0,
                   help="sampler pixelsamples (0: the smallest power of two >= 256 holding every timed sample index "
                        "of every rank of an 8-GPU world, the same at every N: launch.sample_plan)")
    p.add_argument("--cpu-seconds", type=float, default=15.0, help="budget of the CPU-baseline sample")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--pmc", default="auto", choices=["auto", "on", "off"],
                   help="rocprofv3 counter passes for traffic / VALU (auto: at N=1 when rocprofv3 exists)")
    p.add_argument("--kernel", default="persistent", choices=["persistent", "wavefront"])
    p.add_argument("--medium", default="grid", choices=["grid", "nanovdb"],
                   help="S-cloud as GridMedium (default) or as a NanoVDBMedium tree (disney-cloud's type)")
    p.add_argument("--refill-min", type=int, default=0, help="k_paths refill threshold (0 = library default)")
    p.add_argument("--grid-layout", default="fat", choices=["fat", "linear", "brick"])
    p.add_argument("--dda-budget", type=int, default=0, help="k_paths DDA cells per iteration (0 = default)")
    p.add_argument("--tune-walk", default="on", choices=["on", "off"],
                   help="choose k_paths' refill / DDA budget for this scene by on-device probe renders (avr_tune_walk, "
                        "outside the timed region); off: --refill-min / --dda-budget or the library defaults")
    p.add_argument("--zsobol-table", type=int, default=256,
                   help="ZSobol pixel-table dimensions (0 = every digit per sampler call)")
    p.add_argument("--zsobol-pass-table", type=int, default=96,
                   help="ZSobol per-pass table dimensions (0 = off): the digits a pass's sample indices share")
    p.add_argument("--pass-table-ahead", type=int, default=1,
                   help="build the next pass's ZSobol table on a low-priority side stream during k_paths' drain "
                        "(avr_set_pass_table_ahead; 0 = in front of each camera stage)")
    p.add_argument("--sampler", default="zsobol", choices=["zsobol", "independent"],
                   help="pixel sampler (BASELINE.md S-cloud: zsobol, pbrt's default)")
    p.add_argument("--filter", default="gaussian", choices=["gaussian", "box"],
                   help="pixel filter (pbrt's default: gaussian radius 1.5, sigma 0.5)")
    p.add_argument("--mode", default="replay", choices=["replay", "fast"],
                   help="render mode: replay (canonical math, per-sample CPU parity; the headline) or fast "
                        "(hardware transcendentals, statistical parity)")
    p.add_argument("--majorant-res", type=int, default=None,
                   help="GridMedium majorant resolution per axis: 0 = pbrt's 16^3 (replay default), -1 = tuned "
                        "on the device among 1,2,4,8,16 (fast-mode default, outside the timed region)")
    p.add_argument("--occupancy", type=int, default=0,
                   help="NanoVDB: coarse majorant occupancy level in LDS (avr_set_majorant_occupancy; -2 %%, off)")
    p.add_argument("--pixel-order", default="scanline", choices=["scanline", "entry-cell"],
                   help="k_paths pixel order: scanline, or sorted by the majorant cell where the pixel's camera ray "
                        "enters the medium (N1: coherent ray packets, avr_set_pixel_order)")
    p.add_argument("--ray-binning", type=int, default=0,
                   help="wavefront kernels: counting-sort the queues by (majorant cell, octant) before each launch")
    p.add_argument("--nvdb", default=None,
                   help="NanoVDBMedium from this .nvdb file's density grid (needs --medium nanovdb); 'roundtrip' "
                        "writes the synthetic cloud's tree to a temporary .nvdb and reads it back")
    p.add_argument("--fast-leg", type=int, default=1,
                   help="after the replay measurement, time the same steps in fast mode (reported as fast_mode)")
    p.add_argument("--fast-majorant-res", type=int, default=0,
                   help="the fast leg's majorant resolution (0: tuned on the device among 1..16, outside the timed "
                        "region); a fixed value skips the probe renders (e.g. for a kernel-stats run)")
    p.add_argument("--scene", default="cloud", choices=["cloud", "uniform", "explosion", "rgb-explosion"],
                   help="cloud: the metric workload (S-cloud); uniform: BASELINE C2's uniform cube (orthographic, "
                        "use --res 256 --width 512 --height 512); explosion: C5's emissive NanoVDB stand-in with a "
                        "SpectralFilm (pixelsamples >= 4096); rgb-explosion: C5 as an emissive RGB-coefficient RGBGridMedium "
                        "(k_rgb_explosion, 3 x 16 GiB at 1024^3) with a SpectralFilm")
    p.add_argument("--nanovdb-leg", type=int, default=1,
                   help="after the headline (S-cloud GridMedium), time the same sample indices over the same cloud as a "
                        "NanoVDBMedium (disney-cloud's medium type; tree built on the device), reported as `nanovdb`")
    p.add_argument("--nanovdb-steps", type=int, default=8, help="timed steps of the NanoVDB leg (at most --steps)")
    p.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    return p.parse_args(argv)


def log(msg):
    """Progress on stderr (the JSON line stays the only stdout output)."""
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


class heartbeat:
    """`with heartbeat("what"):` logs every `every` s while a long host step runs (NanoVDB
    tree builds, the oracle's scene), so a supervisor watching the output sees progress."""

    def __init__(self, what, every=30.0):
        import threading
        self.what, self.every, self.stop = what, every, threading.Event()
        self.thread = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        t0 = time.perf_counter()
        while not self.stop.wait(self.every):
            log(f"{self.what}: {time.perf_counter() - t0:.0f} s")

    def __enter__(self):
        self.thread.start()
        return self

    def __exit__(self, *exc):
        self.stop.set()
        self.thread.join()
        return False


def host_cpu_info():
    """Host cores this process may use: the affinity mask, capped by a cgroup CPU quota."""
    info = {"nproc": os.cpu_count() or 1}
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = info["nproc"]
    info["affinity"] = aff
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = open(path).read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) // int(per)))
        except (OSError, ValueError):
            pass
    if quota is None:
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = max(1, q // per)
        except (OSError, ValueError):
            pass
    info["cgroup_quota_cpus"] = quota
    info["used"] = min(aff, quota) if quota else aff
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.lower().startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    info["model"] = model
    return info


def cpu_baseline(scene_host, spp_per_step, budget_s, label="S-cloud"):
    """Time the CPU oracle (pbrt VolPath restatement, `port`) on a bounded sample of the
    SAME workload: a strided pixel subset across the whole frame, spp_per_step samples
    each, threaded over every host core this process may use (the reference's ParallelFor
    over AvailableCores(), util/parallel.cpp:307-332)."""
    from oracle import binding
    info = host_cpu_info()
    cores = info["used"]
    log(f"cpu baseline: building the oracle scene ({label})")
    run = binding.OracleRun(scene_host, max_depth=100, seed=0)
    log(f"cpu baseline: timing {budget_s:.0f} s on {cores} threads ({info['model']})")
    f = scene_host.film
    npix = f.width * f.height
    # a strided pixel subset that spans every row/column band of the frame; samples are
    # taken in sampleIndex order, sweep after sweep, until the time budget is used
    stride = 61
    order = np.arange(0, npix, stride, dtype=np.int32)
    chunk = max(512, 32 * cores)   # enough pixels per call to keep every thread busy
    done_s = 0
    swept_spp = 0
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) < budget_s:
        for i in range(0, len(order), chunk):
            px = order[i:i + chunk]
            run.render_list(px, swept_spp, swept_spp + spp_per_step, nthreads=cores)
            done_s += len(px) * spp_per_step
            if (time.perf_counter() - t0) >= budget_s:
                break
        swept_spp += spp_per_step
    t_used = time.perf_counter() - t0
    return {"value": done_s / t_used / 1e6, "unit": "Msamples/s", "cores": cores, "kind": "port",
            "host": info,
            "sample": f"{done_s} samples: pixels every {stride}th of {f.width}x{f.height} ({len(order)} px), "
                      f"sample indices from 0 in sweeps of {spp_per_step}, same {label} "
                      f"scene, {t_used:.1f} s on {cores} threads"}


def pmc_child_argv(args, pixelsamples):
    """The command of one counter-pass child: this configuration, 2 timed steps after 1 warmup,
    at the parent's resolved pixelsamples (not re-planned: the plan depends on --steps)."""
    child = [sys.executable, os.path.join(ROOT, "bench.py"), "--pmc-child", "--no-cpu-baseline", "--pmc", "off",
             "--steps", "2", "--warmup", "1", "--tune-walk", "off"]
    child += ["--pixelsamples", str(int(pixelsamples))]
    for k in ("res", "width", "height", "spp_per_step", "max_paths", "pixel_order", "kernel", "medium",
              "refill_min", "grid_layout",
              "dda_budget", "zsobol_table", "zsobol_pass_table", "pass_table_ahead", "sampler", "filter", "mode", "majorant_res", "ray_binning", "occupancy", "nvdb",
              "scene"):
        if getattr(args, k) is not None:
            child += [f"--{k.replace('_', '-')}", str(getattr(args, k))]
    return child


CAMERA_RE = r"\bk_paths_camera<|k_paths_cameraI"


def traffic_bytes(ctr):
    """HBM bytes of one launch from its counters: the memory-side reads by request size (32 R32 +
    64 R64 + 128 R128) + WRITE_SIZE; None without the size pass. FETCH_SIZE would tally the 128-B
    requests at 64 B (FETCH_CALIBRATION)."""
    if not all(k in ctr for k in RDREQ_SIZES[1:]) or "WRITE_SIZE" not in ctr:
        return None
    rd = 32 * ctr["TCC_EA0_RDREQ_32B_sum"] + 64 * ctr["TCC_EA0_RDREQ_64B_sum"] + 128 * ctr["TCC_EA0_RDREQ_128B_sum"]
    return rd + ctr["WRITE_SIZE"] * 1024


def pmc_passes(args, pixelsamples, kernel_re=r"\bk_paths<|\dk_pathsI", timeout_s=240, side=None, passes=PMC_PASSES):
    """rocprofv3 counter passes of this same bench configuration, one child process per
    pass (--pmc only: no tracing in the same run), each killed after timeout_s. The child
    renders with the parent's RESOLVED pixelsamples (so the same k_paths instantiation and
    ZSobol digit count) and the parent's first timed sample indices (world 1: steps 0 and 1
    render [0, S) and [S, 2S)). Returns (per-launch averages of the dominant kernel's counters,
    error, the set of kernel names matched), or None. kernel_re matches the kernel name,
    demangled or mangled (k_paths itself, not the camera stage k_paths_camera). `side`: an
    optional dict filled with the same per-launch averages of the camera stage (CAMERA_RE)."""
    exe = shutil.which("rocprofv3")
    if exe is None:
        return None, "rocprofv3 not found", set()
    child = pmc_child_argv(args, pixelsamples)
    out = {}
    names = set()
    tmp = tempfile.mkdtemp(prefix="avr_pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        for name, counters in passes:
            d = os.path.join(tmp, name)
            cmd = [exe, "--pmc", *counters, "-d", d, "-o", "run", "--output-format", "csv", "--"] + child
            log(f"pmc pass {name}: {' '.join(counters)}")
            # the child rebuilds the scene (minutes for a host-built NanoVDB tree): log a heartbeat
            # every 30 s so a supervisor that watches the output does not take the pass for a hang
            errf = tempfile.TemporaryFile(dir=tmp)
            proc = subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=errf)
            t0 = time.perf_counter()
            while True:
                try:
                    rc = proc.wait(timeout=30)
                    break
                except subprocess.TimeoutExpired:
                    el = time.perf_counter() - t0
                    if el > timeout_s:
                        proc.kill()
                        proc.wait()
                        return None, f"pmc pass {name} timed out", names
                    log(f"pmc pass {name}: running {el:.0f} s")
            if rc != 0:
                errf.seek(0)
                return None, f"pmc pass {name} exited {rc}: {errf.read().decode(errors='replace')[-300:]}", names
            files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
            if not files:
                return None, f"pmc pass {name}: no counter file", names
            per, per_cam = {}, {}
            for fn in files:
                for row in csv.DictReader(open(fn)):
                    tgt = None
                    if re.search(kernel_re, row["Kernel_Name"]):
                        names.add(row["Kernel_Name"])
                        tgt = per
                    elif side is not None and re.search(CAMERA_RE, row["Kernel_Name"]):
                        tgt = per_cam
                    if tgt is not None:
                        tgt.setdefault(row["Counter_Name"], {}).setdefault(row.get("Dispatch_Id", ""), 0.0)
                        tgt[row["Counter_Name"]][row.get("Dispatch_Id", "")] += float(row["Counter_Value"])
            for dst, src in ((out, per), (side, per_cam)):
                for cn, disp in src.items():
                    # the child's first launch is its warmup; average the timed launches
                    vals = [disp[k] for k in sorted(disp, key=lambda x: int(x) if x.isdigit() else 0)]
                    vals = vals[1:] if len(vals) > 1 else vals
                    dst[cn] = sum(vals) / len(vals)
        return out, None, names
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def broadcast_choice(vals, world, device):
    """Rank 0's choice on every rank (the tuned walk schedule and majorant resolutions), so that
    every rank renders the same k_paths schedule and majorant segments; `vals` a tuple of ints."""
    if world <= 1:
        return tuple(int(v) for v in vals)
    import torch
    import torch.distributed as dist
    t = torch.tensor([int(v) for v in vals], dtype=torch.int64, device=device)
    dist.broadcast(t, src=0)
    return tuple(int(v) for v in t.tolist())


def reduce_step_film(buf, world):
    """The multi-GPU path's one exchange, inside the timed region: SUM-reduce of the packed fp64
    film (avr_film_export_device layout) to rank 0 (RCCL over xGMI; gloo in the CPU tests)."""
    if world > 1:
        import torch.distributed as dist
        dist.reduce(buf, dst=0, op=dist.ReduceOp.SUM)


def max_over_ranks(seconds, world, device):
    """The slowest rank's time (the driver's clock covers the whole world)."""
    if world <= 1:
        return seconds
    import torch
    import torch.distributed as dist
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def step_base(warm_bases, timed_bases, rank, warmup, k):
    """This rank's first sample index of step k (the warmup steps first, then the timed ones)."""
    return warm_bases[rank][k] if k < warmup else timed_bases[rank][k - warmup]


def timed_steps(integ, bases, S, maxdepth, world, buf):
    """Render the sample ranges [b, b + S) for b in bases back to back on the context stream,
    then export the film (and SUM-reduce it over the world), bracketed by barrier + sync;
    returns the max-over-ranks wall time in s."""
    import torch
    import torch.distributed as dist
    integ.ctx.sync()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for b in bases:
        integ.ctx.render(b, b + S, 0, maxdepth)
    integ.ctx.film_export_device(buf.data_ptr())
    reduce_step_film(buf, world)
    integ.ctx.sync()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    return max_over_ranks(time.perf_counter() - t0, world, buf.device)


def nanovdb_leg(args, density, dev, world, rank, S, warm_bases, timed_bases, spp_total, buf):
    """The headline's sample indices over the same S-cloud as a NanoVDBMedium (disney-cloud's
    medium type; media.h:602-685): the sparse tree is classified from the device grid
    (NanoVDBGrid.from_dense on the tensor), uploaded, its 64^3 majorant built on the device
    (pbrt's resolution: replay), library-default walk schedule, then `--nanovdb-steps` timed
    steps like the headline's. Returns the `nanovdb` block of the line."""
    from acceleratedvolrenderer_amd import VolPathIntegrator, scenes
    tb = time.perf_counter()
    grid = scenes.vdb_grid(density)
    scene = scenes.s_cloud_vdb(grid, width=args.width, height=args.height, sampler=args.sampler, spp=spp_total,
                               filter=args.filter)
    integ = VolPathIntegrator(scene, maxdepth=scenes.CLOUD_MAXDEPTH, spp=S, seed=0, device=dev, mode="replay")
    nleaves, ntiles = len(grid.leaf_origins), len(grid.tile_values)
    del grid
    try:
        integ.ctx.set_sampler_table(args.zsobol_table)
        if args.zsobol_pass_table != 96:
            integ.ctx.set_sampler_pass_table(args.zsobol_pass_table)
        if not args.pass_table_ahead:
            integ.ctx.set_pass_table_ahead(0)
        for b in (list(warm_bases[rank]) or list(timed_bases[rank]))[:1]:   # one-off tables, untimed
            integ.ctx.render(b, b + S, 0, scenes.CLOUD_MAXDEPTH)
        integ.ctx.film_clear()
        integ.ctx.reset_stats()
        build_s = time.perf_counter() - tb
        steps = max(1, min(args.steps, args.nanovdb_steps))
        el = timed_steps(integ, timed_bases[rank][:steps], S, scenes.CLOUD_MAXDEPTH, world, buf)
        agg = integ.ctx.stats()
        kernel = integ.ctx.last_kernel()
        launches = max(1, agg["medium_launches"])
        rb = roofline_block(agg, launches, args.sampler, "nanovdb", False, args.zsobol_table > 0,
                            args.zsobol_pass_table > 0)
    finally:
        integ.close()
    npix = args.width * args.height
    return {"workload": f"S-cloud-{args.res} as NanoVDBMedium ({nleaves} leaves, {ntiles} tiles; pbrt's 64^3 majorant, "
                        f"read through L2), same camera / film / sampler / sample indices as the headline, replay mode",
            "value": round(npix * S * steps * world / el / 1e6, 4), "unit": "Msamples/s", "steps": steps,
            "ms_per_step": round(1e3 * el / steps, 3), "instantiation": kernel, "build_s": round(build_s, 2),
            "parity": "tests/test_gpu_fullsize.py::test_fullsize_nanovdb_replay_at_the_driver_configuration",
            "roofline": rb, "dda_steps_per_sample": round(agg["medium_dda_steps"] / (npix * S * steps), 2)}


def main():
    args = parse()
    from acceleratedvolrenderer_amd import launch
    # one process per GPU: start the N ranks before anything touches a GPU
    launch.ensure_world(args.gpus, os.path.abspath(__file__), sys.argv[1:])
    import torch
    import torch.distributed as dist

    world, rank, local_rank = launch.world_from_env()
    if world > 1:
        dist.init_process_group("nccl", init_method="env://")
    torch.cuda.set_device(local_rank)
    dev = local_rank

    from acceleratedvolrenderer_amd import VolPathIntegrator, scenes, capi

    n = args.res
    # --- input generation (excluded from the timed region) ---
    tgen = time.perf_counter()
    density = torch.empty((n, n, n), dtype=torch.float32, device=f"cuda:{dev}")
    gen = capi.Context(dev)
    slab = n * n * 64
    total = n * n * n
    for first in range(0, total, slab):
        cnt = min(slab, total - first)
        gen.generate_cloud(density.data_ptr() + 4 * first, n, first, cnt)
    gen.sync()
    gen.close()
    tgen = time.perf_counter() - tgen
    log(f"density grid {n}^3 generated in {tgen:.2f} s")
    # sample indices (launch.sample_plan): the timed steps of all ranks render disjoint index
    # ranges [(k * world + rank) * S, + S) of one frame at `pixelsamples` spp, the smallest power
    # of two >= steps * world * S and >= 256 (BASELINE config C3's pixelsamples at N = 1 with
    # 4 steps of 64); ZSobol switches to 64-bit indices by itself where Morton(pixel) << log2 spp
    # needs more than 32 bits
    S = args.spp_per_step
    spp_total, warm_bases, timed_bases = launch.sample_plan(
        world, args.steps, args.warmup, S, base_spp=4096 if "explosion" in args.scene else 256,
        pixelsamples=args.pixelsamples)
    wrap = False
    vdb = None
    rgb_grids = None
    maxdepth = scenes.CLOUD_MAXDEPTH
    workload_name = {"cloud": f"S-cloud-{n}", "uniform": f"S-uniform-{n} (C2)",
                     "explosion": f"S-explosion-{n} emissive spectral (C5 stand-in)",
                     "rgb-explosion": f"S-rgb-explosion-{n} emissive RGB-coefficient spectral (C5 stand-in)"}[args.scene]
    if args.scene == "uniform":
        # C2: GridMedium n^3 of 1.0, orthographic; S-uniform's "scatter" variant (distant light + sky)
        density.fill_(1.0)
        scene = scenes.s_uniform(n=n, width=args.width, height=args.height, variant="scatter", density=density)
        from acceleratedvolrenderer_amd.scene import ZSobolSampler, IndependentSampler
        scene.sampler = ZSobolSampler(spp_total) if args.sampler == "zsobol" else IndependentSampler(spp_total)
        maxdepth = 100
    elif args.scene == "rgb-explosion":
        trgb = time.perf_counter()
        del density
        density = None
        torch.cuda.empty_cache()
        rgb_grids = scenes.rgb_explosion_grids(n=n, device=dev)
        scene = scenes.s_rgb_explosion(*rgb_grids, width=args.width, height=args.height, sampler=args.sampler,
                                       spp=spp_total, filter=args.filter)
        tgen += time.perf_counter() - trgb
        maxdepth = 100
    elif args.scene == "explosion":
        tvdb = time.perf_counter()
        del density
        density = None
        torch.cuda.empty_cache()
        vdb, vtemp = scenes.explosion_vdb(n=n)
        scene = scenes.s_explosion(vdb, vtemp, width=args.width, height=args.height, sampler=args.sampler,
                                   spp=spp_total)
        tgen += time.perf_counter() - tvdb
        maxdepth = 100
    elif args.medium == "nanovdb":
        # sparse tree of the same cloud (leaf blocks where the density is nonzero), built on
        # the host; outside the timed region like the grid generation
        tvdb = time.perf_counter()
        if args.nvdb and args.nvdb != "roundtrip":
            from acceleratedvolrenderer_amd.vdb import NanoVDBGrid
            vdb = NanoVDBGrid.read_nvdb(args.nvdb)
        else:
            with heartbeat("NanoVDB tree from the dense grid"):
                vdb = scenes.vdb_grid(density.cpu().numpy())
            if args.nvdb == "roundtrip":
                from acceleratedvolrenderer_amd.vdb import NanoVDBGrid
                tmpf = os.path.join(tempfile.mkdtemp(prefix="avr_nvdb_", dir=os.environ.get("TMPDIR", "/tmp")),
                                    "cloud.nvdb")
                vdb.write_nvdb(tmpf)
                vdb = NanoVDBGrid.read_nvdb(tmpf)
                shutil.rmtree(os.path.dirname(tmpf), ignore_errors=True)
                log(f"NanoVDB grid written to and read back from an .nvdb file ({len(vdb.leaf_origins)} leaves)")
        del density
        density = None
        torch.cuda.empty_cache()
        tgen += time.perf_counter() - tvdb
        scene = scenes.s_cloud_vdb(vdb, width=args.width, height=args.height, sampler=args.sampler, spp=spp_total,
                                   filter=args.filter)
    else:
        scene = scenes.s_cloud(density, width=args.width, height=args.height, sampler=args.sampler, spp=spp_total,
                               filter=args.filter)
    if args.majorant_res and args.majorant_res > 0:
        scene.medium.majorant_res = (args.majorant_res,) * 3
    integ = VolPathIntegrator(scene, maxdepth=maxdepth, spp=args.spp_per_step, seed=0, device=dev,
                              max_paths=args.max_paths, kernel=args.kernel, grid_layout=args.grid_layout,
                              mode=args.mode)
    if args.refill_min:
        integ.ctx.set_refill_min(args.refill_min)
    if args.dda_budget:
        integ.ctx.set_dda_budget(args.dda_budget)
    integ.ctx.set_sampler_table(args.zsobol_table)
    if args.zsobol_pass_table != 96:   # (96: the library default; older libraries lack the call)
        integ.ctx.set_sampler_pass_table(args.zsobol_pass_table)
    if not args.pass_table_ahead:
        integ.ctx.set_pass_table_ahead(0)
    if args.ray_binning:
        integ.ctx.set_ray_binning(1)
    if args.pixel_order == "entry-cell":
        integ.ctx.set_pixel_order(integ.entry_cell_order())
    if args.occupancy:
        integ.ctx.set_majorant_occupancy(1)
    walk_tuned = None
    if args.tune_walk == "on" and args.kernel == "persistent" and not (args.refill_min or args.dda_budget):
        # k_paths' lane schedule for this scene (avr_tune_walk): refill lanes x DDA cells per
        # iteration, 0 = the library default, probe = 8 sample indices of every pixel
        fine = vdb is not None or (scene.medium.majorant_res[0] > 16)
        rc = (0, 12, 16, 24, 32, 40)
        dc = (0, 16, 24, 28, 32, 40) if fine else (0, 8, 10, 12, 16, 24)
        (r_best, d_best), wms = integ.ctx.tune_walk(rc, dc, 0, 8, 0, maxdepth)
        r_best, d_best = broadcast_choice((r_best, d_best), world, f"cuda:{dev}")   # rank 0's, on every rank
        integ.ctx.set_refill_min(r_best)
        integ.ctx.set_dda_budget(d_best)
        walk_tuned = {"refill_min": r_best, "dda_budget": d_best, "refill_candidates": list(rc), "dda_candidates": list(dc),
                      "tie_break": "the default (0, 0) is kept unless a candidate's probe is > 2 % faster than every probe of the "
                                   "default's effective schedule (avr_tune_walk)",
                      "probe_ms": [[round(float(x), 3) for x in row] for row in wms]}
        args.refill_min, args.dda_budget = r_best, d_best   # the counter passes render the same schedule
        log(f"tuned walk: refill {r_best}, DDA {d_best} (0 = default)")
    maj_res = tuple(scene.medium.majorant_res)
    tune_ms = None
    if args.majorant_res == -1 or (args.majorant_res is None and args.mode == "fast"):
        cands = (1, 2, 4, 8, 16) + ((32, 64) if vdb is not None else ())
        maj_res, tune_ms = integ.tune_majorant(candidates=cands, probe=(0, 64))
        if world > 1:   # every rank renders with rank 0's choice
            maj_res = broadcast_choice(maj_res, world, f"cuda:{dev}")
            integ.ctx.set_majorant_res(maj_res)
        log(f"tuned majorant {maj_res} (probe ms {tune_ms})")
        args.majorant_res = maj_res[0]   # the counter passes (child processes) render the same majorant

    def step(k):
        # asynchronous on the context stream: steps queue back to back
        base = step_base(warm_bases, timed_bases, rank, args.warmup, k)
        integ.ctx.render(base, base + S, 0, maxdepth)

    log(f"scene uploaded; pixelsamples {spp_total}; warmup")
    for k in range(args.warmup):
        step(k)
    integ.ctx.film_clear()
    # one-off device tables (ZSobol pixel table) are built by the first (warmup) render
    setup_ms = integ.ctx.stats()["ms_setup"]
    integ.ctx.reset_stats()   # waits for the warmup; counters and kernel times restart
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.warmup, args.warmup + args.steps):
        step(k)
    # final film reduce over RCCL (part of T_render)
    npix = args.width * args.height
    from acceleratedvolrenderer_amd.integrator import film_buffer_size
    buf = torch.empty(film_buffer_size(npix, getattr(scene.film, "nbuckets", 0)), dtype=torch.float64,
                      device=f"cuda:{dev}")
    integ.ctx.film_export_device(buf.data_ptr())
    reduce_step_film(buf, world)
    integ.ctx.sync()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    agg = integ.ctx.stats()   # device counters + per-launch HIP-event times of the timed steps
    # the k_paths instantiation the timed steps ran (before the fast-mode leg launches another)
    timed_kernel = integ.ctx.last_kernel() if agg.get("loop_iterations") else "k_medium"
    elapsed = max_over_ranks(elapsed, world, f"cuda:{dev}")
    if args.pmc_child:
        integ.close()
        return

    samples = npix * S * args.steps * world
    value = samples / elapsed / 1e6

    # Second leg, after the headline (replay) measurement: the same steps in the "fast" render
    # mode (hardware transcendentals, majorant tuned on the device; statistical parity,
    # tests/test_gpu_fast.py), timed the same way. Not the headline value.
    fast_line = None
    if args.mode == "replay" and args.fast_leg and args.kernel == "persistent":
        integ.ctx.set_render_mode("fast")
        cands = (1, 2, 4, 8, 16) + ((32, 64) if vdb is not None else ())
        if args.fast_majorant_res > 0:
            fres, fms = (args.fast_majorant_res,) * 3, {}
            integ.ctx.set_majorant_res(fres)
        else:
            fres, fms = integ.tune_majorant(candidates=cands, probe=(0, 64))
        if world > 1:   # every rank renders with rank 0's choice
            fres = broadcast_choice(fres, world, f"cuda:{dev}")
            integ.ctx.set_majorant_res(fres)
        integ.ctx.film_clear()
        for k in range(args.warmup):
            step(k)
        integ.ctx.film_clear()
        integ.ctx.reset_stats()   # waits for the warmup; the fast leg's own counters and kernel times
        integ.ctx.sync()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        tf = time.perf_counter()
        for k in range(args.warmup, args.warmup + args.steps):
            step(k)
        integ.ctx.film_export_device(buf.data_ptr())
        reduce_step_film(buf, world)
        integ.ctx.sync()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        ef = max_over_ranks(time.perf_counter() - tf, world, f"cuda:{dev}")
        fagg = integ.ctx.stats()
        fast_kernel = integ.ctx.last_kernel()
        flaunches = max(1, fagg["medium_launches"])
        fast_line = {"value": round(samples / ef / 1e6, 4), "unit": "Msamples/s", "ms_per_step": round(1e3 * ef / args.steps, 3),
                     "majorant_res": list(fres), "majorant_probe_ms": {str(k): round(v, 4) for k, v in fms.items()},
                     "instantiation": fast_kernel,
                     "roofline": roofline_block(fagg, flaunches, args.sampler, "nanovdb" if vdb is not None else "grid", False,
                                                args.zsobol_table > 0, args.zsobol_pass_table > 0),
                     "parity": "statistical (hardware log/exp/sin/cos, tuned majorant): tests/test_gpu_fast.py"}
        log(f"fast mode: {fast_line['value']} Msamples/s (majorant {fres})")
    # roofline of the dominant kernel: algorithmic bytes / summed device time of its launches
    med_s = agg["ms_medium"] / 1e3
    launches = max(1, agg["medium_launches"])
    persistent = bool(agg.get("loop_iterations"))   # k_paths counts its wave loop iterations
    medium_kind = "rgb" if args.scene == "rgb-explosion" else ("nanovdb" if vdb is not None else "grid")
    emissive = "explosion" in args.scene
    samples_timed = npix * S * args.steps          # this rank's samples in the timed region
    samples_per_launch = samples_timed / launches
    bytes_parts = impl_parts = None
    rb = None
    if persistent:
        # k_paths fuses delta tracking and ratio tracking: per-unit bytes of kpaths_bytes()
        # (lookups by medium kind + majorant steps read outside LDS + the 16-B sample record + the
        # camera record it reads per path; ZSobol table entries and NanoVDB slots apart as
        # implementation bytes); path state never leaves VGPRs / LDS
        kname = "k_paths (persistent: delta + ratio tracking, density fetch)"
        med_bytes, bytes_parts, impl_parts = kpaths_bytes(agg, args.sampler, medium_kind, emissive,
                                                          args.zsobol_table > 0, args.zsobol_pass_table > 0,
                                                          majorant_in_lds=medium_kind != "nanovdb")
        rb = roofline_block(agg, launches, args.sampler, medium_kind, emissive, args.zsobol_table > 0,
                            args.zsobol_pass_table > 0)
    else:
        kname = "k_medium (wavefront delta tracking + density fetch)"
        med_bytes = BYTES_PER_LOOKUP * agg["medium_lookups"] + BYTES_PER_ITEM * (agg["medium_items_in"] +
                                                                                agg["medium_items_out"])
    achieved = med_bytes / med_s / 1e9 if med_s > 0 else 0.0
    avg_launch_ms = agg["ms_medium"] / launches
    # the camera stage (k_paths_camera), one launch per k_paths launch
    cam_block = None
    if persistent and agg["ms_camera"] > 0:
        # with the tables built ahead (a side stream, untimed) the interval is the camera kernel
        # alone, and so are the bytes: the table build's are left out
        ahead = args.pass_table_ahead and args.sampler == "zsobol" and args.zsobol_pass_table > 0
        cb = camera_bytes(samples_timed, args.sampler, args.zsobol_table > 0, args.zsobol_pass_table, npix,
                          0 if ahead else launches)
        cam_block = {"kernel": "k_paths_camera" if ahead else "k_zsobol_pass_table + k_paths_camera",
                     "pass_table": "built ahead on the side stream (not in this interval)" if ahead else "in this interval",
                     "bytes_per_launch": cb / launches,
                     "avg_launch_ms": round(agg["ms_camera"] / launches, 4),
                     "achieved": round(cb / (agg["ms_camera"] / 1e3) / 1e9, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(cb / (agg["ms_camera"] / 1e3) / 1e9 / HBM_PEAK_GBPS, 5),
                     "bytes_per_sample": round(cb / samples_timed, 2)}
    grid_layout = {0: "linear", 1: "fat", 2: "brick"}[integ.ctx.grid_layout_active()]
    host_density = host_rgb = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and vdb is None:
        if args.scene == "rgb-explosion" and n > RGB_CPU_MAX_RES:
            pass   # no host copy (the CPU baseline is skipped below)
        elif args.scene == "rgb-explosion":
            host_rgb = [t.cpu().numpy() for t in rgb_grids]
        else:
            host_density = density.cpu().numpy()
    integ.close()
    vdb_line = None
    if (args.nanovdb_leg and args.scene == "cloud" and vdb is None and args.kernel == "persistent"
            and args.mode == "replay"):
        torch.cuda.empty_cache()
        log("nanovdb leg: tree from the device grid")
        vdb_line = nanovdb_leg(args, density, dev, world, rank, S, warm_bases, timed_bases, spp_total, buf)
        log(f"nanovdb leg: {vdb_line['value']} Msamples/s ({vdb_line['instantiation']})")
    del density
    rgb_grids = None
    torch.cuda.empty_cache()

    out = None
    if rank == 0:
        cpu = None
        if vdb is not None and n > 256 and not args.no_cpu_baseline and world == 1:
            # the oracle's own NanoVDB tree for a 1024^3 grid takes over 10 minutes to build
            # on the host: the NanoVDB lines at that size carry no CPU baseline
            cpu = {"value": None, "skipped": f"oracle NanoVDB scene build at {n}^3 exceeds the bench's time budget"}
        elif args.scene == "rgb-explosion" and n > RGB_CPU_MAX_RES and not args.no_cpu_baseline and world == 1:
            cpu = {"value": None, "skipped": f"the three RGB-coefficient grids at {n}^3 ({3 * 16 * n ** 3 / 2 ** 30:.0f} GiB) "
                                             f"exceed the host copy the oracle scene needs (limit {RGB_CPU_MAX_RES}^3)"}
        elif not args.no_cpu_baseline and world == 1:
            if vdb is not None:
                host_scene = scene
            elif args.scene == "rgb-explosion":
                host_scene = scenes.s_rgb_explosion(*host_rgb, width=args.width, height=args.height,
                                                    sampler=args.sampler, spp=spp_total, filter=args.filter)
            elif args.scene == "uniform":
                host_scene = scenes.s_uniform(n=n, width=args.width, height=args.height, variant="scatter",
                                              density=host_density)
                host_scene.sampler = scene.sampler
            else:
                host_scene = scenes.s_cloud(host_density, width=args.width, height=args.height,
                                            sampler=args.sampler, spp=spp_total, filter=args.filter)
            with heartbeat("cpu baseline"):
                cpu = cpu_baseline(host_scene, S, args.cpu_seconds, f"{workload_name} {args.medium}")
            host_scene = host_density = host_rgb = None
        # HBM traffic and the VALU limiter from rocprofv3 counter passes of this same
        # configuration (child processes; the guide's gfx950 rule: FETCH_SIZE x2 + WRITE_SIZE)
        traffic, limiter, pmc_note, cache = None, None, "pmc off", None
        traffic_raw = traffic_x2 = None
        want_pmc = args.pmc == "on" or (args.pmc == "auto" and world == 1)
        pmc_kernel = None
        if want_pmc:
            cam_ctr = {}
            ctr, err, names = pmc_passes(args, spp_total,
                                         kernel_re=r"\bk_paths<|\dk_pathsI" if persistent else r"\bk_medium\b|\dk_mediumE",
                                         side=cam_ctr if persistent else None)
            if persistent and ctr is not None:
                # the counters must come from the instantiation the parent timed
                got = {kernel_targs(nm) for nm in names}
                pmc_kernel = sorted(names)[0] if len(names) == 1 else sorted(names)
                if got != {kernel_targs(timed_kernel)}:
                    ctr, err = None, f"pmc child profiled {sorted(names)}, the timed run launched {timed_kernel}"
            if ctr is None:
                pmc_note = err
                log(f"pmc: {err}")
            else:
                pmc_note = (f"rocprofv3 --pmc child passes of this configuration (bench.py pmc_passes, pixelsamples "
                            f"{spp_total}, same instantiation)")
                tb = traffic_bytes(ctr)
                if tb is not None:
                    traffic = round(tb / 1e9, 4)
                if "FETCH_SIZE" in ctr and "WRITE_SIZE" in ctr:
                    traffic_raw = round((ctr["FETCH_SIZE"] + ctr["WRITE_SIZE"]) * 1024 / 1e9, 4)
                    traffic_x2 = round((2 * ctr["FETCH_SIZE"] + ctr["WRITE_SIZE"]) * 1024 / 1e9, 4)
                lookups_pl = (agg["medium_lookups"] + (agg["shadow_lookups"] if persistent else 0)) / launches
                rd = (tb - ctr["WRITE_SIZE"] * 1024) if tb is not None else None
                cache = {
                    "read_bytes_per_lookup": round(rd / lookups_pl, 2) if rd is not None and lookups_pl else None,
                    "read_requests_by_size": ({"32B": ctr["TCC_EA0_RDREQ_32B_sum"], "64B": ctr["TCC_EA0_RDREQ_64B_sum"],
                                               "128B": ctr["TCC_EA0_RDREQ_128B_sum"], "all": ctr.get("TCC_EA0_RDREQ_sum")}
                                              if tb is not None else None),
                    "tcc_hit_rate": (round(ctr["TCC_HIT_sum"] / (ctr["TCC_HIT_sum"] + ctr["TCC_MISS_sum"]), 4)
                                     if ctr.get("TCC_HIT_sum") is not None and ctr.get("TCC_MISS_sum") else None),
                }
                if persistent and "SQ_INSTS_VALU" in ctr and "SQ_WAVE_CYCLES" in ctr:
                    # effective clock from GRBM_GUI_ACTIVE (summed over 8 XCDs) over the launch time
                    clk = (ctr["GRBM_GUI_ACTIVE"] / 8 / (avg_launch_ms / 1e3)) if ctr.get("GRBM_GUI_ACTIVE") else 2.4e9
                    valu_frac = ctr["SQ_INSTS_VALU"] * 2 / (VALU_SIMDS * clk * avg_launch_ms / 1e3)
                    wc = ctr["SQ_WAVE_CYCLES"]
                    limiter = {
                        "kind": "valu-issue + dependent-chain latency" if valu_frac > 4 * achieved / HBM_PEAK_GBPS
                        else "hbm",
                        "valu_issue_frac": round(valu_frac, 4),
                        "valu_wave_insts_per_launch": ctr["SQ_INSTS_VALU"],
                        # per launch: the child renders the same pass size (S sample indices per launch)
                        "valu_wave_insts_per_sample": round(ctr["SQ_INSTS_VALU"] / samples_per_launch, 1),
                        "effective_clock_ghz": round(clk / 1e9, 3),
                        "waves": ctr.get("SQ_WAVES"),
                        "waves_per_simd": round(ctr["SQ_WAVES"] / VALU_SIMDS, 2) if ctr.get("SQ_WAVES") else None,
                        "wave_cycle_split": {"issuing": round(ctr["SQ_ACTIVE_INST_ANY"] / wc, 4),
                                             "dependency/issue stall": round(ctr["SQ_WAIT_INST_ANY"] / wc, 4),
                                             "s_waitcnt (memory/LDS)": round(ctr["SQ_WAIT_ANY"] / wc, 4)},
                    }
                if cam_block is not None and "SQ_INSTS_VALU" in cam_ctr and cam_ctr.get("SQ_WAVE_CYCLES"):
                    # the camera stage's own limiter (the same passes count k_paths_camera separately)
                    cms = cam_block["avg_launch_ms"]
                    cclk = (cam_ctr["GRBM_GUI_ACTIVE"] / 8 / (cms / 1e3)) if cam_ctr.get("GRBM_GUI_ACTIVE") else 2.4e9
                    cwc = cam_ctr["SQ_WAVE_CYCLES"]
                    cam_block["limiter"] = {
                        "valu_issue_frac": round(cam_ctr["SQ_INSTS_VALU"] * 2 / (VALU_SIMDS * cclk * cms / 1e3), 4),
                        "valu_wave_insts_per_sample": round(cam_ctr["SQ_INSTS_VALU"] / samples_per_launch, 2),
                        "waves_per_simd_launched": round(cam_ctr["SQ_WAVES"] / VALU_SIMDS, 2) if cam_ctr.get("SQ_WAVES") else None,
                        "wave_cycle_split": {"issuing": round(cam_ctr["SQ_ACTIVE_INST_ANY"] / cwc, 4),
                                             "dependency/issue stall": round(cam_ctr["SQ_WAIT_INST_ANY"] / cwc, 4),
                                             "s_waitcnt (memory/LDS)": round(cam_ctr["SQ_WAIT_ANY"] / cwc, 4)},
                        "hbm_traffic_GB": (round(traffic_bytes(cam_ctr) / 1e9, 4) if traffic_bytes(cam_ctr) is not None
                                           else None),
                    }
        if want_pmc and fast_line is not None and persistent:
            # the fast leg's HBM traffic: the same counter passes (request sizes, WRITE_SIZE, FETCH_SIZE)
            # of the fast configuration at its majorant resolution
            import copy
            fargs = copy.copy(args)
            fargs.mode, fargs.majorant_res, fargs.fast_leg = "fast", fast_line["majorant_res"][0], 0
            fctr, ferr, fnames = pmc_passes(fargs, spp_total, passes=tuple(x for x in PMC_PASSES
                                                                           if x[0] in ("size", "write", "fetch")))
            if fctr is not None and {kernel_targs(nm) for nm in fnames} != {kernel_targs(fast_line["instantiation"])}:
                fctr, ferr = None, f"pmc child profiled {sorted(fnames)}, the fast leg launched {fast_line['instantiation']}"
            frb = fast_line["roofline"]
            ftb = traffic_bytes(fctr) if fctr is not None else None
            frb["traffic"] = round(ftb / 1e9, 4) if ftb is not None else None
            frb["traffic_over_algorithmic"] = round(ftb / frb["bytes_per_launch"], 3) if ftb and frb["bytes_per_launch"] else None
            frb["traffic_fetch_x2_rule"] = (round((2 * fctr["FETCH_SIZE"] + fctr["WRITE_SIZE"]) * 1024 / 1e9, 4)
                                            if fctr is not None and "FETCH_SIZE" in fctr and "WRITE_SIZE" in fctr else None)
            frb["traffic_source"] = (f"rocprofv3 --pmc child passes of the fast configuration (majorant "
                                     f"{fast_line['majorant_res'][0]}^3), {FETCH_CALIBRATION}" if ftb is not None else ferr)
            if ferr:
                log(f"fast-mode pmc: {ferr}")
        out = {
            "metric": "Msamples/s (whole node) on synthetic S-cloud-1024 720p (disney-cloud stand-in)",
            "value": round(value, 4),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": {"cloud": f"synthetic (CloudMedium::Density {n}^3 generated on device; disney-cloud assets absent)",
                     "uniform": f"synthetic (uniform density {n}^3)",
                     "explosion": f"synthetic (radial density + temperature NanoVDB grids over {n}^3; explosion asset absent)",
                     "rgb-explosion": f"synthetic (k_rgb_explosion RGB-coefficient sigma_a / sigma_s / Le grids {n}^3 generated on device; explosion asset absent)"}[args.scene],
            "config": {"workload": f"{workload_name} {'NanoVDBMedium' if vdb is not None else ('RGBGridMedium' if args.scene == 'rgb-explosion' else 'GridMedium')}, {'orthographic' if args.scene == 'uniform' else 'perspective'} {args.width}x{args.height}, "
                                   f"{S} spp/step/GPU, maxdepth {maxdepth}, {args.sampler} sampler "
                                   f"(pixelsamples {spp_total}), {args.filter} filter, {args.mode} mode",
                       "majorant_res": list(maj_res), "majorant_tuning_ms": tune_ms,
                       "walk_schedule": walk_tuned or {"refill_min": args.refill_min, "dda_budget": args.dda_budget},
                       "global_batch": samples // args.steps, "parallelism": f"sample-shard x{world}",
                       "pixelsamples": spp_total, "sample_indices_distinct": True},
            "roofline": {
                "kernel": kname,
                "instantiation": timed_kernel,
                "pmc_kernel": pmc_kernel,
                # what limits the kernel, from the counter passes (`limiter`); `achieved` /
                # `peak` / `frac` stay priced against the HBM roof (no MFMA work on the path)
                "bound": ("valu" if limiter and limiter["kind"].startswith("valu") else "hbm"),
                "priced_against": "hbm",
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 5),
                "traffic": traffic,
                "traffic_source": pmc_note,
                # counter bytes over §8(d) bytes: > 1 is over-fetch (a whole 64- or 128-B request per
                # 32-B gather, ZSobol tables, NanoVDB slots). `traffic` prices the memory-side reads
                # by request size (traffic_bytes); FETCH_SIZE undoubled / doubled (the guide's x2
                # rule for streaming reads) are kept for comparison: FETCH_CALIBRATION measures
                # which holds for this kernel's 32-B gathers
                "traffic_over_algorithmic": (round(traffic * 1e9 / (med_bytes / launches), 3)
                                             if traffic and med_bytes else None),
                "traffic_basis": (f"TCC_EA0_RDREQ 32B/64B/128B request sizes x bytes + WRITE_SIZE, per launch "
                                  f"(calibration: {FETCH_CALIBRATION})" if traffic is not None else None),
                "traffic_fetch_raw": traffic_raw,
                "traffic_fetch_x2_rule": traffic_x2,
                "bytes_per_launch": med_bytes / launches,
                "bytes_parts_per_launch": ({k: v / launches for k, v in bytes_parts.items()} if bytes_parts else None),
                "implementation_bytes_per_launch": ({k: v / launches for k, v in impl_parts.items()}
                                                    if impl_parts else None),
                "density_fetch": rb["density_fetch"] if rb else None,
                "samples_per_launch": samples_per_launch,
                "avg_launch_ms": avg_launch_ms,
                "launches": launches,
                # the ceiling of this access pattern: a random 32-B fat-entry gather moves one whole
                # 128-B memory-side request per lookup (FETCH_CALIBRATION), so at the achievable
                # 6.3 TB/s at most a quarter of the bytes are the lookup's own
                "attainable": {"random_gather_GBps": HBM_ACHIEVABLE_GBPS * BYTES_PER_LOOKUP / HBM_REQUEST_BYTES,
                               "basis": f"{HBM_ACHIEVABLE_GBPS:.0f} GB/s achievable x {BYTES_PER_LOOKUP} B used per "
                                        f"{HBM_REQUEST_BYTES}-B request",
                               "frac": round(achieved / (HBM_ACHIEVABLE_GBPS * BYTES_PER_LOOKUP / HBM_REQUEST_BYTES), 5)},
                "camera_stage": cam_block,
                "limiter": limiter,
                "cache": cache,
            },
            "fast_mode": fast_line,
            "nanovdb": vdb_line,
            "grid_layout": grid_layout,
            "majorant_occupancy": bool(args.occupancy) if vdb is not None else None,
            "simd_utilisation": (agg["active_lane_iterations"] / (64.0 * agg["loop_iterations"])
                                 if agg.get("loop_iterations") else None),
            "cpu_baseline": cpu,
            "detail": {
                "grid_gen_s": round(tgen, 3),
                "setup_ms": round(setup_ms, 3), "zsobol_table_dims": args.zsobol_table,
                "ms_camera": agg["ms_camera"], "ms_medium": agg["ms_medium"], "ms_shadow": agg["ms_shadow"],
                "ms_film": agg["ms_film"], "medium_lookups": agg["medium_lookups"],
                "shadow_lookups": agg["shadow_lookups"], "medium_items_in": agg["medium_items_in"],
                "loop_iterations": agg.get("loop_iterations"), "medium_dda_steps": agg["medium_dda_steps"],
                "medium_items_out": agg["medium_items_out"], "shadow_items": agg["shadow_items"],
                # wavefront organisation only (k_paths has no separate shadow kernel)
                "shadow_achieved_GBps": (round((BYTES_PER_LOOKUP * agg["shadow_lookups"] + BYTES_PER_ITEM *
                                                agg["shadow_items"]) / (agg["ms_shadow"] / 1e3) / 1e9, 2)
                                         if agg["ms_shadow"] > 0 else None),
            },
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

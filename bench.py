"""Benchmark: Msamples/s of the MI355X volumetric path integrator on the BASELINE.json
metric workload ("disney-cloud 720p" -> synthetic S-cloud-1024):
GridMedium 1024^3 f32 (4 GiB) filled on device with CloudMedium::Density, perspective
1280x720, VolPath maxdepth 100, IndependentSampler seed 0.

A step = one render pass of --spp-per-step sample indices over every pixel (the hot path:
camera rays -> delta tracking -> ratio-tracked shadow rays -> film). Each rank renders
its own disjoint sample indices (weak scaling); the fp64 film is SUM-reduced over RCCL
once at the end of the timed region (T_render ends at the film reduce).

Prints ONE JSON line (rank 0) with roofline (k_paths, the fused delta-tracking /
ratio-tracking / density-fetch kernel; HIP-event time of its launches on the context stream)
and cpu_baseline (the oracle restatement on a bounded sample of the same workload).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# SURVEY.md §8d algorithmic bytes: 32 B per trilinear lookup (8 taps x 4 B) and 132 B per
# work item read / written (ray 24, tMax 4, lambda+pdf 32, beta/r_u/r_l 48, RNG 16, pixel/depth 8).
BYTES_PER_LOOKUP = 32
BYTES_PER_ITEM = 132


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=4)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--res", type=int, default=1024, help="density grid resolution (n^3)")
    p.add_argument("--width", type=int, default=1280)
    p.add_argument("--height", type=int, default=720)
    p.add_argument("--spp-per-step", type=int, default=16)
    p.add_argument("--max-paths", type=int, default=0)
    p.add_argument("--cpu-seconds", type=float, default=15.0, help="budget of the CPU-baseline sample")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--kernel", default="persistent", choices=["persistent", "wavefront"])
    p.add_argument("--medium", default="grid", choices=["grid", "nanovdb"],
                   help="S-cloud as GridMedium (default) or as a NanoVDBMedium tree (disney-cloud's type)")
    p.add_argument("--refill-min", type=int, default=0, help="k_paths refill threshold (0 = library default)")
    p.add_argument("--grid-layout", default="fat", choices=["fat", "linear"])
    p.add_argument("--dda-budget", type=int, default=0, help="k_paths DDA cells per iteration (0 = default)")
    p.add_argument("--zsobol-table", type=int, default=256,
                   help="ZSobol pixel-table dimensions (0 = every digit per sampler call)")
    p.add_argument("--sampler", default="zsobol", choices=["zsobol", "independent"],
                   help="pixel sampler (BASELINE.md S-cloud: zsobol, pbrt's default)")
    p.add_argument("--filter", default="gaussian", choices=["gaussian", "box"],
                   help="pixel filter (pbrt's default: gaussian radius 1.5, sigma 0.5)")
    return p.parse_args()


def log(msg):
    """Progress on stderr (the JSON line stays the only stdout output)."""
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def cpu_baseline(scene_host, spp_per_step, budget_s, label="S-cloud"):
    """Time the CPU oracle (pbrt VolPath restatement, `port`) on a bounded sample of the
    SAME workload: a strided pixel subset across the whole 1280x720 frame, spp_per_step
    samples each, on the host cores this process may use."""
    from oracle import binding
    cores = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    cores = max(1, min(cores, 16, os.cpu_count() or 1))
    log(f"cpu baseline: building the oracle scene ({label})")
    run = binding.OracleRun(scene_host, max_depth=100, seed=0)
    log(f"cpu baseline: timing {budget_s:.0f} s on {cores} threads")
    f = scene_host.film
    npix = f.width * f.height
    # a strided pixel subset that spans every row/column band of the frame; samples are
    # taken in sampleIndex order, sweep after sweep, until the time budget is used
    stride = 61
    order = np.arange(0, npix, stride, dtype=np.int32)
    chunk = 512
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
    done_px = len(order)
    return {"value": done_s / t_used / 1e6, "unit": "Msamples/s", "cores": cores, "kind": "port",
            "sample": f"{done_s} samples: pixels every {stride}th of {f.width}x{f.height} ({done_px} px), "
                      f"sample indices from 0 in sweeps of {spp_per_step}, same {label} "
                      f"scene, {t_used:.1f} s on {cores} threads"}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
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
    # the sampler's pixelsamples covers every sample index the run renders (ZSobol lays out
    # Morton(pixel) << log2(spp) | index): 256 (config C3) unless more are rendered
    S = args.spp_per_step
    needed = (args.warmup + args.steps) * world * S
    spp_total = 256
    while spp_total < needed:
        spp_total *= 2
    # ZSobol's 32-bit index needs Morton(pixel) << log2(spp) < 2^32: at most 2^(32 - 2 log2 res)
    # sample indices (1024 at 720p/1080p). Longer runs wrap the index range: every step still
    # traces S fresh paths per pixel (nothing is reused), later steps repeat earlier indices.
    res_pow2 = 1
    while res_pow2 < max(args.width, args.height):
        res_pow2 *= 2
    spp_cap = 1 << (32 - 2 * (res_pow2.bit_length() - 1))
    wrap = spp_total > spp_cap and args.sampler == "zsobol"
    if wrap:
        spp_total = spp_cap
        if spp_total % S:
            raise SystemExit(f"--spp-per-step {S} must divide the ZSobol index range {spp_total} for this run length")
    vdb = None
    if args.medium == "nanovdb":
        # sparse tree of the same cloud (leaf blocks where the density is nonzero), built on
        # the host; outside the timed region like the grid generation
        tvdb = time.perf_counter()
        vdb = scenes.vdb_grid(density.cpu().numpy())
        del density
        density = None
        torch.cuda.empty_cache()
        tgen += time.perf_counter() - tvdb
        scene = scenes.s_cloud_vdb(vdb, width=args.width, height=args.height, sampler=args.sampler, spp=spp_total,
                                   filter=args.filter)
    else:
        scene = scenes.s_cloud(density, width=args.width, height=args.height, sampler=args.sampler, spp=spp_total,
                               filter=args.filter)
    integ = VolPathIntegrator(scene, maxdepth=scenes.CLOUD_MAXDEPTH, spp=args.spp_per_step, seed=0, device=dev,
                              max_paths=args.max_paths, kernel=args.kernel, grid_layout=args.grid_layout)
    if args.refill_min:
        integ.ctx.set_refill_min(args.refill_min)
    if args.dda_budget:
        integ.ctx.set_dda_budget(args.dda_budget)
    integ.ctx.set_sampler_table(args.zsobol_table)

    def step(k):
        # asynchronous on the context stream: steps queue back to back
        base = ((k * world + rank) * S) % spp_total if wrap else (k * world + rank) * S
        integ.ctx.render(base, base + S, 0, scenes.CLOUD_MAXDEPTH)

    log("scene uploaded; warmup")
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
    buf = torch.empty(4 * npix, dtype=torch.float64, device=f"cuda:{dev}")
    integ.ctx.film_export_device(buf.data_ptr())
    if world > 1:
        dist.reduce(buf, dst=0, op=dist.ReduceOp.SUM)
    integ.ctx.sync()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    agg = integ.ctx.stats()   # device counters + per-launch HIP-event times of the timed steps
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{dev}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    samples = npix * S * args.steps * world
    value = samples / elapsed / 1e6
    # roofline of the dominant kernel: algorithmic bytes / summed device time of its launches
    med_s = agg["ms_medium"] / 1e3
    launches = max(1, agg["medium_launches"])
    if args.kernel == "persistent":
        # k_paths fuses delta tracking and ratio tracking: 32 B per trilinear lookup (both kinds)
        # + the 32 B per-sample record (L, lambda) it writes; path state never leaves VGPRs.
        kname = "k_paths (persistent: delta + ratio tracking, density fetch)"
        med_bytes = BYTES_PER_LOOKUP * (agg["medium_lookups"] + agg["shadow_lookups"]) + 32 * agg["medium_items_in"]
    else:
        kname = "k_medium (wavefront delta tracking + density fetch)"
        med_bytes = BYTES_PER_LOOKUP * agg["medium_lookups"] + BYTES_PER_ITEM * (agg["medium_items_in"] +
                                                                                agg["medium_items_out"])
    achieved = med_bytes / med_s / 1e9 if med_s > 0 else 0.0
    # HBM traffic per launch from the committed rocprofv3 PMC passes of this kernel on this
    # workload (FETCH_SIZE x2 + WRITE_SIZE, MI355X_MICROARCH.md HBM section); bench.py
    # itself cannot read counters. Null when the profile does not match the run.
    traffic, traffic_src, valu = None, None, None
    prof = os.path.join(ROOT, "profiles", f"r01_pmc_k_paths_{args.sampler}_{args.filter}.json")
    if args.kernel == "persistent" and args.medium == "grid" and n == 1024 and S == 16 and os.path.exists(prof):
        pm = json.load(open(prof))
        traffic = round(pm["hbm_traffic_bytes_per_launch"] / 1e9, 3)
        traffic_src = os.path.relpath(prof, ROOT) + " (GB per launch, PMC FETCH_SIZE x2 + WRITE_SIZE)"
        # the bound that is actually close: VALU issue (wave64 op = 2 SIMD cycles)
        valu = {"wave_instructions_per_launch": pm["valu_wave_instructions_per_launch"],
                "issue_fraction": round(pm["valu_issue_fraction"], 4),
                "wave_cycle_split": pm["wave_cycle_split"], "source": os.path.relpath(prof, ROOT)}
    out = None
    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            if vdb is not None:
                host_scene = scene
            else:
                host_density = density.cpu().numpy()
                host_scene = scenes.s_cloud(host_density, width=args.width, height=args.height,
                                            sampler=args.sampler, spp=spp_total, filter=args.filter)
            cpu = cpu_baseline(host_scene, S, args.cpu_seconds, f"S-cloud-{n} {args.medium}")
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
            "data": "synthetic (CloudMedium::Density 1024^3 generated on device; disney-cloud assets absent)",
            "config": {"workload": f"S-cloud-{n} {'NanoVDBMedium' if vdb is not None else 'GridMedium'}, perspective {args.width}x{args.height}, "
                                   f"{S} spp/step/GPU, maxdepth {scenes.CLOUD_MAXDEPTH}, {args.sampler} sampler "
                                   f"(pixelsamples {spp_total}), {args.filter} filter",
                       "global_batch": samples // args.steps, "parallelism": f"sample-shard x{world}",
                       "sample_index_wrap": wrap},
            "roofline": {
                "kernel": kname,
                "bound": "hbm",
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 5),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "bytes_per_launch": med_bytes / launches,
                "avg_launch_ms": agg["ms_medium"] / launches,
                "launches": launches,
            },
            "valu": valu,
            "grid_layout": "fat" if integ.ctx.grid_layout_active() else "linear",
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
                "shadow_achieved_GBps": round((BYTES_PER_LOOKUP * agg["shadow_lookups"] + BYTES_PER_ITEM *
                                               agg["shadow_items"]) / max(1e-9, agg["ms_shadow"] / 1e3) / 1e9, 2),
            },
        }
        print(json.dumps(out), flush=True)
    integ.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

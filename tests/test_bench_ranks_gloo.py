"""bench.py's `--gpus N` rank path on CPU (gloo, world size 2), with the oracle as the renderer
(tests/bench_rank_child.py): the sample plan's timed steps of both ranks, reduced by
bench.reduce_step_film, equal the single-process oracle render of the same sample indices at
the same pixelsamples (the film of one render at pixelsamples spp, up to fp64 summation
order); bench.broadcast_choice gives every rank rank 0's walk schedule and majorant, and
bench.max_over_ranks the slowest rank's time. SCALE stays unmeasured until an 8-GPU node runs
the driver's scaling bench; this is its rank logic."""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = os.path.join(ROOT, "tests", "bench_rank_child.py")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def _env():
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e["OMP_NUM_THREADS"] = "1"
    return e


def test_bench_rank_path_reduces_to_the_one_rank_film():
    steps, warmup, S = 2, 1, 4
    r = subprocess.run([sys.executable, CHILD, "--gpus", "2", "--steps", str(steps), "--warmup", str(warmup),
                        "--spp-per-step", str(S)], capture_output=True, text=True, env=_env(), timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1                               # rank 0 prints
    got = json.loads(lines[0])
    assert got["world"] == 2
    assert got["walk"] == [32, 10] and got["majorant"] == [16, 16, 16]   # rank 0's choice everywhere
    assert got["max_time"] == 2.0                        # the slower rank's clock
    # the same pixelsamples as a 1-GPU (and an 8-GPU) run of the same command
    from acceleratedvolrenderer_amd.launch import sample_plan
    assert got["pixelsamples"] == sample_plan(1, steps, warmup, S)[0] == sample_plan(8, steps, warmup, S)[0]
    idx = sorted(b + i for rank in got["timed"] for b in rank for i in range(S))
    assert idx == list(range(steps * 2 * S))             # every index once, none twice
    # the 1-rank film of the same sample indices, one oracle render in sampleIndex order
    import bench_rank_child
    from oracle import binding
    scene = bench_rank_child.scene_for(got["pixelsamples"])
    rgb1, w1 = binding.OracleRun(scene, max_depth=20, seed=0).render(0, steps * 2 * S, nthreads=4)
    rgb2, w2 = np.array(got["rgb"]), np.array(got["w"])
    assert np.allclose(w2, w1, rtol=1e-12, atol=0) and np.all(w1 > 0)
    assert np.allclose(rgb2, rgb1, rtol=1e-12, atol=1e-300)
    assert np.any(rgb1 > 0)

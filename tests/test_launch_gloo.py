"""bench.py's `--gpus N` launcher (acceleratedvolrenderer_amd/launch.py) on CPU with gloo:
without a launcher environment it starts N ranks itself (torch.distributed.run as a child
process), each rank renders its sample shard and the fp64 film is SUM-reduced to rank 0;
under a launcher a world size different from --gpus is refused."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = os.path.join(ROOT, "tests", "launch_child.py")


def _env():
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e["OMP_NUM_THREADS"] = "1"
    return e


def _run(args, env):
    r = subprocess.run([sys.executable, CHILD] + args, capture_output=True, text=True, env=env, timeout=240)
    return r


def test_launcher_starts_the_world_and_reduces_the_film():
    one = _run(["--gpus", "1"], _env())
    assert one.returncode == 0, one.stderr
    ref = json.loads([x for x in one.stdout.splitlines() if x.startswith("{")][-1])
    assert ref["n_gpus"] == 1
    two = _run(["--gpus", "2"], _env())
    assert two.returncode == 0, two.stderr[-2000:]
    lines = [x for x in two.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1          # rank 0 only
    got = json.loads(lines[0])
    assert got["n_gpus"] == 2
    assert got["w"] == ref["w"]     # every (pixel, sample) exactly once over the shards
    for a, b in zip(got["rgb"], ref["rgb"]):
        assert abs(a - b) <= 1e-12 * abs(b)


def test_launcher_refuses_a_mismatched_world():
    e = _env()
    e.update({"WORLD_SIZE": "3", "RANK": "0", "LOCAL_RANK": "0"})
    r = _run(["--gpus", "2"], e)
    assert r.returncode != 0
    assert "WORLD_SIZE=3" in r.stderr


def test_bench_sample_plan_renders_distinct_indices_at_every_world_size():
    """bench.py's step arithmetic (launch.sample_plan): over the timed steps of all ranks every
    (pixel, sample index) pair is rendered exactly once, inside [0, pixelsamples), for the
    driver's 1/2/4/8-GPU runs."""
    from acceleratedvolrenderer_amd.launch import sample_plan
    for world in (1, 2, 4, 8):
        for steps, warmup, S in ((4, 1, 64), (10, 2, 64), (3, 0, 16), (20, 5, 64)):
            P, warm, timed = sample_plan(world, steps, warmup, S)
            idx = [b + i for r in range(world) for b in timed[r] for i in range(S)]
            assert len(idx) == len(set(idx)) == steps * world * S
            assert min(idx) == 0 and max(idx) < P and P >= 256 and P & (P - 1) == 0
            assert all(0 <= b and b + S <= P for r in range(world) for b in warm[r])
            assert len(warm[0]) == warmup and all(len(t) == steps for t in timed)
    assert sample_plan(1, 4, 1, 64, base_spp=4096)[0] == 4096
    import pytest
    with pytest.raises(ValueError):
        sample_plan(8, 4, 1, 64, pixelsamples=256)
    with pytest.raises(ValueError):
        sample_plan(0, 4, 1, 64)


def test_bench_sample_plan_pixelsamples_is_invariant_in_the_world_size():
    """One bench command runs the same sampler at N = 1, 2, 4 and 8: the
    pixelsamples value, hence the ZSobol index width and the digits per draw (samplers.h:250-254),
    does not depend on the world size, and is sized for the 8-GPU world."""
    from acceleratedvolrenderer_amd.launch import sample_plan
    for steps, warmup, S in ((4, 1, 64), (10, 2, 64), (3, 0, 16), (20, 5, 64), (2, 1, 64)):
        Ps = {sample_plan(world, steps, warmup, S)[0] for world in (1, 2, 4, 8)}
        assert len(Ps) == 1, (steps, S, Ps)
        P = Ps.pop()
        assert P >= steps * 8 * S
    # the driver's command: python bench.py --steps 20 --warmup 5 (64 sample indices per step)
    assert sample_plan(1, 20, 5, 64)[0] == sample_plan(8, 20, 5, 64)[0] == 16384
    assert sample_plan(1, 4, 1, 64)[0] == 2048
    # the index ranges of different world sizes are prefixes of one another's sequence: the
    # timed steps of world N cover [0, steps * N * S)
    for world in (1, 2, 4, 8):
        _, _, timed = sample_plan(world, 20, 5, 64)
        assert sorted(b for r in range(world) for b in timed[r]) == list(range(0, 20 * world * 64, 64))

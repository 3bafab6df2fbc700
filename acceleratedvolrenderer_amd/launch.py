"""One process per GPU: the launcher behind `bench.py --gpus N` and `render_distributed`.

`ensure_world(n, script, argv)` is called before anything touches the GPU. Under a
launcher (WORLD_SIZE set: torchrun / torch.distributed.run) it only checks that the world
size is the one requested. Without one and with n > 1 it starts
`python -m torch.distributed.run --nproc-per-node n --master-addr 127.0.0.1 script argv`
as a CHILD process (never exec: the parent may not replace itself once a GPU runtime is
loaded), waits for it and exits with its status. Each rank then reads RANK / LOCAL_RANK /
WORLD_SIZE from the environment (`world_from_env`).
"""
import os
import socket
import subprocess
import sys


def world_from_env():
    """(world_size, rank, local_rank) from the torch.distributed launcher's environment."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_command(nproc, script, argv):
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={int(nproc)}",
            "--master-addr", "127.0.0.1", "--master-port", str(free_port()), script] + list(argv)


def ensure_world(requested, script, argv, env=None):
    """Return normally when this process is a rank of a world of `requested` processes
    (or requested == 1 without a launcher). Otherwise launch that world as a child and
    exit with its status. Raises SystemExit when a launcher's world size differs."""
    requested = int(requested)
    if requested < 1:
        raise SystemExit(f"--gpus must be >= 1 (got {requested})")
    if "WORLD_SIZE" in os.environ:
        world = int(os.environ["WORLD_SIZE"])
        if world != requested:
            raise SystemExit(f"launched with WORLD_SIZE={world} but --gpus {requested}")
        return
    if requested == 1:
        return
    e = dict(os.environ if env is None else env)
    # dmabuf IPC only on this platform (RCCL / CUDA-tensor sharing across processes)
    e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    rc = subprocess.call(launch_command(requested, script, argv), env=e)
    sys.exit(rc)


PLAN_WORLD = 8   # the largest world bench.py is run at (one 8-GPU node)


def sample_plan(world, steps, warmup, spp_per_step, base_spp=256, pixelsamples=0, plan_world=PLAN_WORLD):
    """Sample indices of `bench.py --gpus N` (weak scaling: every rank renders spp_per_step
    sample indices of every pixel per step; the sampler is indexed by (pixel, sampleIndex),
    samplers.h:252-254, so disjoint index ranges are disjoint paths).

    Returns (pixelsamples, warm, timed): warm[r] / timed[r] are rank r's first sample index of
    each warmup / timed step. Rank r's timed steps are the consecutive block [r * steps * S,
    (r + 1) * steps * S) (rank-major: each rank walks its indices in order, as pbrt's pass loop
    does, so its ZSobol pass tables are built one pass ahead and share their level-A table —
    an interleaved plan measured 0.2 ms per step slower, profiles/r06_pass_stride_probe.json).
    The timed steps of all ranks cover [0, steps * world * S) once — no (pixel, index) pair is
    rendered twice, so the reduced film is one render at pixelsamples spp. pixelsamples is the smallest power of two >= steps * max(world,
    plan_world) * S and >= base_spp (BASELINE config C3: 256), unless given: sized for the
    largest world (8 GPUs) at EVERY world size, so the N = 1, 2, 4 and 8 lines of one command
    run the same ZSobol instantiation with the same number of sample digits per draw
    (samplers.h:250-254: the digit count grows with log2 pixelsamples) and a scaling curve
    measures scaling, not sampler cost. Warmup steps re-render indices of the same range
    (their film is cleared before the timed region)."""
    S = int(spp_per_step)
    if S < 1:
        raise ValueError(f"spp per step must be >= 1 (got {S})")
    if int(world) < 1:
        raise ValueError(f"world size must be >= 1 (got {world})")
    need = int(steps) * int(world) * S
    plan = int(steps) * max(int(world), int(plan_world)) * S
    P = int(pixelsamples) if pixelsamples else max(int(base_spp), 1)
    if not pixelsamples:
        while P < plan:
            P *= 2
    if P < need or P % S:
        raise ValueError(f"pixelsamples {P} cannot hold {steps} steps x {world} ranks x {S} distinct sample indices")
    timed = [[(r * steps + k) * S for k in range(steps)] for r in range(world)]
    warm = [[((r * steps + k) * S) % P for k in range(warmup)] for r in range(world)]
    return P, warm, timed

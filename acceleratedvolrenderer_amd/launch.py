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

"""Build libavr_hip.so in-tree with hipcc for gfx950 (no JIT cache: the .so travels
with the repository snapshot to the GPU box)."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "csrc", "avr_capi.hip")
DEPS = [os.path.join(HERE, "csrc", f) for f in ("avr_capi.hip", "avr_kernels.hip", "avr_numerics.h", "avr_canon.h", "avr_sampling.h", "avr_vdb.h", "avr_envmap.h", "avr_flip.h", "avr_graph.hip", "avr_graph_capi.hip", "avr_graph_host.h")] + [
    os.path.join(ROOT, "include", "avr.h")]
OUT = os.path.join(HERE, "libavr_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

# -ffp-contract=off: same float semantics as pbrt's CPU build (CMakeLists.txt:134-137),
# so a device sample replays the CPU oracle's sample.
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared",
         "-I" + os.path.join(ROOT, "include")]
# RCCL for avr_film_reduce_rccl (in-process multi-GPU film reduce)
LIBS = ["-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]


def up_to_date():
    if not os.path.exists(OUT):
        return False
    t = os.path.getmtime(OUT)
    return all(os.path.getmtime(d) <= t for d in DEPS)


def build(force=False, verbose=False):
    if not force and up_to_date():
        return OUT
    cmd = [HIPCC] + FLAGS + [SRC, "-o", OUT + ".tmp"] + LIBS
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force=True, verbose=True))

"""Build libavr_hip.so in-tree with hipcc for gfx950 (no JIT cache: the .so travels
with the repository snapshot to the GPU box).

The persistent path kernel k_paths has 112 instantiations (medium kind x emission x gray
state x sampler x image light x render mode); they are compiled as eight objects
(csrc/avr_kpaths.hip, one per medium kind and render mode) in parallel with the C-ABI
unit (csrc/avr_capi.hip, -DAVR_KP_SPLIT), then linked."""
import hashlib
import os
import subprocess
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
SRC = os.path.join(CSRC, "avr_capi.hip")
KPATHS = os.path.join(CSRC, "avr_kpaths.hip")
DEPS = [os.path.join(CSRC, f) for f in (
    "avr_capi.hip", "avr_kernels.hip", "avr_kpaths.hip", "avr_kpaths_list.h", "avr_numerics.h", "avr_canon.h",
    "avr_sampling.h", "avr_vdb.h", "avr_envmap.h", "avr_flip.h", "avr_graph.hip", "avr_graph_capi.hip",
    "avr_graph_host.h", "avr_boundary.h", "avr_fastdiv.h", "avr_image_kernels.h")] + [os.path.join(ROOT, "include", "avr.h")]
OUT = os.path.join(HERE, "libavr_hip.so")
OBJDIR = os.path.join(ROOT, "build", "obj")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# (medium kind, fast) per k_paths object: 0 GridMedium, 1 Homogeneous/Cloud, 3 NanoVDB, 4 RGB grid
KP_UNITS = [(m, f) for f in (0, 1) for m in (0, 1, 3, 4)]

# -ffp-contract=off: same float semantics as pbrt's CPU build (CMakeLists.txt:134-137),
# so a device sample replays the CPU oracle's sample.
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC",
         "-I" + os.path.join(ROOT, "include")]
# k_paths units' extra flags. Rounds 4-5 built them without MachineLICM (-mllvm
# -disable-machine-licm): the hoisted invariants did not fit 4 waves/SIMD next to the kernel
# arguments spilled to VGPR lanes. Since k_paths reloads its kernel arguments where it uses them
# (fresh_params, round 6: 126 -> 107 VGPRs), the hoisting fits (128 VGPRs, no scratch) and wins
# +0.6 % (profiles/r06_ab_walk.json). `python -m acceleratedvolrenderer_amd.build <variant>
# --no-licm` builds the old way.
KP_FLAGS = []
NO_LICM = ["-mllvm", "-disable-machine-licm"]
# RCCL for avr_film_reduce_rccl (in-process multi-GPU film reduce)
LIBS = ["-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]


def source_hash(defines=()):
    """sha256 over every source the library is built from, the compiler flags and the unit
    list: the library is rebuilt whenever this differs from the hash recorded next to it."""
    h = hashlib.sha256()
    for d in DEPS:
        h.update(os.path.basename(d).encode() + b"\0")
        with open(d, "rb") as f:
            h.update(f.read())
    h.update(repr((FLAGS, KP_FLAGS, LIBS, KP_UNITS, list(defines))).encode())
    return h.hexdigest()


def up_to_date():
    """True when libavr_hip.so exists and was built from exactly the current sources (the
    recorded source hash matches; file times alone can make a stale library look new)."""
    if not os.path.exists(OUT) or not os.path.exists(OUT + ".srchash"):
        return False
    with open(OUT + ".srchash") as f:
        return f.read().strip() == source_hash()


def _compile(args):
    src, obj, defs, verbose = args
    cmd = [HIPCC] + FLAGS + defs + ["-c", src, "-o", obj]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    return obj


def build(force=False, verbose=False, jobs=None, variant=None, defines=(), kp_flags=None):
    """Build the library. `variant` + `defines` (e.g. ["-DAVR_PATHS_WAVES_GRAY=4"]) build an
    experiment copy into variants/<variant>/libavr_hip.so instead (load it with AVR_LIB);
    `kp_flags` replaces the k_paths units' KP_FLAGS in such a copy."""
    out, objdir = OUT, OBJDIR
    if variant:
        out = os.path.join(ROOT, "variants", variant, "libavr_hip.so")
        objdir = os.path.join(ROOT, "variants", variant, "obj")
    elif not force and up_to_date():
        return OUT
    os.makedirs(objdir, exist_ok=True)
    defines = list(defines)
    units = [(SRC, os.path.join(objdir, "avr_capi.o"), ["-DAVR_KP_SPLIT"] + defines, verbose)]
    for med, fast in KP_UNITS:
        units.append((KPATHS, os.path.join(objdir, f"avr_kpaths_m{med}_f{fast}.o"),
                      (KP_FLAGS if kp_flags is None else list(kp_flags)) + [f"-DAVR_KP_MED={med}", f"-DAVR_KP_FAST={fast}"]
                      + defines, verbose))
    jobs = jobs or max(1, min(len(units), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4))))
    with ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(_compile, units))
    cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC"] + objs + ["-o", out + ".tmp"] + LIBS
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(out + ".tmp", out)
    with open(out + ".srchash", "w") as f:
        f.write(source_hash(defines) + "\n")
    return out


if __name__ == "__main__":
    import sys
    if len(sys.argv) > 1:   # python -m acceleratedvolrenderer_amd.build <variant> [--no-licm] -DNAME=VALUE ...
        print(build(verbose=True, variant=sys.argv[1], defines=[a for a in sys.argv[2:] if a != "--no-licm"],
                    kp_flags=NO_LICM if "--no-licm" in sys.argv[2:] else None))
    else:
        print(build(force=True, verbose=True))

"""Static ISA statistics of one k_paths instantiation (SGPR-spill reloads, hazard nops, totals).

usage: python tools/isa_stats.py [kernel-mangled-name-substring] [-D...]
Compiles csrc/avr_kpaths.hip (grid medium, replay) with --save-temps into /tmp/avr_isa."""
import os
import re
import subprocess
import sys
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from acceleratedvolrenderer_amd import build as B  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("-D") else \
        "_ZN3avr7k_pathsILb0ELb1ELi2ELi0ELb0ELb0EEEvNS_6ParamsE"
    defs = [a for a in sys.argv[1:] if a.startswith("-D")]
    out = "/tmp/avr_isa"
    os.makedirs(out, exist_ok=True)
    med = next((d.split("=")[1] for d in defs if d.startswith("-DAVR_KP_MED=")), "0")
    fast = next((d.split("=")[1] for d in defs if d.startswith("-DAVR_KP_FAST=")), "0")
    defs = [d for d in defs if not d.startswith(("-DAVR_KP_MED=", "-DAVR_KP_FAST="))]
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                           "-fPIC", "-I" + os.path.join(ROOT, "include"), *B.KP_FLAGS,   # the k_paths units' flags
                           f"-DAVR_KP_MED={med}", f"-DAVR_KP_FAST={fast}",
                           *defs, "--save-temps", "-c", os.path.join(ROOT, "acceleratedvolrenderer_amd", "csrc", "avr_kpaths.hip"),
                           "-o", os.path.join(out, "kp.o")], cwd=out, stderr=subprocess.DEVNULL)
    s = open(os.path.join(out, "avr_kpaths-hip-amdgcn-amd-amdhsa-gfx950.s")).read()
    i = s.index(name + ":")
    j = s.index(".Lfunc_end", i)
    ins = [l.strip().split()[0] for l in s[i:j].splitlines() if l.startswith("\t") and not l.strip().startswith((".", ";"))]
    c = Counter(ins)
    print(f"{name}: {len(ins)} instrs, v_readlane {c['v_readlane_b32']}, v_writelane {c['v_writelane_b32']}, "
          f"s_nop {c['s_nop']}, scratch ops {sum(v for k, v in c.items() if k.startswith('scratch_'))}")
    m = re.search(r"\.sgpr_count:\s+(\d+)", s[j:])
    v = re.search(r"\.vgpr_count:\s+(\d+)", s[j:])


if __name__ == "__main__":
    main()

"""Digest of the gfx950 ISA of every unit the library is built from (the eight k_paths objects
and the C-ABI unit), compiled with build.py's exact flags and --save-temps.

usage: python tools/isa_digest.py [out.json] [--root DIR] [-DNAME=VALUE ...]
Per unit: sha256 over the device assembly (comments and .file / .ident stripped) and, per
kernel symbol, sha256 over its instruction mnemonics in order (`ops`: register numbers,
immediates and LDS / kernel-argument offsets ignored) plus its instruction count. --root
compiles another checkout (e.g. a `git worktree` of the previous commit) with this tree's
flags. Used to show that removing measurement-only switches left the default kernels'
instruction streams unchanged."""
import hashlib
import json
import os
import re
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from acceleratedvolrenderer_amd import build as B  # noqa: E402


def unit_asm(args):
    src, flags, tag, tmp = args
    d = os.path.join(tmp, tag)
    os.makedirs(d, exist_ok=True)
    subprocess.check_call([B.HIPCC] + B.FLAGS + flags + ["--save-temps", "-c", src, "-o", os.path.join(d, "u.o")],
                          cwd=d, stderr=subprocess.DEVNULL)
    s = [f for f in os.listdir(d) if f.endswith("gfx950.s")]
    text = open(os.path.join(d, s[0])).read()
    keep = []
    for line in text.splitlines():
        t = line.strip()
        if not t or t.startswith(";") or t.startswith(".ident") or t.startswith(".file"):
            continue
        keep.append(re.sub(r"\s*;.*$", "", line))
    body = "\n".join(keep)
    nins = sum(1 for l in keep if l.startswith("\t") and not l.strip().startswith("."))
    kern = {}
    cur = None
    for l in keep:
        m = re.match(r"^(_Z\w+):\s*$", l)
        if m:
            cur = m.group(1)
            kern[cur] = []
        elif l.startswith(".Lfunc_end"):
            cur = None
        elif cur and l.startswith("\t") and not l.strip().startswith("."):
            kern[cur].append(l.split()[0])
    ops = {k: {"ops": hashlib.sha256(" ".join(v).encode()).hexdigest()[:16], "n": len(v)} for k, v in kern.items() if v}
    return tag, hashlib.sha256(body.encode()).hexdigest(), nins, ops


def main():
    argv = sys.argv[1:]
    out = next((a for a in argv if a.endswith(".json")), None)
    defs = [a for a in argv if a.startswith("-D")]
    root = argv[argv.index("--root") + 1] if "--root" in argv else ROOT
    csrc = os.path.join(root, "acceleratedvolrenderer_amd", "csrc")
    src, kpaths = os.path.join(csrc, "avr_capi.hip"), os.path.join(csrc, "avr_kpaths.hip")
    defs += ["-I" + os.path.join(root, "include")]
    units = [(src, ["-DAVR_KP_SPLIT"] + defs, "capi")]
    for med, fast in B.KP_UNITS:
        units.append((kpaths, B.KP_FLAGS + [f"-DAVR_KP_MED={med}", f"-DAVR_KP_FAST={fast}"] + defs, f"kp_m{med}_f{fast}"))
    with tempfile.TemporaryDirectory(prefix="avr_isa_") as tmp:
        with ThreadPoolExecutor(min(len(units), os.cpu_count() or 4)) as ex:
            res = list(ex.map(unit_asm, [(s, f, t, tmp) for s, f, t in units]))
    dig = {t: {"sha256": h, "instructions": n, "kernels": ops} for t, h, n, ops in res}
    for t, v in dig.items():
        print(f"{t:12s} {v['sha256'][:16]}  {v['instructions']} instrs")
    if out:
        json.dump(dig, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()

"""Per-kernel register / scratch / occupancy table from a hipcc -Rpass-analysis=kernel-resource-usage log.

usage: python tools/kres.py build.log [name-filter]"""
import re
import subprocess
import sys


def table(path, filt=""):
    rows, cur = [], None
    for line in open(path):
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        for key, pat in (("vgpr", r"VGPRs: (\d+)"), ("sgpr", r"TotalSGPRs: (\d+)"), ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"),
                         ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"), ("lds", r"LDS Size \[bytes/block\]: (\d+)")):
            m = re.search(pat, line)
            if m and cur is not None:
                cur[key] = int(m.group(1))
    names = [r["name"] for r in rows]
    dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.splitlines()
    for r, d in zip(rows, dem):
        if filt in d:
            print(f"{r.get('vgpr', '?'):>4} vgpr {r.get('sgpr', '?'):>4} sgpr {r.get('scratch', 0):>3} B scratch "
                  f"occ {r.get('occ', '?')} lds {r.get('lds', '?'):>6}  {d[:150]}")


if __name__ == "__main__":
    table(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")

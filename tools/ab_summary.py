"""Collect bench.py A/B lines (gpurun_out/.../ab_<tag>.json) into one summary JSON for profiles/.

usage: python tools/ab_summary.py out.json "title" dir:tag=description ...  [extra.json=key ...]"""
import json
import os
import sys


def line(path):
    d = json.load(open(path))
    de, r = d["detail"], d["roofline"]
    n = d["steps"]
    return {"Msamples_per_s": round(d["value"], 1), "ms_per_step": round(d["ms_per_step"], 3),
            "k_paths_ms": round(r["avg_launch_ms"], 3), "camera_ms": round(de["ms_camera"] / n, 3),
            "film_ms": round(de["ms_film"] / n, 3), "pixelsamples": d["config"].get("pixelsamples"),
            "grid_layout": d["config"].get("grid_layout"), "instantiation": r.get("instantiation")}


def main():
    out, title = sys.argv[1], sys.argv[2]
    res = {"title": title, "lines": {}, "extra": {}}
    for a in sys.argv[3:]:
        k, desc = a.split("=", 1)
        if k.endswith(".json"):
            res["extra"][desc] = json.load(open(k))
            continue
        d, tag = k.split(":")
        res["lines"][tag] = dict(description=desc, **line(os.path.join(d, f"ab_{tag}.json")))
    json.dump(res, open(out, "w"), indent=1)
    for t, v in res["lines"].items():
        print(f"{t:10s} {v['Msamples_per_s']:8.1f}  k_paths {v['k_paths_ms']:7.3f}  camera {v['camera_ms']:6.3f}  {v['description']}")


if __name__ == "__main__":
    main()

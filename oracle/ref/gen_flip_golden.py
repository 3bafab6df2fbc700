"""Golden FLIP error maps from the reference's own FLIP (src/ext/flip/flip.cpp, built
unmodified into oracle/_ref/flip_ref by oracle/ref/Makefile) — test infrastructure.
Writes tests/golden/flip_vectors.npz: per case the test / reference images (H, W, 3),
the ppd and the expected error map."""
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
EXE = os.path.join(REPO, "oracle", "_ref", "flip_ref")


def cases():
    rng = np.random.default_rng(7)
    h, w = 32, 40
    y, x = np.mgrid[0:h, 0:w]
    ref = np.stack([0.5 + 0.4 * np.sin(x / 5), 0.5 + 0.4 * np.cos(y / 4), (x * y) / (h * w)], 2)
    test = np.clip(ref + rng.normal(0, 0.05, ref.shape), 0, 1)
    yield "smooth_noise", test, ref, 0.0
    edges = np.zeros((h, w, 3))
    edges[:, w // 2:] = 0.9
    edges[h // 3: h // 3 + 3] = [0.2, 0.8, 0.1]
    yield "edges_ppd20", np.clip(edges + rng.normal(0, 0.02, edges.shape), 0, 1), edges, 20.0
    yield "identical", ref, ref, 0.0


def main():
    if not os.path.exists(EXE):
        subprocess.check_call(["make", "-s", "../_ref/flip_ref"], cwd=HERE)
    out = {}
    with tempfile.TemporaryDirectory() as d:
        for name, test, ref, ppd in cases():
            test = np.ascontiguousarray(test, np.float32)
            ref = np.ascontiguousarray(ref, np.float32)
            h, w = ref.shape[:2]
            test.tofile(os.path.join(d, "t.f32"))
            ref.tofile(os.path.join(d, "r.f32"))
            subprocess.check_call([EXE, os.path.join(d, "t.f32"), os.path.join(d, "r.f32"), str(w), str(h), repr(ppd),
                                   os.path.join(d, "o.f32")])
            out[name + "_test"] = test
            out[name + "_ref"] = ref
            out[name + "_ppd"] = np.float32(ppd)
            out[name + "_flip"] = np.fromfile(os.path.join(d, "o.f32"), np.float32).reshape(h, w)
    dst = os.path.join(REPO, "tests", "golden", "flip_vectors.npz")
    np.savez_compressed(dst, **out)
    print("wrote", dst, sorted(k for k in out if k.endswith("_flip")))


if __name__ == "__main__":
    sys.exit(main())

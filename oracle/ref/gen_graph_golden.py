"""Regenerate tests/golden/graph_vectors.json from the REAL reference (test infrastructure).

Builds oracle/_ref/graph_ref (oracle/ref/Makefile: our harness graph_ref.cpp over the
unmodified pbrt sources and the reference's vendored Eigen headers) and stores its output:
sphere GetHits results (graph/util.h:419-463 over pbrt's Sphere) and LightingCalculator
transport iterations (lighting_calculator.cpp:23-82 with Eigen). Float values are uint32 bits.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))


def main():
    if not os.path.isdir("/root/reference/src/pbrt"):
        sys.exit("reference sources not present; golden vectors are committed")
    subprocess.check_call(["make", "-s", "-j8"], cwd=HERE)
    out = subprocess.check_output([os.path.join(REPO, "oracle", "_ref", "graph_ref")])
    with open(os.path.join(REPO, "tests", "golden", "graph_vectors.json"), "wb") as f:
        f.write(out)
    print("wrote", len(out), "bytes")


if __name__ == "__main__":
    main()

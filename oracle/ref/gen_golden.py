"""Regenerate the golden vectors pinned against the REAL reference.

Test infrastructure only. Builds oracle/_ref/ref_harness from the unmodified
pbrt-v4 sources under /root/reference (oracle/ref/Makefile), runs it and writes
  tests/golden/ref_vectors.json                — golden vectors (uint32 float bits)
  acceleratedvolrenderer_amd/data/spectra_f32.bin — CIE 1931 x̄ȳz̄, D65 (471 each,
      360..830 nm), sRGB RGBFromXYZ (9), D65 photometric scale, CIE_Y_integral
The RGB -> spectrum goldens read the sRGB table that the reference's own rgb2spec_opt
writes into oracle/_ref (Makefile); the table stays there (not committed).
The spectral tables are published CIE / ITU data as the reference holds them;
they are inputs to the film, not code.
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
    exe = os.path.join(REPO, "oracle", "_ref", "ref_harness")
    tables = os.path.join(REPO, "acceleratedvolrenderer_amd", "data", "spectra_f32.bin")
    rgbtable = os.path.join(REPO, "oracle", "_ref", "srgb_table.inc")
    out = subprocess.check_output([exe, "--tables", tables, "--rgbtable", rgbtable])
    with open(os.path.join(REPO, "tests", "golden", "ref_vectors.json"), "wb") as f:
        f.write(out)
    print("wrote", len(out), "bytes of golden vectors and", os.path.getsize(tables), "bytes of tables")


if __name__ == "__main__":
    main()

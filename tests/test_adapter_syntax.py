"""The pbrt adapter (tools/adapter/mi355x_integrator.cpp) against pbrt's own
headers: with the documented accessor patch applied to temporary copies of media.h, film.h,
cameras.h, lights.h and filters.h (tools/adapter/pbrt_accessors.py), `g++ -fsyntax-only`
parses the adapter — its pbrt::Integrator subclass (cpu/integrators.h:34-77), every pbrt call
it makes and every avr_* call against include/avr.h. Nothing is built or run: NanoVDB, an
absent submodule that media.h includes, is replaced by declarations of the four names media.h
uses (SURVEY §8c's syntax shims). Skipped where the reference sources are absent (the GPU box)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/src"
sys.path.insert(0, os.path.join(ROOT, "tools", "adapter"))

NANOVDB_SHIM = {
    "nanovdb/NanoVDB.h": """#pragma once
#include <cstdint>
namespace nanovdb {
template <typename T> struct Vec3 {
    T v[3];
    Vec3() = default;
    Vec3(T x, T y, T z) : v{x, y, z} {}
    T operator[](int i) const { return v[i]; }
};
struct FloatTree {};
struct FloatGrid {
    using TreeType = FloatTree;
    template <typename V> V worldToIndexF(const V &p) const;
    const FloatTree &tree() const;
};
}  // namespace nanovdb
""",
    "nanovdb/util/GridHandle.h": """#pragma once
#include <nanovdb/NanoVDB.h>
namespace nanovdb {
template <typename BufferT> class GridHandle {
  public:
    template <typename T> const FloatGrid *grid(uint32_t n = 0) const;
};
}  // namespace nanovdb
""",
    "nanovdb/util/SampleFromVoxels.h": """#pragma once
#include <nanovdb/NanoVDB.h>
namespace nanovdb {
template <typename TreeT, int Order, bool UseCache> struct SampleFromVoxels {
    explicit SampleFromVoxels(const TreeT &);
    template <typename V> float operator()(const V &) const;
};
}  // namespace nanovdb
""",
}


def _tree(tmp_path):
    import pbrt_accessors
    shim = tmp_path / "shim"
    for rel, text in NANOVDB_SHIM.items():
        p = shim / rel
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_text(text)
    patched = tmp_path / "patched"
    pbrt_accessors.patch_headers(REF, str(patched))
    return shim, patched


def _syntax(src, shim, patched):
    cmd = ["g++", "-std=c++17", "-fsyntax-only", "-DPBRT_IS_LINUX", f"-I{patched}", f"-I{shim}", f"-I{REF}",
           f"-I{REF}/ext", f"-I{ROOT}/include", str(src)]
    return subprocess.run(cmd, capture_output=True, text=True)


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "pbrt")), reason="reference sources absent")
def test_adapter_parses_against_pbrt_headers(tmp_path):
    shim, patched = _tree(tmp_path)
    r = _syntax(os.path.join(ROOT, "tools", "adapter", "mi355x_integrator.cpp"), shim, patched)
    assert r.returncode == 0, r.stderr[-4000:]


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "pbrt")), reason="reference sources absent")
def test_adapter_check_is_not_vacuous(tmp_path):
    """The same check rejects the adapter without the accessor patch (pbrt's private members),
    and rejects a wrong avr_* argument list: it really parses both sides."""
    shim, patched = _tree(tmp_path)
    r = _syntax(os.path.join(ROOT, "tools", "adapter", "mi355x_integrator.cpp"), shim, tmp_path / "none")
    assert r.returncode != 0 and "SigmaASpec" in r.stderr
    bad = tmp_path / "bad.cpp"
    text = open(os.path.join(ROOT, "tools", "adapter", "mi355x_integrator.cpp")).read()
    bad.write_text(text.replace("avr_camera(ctx, camType, cfr, rfc)", "avr_camera(ctx, cfr, rfc)"))
    r = _syntax(bad, shim, patched)
    assert r.returncode != 0 and "avr_camera" in r.stderr

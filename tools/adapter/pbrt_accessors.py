"""The accessor patch of INTEGRATION.md §2a, applied to COPIES of pbrt's headers (never to
/root/reference, never committed): read accessors for the private members the adapter
(tools/adapter/mi355x_integrator.cpp) hands to the C-ABI, in the style of the accessors the
fork already added (media.h:460-461, 617-618), plus RGBFilm::AddPixelSums to merge the
device's fp64 sums. Each entry names a class and the member functions inserted right after
the first `public:` of its definition; the inserted lines are this repository's own code.

usage: python tools/adapter/pbrt_accessors.py <pbrt src dir> <out dir>   (writes <out>/pbrt/*.h)
"""
import os
import re
import sys

# header -> [(class name, accessor lines)]
ACCESSORS = {
    "media.h": [
        ("HGPhaseFunction", ["Float G() const { return g; }"]),
        ("GridMedium", [
            "const Bounds3f &Bounds() const { return bounds; }",
            "const Transform &RenderFromMedium() const { return renderFromMedium; }",
            "const SampledGrid<Float> &Density() const { return densityGrid; }",
            "const DenselySampledSpectrum &SigmaASpec() const { return sigma_a_spec; }",
            "const DenselySampledSpectrum &SigmaSSpec() const { return sigma_s_spec; }",
            "const DenselySampledSpectrum &LeSpec() const { return Le_spec; }",
            "const SampledGrid<Float> &LeScaleGrid() const { return LeScale; }",
            "const pstd::optional<SampledGrid<Float>> &TemperatureGrid() const { return temperatureGrid; }",
            "Float TemperatureScale() const { return temperatureScale; }",
            "Float TemperatureOffset() const { return temperatureOffset; }",
            "Float G() const { return phase.G(); }",
        ]),
        ("CloudMedium", [
            "const DenselySampledSpectrum &SigmaASpec() const { return sigma_a_spec; }",
            "const DenselySampledSpectrum &SigmaSSpec() const { return sigma_s_spec; }",
            "Float G() const { return phase.G(); }",
            "Float DensityScale() const { return density; }",
            "Float Wispiness() const { return wispiness; }",
            "Float Frequency() const { return frequency; }",
        ]),
    ],
    "film.h": [
        ("PixelSensor", [
            "const DenselySampledSpectrum &RBar() const { return r_bar; }",
            "const DenselySampledSpectrum &GBar() const { return g_bar; }",
            "const DenselySampledSpectrum &BBar() const { return b_bar; }",
            "Float ImagingRatio() const { return imagingRatio; }",
        ]),
        ("RGBFilm", [
            "Float MaxComponentValue() const { return maxComponentValue; }",
            "void AddPixelSums(Point2i p, const double rgb[3], double w) {",
            "    Pixel &px = pixels[p];",
            "    for (int c = 0; c < 3; ++c) px.rgbSum[c] += rgb[c];",
            "    px.weightSum += w;",
            "}",
        ]),
    ],
    "cameras.h": [
        ("ProjectiveCamera", ["const Transform &CameraFromRaster() const { return cameraFromRaster; }"]),
    ],
    "lights.h": [
        ("UniformInfiniteLight", [
            "DenselySampledSpectrum GetLEmit() {",
            "    DenselySampledSpectrum spectrum = *Lemit;",
            "    spectrum.Scale(scale);",
            "    return spectrum;",
            "}",
        ]),
    ],
    "filters.h": [
        ("GaussianFilter", ["Float Sigma() const { return sigma; }"]),
    ],
}


def patch_text(text, entries):
    """The header text with each class's accessors inserted after its first `public:`."""
    lines = text.split("\n")
    for cls, acc in entries:
        start = next((i for i, l in enumerate(lines) if re.match(rf"^class {cls}\b[^;]*$", l)), None)
        if start is None:
            raise ValueError(f"class {cls} not found")
        pub = next((i for i in range(start, min(start + 40, len(lines))) if lines[i].strip() == "public:"), None)
        if pub is None:
            raise ValueError(f"no public: in class {cls}")
        lines[pub + 1:pub + 1] = ["    // (adapter accessors, tools/adapter/pbrt_accessors.py)"] + ["    " + a for a in acc]
    return "\n".join(lines)


def patch_headers(src, out):
    """Copies of pbrt/<header> with the accessors, under <out>/pbrt/; returns the paths."""
    os.makedirs(os.path.join(out, "pbrt"), exist_ok=True)
    paths = []
    for h, entries in ACCESSORS.items():
        with open(os.path.join(src, "pbrt", h)) as f:
            text = f.read()
        p = os.path.join(out, "pbrt", h)
        with open(p, "w") as f:
            f.write(patch_text(text, entries))
        paths.append(p)
    return paths


if __name__ == "__main__":
    print("\n".join(patch_headers(sys.argv[1], sys.argv[2])))

// ref_harness.cpp — ORACLE TEST INFRASTRUCTURE (never shipped, never on the product path).
//
// Our own harness, compiled against the UNMODIFIED pbrt-v4 sources under
// /root/reference/src (AcceleratedVolRenderer fork) by oracle/ref/Makefile.
// It calls the reference's own numerics and prints golden vectors that pin
// the CPU restatement in oracle/volpath_oracle.cpp:
//   RNG (util/rng.h:25-160), Hash/MixBits (util/hash.h:19-106),
//   FastExp (util/math.h:450-471), SampleExponential / SampleDiscrete /
//   SampleVisibleWavelengths (util/sampling.h:79-225), SampleHenyeyGreenstein
//   (util/sampling.cpp:348-372), HenyeyGreenstein (util/scattering.h:49-58),
//   SampledGrid::Lookup/MaxValue (util/containers.h:765-870),
//   Bounds3::IntersectP (util/vecmath.h:1547-1571),
//   Transform::operator()/ApplyInverse(Ray) (util/transform.h:340-433),
//   IndependentSampler (samplers.h:442-476), ZSobolSampler (samplers.h:225-330),
//   SobolSample + FastOwenScrambler (util/lowdiscrepancy.h:168-237),
//   GaussianFilter / FilterSampler (filters.h:26-118, filters.cpp:133-147),
//   Noise/DNoise (util/noise.cpp),
//   Blackbody (util/spectrum.h:69-80), CIE/D65 tables (util/spectrum.cpp),
//   sRGB RGBFromXYZ (util/colorspace.cpp).
// Output: JSON on stdout (golden vectors) and, with --tables <file>, a raw
// little-endian float32 table file consumed by oracle/ref/gen_golden.py.
#include <pbrt/util/rng.h>
#include <pbrt/util/hash.h>
#include <pbrt/util/math.h>
#include <pbrt/util/containers.h>
#include <pbrt/util/vecmath.h>
#include <pbrt/util/sampling.h>
#include <pbrt/util/spectrum.h>
#include <pbrt/util/scattering.h>
#include <pbrt/util/transform.h>
#include <pbrt/util/noise.h>
#include <pbrt/util/colorspace.h>
#include <pbrt/util/image.h>
#include <pbrt/samplers.h>
#include <pbrt/filters.h>

#include <cstdio>
#include <cstring>
#include <vector>
#include <string>

using namespace pbrt;

// Reads the sRGB RGBToSpectrumTable data that the reference's rgb2spec_opt wrote
// (oracle/ref/Makefile): the 64 z nodes, then 3 x 64^3 x 3 coefficients.
static bool ReadRgbTable(const char *path, std::vector<float> &scale, std::vector<float> &data) {
    FILE *f = fopen(path, "rb");
    if (!f) return false;
    std::string text;
    char buf[1 << 16];
    size_t n;
    while ((n = fread(buf, 1, sizeof(buf), f)) > 0) text.append(buf, n);
    fclose(f);
    auto parse = [&](const char *marker, size_t count, std::vector<float> &out) {
        size_t pos = text.find(marker);
        if (pos == std::string::npos) return false;
        pos = text.find('=', pos) + 1;
        const char *c = text.c_str() + pos;
        while (out.size() < count && *c) {
            if ((*c >= '0' && *c <= '9') || *c == '-' || *c == '.') {
                char *end;
                out.push_back(strtof(c, &end));
                c = end;
            } else {
                ++c;
            }
        }
        return out.size() == count;
    };
    return parse("ToSpectrumTable_Scale", 64, scale) && parse("ToSpectrumTable_Data", 3 * 64 * 64 * 64 * 3, data);
}

static uint32_t fb(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }

struct J {
    bool first = true;
    void key(const char *k) { printf("%s\"%s\":", first ? "" : ",", k); first = false; }
};

static void arr_u32(const std::vector<uint32_t> &v) {
    printf("[");
    for (size_t i = 0; i < v.size(); ++i) printf("%s%u", i ? "," : "", v[i]);
    printf("]");
}
static void arr_u64(const std::vector<uint64_t> &v) {
    printf("[");
    for (size_t i = 0; i < v.size(); ++i) printf("%s\"%llu\"", i ? "," : "", (unsigned long long)v[i]);
    printf("]");
}

int main(int argc, char **argv) {
    Allocator alloc;
    Spectra::Init(alloc);
    const char *tablePath = nullptr, *rgbTablePath = nullptr;
    for (int i = 1; i < argc; ++i) {
        if (!strcmp(argv[i], "--tables") && i + 1 < argc) tablePath = argv[++i];
        if (!strcmp(argv[i], "--rgbtable") && i + 1 < argc) rgbTablePath = argv[++i];
    }

    printf("{");
    J j;

    // ---- RNG streams ------------------------------------------------------
    {
        j.key("rng");
        printf("[");
        const uint64_t seqs[][2] = {{0, 0}, {1, 2}, {12345, 678}, {0xdeadbeefcafeULL, 99}};
        for (int s = 0; s < 4; ++s) {
            RNG rng(seqs[s][0], seqs[s][1]);
            std::vector<uint32_t> u32, f32;
            for (int i = 0; i < 16; ++i) u32.push_back(rng.Uniform<uint32_t>());
            for (int i = 0; i < 8; ++i) f32.push_back(fb(rng.Uniform<float>()));
            rng.Advance(100000);
            std::vector<uint32_t> adv;
            for (int i = 0; i < 4; ++i) adv.push_back(rng.Uniform<uint32_t>());
            RNG r1(seqs[s][0]);  // single-arg SetSequence (MixBits seed)
            std::vector<uint32_t> single;
            for (int i = 0; i < 4; ++i) single.push_back(r1.Uniform<uint32_t>());
            printf("%s{\"seq\":\"%llu\",\"seed\":\"%llu\",\"u32\":", s ? "," : "",
                   (unsigned long long)seqs[s][0], (unsigned long long)seqs[s][1]);
            arr_u32(u32); printf(",\"f32\":"); arr_u32(f32);
            printf(",\"adv100000\":"); arr_u32(adv);
            printf(",\"single\":"); arr_u32(single); printf("}");
        }
        printf("]");
    }

    // ---- Hash -------------------------------------------------------------
    {
        j.key("hash_float");
        printf("[");
        const float fs[] = {0.f, 0.25f, 0.5f, 0.999f, 0.1234567f, 1e-7f, 0.75f};
        for (int i = 0; i < 7; ++i)
            printf("%s[%u,\"%llu\"]", i ? "," : "", fb(fs[i]), (unsigned long long)Hash(fs[i]));
        printf("]");
        j.key("hash_pixel_seed");
        printf("[");
        const int ps[][3] = {{0, 0, 0}, {1, 2, 0}, {511, 511, 0}, {17, 3, 7}, {1279, 719, 42}};
        for (int i = 0; i < 5; ++i)
            printf("%s[%d,%d,%d,\"%llu\"]", i ? "," : "", ps[i][0], ps[i][1], ps[i][2],
                   (unsigned long long)Hash(Point2i(ps[i][0], ps[i][1]), ps[i][2]));
        printf("]");
        j.key("hash_point3f");
        printf("[");
        const float pts[][3] = {{0.f, 0.f, 0.f}, {0.5f, 0.25f, -1.f}, {1e3f, -2.5f, 3.75f}};
        for (int i = 0; i < 3; ++i)
            printf("%s[%u,%u,%u,\"%llu\"]", i ? "," : "", fb(pts[i][0]), fb(pts[i][1]),
                   fb(pts[i][2]),
                   (unsigned long long)Hash(Point3f(pts[i][0], pts[i][1], pts[i][2])));
        printf("]");
        j.key("mixbits");
        std::vector<uint64_t> in{0, 1, 12345, 0xffffffffffffffffULL}, out;
        for (uint64_t v : in) out.push_back(MixBits(v));
        printf("{\"in\":"); arr_u64(in); printf(",\"out\":"); arr_u64(out); printf("}");
    }

    // ---- FastExp / SampleExponential / SampleDiscrete ----------------------
    {
        j.key("fastexp");
        std::vector<uint32_t> xs, ys;
        for (int i = 0; i <= 160; ++i) {
            float x = -20.f + 0.25f * i;
            xs.push_back(fb(x)); ys.push_back(fb(FastExp(x)));
        }
        const float extra[] = {-0.f, -87.f, -100.f, -1e-6f, -3.4028235e38f, 88.f, 1e-3f};
        for (float x : extra) { xs.push_back(fb(x)); ys.push_back(fb(FastExp(x))); }
        printf("{\"x\":"); arr_u32(xs); printf(",\"y\":"); arr_u32(ys); printf("}");

        j.key("sample_exponential");
        std::vector<uint32_t> us, as, ts;
        const float uu[] = {0.f, 0.1f, 0.5f, 0.9f, 0.99999994f, 0.3333f};
        const float aa[] = {0.5f, 1.f, 4.f, 123.456f};
        for (float u : uu)
            for (float a : aa) { us.push_back(fb(u)); as.push_back(fb(a)); ts.push_back(fb(SampleExponential(u, a))); }
        printf("{\"u\":"); arr_u32(us); printf(",\"a\":"); arr_u32(as); printf(",\"t\":"); arr_u32(ts); printf("}");

        j.key("sample_discrete");
        printf("[");
        const float w[][3] = {{0.2f, 0.5f, 0.3f}, {0.f, 1.f, 0.f}, {0.75f, 0.f, 0.25f}, {1.f, 1.f, 1e-8f}};
        const float ud[] = {0.f, 0.1f, 0.2f, 0.5f, 0.7f, 0.75f, 0.9f, 0.99999994f};
        bool f = true;
        for (int a = 0; a < 4; ++a)
            for (float u : ud) {
                int m = SampleDiscrete({w[a][0], w[a][1], w[a][2]}, u, nullptr, nullptr);
                printf("%s[%u,%u,%u,%u,%d]", f ? "" : ",", fb(w[a][0]), fb(w[a][1]), fb(w[a][2]), fb(u), m);
                f = false;
            }
        printf("]");
    }

    // ---- Wavelength sampling ----------------------------------------------
    {
        j.key("sample_visible");
        printf("[");
        for (int i = 0; i <= 32; ++i) {
            float u = i / 32.f;
            if (i == 32) u = 0.99999994f;
            SampledWavelengths l = SampledWavelengths::SampleVisible(u);
            SampledSpectrum pdf = l.PDF();
            printf("%s[%u,%u,%u,%u,%u,%u,%u,%u,%u]", i ? "," : "", fb(u), fb(l[0]), fb(l[1]),
                   fb(l[2]), fb(l[3]), fb(pdf[0]), fb(pdf[1]), fb(pdf[2]), fb(pdf[3]));
        }
        printf("]");
    }

    // SampledWavelengths::SampleUniform (spectrum.h:287-306): SpectralFilm::SampleWavelengths
    {
        j.key("sample_uniform");
        printf("[");
        const float ranges[][2] = {{360.f, 830.f}, {400.f, 700.f}, {380.f, 780.f}, {361.5f, 829.25f}};
        bool f = true;
        for (auto &r : ranges)
            for (int i = 0; i <= 32; ++i) {
                float u = i / 32.f;
                if (i == 32) u = 0.99999994f;
                SampledWavelengths l = SampledWavelengths::SampleUniform(u, r[0], r[1]);
                SampledSpectrum pdf = l.PDF();
                printf("%s[%u,%u,%u,%u,%u,%u,%u,%u,%u,%u,%u]", f ? "" : ",", fb(u), fb(r[0]), fb(r[1]), fb(l[0]),
                       fb(l[1]), fb(l[2]), fb(l[3]), fb(pdf[0]), fb(pdf[1]), fb(pdf[2]), fb(pdf[3]));
                f = false;
            }
        printf("]");
    }

    // ---- Henyey-Greenstein --------------------------------------------------
    {
        j.key("hg_eval");
        printf("[");
        const float gs[] = {0.f, 0.3f, -0.5f, 0.877f, 0.995f};
        bool f = true;
        for (float g : gs)
            for (int i = 0; i <= 8; ++i) {
                float c = -1.f + 0.25f * i;
                printf("%s[%u,%u,%u]", f ? "" : ",", fb(c), fb(g), fb(HenyeyGreenstein(c, g)));
                f = false;
            }
        printf("]");
        j.key("hg_sample");
        printf("[");
        f = true;
        const float wos[][3] = {{0.f, 0.f, 1.f}, {0.f, 0.f, -1.f}, {0.36f, -0.48f, 0.8f}, {-0.6f, 0.f, -0.8f}};
        const float us[][2] = {{0.1f, 0.2f}, {0.5f, 0.5f}, {0.9f, 0.05f}, {0.0f, 0.999f}};
        for (float g : gs)
            for (auto &wo : wos)
                for (auto &u : us) {
                    Float pdf;
                    Vector3f wi = SampleHenyeyGreenstein(Vector3f(wo[0], wo[1], wo[2]), g, Point2f(u[0], u[1]), &pdf);
                    printf("%s[%u,%u,%u,%u,%u,%u,%u,%u,%u,%u]", f ? "" : ",", fb(wo[0]), fb(wo[1]), fb(wo[2]),
                           fb(g), fb(u[0]), fb(u[1]), fb(wi.x), fb(wi.y), fb(wi.z), fb(pdf));
                    f = false;
                }
        printf("]");
    }

    // ---- SampledGrid --------------------------------------------------------
    {
        const int nx = 5, ny = 4, nz = 3;
        std::vector<float> v(nx * ny * nz);
        RNG rng(7, 11);
        for (auto &x : v) x = rng.Uniform<float>() * 3.f;
        SampledGrid<float> g(v, nx, ny, nz, alloc);
        j.key("grid");
        printf("{\"nx\":%d,\"ny\":%d,\"nz\":%d,\"values\":", nx, ny, nz);
        std::vector<uint32_t> vb; for (float x : v) vb.push_back(fb(x));
        arr_u32(vb);
        printf(",\"lookup\":[");
        for (int i = 0; i < 64; ++i) {
            Point3f p(rng.Uniform<float>() * 1.4f - 0.2f, rng.Uniform<float>() * 1.4f - 0.2f,
                      rng.Uniform<float>() * 1.4f - 0.2f);
            printf("%s[%u,%u,%u,%u]", i ? "," : "", fb(p.x), fb(p.y), fb(p.z), fb(g.Lookup(p)));
        }
        printf("],\"maxvalue\":[");
        for (int i = 0; i < 32; ++i) {
            Point3f a(rng.Uniform<float>(), rng.Uniform<float>(), rng.Uniform<float>());
            Point3f b(rng.Uniform<float>(), rng.Uniform<float>(), rng.Uniform<float>());
            Bounds3f bb(a, b);
            printf("%s[%u,%u,%u,%u,%u,%u,%u]", i ? "," : "", fb(bb.pMin.x), fb(bb.pMin.y), fb(bb.pMin.z),
                   fb(bb.pMax.x), fb(bb.pMax.y), fb(bb.pMax.z), fb(g.MaxValue(bb)));
        }
        printf("]}");

        // 16^3 majorant of a 20^3 grid exactly as GridMedium's ctor does it
        // (media.cpp:241-246 with MajorantGrid::VoxelBounds, media.h:123-127).
        const int n = 20;
        std::vector<float> w(n * n * n);
        for (auto &x : w) x = rng.Uniform<float>();
        SampledGrid<float> g2(w, n, n, n, alloc);
        j.key("majorant16");
        printf("{\"n\":%d,\"values\":", n);
        std::vector<uint32_t> wb; for (float x : w) wb.push_back(fb(x));
        arr_u32(wb);
        std::vector<uint32_t> mj;
        for (int z = 0; z < 16; ++z)
            for (int y = 0; y < 16; ++y)
                for (int x = 0; x < 16; ++x) {
                    Point3f p0(Float(x) / 16, Float(y) / 16, Float(z) / 16);
                    Point3f p1(Float(x + 1) / 16, Float(y + 1) / 16, Float(z + 1) / 16);
                    mj.push_back(fb(g2.MaxValue(Bounds3f(p0, p1))));
                }
        printf(",\"majorant\":"); arr_u32(mj); printf("}");
    }

    // ---- Bounds3::IntersectP -------------------------------------------------
    {
        j.key("intersectp");
        printf("[");
        RNG rng(3, 5);
        Bounds3f b(Point3f(-0.5f, 0.f, 1.f), Point3f(0.5f, 2.f, 1.25f));
        for (int i = 0; i < 48; ++i) {
            Point3f o(rng.Uniform<float>() * 4 - 2, rng.Uniform<float>() * 4 - 1, rng.Uniform<float>() * 4 - 1);
            Vector3f d(rng.Uniform<float>() * 2 - 1, rng.Uniform<float>() * 2 - 1, rng.Uniform<float>() * 2 - 1);
            if (i % 8 == 0) d.x = 0.f;
            float tMax = (i % 3 == 0) ? Infinity : 3.f;
            Float t0 = -1, t1 = -1;
            bool hit = b.IntersectP(o, d, tMax, &t0, &t1);
            printf("%s[%u,%u,%u,%u,%u,%u,%u,%d,%u,%u]", i ? "," : "", fb(o.x), fb(o.y), fb(o.z), fb(d.x),
                   fb(d.y), fb(d.z), fb(tMax), hit ? 1 : 0, fb(hit ? t0 : 0.f), fb(hit ? t1 : 0.f));
        }
        printf("]");
    }

    // ---- Transform (Ray) with interval-error origin offset ------------------
    {
        j.key("transform_ray");
        printf("[");
        Transform ts[3] = {
            Transform(SquareMatrix<4>(1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1)),
            Translate(Vector3f(-0.5f, 0.25f, 3.f)) * Scale(2.f, 2.f, 0.5f),
            Translate(Vector3f(1.f, -2.f, 0.5f)) * Rotate(30.f, Vector3f(0.f, 1.f, 0.f))};
        RNG rng(9, 1);
        bool f = true;
        for (int k = 0; k < 3; ++k) {
            SquareMatrix<4> m = ts[k].GetMatrix(), mi = ts[k].GetInverseMatrix();
            for (int i = 0; i < 8; ++i) {
                Point3f o(rng.Uniform<float>() * 4 - 2, rng.Uniform<float>() * 4 - 2, rng.Uniform<float>() * 4 - 2);
                Vector3f d(rng.Uniform<float>() * 2 - 1, rng.Uniform<float>() * 2 - 1, rng.Uniform<float>() * 2 - 1);
                Float tMaxF = 10.f, tMaxI = 10.f;
                Ray rf = ts[k](Ray(o, d), &tMaxF);
                Ray ri = ts[k].ApplyInverse(Ray(o, d), &tMaxI);
                printf("%s{\"m\":[", f ? "" : ",");
                for (int a = 0; a < 16; ++a) printf("%s%u", a ? "," : "", fb(m[a / 4][a % 4]));
                printf("],\"minv\":[");
                for (int a = 0; a < 16; ++a) printf("%s%u", a ? "," : "", fb(mi[a / 4][a % 4]));
                printf("],\"o\":[%u,%u,%u],\"d\":[%u,%u,%u]", fb(o.x), fb(o.y), fb(o.z), fb(d.x), fb(d.y), fb(d.z));
                printf(",\"fwd\":[%u,%u,%u,%u,%u,%u,%u]", fb(rf.o.x), fb(rf.o.y), fb(rf.o.z), fb(rf.d.x), fb(rf.d.y),
                       fb(rf.d.z), fb(tMaxF));
                printf(",\"inv\":[%u,%u,%u,%u,%u,%u,%u]}", fb(ri.o.x), fb(ri.o.y), fb(ri.o.z), fb(ri.d.x), fb(ri.d.y),
                       fb(ri.d.z), fb(tMaxI));
                f = false;
            }
        }
        printf("]");
    }

    // ---- IndependentSampler -------------------------------------------------
    {
        j.key("independent_sampler");
        printf("[");
        const int cases[][4] = {{0, 0, 0, 0}, {3, 7, 0, 0}, {3, 7, 5, 0}, {100, 200, 255, 42}, {511, 0, 1, 0}};
        for (int c = 0; c < 5; ++c) {
            IndependentSampler s(256, cases[c][3]);
            s.StartPixelSample(Point2i(cases[c][0], cases[c][1]), cases[c][2], 0);
            std::vector<uint32_t> v;
            for (int i = 0; i < 12; ++i) v.push_back(fb(s.Get1D()));
            IndependentSampler s2(256, cases[c][3]);
            s2.StartPixelSample(Point2i(cases[c][0], cases[c][1]), cases[c][2], 6);
            std::vector<uint32_t> v6;
            for (int i = 0; i < 3; ++i) v6.push_back(fb(s2.Get1D()));
            printf("%s{\"px\":%d,\"py\":%d,\"s\":%d,\"seed\":%d,\"dims\":", c ? "," : "", cases[c][0],
                   cases[c][1], cases[c][2], cases[c][3]);
            arr_u32(v); printf(",\"from_dim6\":"); arr_u32(v6); printf("}");
        }
        printf("]");
    }

    // ---- ZSobolSampler (samplers.h:225-330), FastOwen randomisation ---------
    // Call pattern per case: the dimension consumption of one VolPath sample (SURVEY
    // Appendix A): 1D (lambda), pixel 2D (filter), 1D (time), 2D (lens), then 1D x3 per
    // segment and 1D + 2D + 2D per scatter, repeated.
    {
        j.key("zsobol");
        printf("[");
        struct Case { int spp, resx, resy, px, py, s, seed; };
        const Case cases[] = {{16, 1280, 720, 0, 0, 0, 0},     {16, 1280, 720, 17, 5, 3, 0},
                              {16, 1280, 720, 1279, 719, 15, 0}, {16, 1280, 720, 640, 360, 7, 7},
                              {1, 1280, 720, 100, 200, 0, 0},    {2, 1280, 720, 100, 200, 1, 0},
                              {8, 1280, 720, 33, 44, 5, 3},      {64, 1920, 1080, 1919, 1079, 63, 0},
                              {256, 1280, 720, 321, 123, 200, 0}, {4, 32, 32, 31, 0, 2, 1},
                              // indices past 2^32 (config C5's 4096 spp at 720p and beyond)
                              {4096, 1280, 720, 1279, 719, 4095, 0}, {4096, 1280, 720, 640, 360, 1234, 0},
                              {8192, 1280, 720, 77, 700, 5000, 2}, {65536, 1920, 1080, 1500, 1000, 65535, 0},
                              {4096, 1920, 1080, 3, 1079, 17, 5}};
        const char *pattern = "1212111111221112211122";
        int ci = 0;
        for (const Case &c : cases) {
            ZSobolSampler zs(c.spp, Point2i(c.resx, c.resy), RandomizeStrategy::FastOwen, c.seed);
            zs.StartPixelSample(Point2i(c.px, c.py), c.s, 0);
            std::vector<uint32_t> v;
            for (const char *q = pattern; *q; ++q) {
                if (*q == '1') v.push_back(fb(zs.Get1D()));
                else { Point2f u = (q == pattern + 1) ? zs.GetPixel2D() : zs.Get2D(); v.push_back(fb(u.x)); v.push_back(fb(u.y)); }
            }
            printf("%s{\"spp\":%d,\"resx\":%d,\"resy\":%d,\"px\":%d,\"py\":%d,\"s\":%d,\"seed\":%d,\"pattern\":\"%s\",\"u\":",
                   ci++ ? "," : "", c.spp, c.resx, c.resy, c.px, c.py, c.s, c.seed, pattern);
            arr_u32(v);
            printf("}");
        }
        printf("]");
        // SobolSample(a, dim, FastOwenScrambler(seed)) for dims 0, 1 (the two ZSobol uses)
        j.key("sobol_fastowen");
        printf("[");
        RNG rng(5, 9);
        for (int i = 0; i < 96; ++i) {
            // 64 indices below 2^32, then 32 up to the 2^52 table limit (SobolMatrixSize 52)
            uint64_t a = i < 8 ? (uint64_t)i : (uint64_t)rng.Uniform<uint32_t>();
            if (i >= 64) a |= ((uint64_t)rng.Uniform<uint32_t>() & 0xfffffu) << 32;
            uint32_t seed = rng.Uniform<uint32_t>();
            printf("%s[\"%llu\",%u,%u,%u,%u,%u]", i ? "," : "", (unsigned long long)a, seed,
                   fb(SobolSample(a, 0, FastOwenScrambler(seed))), fb(SobolSample(a, 1, FastOwenScrambler(seed))),
                   fb(SobolSample(a, 0, NoRandomizer())), fb(SobolSample(a, 1, NoRandomizer())));
        }
        printf("]");
    }

    // ---- GaussianFilter sampling (filters.h:80-118, filters.cpp:133-147) -----
    {
        j.key("gaussian_filter");
        printf("[");
        const float cfg[][3] = {{1.5f, 1.5f, 0.5f}, {0.5f, 0.5f, 0.5f}, {2.f, 1.f, 0.75f}};
        RNG rng(11, 3);
        for (int c = 0; c < 3; ++c) {
            GaussianFilter gf(Vector2f(cfg[c][0], cfg[c][1]), cfg[c][2]);
            printf("%s{\"rx\":%u,\"ry\":%u,\"sigma\":%u,\"samples\":[", c ? "," : "", fb(cfg[c][0]), fb(cfg[c][1]),
                   fb(cfg[c][2]));
            for (int i = 0; i < 96; ++i) {
                Point2f u(rng.Uniform<Float>(), rng.Uniform<Float>());
                if (i == 0) u = Point2f(0.f, 0.f);
                if (i == 1) u = Point2f(0.99999994f, 0.99999994f);
                if (i == 2) u = Point2f(0.5f, 0.5f);
                FilterSample fs = gf.Sample(u);
                printf("%s[%u,%u,%u,%u,%u]", i ? "," : "", fb(u.x), fb(u.y), fb(fs.p.x), fb(fs.p.y), fb(fs.weight));
            }
            printf("]}");
        }
        printf("]");
    }

    // ---- Perlin noise (CloudMedium density generator inputs) ---------------
    {
        j.key("noise");
        printf("[");
        RNG rng(21, 4);
        for (int i = 0; i < 40; ++i) {
            Point3f p(rng.Uniform<float>() * 20 - 5, rng.Uniform<float>() * 20 - 5, rng.Uniform<float>() * 20 - 5);
            Vector3f dn = DNoise(p);
            printf("%s[%u,%u,%u,%u,%u,%u,%u]", i ? "," : "", fb(p.x), fb(p.y), fb(p.z), fb(Noise(p)), fb(dn.x),
                   fb(dn.y), fb(dn.z));
        }
        printf("]");
    }

    // ---- Blackbody ----------------------------------------------------------
    {
        j.key("blackbody");
        printf("[");
        const float Ts[] = {1000.f, 3000.f, 6500.f};
        const float ls[] = {360.f, 483.f, 600.f, 830.f};
        bool f = true;
        for (float T : Ts) {
            BlackbodySpectrum bb(T);
            for (float l : ls) {
                printf("%s[%u,%u,%u,%u]", f ? "" : ",", fb(T), fb(l), fb(Blackbody(l, T)), fb(bb(l)));
                f = false;
            }
        }
        printf("]");
    }

    // ---- Spectral tables ----------------------------------------------------
    {
        // sRGB as constructed in colorspace.cpp (primaries + stdillum-D65); the
        // RGB->spectrum table pointer is irrelevant to RGBFromXYZ.
        Spectrum d65 = GetNamedSpectrum("stdillum-D65");
        RGBColorSpace srgb(Point2f(.64, .33), Point2f(.3, .6), Point2f(.15, .06), d65, nullptr, alloc);
        DenselySampledSpectrum illum(d65, alloc);
        Float photometric = SpectrumToPhotometric(&illum);
        j.key("srgb_rgb_from_xyz");
        printf("[");
        for (int a = 0; a < 9; ++a) printf("%s%u", a ? "," : "", fb(srgb.RGBFromXYZ[a / 3][a % 3]));
        printf("]");
        j.key("d65_photometric");
        printf("%u", fb(photometric));
        j.key("d65_scale");
        printf("%u", fb(1.f / photometric));
        if (tablePath) {
            FILE *fp = fopen(tablePath, "wb");
            std::vector<float> t;
            for (int l = 360; l <= 830; ++l) t.push_back(Spectra::X()(l));
            for (int l = 360; l <= 830; ++l) t.push_back(Spectra::Y()(l));
            for (int l = 360; l <= 830; ++l) t.push_back(Spectra::Z()(l));
            for (int l = 360; l <= 830; ++l) t.push_back(illum(l));
            for (int a = 0; a < 9; ++a) t.push_back(srgb.RGBFromXYZ[a / 3][a % 3]);
            t.push_back(1.f / photometric);
            t.push_back(CIE_Y_integral);
            fwrite(t.data(), 4, t.size(), fp);
            fclose(fp);
        }
    }
    // ---- RGB -> spectrum (RGBGridMedium's grids) ----------------------------------
    // RGBToSpectrumTable::operator() (color.cpp:31-68) on the table rgb2spec_opt produced,
    // RGBSigmoidPolynomial eval / MaxValue (color.h:332-365), RGBUnboundedSpectrum and
    // RGBIlluminantSpectrum (spectrum.h:560-631, spectrum.cpp:236-247) in sRGB.
    std::vector<float> zNodes, coeffs;
    if (rgbTablePath && ReadRgbTable(rgbTablePath, zNodes, coeffs)) {
        RGBToSpectrumTable table(zNodes.data(), (const RGBToSpectrumTable::CoefficientArray *)coeffs.data());
        Spectrum d65 = GetNamedSpectrum("stdillum-D65");
        RGBColorSpace srgb(Point2f(.64, .33), Point2f(.3, .6), Point2f(.15, .06), d65, &table, alloc);
        const float ls[] = {360.f, 412.5f, 500.3f, 555.f, 611.7f, 700.f, 829.6f};
        std::vector<RGB> rgbs = {RGB(0, 0, 0), RGB(1, 1, 1), RGB(.5f, .5f, .5f), RGB(.25f, .25f, .25f),
                                 RGB(1, 0, 0), RGB(0, 1, 0), RGB(0, 0, 1), RGB(.9f, .1f, .3f),
                                 RGB(.2f, .7f, .4f), RGB(.05f, .02f, .9f), RGB(1e-4f, 2e-4f, 3e-4f)};
        RNG rng(77, 5);
        for (int i = 0; i < 40; ++i)
            rgbs.push_back(RGB(rng.Uniform<float>(), rng.Uniform<float>(), rng.Uniform<float>()));
        j.key("rgb_table");   // rgb in [0,1]: [r,g,b, rsp(l) x 7, MaxValue]
        printf("[");
        for (size_t i = 0; i < rgbs.size(); ++i) {
            RGBSigmoidPolynomial rsp = table(rgbs[i]);
            printf("%s[%u,%u,%u", i ? "," : "", fb(rgbs[i].r), fb(rgbs[i].g), fb(rgbs[i].b));
            for (float l : ls) printf(",%u", fb(rsp(l)));
            printf(",%u]", fb(rsp.MaxValue()));
        }
        printf("]");
        // unbounded / illuminant: rgb scaled past 1
        j.key("rgb_unbounded");   // [r,g,b, s(l) x 7, MaxValue]
        printf("[");
        for (size_t i = 0; i < rgbs.size(); ++i) {
            RGB c = rgbs[i] * (i % 3 == 0 ? 7.5f : (i % 3 == 1 ? 0.3f : 1.f));
            RGBUnboundedSpectrum s(srgb, c);
            printf("%s[%u,%u,%u", i ? "," : "", fb(c.r), fb(c.g), fb(c.b));
            for (float l : ls) printf(",%u", fb(s(l)));
            printf(",%u]", fb(s.MaxValue()));
        }
        printf("]");
        j.key("rgb_illuminant");   // [r,g,b, s(l) x 7]
        printf("[");
        for (size_t i = 0; i < rgbs.size(); ++i) {
            RGB c = rgbs[i] * (i % 2 ? 3.f : 1.f);
            RGBIlluminantSpectrum s(srgb, c);
            printf("%s[%u,%u,%u", i ? "," : "", fb(c.r), fb(c.g), fb(c.b));
            for (float l : ls) printf(",%u", fb(s(l)));
            printf("]");
        }
        printf("]");
    }
    // ---- ImageInfiniteLight pieces ---------------------------------------------
    // EqualAreaSquareToSphere / EqualAreaSphereToSquare (util/math.cpp:292-361),
    // RemapPixelCoords with WrapMode::OctahedralSphere (util/image.h:96-123),
    // PiecewiseConstant2D Sample / PDF (util/sampling.h:698-779)
    {
        RNG rng(31, 7);
        j.key("equal_area");   // [u, v, x, y, z, u', v'] with (u', v') = SphereToSquare(x, y, z)
        printf("[");
        std::vector<Point2f> pts = {{0, 0}, {1, 1}, {0.5f, 0.5f}, {0, 1}, {1, 0}, {0.25f, 0.75f}, {0.5f, 0}};
        for (int i = 0; i < 60; ++i) pts.push_back({rng.Uniform<float>(), rng.Uniform<float>()});
        for (size_t i = 0; i < pts.size(); ++i) {
            Vector3f w = EqualAreaSquareToSphere(pts[i]);
            Point2f q = EqualAreaSphereToSquare(w);
            printf("%s[%u,%u,%u,%u,%u,%u,%u]", i ? "," : "", fb(pts[i].x), fb(pts[i].y), fb(w.x), fb(w.y), fb(w.z),
                   fb(q.x), fb(q.y));
        }
        printf("]");
        j.key("equal_area_dirs");   // [x, y, z, u, v] for normalised random directions
        printf("[");
        for (int i = 0; i < 60; ++i) {
            Vector3f d = Normalize(Vector3f(rng.Uniform<float>() * 2 - 1, rng.Uniform<float>() * 2 - 1,
                                            rng.Uniform<float>() * 2 - 1));
            Point2f q = EqualAreaSphereToSquare(d);
            printf("%s[%u,%u,%u,%u,%u]", i ? "," : "", fb(d.x), fb(d.y), fb(d.z), fb(q.x), fb(q.y));
        }
        printf("]");
        j.key("octahedral_wrap");   // [res, x, y, x', y']
        printf("[");
        bool f = true;
        for (int res : {1, 8}) {
            for (int x = -2; x <= res + 1; ++x)
                for (int y = -2; y <= res + 1; ++y) {
                    Point2i pp(x, y);
                    RemapPixelCoords(&pp, Point2i(res, res), WrapMode::OctahedralSphere);
                    printf("%s[%d,%d,%d,%d,%d]", f ? "" : ",", res, x, y, pp.x, pp.y);
                    f = false;
                }
        }
        printf("]");
        // a 7 x 5 function with a zero row and zero entries
        const int nu = 7, nv = 5;
        std::vector<Float> func(nu * nv);
        for (int i = 0; i < nu * nv; ++i) func[i] = (i / nu == 2) ? 0.f : (i % 3 == 0 ? 0.f : rng.Uniform<float>() * 3);
        PiecewiseConstant2D d2(func, nu, nv);
        j.key("pc2d_func");
        printf("[");
        for (int i = 0; i < nu * nv; ++i) printf("%s%u", i ? "," : "", fb(func[i]));
        printf("]");
        j.key("pc2d_sample");   // [u0, u1, x, y, pdf, PDF(x, y)]
        printf("[");
        for (int i = 0; i < 50; ++i) {
            Point2f u(rng.Uniform<float>(), rng.Uniform<float>());
            Float pdf;
            Point2f q = d2.Sample(u, &pdf);
            printf("%s[%u,%u,%u,%u,%u,%u]", i ? "," : "", fb(u.x), fb(u.y), fb(q.x), fb(q.y), fb(pdf), fb(d2.PDF(q)));
        }
        printf("]");
    }
    printf("}\n");
    return 0;
}

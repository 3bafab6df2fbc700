"""The device's pixel-sample generation (acceleratedvolrenderer_amd/csrc/avr_sampling.h),
compiled for the host, against the golden vectors of the reference itself: ZSobolSampler
streams (samplers.h:225-330) and SobolSample with FastOwen scrambling for the two Sobol'
dimensions ZSobol uses (lowdiscrepancy.h:168-237; here computed without the matrix table)."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def hdr(tmp_path_factory):
    d = tmp_path_factory.mktemp("smp")
    src = d / "shim.cpp"
    src.write_text(
        "#define AVR_HD inline\n"
        f'#include "{ROOT}/acceleratedvolrenderer_amd/csrc/avr_sampling.h"\n'
        "using namespace avr::smp;\n"
        'extern "C" {\n'
        "void zs(int spp, int rx, int ry, int px, int py, int s, int seed, const char *pat, float *out) {\n"
        "  ZSobolParams zp = zsobol_params(spp, rx, ry, seed); ZSobol z; z.start(px, py, s, zp);\n"
        "  for (; *pat; ++pat) { if (*pat == '1') *out++ = z.get1d(zp); else { z.get2d(zp, out, out + 1); out += 2; } }\n"
        "}\n"
        "int zs_split(int spp, int rx, int ry, int dmax, int n, const int *q, unsigned long long *full,\n"
        "             unsigned long long *tab) {\n"
        "  ZSobolParams zp = zsobol_params(spp, rx, ry, 0);\n"
        "  size_t rows = (size_t)encode_morton2(rx - 1, ry - 1) + 1;\n"
        "  unsigned *t = new unsigned[rows * dmax];\n"
        "  for (int y = 0; y < ry; ++y) for (int x = 0; x < rx; ++x) for (int d = 0; d < dmax; ++d) {\n"
        "    unsigned pm = (unsigned)encode_morton2(x, y); t[(size_t)pm * dmax + d] = zsobol_upper(pm, d, zp); }\n"
        "  for (int i = 0; i < n; ++i) {\n"
        "    unsigned long long m = (encode_morton2(q[4 * i], q[4 * i + 1]) << zp.log2spp) | (unsigned)q[4 * i + 2];\n"
        "    ZSobolParams zt = zp; zt.upper = t; zt.dmax = dmax;\n"
        "    if (zsobol_wide(zp)) { full[i] = zsobol_index<unsigned long long>(m, q[4 * i + 3], zp);\n"
        "      tab[i] = zsobol_index<unsigned long long>(m, q[4 * i + 3], zt); }\n"
        "    else { full[i] = zsobol_index<unsigned>((unsigned)m, q[4 * i + 3], zp);\n"
        "      tab[i] = zsobol_index<unsigned>((unsigned)m, q[4 * i + 3], zt); } }\n"
        "  delete[] t; return zsobol_split(zp); }\n"
        "void zs_pass(int spp, int rx, int ry, int n, const int *q, unsigned long long *full,\n"
        "             unsigned long long *pass) {\n"
        "  ZSobolParams zp = zsobol_params(spp, rx, ry, 0);\n"
        "  for (int i = 0; i < n; ++i) {\n"
        "    const int *r = q + 6 * i; int base = r[4], S = r[5], plo = 0;\n"
        "    while ((base >> plo) != ((base + S - 1) >> plo)) ++plo;\n"
        "    unsigned pm = (unsigned)encode_morton2(r[0], r[1]); unsigned d = (unsigned)r[3];\n"
        "    unsigned long long mb = ((unsigned long long)pm << zp.log2spp) | (unsigned)base;\n"
        "    unsigned long long ms = ((unsigned long long)pm << zp.log2spp) | (unsigned)r[2];\n"
        "    unsigned up = zsobol_upper(pm, d, zp);\n"
        "    ZSobolParams zt = zp; zt.plo = plo;\n"
        "    if (zsobol_wide(zp)) { full[i] = zsobol_index<unsigned long long>(ms, d, zp);\n"
        "      pass[i] = zsobol_index_pass<unsigned long long>(ms, d, zt, zsobol_pass_entry<unsigned long long>(mb, d, zp, plo, up)); }\n"
        "    else { full[i] = zsobol_index<unsigned>((unsigned)ms, d, zp);\n"
        "      pass[i] = zsobol_index_pass<unsigned>((unsigned)ms, d, zt, zsobol_pass_entry<unsigned>((unsigned)mb, d, zp, plo, up)); } } }\n"
        "int zperm_bytes_check() {\n"
        "  unsigned char t[24]; const unsigned long long W[3] = {kZPermW0, kZPermW1, kZPermW2};\n"
        "  for (int p = 0; p < 24; ++p) t[p] = (unsigned char)(W[p >> 3] >> ((p & 7) * 8));\n"
        "  int bad = 0; for (unsigned p = 0; p < 24; ++p) for (unsigned d = 0; d < 4; ++d)\n"
        "    bad += zperm_t(t, p, d) != zperm(p, d) || zperm_t(nullptr, p, d) != zperm(p, d);\n"
        "  for (unsigned p = 0; p < 24; ++p) { unsigned m = 0; for (unsigned d = 0; d < 4; ++d) m |= 1u << zperm(p, d);\n"
        "    bad += m != 15u; }\n"
        "  return bad; }\n"
        "int zs_pass_from(int spp, int rx, int ry, int n, const int *q) {\n"
        "  ZSobolParams zp = zsobol_params(spp, rx, ry, 0); int bad = 0;\n"
        "  for (int i = 0; i < n; ++i) {\n"
        "    const int *r = q + 6 * i; int base = r[4], S = r[5], plo = 0;\n"
        "    while ((base >> plo) != ((base + S - 1) >> plo)) ++plo;\n"
        "    if (plo + 2 > zp.log2spp) continue;\n"
        "    unsigned pm = (unsigned)encode_morton2(r[0], r[1]); unsigned d = (unsigned)r[3];\n"
        "    unsigned long long mb = ((unsigned long long)pm << zp.log2spp) | (unsigned)base;\n"
        "    unsigned up = zsobol_upper(pm, d, zp);\n"
        "    if (zsobol_wide(zp)) bad += zsobol_pass_entry_from<unsigned long long>(mb, d, zp, plo,\n"
        "        zsobol_pass_entry<unsigned long long>(mb, d, zp, plo + 2, up)) != zsobol_pass_entry<unsigned long long>(mb, d, zp, plo, up);\n"
        "    else bad += zsobol_pass_entry_from<unsigned>((unsigned)mb, d, zp, plo,\n"
        "        zsobol_pass_entry<unsigned>((unsigned)mb, d, zp, plo + 2, up)) != zsobol_pass_entry<unsigned>((unsigned)mb, d, zp, plo, up); }\n"
        "  return bad; }\n"
        "int fi_check(const float *cdf, int n, int nu, const float *u) {\n"
        "  unsigned char g[kFilterGuideK + 1]; filter_guide_build(cdf, n, g); int bad = 0;\n"
        "  for (int i = 0; i < nu; ++i) bad += find_interval_guided(cdf, n, g, u[i]) != find_interval(cdf, n, u[i]);\n"
        "  return bad; }\n"
        "static void pcb(const float *f, int n, float mn, float mx, float *cdf, float *fi) {\n"
        "  cdf[0] = 0; for (int i = 1; i <= n; ++i) cdf[i] = cdf[i - 1] + __builtin_fabsf(f[i - 1]) * (mx - mn) / n;\n"
        "  *fi = cdf[n]; if (*fi == 0) for (int i = 1; i <= n; ++i) cdf[i] = float(i) / float(n);\n"
        "  else for (int i = 1; i <= n; ++i) cdf[i] /= *fi; }\n"
        "int fs_check(int nx, int ny, float rx, float ry, const float *f, int nu, const float *u) {\n"
        "  float *cc = new float[ny * (nx + 1)], *ci = new float[ny], *mc = new float[ny + 1], mi;\n"
        "  for (int y = 0; y < ny; ++y) pcb(f + y * nx, nx, -rx, rx, cc + y * (nx + 1), ci + y);\n"
        "  pcb(ci, ny, -ry, ry, mc, &mi);\n"
        "  unsigned char *g = new unsigned char[(ny + 1) * (kFilterGuideK + 1)]; float *w = new float[nx * ny];\n"
        "  for (int y = 0; y < ny; ++y) filter_guide_build(cc + y * (nx + 1), nx, g + y * (kFilterGuideK + 1));\n"
        "  filter_guide_build(mc, ny, g + ny * (kFilterGuideK + 1));\n"
        "  for (int y = 0; y < ny; ++y) for (int x = 0; x < nx; ++x) w[y * nx + x] = filter_cell_weight(f, ci, mi, nx, y, x);\n"
        "  FilterTables a{nx, ny, rx, ry, f, cc, ci, mc, mi, nullptr, nullptr}, b = a; b.guide = g; b.wt = w;\n"
        "  int bad = 0;\n"
        "  for (int i = 0; i < nu; ++i) { float p[3], q[3];\n"
        "    gaussian_filter_sample(a, u[2 * i], u[2 * i + 1], p, p + 1, p + 2);\n"
        "    gaussian_filter_sample(b, u[2 * i], u[2 * i + 1], q, q + 1, q + 2);\n"
        "    bad += __builtin_memcmp(p, q, sizeof p) != 0; }\n"
        "  delete[] cc; delete[] ci; delete[] mc; delete[] g; delete[] w; return bad; }\n"
        "float sob(unsigned long long a, int dim, unsigned seed, int scr) {\n"
        "  unsigned v = sobol_bits64((unsigned)a, (unsigned)(a >> 32), dim);\n"
        "  return u32_to_unit(scr ? fast_owen(v, seed) : v); }\n"
        "}\n")
    so = d / "shim.so"
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-shared", "-fPIC", str(src), "-o", str(so)])
    L = ctypes.CDLL(str(so))
    L.zs.argtypes = [ctypes.c_int] * 7 + [ctypes.c_char_p, ctypes.POINTER(ctypes.c_float)]
    L.zs_split.restype = ctypes.c_int
    L.sob.restype = ctypes.c_float
    L.sob.argtypes = [ctypes.c_ulonglong, ctypes.c_int, ctypes.c_uint, ctypes.c_int]
    return L


def test_header_zsobol_streams_match_reference(hdr, golden):
    for c in golden["zsobol"]:
        n = sum(1 if ch == "1" else 2 for ch in c["pattern"])
        out = np.zeros(n, np.float32)
        hdr.zs(c["spp"], c["resx"], c["resy"], c["px"], c["py"], c["s"], c["seed"], c["pattern"].encode(),
               out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
        assert out.view(np.uint32).tolist() == c["u"], c


def test_header_sobol_bits_match_reference(hdr, golden):
    for a, seed, f0, f1, p0, p1 in golden["sobol_fastowen"]:
        a = int(a)
        got = [hdr.sob(a, 0, seed, 1), hdr.sob(a, 1, seed, 1), hdr.sob(a, 0, 0, 0), hdr.sob(a, 1, 0, 0)]
        assert np.array(got, np.float32).view(np.uint32).tolist() == [f0, f1, p0, p1]


@pytest.mark.parametrize("spp,rx,ry", [(1, 37, 21), (2, 37, 21), (16, 37, 21), (128, 37, 21), (256, 37, 21),
                                        (4096, 1280, 720), (8192, 300, 200), (65536, 1100, 900)])
def test_zsobol_pixel_table_split(hdr, spp, rx, ry):
    """GetSampleIndex = (pixel-only digits, tabulated per Morton(pixel) x dimension) | (sample
    digits): identical to the untabulated index, including dimensions past the table, for
    32-bit and (4096 spp at 720p and up) 64-bit indices."""
    rng = np.random.default_rng(spp)
    dmax, n = 12, 4000
    q = np.stack([rng.integers(0, rx, n), rng.integers(0, ry, n), rng.integers(0, spp, n),
                  rng.integers(0, 2 * dmax, n)], 1).astype(np.int32)
    full = np.zeros(n, np.uint64)
    tab = np.zeros(n, np.uint64)
    U = ctypes.POINTER(ctypes.c_ulonglong)
    split = hdr.zs_split(spp, rx, ry, dmax, n, q.ctypes.data_as(ctypes.POINTER(ctypes.c_int)),
                         full.ctypes.data_as(U), tab.ctypes.data_as(U))
    assert np.array_equal(full, tab)
    assert split == (int(np.log2(spp)) + (int(np.log2(spp)) & 1)) // 2


@pytest.mark.parametrize("spp,rx,ry", [(1, 37, 21), (2, 37, 21), (8, 37, 21), (128, 37, 21), (256, 37, 21),
                                        (2048, 1280, 720), (16384, 1280, 720), (8192, 300, 200), (65536, 1100, 900)])
def test_zsobol_pass_table(hdr, spp, rx, ry):
    """The per-pass table (avr_set_sampler_pass_table): a pass of S sample indices from `base`
    shares the digits above its lowest differing bits (and the permutation of the digit just
    below); the index rebuilt from its entry plus the digits computed per draw equals the
    untabulated GetSampleIndex for every sample of the pass — aligned passes (the bench's 64),
    unaligned ranges straddling digit boundaries, single indices and whole-pixel passes."""
    rng = np.random.default_rng(spp + 7)
    n = 6000
    rows = []
    for _ in range(n):
        S = int(rng.choice([1, 2, 3, 4, 16, 64, 100, spp]))
        S = min(S, spp)
        if rng.random() < 0.5 and spp % S == 0:
            base = int(rng.integers(0, spp // S)) * S            # aligned pass
        else:
            base = int(rng.integers(0, spp - S + 1))             # any range
        s = base + int(rng.integers(0, S))
        rows.append((int(rng.integers(0, rx)), int(rng.integers(0, ry)), s, int(rng.integers(0, 40)), base, S))
    q = np.array(rows, np.int32)
    full = np.zeros(n, np.uint64)
    pas = np.zeros(n, np.uint64)
    U = ctypes.POINTER(ctypes.c_ulonglong)
    hdr.zs_pass(spp, rx, ry, n, q.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), full.ctypes.data_as(U),
                pas.ctypes.data_as(U))
    assert np.array_equal(full, pas)
    # the two-level build: the entry for plo from the one for plo + 2 (built once per 4 passes)
    assert hdr.zs_pass_from(spp, rx, ry, n, q.ctypes.data_as(ctypes.POINTER(ctypes.c_int))) == 0


def _pc1d_cdf(f, lo, hi):
    """pc1d_build in float32, in the host build's operation order"""
    n = len(f)
    cdf = np.zeros(n + 1, np.float32)
    w = np.float32(hi) - np.float32(lo)
    for i in range(1, n + 1):
        cdf[i] = np.float32(cdf[i - 1] + np.float32(np.float32(abs(f[i - 1])) * w) / np.float32(n))
    tot = cdf[n]
    if tot == 0:
        return np.array([np.float32(i) / np.float32(n) for i in range(n + 1)], np.float32)
    return (cdf / tot).astype(np.float32)


def test_filter_guided_find_interval_identical(hdr):
    """The camera stage's guided FindInterval (a 128-bucket guide per CDF) returns the binary
    search's interval for every u: Gaussian-filter rows, random CDFs with empty cells and ties,
    an all-zero function (cdf = i / n), n = 1 .. 128; u at every CDF value and its neighbours,
    at every bucket edge k / 128 and its neighbours, and at random points (plus u = 1 and
    negative u, which take the full search)."""
    rng = np.random.default_rng(5)
    F = ctypes.POINTER(ctypes.c_float)
    x = (np.arange(48, dtype=np.float32) + np.float32(0.5)) / np.float32(48)
    g = np.maximum(0, np.exp(-((-1.5 + 3 * x) ** 2) / 0.5) - np.exp(-4.5)).astype(np.float32)
    cases = [g, g * np.float32(1e-3), np.outer(g, g)[7]]
    for n in (1, 2, 3, 7, 48, 64, 127, 128):
        f = rng.random(n).astype(np.float32)
        f[rng.random(n) < 0.3] = 0
        cases.append(f)
        cases.append(np.zeros(n, np.float32))
        cases.append(np.round(rng.random(n) * 3).astype(np.float32))   # ties
    edges = np.arange(129, dtype=np.float32) / np.float32(128)
    for f in cases:
        cdf = _pc1d_cdf(f, -1.5, 1.5)
        pts = np.concatenate([cdf, edges]).astype(np.float32)
        u = np.concatenate([pts, np.nextafter(pts, np.float32(2)), np.nextafter(pts, np.float32(-1)),
                            rng.random(4000).astype(np.float32), np.array([0, np.nextafter(np.float32(1), np.float32(0)), 1, -0.25], np.float32)])
        u = np.ascontiguousarray(u.astype(np.float32))
        assert hdr.fi_check(cdf.ctypes.data_as(F), len(f), len(u), u.ctypes.data_as(F)) == 0, len(f)


@pytest.mark.parametrize("r,sigma", [(1.5, 0.5), (0.5, 0.5), (2.0, 0.3), (1.0, 1.0)])
def test_filter_guided_weighted_sample_identical(hdr, r, sigma):
    """GaussianFilter::Sample through the camera stage's tables (128-bucket guides + the cell
    weights f / (pdf0 pdf1) evaluated on the host) returns the point and weight of the plain
    binary-search, divide-per-sample path bit for bit: pbrt's default radius and others, random
    u pairs plus u at 0 and just below 1."""
    n = int(32 * r)
    x = (np.arange(n, dtype=np.float32) + np.float32(0.5)) / np.float32(n)
    p = ((np.float32(1) - x) * np.float32(-r) + x * np.float32(r)).astype(np.float32)
    g1 = np.maximum(0, np.exp(-p.astype(np.float64) ** 2 / (2 * sigma ** 2)) - np.exp(-r * r / (2 * sigma ** 2)))
    f = np.ascontiguousarray(np.outer(g1, g1).astype(np.float32))
    rng = np.random.default_rng(3)
    u = rng.random((20000, 2)).astype(np.float32)
    u[:4] = [[0, 0], [0, np.nextafter(np.float32(1), np.float32(0))], [np.nextafter(np.float32(1), np.float32(0)), 0.5],
             [0.5, 0.5]]
    u = np.ascontiguousarray(u)
    F = ctypes.POINTER(ctypes.c_float)
    hdr.fs_check.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_float, F, ctypes.c_int, F]
    assert hdr.fs_check(n, n, r, r, f.ctypes.data_as(F), len(u), u.ctypes.data_as(F)) == 0


def test_zperm_byte_table(hdr):
    """The 24-byte permutation table the camera stage and k_paths stage in LDS (zperm_t) gives
    zperm's digit for every permutation and digit, and every entry is a permutation of 0..3."""
    assert hdr.zperm_bytes_check() == 0

// FLIP (Andersson et al., HPG 2020) as the reference vendors it for `imgtool diff --metric
// FLIP` (src/ext/flip/flip.cpp:470-1110): per-pixel colour transforms, the CSF spatial filter
// in YCxCz, Hunt-adjusted L*a*b* HyAB colour difference, edge / point feature detectors on
// the achromatic channel, error = cdiff^(1 - fdiff). Standalone (no HIP headers): the device
// kernels (k_flip_*) and the host-compiled tests share these functions; every convolution sums
// its taps in the reference's order (rows, then columns), borders replicated.
#pragma once

#include <algorithm>
#include <cmath>
#include <vector>

#ifndef AVR_HD
#define AVR_HD __host__ __device__ __forceinline__
#endif

#include "avr_canon.h"

namespace avr {
namespace flip {

// powf: on the host the libm the reference links; on the device exp(y log x) in f64 by the
// canonical sequences of avr_canon.h, rounded once (the correctly rounded float except within
// ~1e-16 of a midpoint), which is what a faithful host powf returns for these inputs.
AVR_HD float pow_(float x, float y) {
#if defined(__HIP_DEVICE_COMPILE__)
    if (y == 0.0f) return 1.0f;
    if (x == 0.0f) return 0.0f;   // y > 0 on every call site
    return (float)canon::exp_d((double)y * canon::log_d((double)x));
#else
    return powf(x, y);
#endif
}

constexpr float kQc = 0.7f, kPc = 0.4f, kPt = 0.95f, kW = 0.082f, kQf = 0.5f;
constexpr float kIllX = 0.950428545377181f, kIllY = 1.0f, kIllZ = 1.088900370798128f;   // D65

struct C3 { float x, y, z; };

AVR_HD float srgb2lin(float c) { return c <= 0.04045f ? c / 12.92f : pow_((c + 0.055f) / 1.055f, 2.4f); }

AVR_HD C3 lin2xyz(C3 v) {
    const float a11 = 10135552.0f / 24577794.0f, a12 = 8788810.0f / 24577794.0f, a13 = 4435075.0f / 24577794.0f;
    const float a21 = 2613072.0f / 12288897.0f, a22 = 8788810.0f / 12288897.0f, a23 = 887015.0f / 12288897.0f;
    const float a31 = 1425312.0f / 73733382.0f, a32 = 8788810.0f / 73733382.0f, a33 = 70074185.0f / 73733382.0f;
    return {a11 * v.x + a12 * v.y + a13 * v.z, a21 * v.x + a22 * v.y + a23 * v.z, a31 * v.x + a32 * v.y + a33 * v.z};
}
AVR_HD C3 xyz2lin(C3 v) {
    const float a11 = 3.241003232976358f, a12 = -1.537398969488785f, a13 = -0.498615881996363f;
    const float a21 = -0.969224252202516f, a22 = 1.875929983695176f, a23 = 0.041554226340085f;
    const float a31 = 0.055639419851975f, a32 = -0.204011206123910f, a33 = 1.057148977187533f;
    return {a11 * v.x + a12 * v.y + a13 * v.z, a21 * v.x + a22 * v.y + a23 * v.z, a31 * v.x + a32 * v.y + a33 * v.z};
}
AVR_HD C3 xyz2ycxcz(C3 v) {
    const float x = v.x / kIllX, y = v.y / kIllY, z = v.z / kIllZ;
    return {116.0f * y - 16.0f, 500.0f * (x - y), 200.0f * (y - z)};
}
AVR_HD C3 ycxcz2xyz(C3 v) {
    const float Yy = (v.x + 16.0f) / 116.0f, Cx = v.y / 500.0f, Cz = v.z / 200.0f;
    return {(Yy + Cx) * kIllX, Yy * kIllY, (Yy - Cz) * kIllZ};
}
AVR_HD float lab_f(float t) { return t > 0.008856 ? pow_(t, 1.0f / 3.0f) : 7.787f * t + 16.0f / 116.0f; }
AVR_HD C3 xyz2lab(C3 v) {
    const float x = fabsf(v.x) / kIllX, y = fabsf(v.y) / kIllY, z = fabsf(v.z) / kIllZ;
    const float fx = lab_f(x), fy = lab_f(y), fz = lab_f(z);
    return {116.0f * fy - 16.0f, 500.0f * (fx - fy), 200.0f * (fy - fz)};
}
AVR_HD float hunt(float l, float c) { return 0.01f * l * c; }
AVR_HD float hyab(C3 a, C3 b) {
    return fabsf(a.x - b.x) + sqrtf((a.y - b.y) * (a.y - b.y) + (a.z - b.z) * (a.z - b.z));
}
AVR_HD float fmin_(float a, float b) { return b < a ? b : a; }   // std::min
AVR_HD float fmax_(float a, float b) { return a < b ? b : a; }   // std::max

// sRGB pixel -> YCxCz (computeFLIPError's first loop)
AVR_HD C3 to_ycxcz(C3 s) { return xyz2ycxcz(lin2xyz({srgb2lin(s.x), srgb2lin(s.y), srgb2lin(s.z)})); }

// preprocess after the CSF convolution: YCxCz -> XYZ -> linear RGB clamped to [0,1] -> XYZ -> Lab,
// then the Hunt adjustment
AVR_HD C3 to_lab_hunt(C3 f) {
    C3 l = xyz2lin(ycxcz2xyz(f));
    l = {fmax_(fmin_(l.x, 1.0f), 0.0f), fmax_(fmin_(l.y, 1.0f), 0.0f), fmax_(fmin_(l.z, 1.0f), 0.0f)};
    const C3 lab = xyz2lab(lin2xyz(l));
    return {lab.x, hunt(lab.x, lab.y), hunt(lab.x, lab.z)};
}

// colour difference of two preprocessed pixels (computeColorDifference), cmax from computeMaxDistance
AVR_HD float color_diff(C3 ref, C3 test, float cmax) {
    const float pccmax = kPc * cmax;
    float e = pow_(hyab(ref, test), kQc);
    if (e < pccmax) e *= kPt / pccmax;
    else e = kPt + ((e - pccmax) / (cmax - pccmax)) * (1.0f - kPt);
    return e;
}

// feature difference from the four detector responses (computeFeatureDifference)
AVR_HD float feature_diff(float ex_r, float ey_r, float ex_t, float ey_t, float px_r, float py_r, float px_t,
                          float py_t) {
    const float eR = sqrtf(ex_r * ex_r + ey_r * ey_r), eT = sqrtf(ex_t * ex_t + ey_t * ey_t);
    const float pR = sqrtf(px_r * px_r + py_r * py_r), pT = sqrtf(px_t * px_t + py_t * py_t);
    const float nf = 1.0f / sqrtf(2.0f);
    return pow_(nf * fmax_(fabsf(eR - eT), fabsf(pR - pT)), kQf);
}

// A pixel's YCxCz (x, y, z) and achromatic channel (Y + 16) / 116 (w), as k_flip_prep stores it
struct F4 { float x, y, z, w; };
AVR_HD F4 prep_pixel(float r, float g, float b) {
    const C3 c = to_ycxcz({r, g, b});
    return {c.x, c.y, c.z, (c.x + 16.0f) / 116.0f};
}

// The FLIP error of pixel (x, y): both CSF convolutions (spatial filter sf, radius rs, 3
// weights per tap), Lab + Hunt, colour difference; the edge / point detector responses (ef, pf,
// radius rd, 2 weights per tap) of both achromatic channels; cdiff^(1 - fdiff).
AVR_HD float error_at(const F4 *ycT, const F4 *ycR, int w, int h, int x, int y, const float *sf, int rs,
                      const float *ef, const float *pf, int rd, float cmax) {
    const int sw = 2 * rs + 1, dw = 2 * rd + 1;
    C3 sR = {0.0f, 0.0f, 0.0f}, sT = {0.0f, 0.0f, 0.0f};
    for (int iy = -rs; iy <= rs; iy++) {
        const int yy = y + iy < 0 ? 0 : (y + iy > h - 1 ? h - 1 : y + iy);
        for (int ix = -rs; ix <= rs; ix++) {
            const int xx = x + ix < 0 ? 0 : (x + ix > w - 1 ? w - 1 : x + ix);
            const float *wt = sf + 3 * ((iy + rs) * sw + (ix + rs));
            const F4 r = ycR[yy * w + xx], t = ycT[yy * w + xx];
            sR = {sR.x + wt[0] * r.x, sR.y + wt[1] * r.y, sR.z + wt[2] * r.z};
            sT = {sT.x + wt[0] * t.x, sT.y + wt[1] * t.y, sT.z + wt[2] * t.z};
        }
    }
    const float cd = color_diff(to_lab_hunt(sR), to_lab_hunt(sT), cmax);
    float exR = 0.0f, eyR = 0.0f, exT = 0.0f, eyT = 0.0f, pxR = 0.0f, pyR = 0.0f, pxT = 0.0f, pyT = 0.0f;
    for (int iy = -rd; iy <= rd; iy++) {
        const int yy = y + iy < 0 ? 0 : (y + iy > h - 1 ? h - 1 : y + iy);
        for (int ix = -rd; ix <= rd; ix++) {
            const int xx = x + ix < 0 ? 0 : (x + ix > w - 1 ? w - 1 : x + ix);
            const int k = 2 * ((iy + rd) * dw + (ix + rd));
            const float cR = ycR[yy * w + xx].w, cT = ycT[yy * w + xx].w;
            exR = exR + ef[k] * cR;
            eyR = eyR + ef[k + 1] * cR;
            exT = exT + ef[k] * cT;
            eyT = eyT + ef[k + 1] * cT;
            pxR = pxR + pf[k] * cR;
            pyR = pyR + pf[k + 1] * cR;
            pxT = pxT + pf[k] * cT;
            pyT = pyT + pf[k + 1] * cT;
        }
    }
    const float fd = feature_diff(exR, eyR, exT, eyT, pxR, pyR, pxT, pyT);
    return pow_(cd, 1.0f - fd);
}

// ---- host side: filters and the max distance (generateSpatialFilter, generateDetectionFilters,
// computeMaxDistance), built with the host libm exactly as the reference builds them
inline float ppd_default() { return 0.7f * (3840.0f / 0.7f) * (float(M_PI) / 180.0f); }   // calculatePPD

inline float gauss_sum(float x2, float a1, float b1, float a2, float b2) {
    const float pi = float(M_PI), pi_sq = float(M_PI * M_PI);
    return a1 * sqrtf(pi / b1) * expf(-pi_sq * x2 / b1) + a2 * sqrtf(pi / b2) * expf(-pi_sq * x2 / b2);
}

// spatial filter: (2r+1)^2 taps x 3 channels, normalised per channel
inline int spatial_filter(float ppd, std::vector<float> &w) {
    const float deltaX = 1.0f / ppd, pi_sq = float(M_PI * M_PI);
    const C3 a1 = {1.0f, 1.0f, 34.1f}, b1 = {0.0047f, 0.0053f, 0.04f}, a2 = {0.0f, 0.0f, 13.5f},
             b2 = {1.0e-5f, 1.0e-5f, 0.025f};
    const float maxScale = std::max(std::max(std::max(b1.x, b1.y), std::max(b1.z, b2.x)), std::max(b2.y, b2.z));
    const int radius = int(std::ceil(3.0f * sqrtf(maxScale / (2.0f * pi_sq)) * ppd));
    const int width = 2 * radius + 1;
    w.assign((size_t)width * width * 3, 0.f);
    C3 sum = {0.0f, 0.0f, 0.0f};
    for (int y = 0; y < width; y++) {
        const float iy = (y - radius) * deltaX;
        for (int x = 0; x < width; x++) {
            const float ix = (x - radius) * deltaX;
            const float dist2 = ix * ix + iy * iy;
            const C3 v = {gauss_sum(dist2, a1.x, b1.x, a2.x, b2.x), gauss_sum(dist2, a1.y, b1.y, a2.y, b2.y),
                          gauss_sum(dist2, a1.z, b1.z, a2.z, b2.z)};
            float *o = &w[3 * ((size_t)y * width + x)];
            o[0] = v.x; o[1] = v.y; o[2] = v.z;
            sum = {sum.x + v.x, sum.y + v.y, sum.z + v.z};
        }
    }
    for (size_t i = 0; i < (size_t)width * width; ++i) {
        w[3 * i] /= sum.x;
        w[3 * i + 1] /= sum.y;
        w[3 * i + 2] /= sum.z;
    }
    return radius;
}

// edge (point = false) or point detector: (2r+1)^2 taps x 2 components (x, y)
inline int detection_filter(float ppd, bool point, std::vector<float> &w) {
    const float stdDev = 0.5f * kW * ppd;
    const int radius = int(std::ceil(3.0f * stdDev));
    const int width = 2 * radius + 1;
    w.assign((size_t)width * width * 2, 0.f);
    float negX = 0.0f, posX = 0.0f, negY = 0.0f, posY = 0.0f;
    for (int y = 0; y < width; y++) {
        const int yy = y - radius;
        for (int x = 0; x < width; x++) {
            const int xx = x - radius;
            const float G = expf(-(float(xx) * float(xx) + float(yy) * float(yy)) / (2.0f * stdDev * stdDev));
            float wx, wy;
            if (point) {
                wx = (float(xx) * float(xx) / (stdDev * stdDev) - 1.0f) * G;
                wy = (float(yy) * float(yy) / (stdDev * stdDev) - 1.0f) * G;
            } else {
                wx = -float(xx) * G;
                wy = -float(yy) * G;
            }
            w[2 * ((size_t)y * width + x)] = wx;
            w[2 * ((size_t)y * width + x) + 1] = wy;
            if (wx > 0.0f) posX += wx; else negX += -wx;
            if (wy > 0.0f) posY += wy; else negY += -wy;
        }
    }
    for (size_t i = 0; i < (size_t)width * width; ++i) {
        const float px = w[2 * i], py = w[2 * i + 1];
        w[2 * i] = px / (px > 0.0f ? posX : negX);
        w[2 * i + 1] = py / (py > 0.0f ? posY : negY);
    }
    return radius;
}

inline float max_distance() {   // computeMaxDistance
    const C3 g = xyz2lab(lin2xyz({0.0f, 1.0f, 0.0f})), b = xyz2lab(lin2xyz({0.0f, 0.0f, 1.0f}));
    const C3 gh = {g.x, hunt(g.x, g.y), hunt(g.x, g.z)}, bh = {b.x, hunt(b.x, b.y), hunt(b.x, b.z)};
    return powf(hyab(gh, bh), kQc);
}

}  // namespace flip
}  // namespace avr

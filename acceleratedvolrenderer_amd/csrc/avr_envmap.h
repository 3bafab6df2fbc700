// ImageInfiniteLight pieces shared by the device kernels and the host-compiled tests
// (lights.h:552-640, lights.cpp:1007-1052): the equal-area square <-> sphere mapping
// (util/math.cpp:292-361), nearest-pixel lookup with the octahedral wrap (util/image.h:96-123,
// 353-357) and PiecewiseConstant2D over [0,1]^2 (util/sampling.h:698-779). Standalone (no HIP
// headers); sin/cos follow the canonical convention of avr_canon.h.
#pragma once

#include <cstddef>
#include <cstdint>

#include "avr_canon.h"
#include "avr_sampling.h"

namespace avr {
namespace env {

AVR_HD float copysign_(float mag, float sgn) { return __builtin_copysignf(mag, sgn); }
AVR_HD float safe_sqrt_(float x) { return __builtin_sqrtf(x > 0.f ? x : 0.f); }

// EqualAreaSquareToSphere (util/math.cpp:292-315)
AVR_HD void square_to_sphere(float px, float py, float *ox, float *oy, float *oz) {
    const float u = 2 * px - 1, v = 2 * py - 1;
    const float up = __builtin_fabsf(u), vp = __builtin_fabsf(v);
    const float signedDistance = 1 - (up + vp);
    const float d = __builtin_fabsf(signedDistance);
    const float r = 1 - d;
    const float phi = (r == 0 ? 1 : (vp - up) / r + 1) * 3.14159265358979323846f / 4;
    const float z = copysign_(1 - r * r, signedDistance);
    float s, c;
    canon::sincos_f(phi, &s, &c);
    const float cosPhi = copysign_(c, u), sinPhi = copysign_(s, v);
    *ox = cosPhi * r * safe_sqrt_(2 - r * r);
    *oy = sinPhi * r * safe_sqrt_(2 - r * r);
    *oz = z;
}

// EqualAreaSphereToSquare (util/math.cpp:317-361): atan by a 6th-degree minimax polynomial
// evaluated with FMA (EvaluatePolynomial, util/math.h)
AVR_HD void sphere_to_square(float dx, float dy, float dz, float *ou, float *ov) {
    const float x = __builtin_fabsf(dx), y = __builtin_fabsf(dy), z = __builtin_fabsf(dz);
    const float r = safe_sqrt_(1 - z);
    const float a = x < y ? y : x;   // std::max(x, y)
    float b = y < x ? y : x;         // std::min(x, y)
    b = a == 0 ? 0 : b / a;
    // double literals rounded to float, as `const Float t1 = 0.40...e-5;` does
    const float t1 = (float)0.406758566246788489601959989e-5, t2 = (float)0.636226545274016134946890922156,
                t3 = (float)0.61572017898280213493197203466e-2, t4 = (float)-0.247333733281268944196501420480,
                t5 = (float)0.881770664775316294736387951347e-1, t6 = (float)0.419038818029165735901852432784e-1,
                t7 = (float)-0.251390972343483509333252996350e-1;
    float phi = __builtin_fmaf(b, __builtin_fmaf(b, __builtin_fmaf(b, __builtin_fmaf(b, __builtin_fmaf(b,
                __builtin_fmaf(b, t7, t6), t5), t4), t3), t2), t1);
    if (x < y) phi = 1 - phi;
    float v = phi * r;
    float u = r - v;
    if (dz < 0) {
        const float t = u;
        u = v;
        v = t;
        u = 1 - u;
        v = 1 - v;
    }
    u = copysign_(u, dx);
    v = copysign_(v, dy);
    *ou = 0.5f * (u + 1);
    *ov = 0.5f * (v + 1);
}

// Image::LookupNearestChannel(p, c, WrapMode::OctahedralSphere) pixel index
AVR_HD int octahedral_pixel(float u, float v, int res) {
    int px = (int)(u * res), py = (int)(v * res);
    if (px < 0) {
        px = -px;
        py = res - 1 - py;
    } else if (px >= res) {
        px = 2 * res - 1 - px;
        py = res - 1 - py;
    }
    if (py < 0) {
        px = res - 1 - px;
        py = -py;
    } else if (py >= res) {
        px = res - 1 - px;
        py = 2 * res - 1 - py;
    }
    if (res == 1) px = py = 0;
    return py * res + px;
}

// PiecewiseConstant2D over the domain [0,1]^2 (tables laid out as smp::FilterTables:
// f[ny*nx] | ccdf[ny*(nx+1)] | cint[ny] | mcdf[ny+1])
struct Distrib2D {
    int nx, ny;
    const float *f, *ccdf, *cint, *mcdf;
    float mint;
};
AVR_HD void distrib_sample(const Distrib2D &D, float u0, float u1, float *su, float *sv, float *pdf) {
    float pdf1, pdf0;
    int v, uo;
    *sv = smp::pc1d_sample(D.mcdf, D.cint, D.ny, D.mint, 0.f, 1.f, u1, &pdf1, &v);
    *su = smp::pc1d_sample(D.ccdf + (size_t)v * (D.nx + 1), D.f + (size_t)v * D.nx, D.nx, D.cint[v], 0.f, 1.f, u0,
                           &pdf0, &uo);
    *pdf = pdf0 * pdf1;
}
AVR_HD float distrib_pdf(const Distrib2D &D, float u, float v) {   // Bounds2f(0,1).Offset(p) = p
    int iu = (int)(u * D.nx), iv = (int)(v * D.ny);
    iu = iu < 0 ? 0 : (iu > D.nx - 1 ? D.nx - 1 : iu);
    iv = iv < 0 ? 0 : (iv > D.ny - 1 ? D.ny - 1 : iv);
    return D.f[(size_t)iv * D.nx + iu] / D.mint;
}

}  // namespace env
}  // namespace avr

// Canonical transcendentals for the path's float libm calls (log, atanh, sin/cos, cosh).
//
// pbrt calls the float overloads of std::log / atanh / sin / cos / cosh (sampling.h:163-171,
// 222-225; vecmath.h:1666). Their last-ulp results are platform-specific. This header fixes
// one convention instead: each function is evaluated in f64 by a fixed sequence of IEEE
// operations (+ - * / and fma, all correctly rounded on CPU and GPU), accurate to a few f64
// ulps, then rounded once to float. The result is the correctly rounded float except when
// the true value lies within ~1e-16 (relative) of a rounding midpoint. The oracle's
// "canonical" libm mode restates the same sequences (oracle/volpath_oracle.cpp), so device
// and oracle agree bit for bit by construction.
//
// Cheaper than ocml's f64 routines (which carry double-double internals): log ~30 f64 ops,
// sincos ~35, for the inputs this path produces (log: (0, 1]; atanh: (-1, 1);
// sincos: [0, 2pi); cosh: |x| < 3).
#pragma once

#include <cmath>
#include <cstdint>
#include <cstring>

#ifndef AVR_HD
#define AVR_HD __host__ __device__ __forceinline__
#endif

namespace avr {
namespace canon {

AVR_HD uint64_t dbits(double x) { uint64_t b; memcpy(&b, &x, 8); return b; }
AVR_HD double dfrom(uint64_t b) { double x; memcpy(&x, &b, 8); return x; }

// f64 polynomial coefficients. On the device each one is materialised at its use by a
// volatile s_mov_b32 pair (SALU, operand of the v_fma_f64): left to itself the compiler
// hoists every f64 constant of the kernel into VGPRs for its whole lifetime (~40 VGPRs in
// the path kernel) and spills. On the host: the plain literal.
#if defined(__HIP_DEVICE_COMPILE__)
template <uint64_t B>
__device__ __forceinline__ double kd() {
    uint32_t lo, hi;
    asm volatile("s_mov_b32 %0, %2\n\ts_mov_b32 %1, %3"
                 : "=s"(lo), "=s"(hi)
                 : "i"((uint32_t)(B & 0xffffffffu)), "i"((uint32_t)(B >> 32)));
    return dfrom(((uint64_t)hi << 32) | lo);
}
#define AVR_KD(bits, value) (::avr::canon::kd<bits>())
#else
#define AVR_KD(bits, value) (value)
#endif

// 2*atanh(s)/(2s) = 1 + z/3 + z^2/5 + ... + z^11/23 with z = s^2 (|s| <= 0.1716, z^12/25 < 2e-20)
AVR_HD double atanh_series(double z) {
    double p = AVR_KD(0x3fa642c8590b2164ull, 0x1.642c8590b2164p-5);
    p = fma(p, z, AVR_KD(0x3fa8618618618618ull, 0x1.8618618618618p-5));
    p = fma(p, z, AVR_KD(0x3faaf286bca1af28ull, 0x1.af286bca1af28p-5));
    p = fma(p, z, AVR_KD(0x3fae1e1e1e1e1e1eull, 0x1.e1e1e1e1e1e1ep-5));
    p = fma(p, z, AVR_KD(0x3fb1111111111111ull, 0x1.1111111111111p-4));
    p = fma(p, z, AVR_KD(0x3fb3b13b13b13b14ull, 0x1.3b13b13b13b14p-4));
    p = fma(p, z, AVR_KD(0x3fb745d1745d1746ull, 0x1.745d1745d1746p-4));
    p = fma(p, z, AVR_KD(0x3fbc71c71c71c71cull, 0x1.c71c71c71c71cp-4));
    p = fma(p, z, AVR_KD(0x3fc2492492492492ull, 0x1.2492492492492p-3));
    p = fma(p, z, AVR_KD(0x3fc999999999999aull, 0x1.999999999999ap-3));
    p = fma(p, z, AVR_KD(0x3fd5555555555555ull, 0x1.5555555555555p-2));
    p = fma(p, z, 1.0);
    return p;
}

constexpr double kLn2Hi = 0x1.62e42fee00000p-1;    // 32 significant bits: k * kLn2Hi is exact
constexpr double kLn2Lo = 0x1.a39ef35793c76p-33;
constexpr double kSqrt2 = 0x1.6a09e667f3bcdp+0;
constexpr double kPio2Hi = 0x1.921fb54400000p+0;   // 33 significant bits
constexpr double kPio2Lo = 0x1.0b4611a626331p-34;
constexpr double kTwoOverPi = 0x1.45f306dc9c883p-1;
constexpr double kInvLn2 = 0x1.71547652b82fep+0;

// log(x) for a positive normal f64 (every float converts to one); 0 -> -inf, <0/NaN -> NaN
AVR_HD double log_d(double x) {
    if (!(x > 0)) return x == 0 ? -__builtin_inf() : __builtin_nan("");
    if (x == __builtin_inf()) return x;
    const uint64_t b = dbits(x);
    int e = (int)((b >> 52) & 0x7ff) - 1023;
    double m = dfrom((b & 0x000fffffffffffffull) | 0x3ff0000000000000ull);   // [1, 2)
    if (m > kSqrt2) { m = m * 0.5; e += 1; }   // [sqrt(1/2), sqrt(2)]
    const double s = (m - 1.0) / (m + 1.0);
    const double t = 2.0 * s * atanh_series(s * s);
    const double de = (double)e;
    return fma(de, AVR_KD(0x3fe62e42fee00000ull, 0x1.62e42fee00000p-1), fma(de, AVR_KD(0x3dea39ef35793c76ull, 0x1.a39ef35793c76p-33), t));
}

AVR_HD double atanh_d(double x) {   // |x| < 1
    const double ax = x < 0 ? -x : x;
    if (ax <= 0.171) return x * atanh_series(x * x);
    return 0.5 * log_d((1.0 + x) / (1.0 - x));
}

// sin and cos for |x| < 2^19 (two-part Cody-Waite reduction by pi/2)
AVR_HD void sincos_d(double x, double *sn, double *cs) {
    const double kf = __builtin_rint(x * AVR_KD(0x3fe45f306dc9c883ull, 0x1.45f306dc9c883p-1));
    const double r = (x - kf * AVR_KD(0x3ff921fb54400000ull, 0x1.921fb54400000p+0)) - kf * AVR_KD(0x3dd0b4611a626331ull, 0x1.0b4611a626331p-34);
    const double z = r * r;
    // sin r = r (1 - z/3! + ... - z^7/15!), cos r = 1 - z (1/2! - z/4! + ... - z^7/16!):
    // truncation below 5e-17 (relative) for |r| <= pi/4
    double ps = AVR_KD(0xbd6ae7f3e733b81full, -0x1.ae7f3e733b81fp-41);   // -1/15!
    ps = fma(ps, z, AVR_KD(0x3de6124613a86d09ull, 0x1.6124613a86d09p-33));   // 1/13!
    ps = fma(ps, z, AVR_KD(0xbe5ae64567f544e4ull, -0x1.ae64567f544e4p-26));   // -1/11!
    ps = fma(ps, z, AVR_KD(0x3ec71de3a556c734ull, 0x1.71de3a556c734p-19));   // 1/9!
    ps = fma(ps, z, AVR_KD(0xbf2a01a01a01a01aull, -0x1.a01a01a01a01ap-13));   // -1/7!
    ps = fma(ps, z, AVR_KD(0x3f81111111111111ull, 0x1.1111111111111p-7));   // 1/5!
    ps = fma(ps, z, AVR_KD(0xbfc5555555555555ull, -0x1.5555555555555p-3));   // -1/3!
    ps = fma(ps, z, 1.0);
    double pc = AVR_KD(0xbd2ae7f3e733b81full, -0x1.ae7f3e733b81fp-45);   // -1/16!
    pc = fma(pc, z, AVR_KD(0x3da93974a8c07c9dull, 0x1.93974a8c07c9dp-37));   // 1/14!
    pc = fma(pc, z, AVR_KD(0xbe21eed8eff8d898ull, -0x1.1eed8eff8d898p-29));   // -1/12!
    pc = fma(pc, z, AVR_KD(0x3e927e4fb7789f5cull, 0x1.27e4fb7789f5cp-22));   // 1/10!
    pc = fma(pc, z, AVR_KD(0xbefa01a01a01a01aull, -0x1.a01a01a01a01ap-16));   // -1/8!
    pc = fma(pc, z, AVR_KD(0x3f56c16c16c16c17ull, 0x1.6c16c16c16c17p-10));   // 1/6!
    pc = fma(pc, z, AVR_KD(0xbfa5555555555555ull, -0x1.5555555555555p-5));   // -1/4!
    pc = fma(pc, z, 0.5);
    const double sr = r * ps;
    const double cr = fma(-z, pc, 1.0);
    const int q = (int)kf & 3;
    *sn = q == 0 ? sr : (q == 1 ? cr : (q == 2 ? -sr : -cr));
    *cs = q == 0 ? cr : (q == 1 ? -sr : (q == 2 ? -cr : sr));
}

// exp(x) for |x| < 708
AVR_HD double exp_d(double x) {
    const double kf = __builtin_rint(x * kInvLn2);
    const double r = (x - kf * kLn2Hi) - kf * kLn2Lo;   // |r| <= 0.3466
    double p = 0x1.952c77030ad4ap-49;       // 1/17! (Taylor to r^17: 0.347^18/18! < 1e-24)
    p = fma(p, r, 0x1.ae7f3e733b81fp-45);   // 1/16!
    p = fma(p, r, 0x1.ae7f3e733b81fp-41);   // 1/15!
    p = fma(p, r, 0x1.93974a8c07c9dp-37);   // 1/14!
    p = fma(p, r, 0x1.6124613a86d09p-33);   // 1/13!
    p = fma(p, r, 0x1.1eed8eff8d898p-29);   // 1/12!
    p = fma(p, r, 0x1.ae64567f544e4p-26);   // 1/11!
    p = fma(p, r, 0x1.27e4fb7789f5cp-22);   // 1/10!
    p = fma(p, r, 0x1.71de3a556c734p-19);   // 1/9!
    p = fma(p, r, 0x1.a01a01a01a01ap-16);   // 1/8!
    p = fma(p, r, 0x1.a01a01a01a01ap-13);   // 1/7!
    p = fma(p, r, 0x1.6c16c16c16c17p-10);   // 1/6!
    p = fma(p, r, 0x1.1111111111111p-7);    // 1/5!
    p = fma(p, r, 0x1.5555555555555p-5);    // 1/4!
    p = fma(p, r, 0x1.5555555555555p-3);    // 1/3!
    p = fma(p, r, 0.5);
    p = fma(p, r, 1.0);
    p = fma(p, r, 1.0);
    const int k = (int)kf;
    return p * dfrom((uint64_t)(k + 1023) << 52);
}

AVR_HD double cosh_d(double x) {
    const double e = exp_d(x < 0 ? -x : x);
    return 0.5 * (e + 1.0 / e);
}

// float interface: one rounding of the f64 value
AVR_HD float log_f(float x) { return (float)log_d((double)x); }
AVR_HD float atanh_f(float x) { return (float)atanh_d((double)x); }
AVR_HD float cosh_f(float x) { return (float)cosh_d((double)x); }
AVR_HD void sincos_f(float x, float *s, float *c) {
    double sd, cd;
    sincos_d((double)x, &sd, &cd);
    *s = (float)sd;
    *c = (float)cd;
}

}  // namespace canon
}  // namespace avr

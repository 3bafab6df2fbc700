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
// The path's log, atanh and cosh use table-driven sequences (log: 7-bit mantissa table +
// degree-8 log1p, no division, ~14 f64 ops; atanh: two such logs; cosh: 2^(j/64) table +
// degree-6 exp polynomial for e^x and e^-x, no division); sincos a Cody-Waite reduction +
// degree-15/16 polynomials. Tables: tools/gen_canon_tables.py (decimal arithmetic, every entry
// the double nearest to the exact value), the same literals in the oracle. The older
// series forms (log_d, exp_d) remain for FLIP's pow (avr_flip.h).
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
// a * b + K with K read straight from its SGPR pair (VOP3 v_fma_f64): the compiler's own choice
// for fma(a, b, K) is v_fmac_f64 after two v_mov_b32 copying K into the accumulator — two extra
// VALU issues per polynomial step of the canonical f64 sequences
template <uint64_t B>
__device__ __forceinline__ double fmak(double a, double b) {
    const double c = kd<B>();
    double r;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(c));
    return r;
}
#ifndef AVR_FMAK_ASM
#define AVR_FMAK_ASM 1
#endif
#if AVR_FMAK_ASM
#define AVR_FMAK(a, b, bits, value) (::avr::canon::fmak<bits>((a), (b)))
#else
#define AVR_FMAK(a, b, bits, value) (fma((a), (b), ::avr::canon::kd<bits>()))
#endif
#else
#define AVR_KD(bits, value) (value)
#define AVR_FMAK(a, b, bits, value) (fma((a), (b), (value)))
#endif

// 2*atanh(s)/(2s) = 1 + z/3 + z^2/5 + ... + z^11/23 with z = s^2 (|s| <= 0.1716, z^12/25 < 2e-20)
AVR_HD double atanh_series(double z) {
    double p = AVR_KD(0x3fa642c8590b2164ull, 0x1.642c8590b2164p-5);
    p = AVR_FMAK(p, z, 0x3fa8618618618618ull, 0x1.8618618618618p-5);
    p = AVR_FMAK(p, z, 0x3faaf286bca1af28ull, 0x1.af286bca1af28p-5);
    p = AVR_FMAK(p, z, 0x3fae1e1e1e1e1e1eull, 0x1.e1e1e1e1e1e1ep-5);
    p = AVR_FMAK(p, z, 0x3fb1111111111111ull, 0x1.1111111111111p-4);
    p = AVR_FMAK(p, z, 0x3fb3b13b13b13b14ull, 0x1.3b13b13b13b14p-4);
    p = AVR_FMAK(p, z, 0x3fb745d1745d1746ull, 0x1.745d1745d1746p-4);
    p = AVR_FMAK(p, z, 0x3fbc71c71c71c71cull, 0x1.c71c71c71c71cp-4);
    p = AVR_FMAK(p, z, 0x3fc2492492492492ull, 0x1.2492492492492p-3);
    p = AVR_FMAK(p, z, 0x3fc999999999999aull, 0x1.999999999999ap-3);
    p = AVR_FMAK(p, z, 0x3fd5555555555555ull, 0x1.5555555555555p-2);
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
    ps = AVR_FMAK(ps, z, 0x3de6124613a86d09ull, 0x1.6124613a86d09p-33);   // 1/13!
    ps = AVR_FMAK(ps, z, 0xbe5ae64567f544e4ull, -0x1.ae64567f544e4p-26);   // -1/11!
    ps = AVR_FMAK(ps, z, 0x3ec71de3a556c734ull, 0x1.71de3a556c734p-19);   // 1/9!
    ps = AVR_FMAK(ps, z, 0xbf2a01a01a01a01aull, -0x1.a01a01a01a01ap-13);   // -1/7!
    ps = AVR_FMAK(ps, z, 0x3f81111111111111ull, 0x1.1111111111111p-7);   // 1/5!
    ps = AVR_FMAK(ps, z, 0xbfc5555555555555ull, -0x1.5555555555555p-3);   // -1/3!
    ps = fma(ps, z, 1.0);
    double pc = AVR_KD(0xbd2ae7f3e733b81full, -0x1.ae7f3e733b81fp-45);   // -1/16!
    pc = AVR_FMAK(pc, z, 0x3da93974a8c07c9dull, 0x1.93974a8c07c9dp-37);   // 1/14!
    pc = AVR_FMAK(pc, z, 0xbe21eed8eff8d898ull, -0x1.1eed8eff8d898p-29);   // -1/12!
    pc = AVR_FMAK(pc, z, 0x3e927e4fb7789f5cull, 0x1.27e4fb7789f5cp-22);   // 1/10!
    pc = AVR_FMAK(pc, z, 0xbefa01a01a01a01aull, -0x1.a01a01a01a01ap-16);   // -1/8!
    pc = AVR_FMAK(pc, z, 0x3f56c16c16c16c17ull, 0x1.6c16c16c16c17p-10);   // 1/6!
    pc = AVR_FMAK(pc, z, 0xbfa5555555555555ull, -0x1.5555555555555p-5);   // -1/4!
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

// ---- tables (tools/gen_canon_tables.py) ----
// 1 / c_k and log(c_k), c_k = 1 + k / 128
constexpr double kLogInvC[128] = {
    0x1.0000000000000p+0, 0x1.fc07f01fc07f0p-1, 0x1.f81f81f81f820p-1, 0x1.f44659e4a4271p-1,
    0x1.f07c1f07c1f08p-1, 0x1.ecc07b301ecc0p-1, 0x1.e9131abf0b767p-1, 0x1.e573ac901e574p-1,
    0x1.e1e1e1e1e1e1ep-1, 0x1.de5d6e3f8868ap-1, 0x1.dae6076b981dbp-1, 0x1.d77b654b82c34p-1,
    0x1.d41d41d41d41dp-1, 0x1.d0cb58f6ec074p-1, 0x1.cd85689039b0bp-1, 0x1.ca4b3055ee191p-1,
    0x1.c71c71c71c71cp-1, 0x1.c3f8f01c3f8f0p-1, 0x1.c0e070381c0e0p-1, 0x1.bdd2b899406f7p-1,
    0x1.bacf914c1bad0p-1, 0x1.b7d6c3dda338bp-1, 0x1.b4e81b4e81b4fp-1, 0x1.b2036406c80d9p-1,
    0x1.af286bca1af28p-1, 0x1.ac5701ac5701bp-1, 0x1.a98ef606a63bep-1, 0x1.a6d01a6d01a6dp-1,
    0x1.a41a41a41a41ap-1, 0x1.a16d3f97a4b02p-1, 0x1.9ec8e951033d9p-1, 0x1.9c2d14ee4a102p-1,
    0x1.999999999999ap-1, 0x1.970e4f80cb872p-1, 0x1.948b0fcd6e9e0p-1, 0x1.920fb49d0e229p-1,
    0x1.8f9c18f9c18fap-1, 0x1.8d3018d3018d3p-1, 0x1.8acb90f6bf3aap-1, 0x1.886e5f0abb04ap-1,
    0x1.8618618618618p-1, 0x1.83c977ab2beddp-1, 0x1.8181818181818p-1, 0x1.7f405fd017f40p-1,
    0x1.7d05f417d05f4p-1, 0x1.7ad2208e0ecc3p-1, 0x1.78a4c8178a4c8p-1, 0x1.767dce434a9b1p-1,
    0x1.745d1745d1746p-1, 0x1.724287f46debcp-1, 0x1.702e05c0b8170p-1, 0x1.6e1f76b4337c7p-1,
    0x1.6c16c16c16c17p-1, 0x1.6a13cd1537290p-1, 0x1.6816816816817p-1, 0x1.661ec6a5122f9p-1,
    0x1.642c8590b2164p-1, 0x1.623fa77016240p-1, 0x1.6058160581606p-1, 0x1.5e75bb8d015e7p-1,
    0x1.5c9882b931057p-1, 0x1.5ac056b015ac0p-1, 0x1.58ed2308158edp-1, 0x1.571ed3c506b3ap-1,
    0x1.5555555555555p-1, 0x1.5390948f40febp-1, 0x1.51d07eae2f815p-1, 0x1.5015015015015p-1,
    0x1.4e5e0a72f0539p-1, 0x1.4cab88725af6ep-1, 0x1.4afd6a052bf5bp-1, 0x1.49539e3b2d067p-1,
    0x1.47ae147ae147bp-1, 0x1.460cbc7f5cf9ap-1, 0x1.446f86562d9fbp-1, 0x1.42d6625d51f87p-1,
    0x1.4141414141414p-1, 0x1.3fb013fb013fbp-1, 0x1.3e22cbce4a902p-1, 0x1.3c995a47babe7p-1,
    0x1.3b13b13b13b14p-1, 0x1.3991c2c187f63p-1, 0x1.3813813813814p-1, 0x1.3698df3de0748p-1,
    0x1.3521cfb2b78c1p-1, 0x1.33ae45b57bcb2p-1, 0x1.323e34a2b10bfp-1, 0x1.30d190130d190p-1,
    0x1.2f684bda12f68p-1, 0x1.2e025c04b8097p-1, 0x1.2c9fb4d812ca0p-1, 0x1.2b404ad012b40p-1,
    0x1.29e4129e4129ep-1, 0x1.288b01288b013p-1, 0x1.27350b8812735p-1, 0x1.25e22708092f1p-1,
    0x1.2492492492492p-1, 0x1.23456789abcdfp-1, 0x1.21fb78121fb78p-1, 0x1.20b470c67c0d9p-1,
    0x1.1f7047dc11f70p-1, 0x1.1e2ef3b3fb874p-1, 0x1.1cf06ada2811dp-1, 0x1.1bb4a4046ed29p-1,
    0x1.1a7b9611a7b96p-1, 0x1.19453808ca29cp-1, 0x1.1811811811812p-1, 0x1.16e0689427379p-1,
    0x1.15b1e5f75270dp-1, 0x1.1485f0e0acd3bp-1, 0x1.135c81135c811p-1, 0x1.12358e75d3033p-1,
    0x1.1111111111111p-1, 0x1.0fef010fef011p-1, 0x1.0ecf56be69c90p-1, 0x1.0db20a88f4696p-1,
    0x1.0c9714fbcda3bp-1, 0x1.0b7e6ec259dc8p-1, 0x1.0a6810a6810a7p-1, 0x1.0953f39010954p-1,
    0x1.0842108421084p-1, 0x1.073260a47f7c6p-1, 0x1.0624dd2f1a9fcp-1, 0x1.05197f7d73404p-1,
    0x1.0410410410410p-1, 0x1.03091b51f5e1ap-1, 0x1.0204081020408p-1, 0x1.0101010101010p-1,
};
constexpr double kLogC[128] = {
    0x0.0p+0, 0x1.fe02a6b106789p-8, 0x1.fc0a8b0fc03e4p-7, 0x1.7b91b07d5b11bp-6,
    0x1.f829b0e783300p-6, 0x1.39e87b9febd60p-5, 0x1.77458f632dcfcp-5, 0x1.b42dd711971bfp-5,
    0x1.f0a30c01162a6p-5, 0x1.16536eea37ae1p-4, 0x1.341d7961bd1d1p-4, 0x1.51b073f06183fp-4,
    0x1.6f0d28ae56b4cp-4, 0x1.8c345d6319b21p-4, 0x1.a926d3a4ad563p-4, 0x1.c5e548f5bc743p-4,
    0x1.e27076e2af2e6p-4, 0x1.fec9131dbeabbp-4, 0x1.0d77e7cd08e59p-3, 0x1.1b72ad52f67a0p-3,
    0x1.29552f81ff523p-3, 0x1.371fc201e8f74p-3, 0x1.44d2b6ccb7d1ep-3, 0x1.526e5e3a1b438p-3,
    0x1.5ff3070a793d4p-3, 0x1.6d60fe719d21dp-3, 0x1.7ab890210d909p-3, 0x1.87fa06520c911p-3,
    0x1.9525a9cf456b4p-3, 0x1.a23bc1fe2b563p-3, 0x1.af3c94e80bff3p-3, 0x1.bc286742d8cd6p-3,
    0x1.c8ff7c79a9a22p-3, 0x1.d5c216b4fbb91p-3, 0x1.e27076e2af2e6p-3, 0x1.ef0adcbdc5936p-3,
    0x1.fb9186d5e3e2bp-3, 0x1.0402594b4d041p-2, 0x1.0a324e27390e3p-2, 0x1.1058bf9ae4ad5p-2,
    0x1.1675cababa60ep-2, 0x1.1c898c16999fbp-2, 0x1.22941fbcf7966p-2, 0x1.2895a13de86a3p-2,
    0x1.2e8e2bae11d31p-2, 0x1.347dd9a987d55p-2, 0x1.3a64c556945eap-2, 0x1.404308686a7e4p-2,
    0x1.4618bc21c5ec2p-2, 0x1.4be5f957778a1p-2, 0x1.51aad872df82dp-2, 0x1.5767717455a6cp-2,
    0x1.5d1bdbf5809cap-2, 0x1.62c82f2b9c795p-2, 0x1.686c81e9b14afp-2, 0x1.6e08eaa2ba1e4p-2,
    0x1.739d7f6bbd007p-2, 0x1.792a55fdd47a2p-2, 0x1.7eaf83b82afc3p-2, 0x1.842d1da1e8b17p-2,
    0x1.89a3386c1425bp-2, 0x1.8f11e873662c7p-2, 0x1.947941c2116fbp-2, 0x1.99d958117e08bp-2,
    0x1.9f323ecbf984cp-2, 0x1.a484090e5bb0ap-2, 0x1.a9cec9a9a084ap-2, 0x1.af1293247786bp-2,
    0x1.b44f77bcc8f63p-2, 0x1.b9858969310fbp-2, 0x1.beb4d9da71b7cp-2, 0x1.c3dd7a7cdad4dp-2,
    0x1.c8ff7c79a9a22p-2, 0x1.ce1af0b85f3ebp-2, 0x1.d32fe7e00ebd5p-2, 0x1.d83e7258a2f3ep-2,
    0x1.dd46a04c1c4a1p-2, 0x1.e24881a7c6c26p-2, 0x1.e744261d68788p-2, 0x1.ec399d2468cc0p-2,
    0x1.f128f5faf06edp-2, 0x1.f6123fa7028acp-2, 0x1.faf588f78f31fp-2, 0x1.ffd2e0857f498p-2,
    0x1.02552a5a5d0ffp-1, 0x1.04bdf9da926d2p-1, 0x1.0723e5c1cdf40p-1, 0x1.0986f4f573521p-1,
    0x1.0be72e4252a83p-1, 0x1.0e44985d1cc8cp-1, 0x1.109f39e2d4c97p-1, 0x1.12f719593efbcp-1,
    0x1.154c3d2f4d5eap-1, 0x1.179eabbd899a1p-1, 0x1.19ee6b467c96fp-1, 0x1.1c3b81f713c25p-1,
    0x1.1e85f5e7040d0p-1, 0x1.20cdcd192ab6ep-1, 0x1.23130d7bebf43p-1, 0x1.2555bce98f7cbp-1,
    0x1.2795e1289b11bp-1, 0x1.29d37fec2b08bp-1, 0x1.2c0e9ed448e8cp-1, 0x1.2e47436e40268p-1,
    0x1.307d7334f10bep-1, 0x1.32b1339121d71p-1, 0x1.34e289d9ce1d3p-1, 0x1.37117b54747b6p-1,
    0x1.393e0d3562a1ap-1, 0x1.3b68449fffc23p-1, 0x1.3d9026a7156fbp-1, 0x1.3fb5b84d16f42p-1,
    0x1.41d8fe84672aep-1, 0x1.43f9fe2f9ce67p-1, 0x1.4618bc21c5ec2p-1, 0x1.48353d1ea88dfp-1,
    0x1.4a4f85db03ebbp-1, 0x1.4c679afccee3ap-1, 0x1.4e7d811b75bb1p-1, 0x1.50913cc01686bp-1,
    0x1.52a2d265bc5abp-1, 0x1.54b2467999498p-1, 0x1.56bf9d5b3f399p-1, 0x1.58cadb5cd7989p-1,
    0x1.5ad404c359f2dp-1, 0x1.5cdb1dc6c1765p-1, 0x1.5ee02a9241675p-1, 0x1.60e32f44788d9p-1,
};
// 2^(j / 64)
constexpr double kExp2J64[64] = {
    0x1.0000000000000p+0, 0x1.02c9a3e778061p+0, 0x1.059b0d3158574p+0, 0x1.0874518759bc8p+0,
    0x1.0b5586cf9890fp+0, 0x1.0e3ec32d3d1a2p+0, 0x1.11301d0125b51p+0, 0x1.1429aaea92de0p+0,
    0x1.172b83c7d517bp+0, 0x1.1a35beb6fcb75p+0, 0x1.1d4873168b9aap+0, 0x1.2063b88628cd6p+0,
    0x1.2387a6e756238p+0, 0x1.26b4565e27cddp+0, 0x1.29e9df51fdee1p+0, 0x1.2d285a6e4030bp+0,
    0x1.306fe0a31b715p+0, 0x1.33c08b26416ffp+0, 0x1.371a7373aa9cbp+0, 0x1.3a7db34e59ff7p+0,
    0x1.3dea64c123422p+0, 0x1.4160a21f72e2ap+0, 0x1.44e086061892dp+0, 0x1.486a2b5c13cd0p+0,
    0x1.4bfdad5362a27p+0, 0x1.4f9b2769d2ca7p+0, 0x1.5342b569d4f82p+0, 0x1.56f4736b527dap+0,
    0x1.5ab07dd485429p+0, 0x1.5e76f15ad2148p+0, 0x1.6247eb03a5585p+0, 0x1.6623882552225p+0,
    0x1.6a09e667f3bcdp+0, 0x1.6dfb23c651a2fp+0, 0x1.71f75e8ec5f74p+0, 0x1.75feb564267c9p+0,
    0x1.7a11473eb0187p+0, 0x1.7e2f336cf4e62p+0, 0x1.82589994cce13p+0, 0x1.868d99b4492edp+0,
    0x1.8ace5422aa0dbp+0, 0x1.8f1ae99157736p+0, 0x1.93737b0cdc5e5p+0, 0x1.97d829fde4e50p+0,
    0x1.9c49182a3f090p+0, 0x1.a0c667b5de565p+0, 0x1.a5503b23e255dp+0, 0x1.a9e6b5579fdbfp+0,
    0x1.ae89f995ad3adp+0, 0x1.b33a2b84f15fbp+0, 0x1.b7f76f2fb5e47p+0, 0x1.bcc1e904bc1d2p+0,
    0x1.c199bdd85529cp+0, 0x1.c67f12e57d14bp+0, 0x1.cb720dcef9069p+0, 0x1.d072d4a07897cp+0,
    0x1.d5818dcfba487p+0, 0x1.da9e603db3285p+0, 0x1.dfc97337b9b5fp+0, 0x1.e502ee78b3ff6p+0,
    0x1.ea4afa2a490dap+0, 0x1.efa1bee615a27p+0, 0x1.f50765b6e4540p+0, 0x1.fa7c1819e90d8p+0,
};
constexpr double kLn2_64Hi = 0x1.62e42fee00000p-7;    // 32 significant bits: n * kLn2_64Hi exact for |n| < 2^21
constexpr double kLn2_64Lo = 0x1.a39ef35793c76p-39;
constexpr double k64OverLn2 = 0x1.71547652b82fep+6;

// log(x) for a positive normal f64; 0 -> -inf, <0/NaN -> NaN. x = 2^e m, m in [1, 2); k = the
// fraction of m rounded to 7 bits (k = 128: m / 2 and e + 1, so k = 0 and c = 1 around x = 1);
// r = (m - c_k) / c_k (m - c_k exact) with |r| <= 2^-8; log1p(r) = r + r^2 q(r) to degree 8.
AVR_HD double log_t(double x, const double *invc = kLogInvC, const double *logc = kLogC) {
    if (!(x > 0)) return x == 0 ? -__builtin_inf() : __builtin_nan("");
    if (x == __builtin_inf()) return x;
    const uint64_t b = dbits(x);
    int e = (int)((b >> 52) & 0x7ff) - 1023;
    const uint64_t frac = b & 0x000fffffffffffffull;
    int k = (int)((frac + (1ull << 44)) >> 45);
    double m = dfrom(frac | 0x3ff0000000000000ull);
    if (k == 128) {
        m = m * 0.5;
        e += 1;
        k = 0;
    }
    const double c = 1.0 + (double)k * 0x1p-7;
    const double r = (m - c) * invc[k];
    double q = AVR_KD(0xbfc0000000000000ull, -0x1.0000000000000p-3);            // -1/8
    q = AVR_FMAK(q, r, 0x3fc2492492492492ull, 0x1.2492492492492p-3);         // 1/7
    q = AVR_FMAK(q, r, 0xbfc5555555555555ull, -0x1.5555555555555p-3);        // -1/6
    q = AVR_FMAK(q, r, 0x3fc999999999999aull, 0x1.999999999999ap-3);         // 1/5
    q = AVR_FMAK(q, r, 0xbfd0000000000000ull, -0.25);
    q = AVR_FMAK(q, r, 0x3fd5555555555555ull, 0x1.5555555555555p-2);         // 1/3
    q = fma(q, r, -0.5);
    const double l1 = fma(r * r, q, r);
    const double de = (double)e;
    return fma(de, AVR_KD(0x3fe62e42fee00000ull, 0x1.62e42fee00000p-1),
               fma(de, AVR_KD(0x3dea39ef35793c76ull, 0x1.a39ef35793c76p-33), logc[k] + l1));
}

// atanh(x), |x| < 1: (log(1 + x) - log(1 - x)) / 2 (1 +- x exact for |x| >= 2^-29); x itself
// below 2^-26 (atanh(x) = x (1 + x^2/3 + ...) rounds to x there)
AVR_HD double atanh_t(double x, const double *invc = kLogInvC, const double *logc = kLogC) {
    const double ax = x < 0 ? -x : x;
    if (ax < 0x1p-26) return x;
    return 0.5 * (log_t(1.0 + x, invc, logc) - log_t(1.0 - x, invc, logc));
}

// e^(s r) 2^(n/64) pieces: n = rint(x 64 / ln2), r = x - n ln2/64 (two-part), |r| <= ln2/128;
// e^r to degree 6
AVR_HD double exp_poly6(double r) {
    double p = AVR_KD(0x3f56c16c16c16c17ull, 0x1.6c16c16c16c17p-10);            // 1/720
    p = AVR_FMAK(p, r, 0x3f81111111111111ull, 0x1.1111111111111p-7);         // 1/120
    p = AVR_FMAK(p, r, 0x3fa5555555555555ull, 0x1.5555555555555p-5);         // 1/24
    p = AVR_FMAK(p, r, 0x3fc5555555555555ull, 0x1.5555555555555p-3);         // 1/6
    p = fma(p, r, 0.5);
    p = fma(p, r, 1.0);
    p = fma(p, r, 1.0);
    return p;
}
AVR_HD double exp_scale(int n, const double *e2j = kExp2J64) {   // 2^(n / 64) = 2^(n >> 6) * kExp2J64[n & 63]
    return e2j[n & 63] * dfrom((uint64_t)((n >> 6) + 1023) << 52);
}
// cosh(x) = (e^|x| + e^-|x|) / 2 for |x| < 700, both exponentials from one reduction
AVR_HD double cosh_t(double x, const double *e2j = kExp2J64) {
    const double ax = x < 0 ? -x : x;
    const double nf = __builtin_rint(ax * k64OverLn2);
    const double r = (ax - nf * kLn2_64Hi) - nf * kLn2_64Lo;
    const int n = (int)nf;
    const double ep = exp_poly6(r) * exp_scale(n, e2j);
    const double em = exp_poly6(-r) * exp_scale(-n, e2j);
    return 0.5 * (ep + em);
}

// float interface: one rounding of the f64 value
AVR_HD float log_f(float x) { return (float)log_t((double)x); }
AVR_HD float atanh_f(float x) { return (float)atanh_t((double)x); }
AVR_HD float cosh_f(float x) { return (float)cosh_t((double)x); }
// the same functions reading their tables from a staged copy (LDS): kLogInvC | kLogC | kExp2J64
constexpr int kCanonTabDoubles = 128 + 128 + 64;
AVR_HD float atanh_f(float x, const double *tabs) { return (float)atanh_t((double)x, tabs, tabs + 128); }
AVR_HD float cosh_f(float x, const double *tabs) { return (float)cosh_t((double)x, tabs + 256); }
AVR_HD void sincos_f(float x, float *s, float *c) {
    double sd, cd;
    sincos_d((double)x, &sd, &cd);
    *s = (float)sd;
    *c = (float)cd;
}

}  // namespace canon
}  // namespace avr

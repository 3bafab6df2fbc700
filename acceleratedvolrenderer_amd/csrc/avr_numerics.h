// avr_numerics.h — device numerics of the MI355X volumetric path integrator.
//
// Bit-level semantics follow pbrt-v4 as in the AcceleratedVolRenderer reference
// (paths relative to /root/reference/src/pbrt); the operation order of every
// float expression matches the CPU build (compiled here with -ffp-contract=off,
// as CMakeLists.txt:134-137 does for pbrt), so a device sample replays the CPU
// VolPathIntegrator's sample up to libm ulps in log/atanh/cosh/sin/cos.
//  - PCG32 RNG            util/rng.h:25-160
//  - MurmurHash64A/MixBits util/hash.h:19-106
//  - FastExp (CPU poly)   util/math.h:450-471 (the CPU branch, not __expf, so the
//                         GPU replays the CPU sample stream — SURVEY Appendix B)
//  - interval offsets     util/float.h:164-227, util/math.h:818-1014, transform.h:340-433
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define AVR_HD __host__ __device__ __forceinline__
#include "avr_canon.h"
#include "avr_fastdiv.h"

namespace avr {

constexpr float kOneMinusEpsilon = 0x1.fffffep-1f;
constexpr float kInf = __builtin_huge_valf();
constexpr float kFloatMax = 3.40282346638528859812e+38f;
constexpr float kPi = 3.14159265358979323846f;
constexpr float kInv4Pi = 0.07957747154594766788f;
constexpr float kLn2 = 0.693147180559945309f;
constexpr float kShadowEpsilon = 0.0001f;
constexpr float kMachineEpsilon = 5.96046448e-08f;  // FLT_EPSILON/2
AVR_HD float gamma_n(int n) { return (n * kMachineEpsilon) / (1 - n * kMachineEpsilon); }
constexpr int kLambdaMin = 360, kNTable = 471;

AVR_HD uint32_t f2u(float f) { return __builtin_bit_cast(uint32_t, f); }
AVR_HD float u2f(uint32_t u) { return __builtin_bit_cast(float, u); }

AVR_HD float next_up(float v) {
    if (__builtin_isinf(v) && v > 0.f) return v;
    if (v == -0.f) v = 0.f;
    uint32_t ui = f2u(v);
    if (v >= 0) ++ui; else --ui;
    return u2f(ui);
}
AVR_HD float next_down(float v) {
    if (__builtin_isinf(v) && v < 0.f) return v;
    if (v == 0.f) v = -0.f;
    uint32_t ui = f2u(v);
    if (v > 0) --ui; else ++ui;
    return u2f(ui);
}
AVR_HD float fminf_(float a, float b) { return a < b ? a : b; }   // std::min semantics
AVR_HD float fmaxf_(float a, float b) { return a < b ? b : a; }   // std::max semantics
AVR_HD float lerp(float x, float a, float b) { return (1 - x) * a + x * b; }
AVR_HD float sqr(float v) { return v * v; }
AVR_HD float clampf(float v, float lo, float hi) { return v < lo ? lo : (v > hi ? hi : v); }


// util/math.h:450-471, CPU branch (EvaluatePolynomial = nested std::fma)
AVR_HD float fast_exp(float x) {
    float xp = x * 1.442695041f;
    float fxp = __builtin_floorf(xp), f = xp - fxp;
    int i = (int)fxp;
    float twoToF = __builtin_fmaf(f, __builtin_fmaf(f, __builtin_fmaf(f, 0.0781455737f, 0.226173572f), 0.695556856f), 1.f);
    int exponent = (int)(f2u(twoToF) >> 23) - 127 + i;
    if (exponent < -126) return 0;
    if (exponent > 127) return kInf;
    uint32_t bits = f2u(twoToF);
    bits &= 0x807FFFFFu;
    bits |= (uint32_t)(exponent + 127) << 23;
    return u2f(bits);
}
// fast_exp(x) for x in (-40, 0]: x log2(e) > -57.8, so the exponent stays inside [-58, 0] and
// neither range check can fire — the same bits without them (the walk's reject factor, whose
// caller only uses it when A = -x < 40)
AVR_HD float fast_exp_m40(float x) {
    float xp = x * 1.442695041f;
    float fxp = __builtin_floorf(xp), f = xp - fxp;
    int i = (int)fxp;
    float twoToF = __builtin_fmaf(f, __builtin_fmaf(f, __builtin_fmaf(f, 0.0781455737f, 0.226173572f), 0.695556856f), 1.f);
    uint32_t bits = f2u(twoToF);
    return u2f(bits + ((uint32_t)i << 23));
}

// ---------------------------------------------------------------------------
// MurmurHash64A specialised to the byte lengths the path hashes (4, 12 bytes)
AVR_HD uint64_t murmur_tail_finish(uint64_t h) {
    const uint64_t m = 0xc6a4a7935bd1e995ull;
    h ^= h >> 47; h *= m; h ^= h >> 47;
    return h;
}
AVR_HD uint64_t hash_u32(uint32_t w) {  // Hash(float) / 4-byte key
    const uint64_t m = 0xc6a4a7935bd1e995ull;
    uint64_t h = 0 ^ (4ull * m);
    h ^= (uint64_t)w;   // bytes 0..3 little endian == the word
    h *= m;
    return murmur_tail_finish(h);
}
AVR_HD uint64_t hash_3u32(uint32_t a, uint32_t b, uint32_t c) {  // 12-byte key
    const uint64_t m = 0xc6a4a7935bd1e995ull;
    uint64_t h = 0 ^ (12ull * m);
    uint64_t k = (uint64_t)a | ((uint64_t)b << 32);
    k *= m; k ^= k >> 47; k *= m;
    h ^= k; h *= m;
    h ^= (uint64_t)c;
    h *= m;
    return murmur_tail_finish(h);
}
AVR_HD uint64_t mix_bits(uint64_t v) {
    v ^= (v >> 31); v *= 0x7fb5d329728ea185ull; v ^= (v >> 27); v *= 0x81dadef4bc2dd44dull; v ^= (v >> 33);
    return v;
}

// PCG32 — util/rng.h
struct Pcg32 {
    uint64_t state, inc;
    AVR_HD void set_sequence(uint64_t seq, uint64_t seed) {
        state = 0u;
        inc = (seq << 1u) | 1u;
        next_u32();
        state += seed;
        next_u32();
    }
    AVR_HD uint32_t next_u32() {
        uint64_t old = state;
        state = old * 0x5851f42d4c957f2dULL + inc;
        uint32_t xorshifted = (uint32_t)(((old >> 18u) ^ old) >> 27u);
        uint32_t rot = (uint32_t)(old >> 59u);
        return (xorshifted >> rot) | (xorshifted << ((~rot + 1u) & 31));
    }
    // std::min(OneMinusEpsilon, v * 2^-32) (rng.h:128-130): the product is never NaN, so the
    // hardware minimum (one v_min_f32 instead of a compare and a select) gives the same value
    AVR_HD float uniform() { return __builtin_fminf(kOneMinusEpsilon, (float)next_u32() * 0x1p-32f); }
    AVR_HD void advance(uint64_t delta) {
        uint64_t curMult = 0x5851f42d4c957f2dULL, curPlus = inc, accMult = 1u, accPlus = 0u;
        while (delta > 0) {
            if (delta & 1) { accMult *= curMult; accPlus = accPlus * curMult + curPlus; }
            curPlus = (curMult + 1) * curPlus;
            curMult *= curMult;
            delta /= 2;
        }
        state = accMult * state + accPlus;
    }
};

// ---------------------------------------------------------------------------
struct V3 { float x, y, z; };
AVR_HD V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
AVR_HD V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
AVR_HD V3 operator*(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
AVR_HD V3 operator*(float s, V3 a) { return {s * a.x, s * a.y, s * a.z}; }
AVR_HD V3 operator/(V3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }
AVR_HD V3 operator-(V3 a) { return {-a.x, -a.y, -a.z}; }
AVR_HD float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
AVR_HD float length_sq(V3 v) { return sqr(v.x) + sqr(v.y) + sqr(v.z); }
AVR_HD float length(V3 v) { return __builtin_sqrtf(length_sq(v)); }
AVR_HD V3 normalize(V3 v) { return v / length(v); }
AVR_HD float comp(V3 v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : v.z); }

// Four-wavelength spectrum (NSpectrumSamples = 4, spectrum.h:36)
struct Spec {
    float v0, v1, v2, v3;
    static AVR_HD Spec c(float a) { return {a, a, a, a}; }
    AVR_HD bool nonzero() const { return v0 != 0 || v1 != 0 || v2 != 0 || v3 != 0; }
    AVR_HD float avg() const { return (((v0 + v1) + v2) + v3) / 4; }
    AVR_HD float maxc() const { return fmaxf_(fmaxf_(fmaxf_(v0, v1), v2), v3); }
};
AVR_HD Spec operator+(Spec a, Spec b) { return {a.v0 + b.v0, a.v1 + b.v1, a.v2 + b.v2, a.v3 + b.v3}; }
AVR_HD Spec operator-(Spec a, Spec b) { return {a.v0 - b.v0, a.v1 - b.v1, a.v2 - b.v2, a.v3 - b.v3}; }
AVR_HD Spec operator*(Spec a, Spec b) { return {a.v0 * b.v0, a.v1 * b.v1, a.v2 * b.v2, a.v3 * b.v3}; }
AVR_HD Spec operator/(Spec a, Spec b) { return {a.v0 / b.v0, a.v1 / b.v1, a.v2 / b.v2, a.v3 / b.v3}; }
AVR_HD Spec operator*(Spec a, float s) { return {a.v0 * s, a.v1 * s, a.v2 * s, a.v3 * s}; }
AVR_HD Spec operator/(Spec a, float s) { return {a.v0 / s, a.v1 / s, a.v2 / s, a.v3 / s}; }
AVR_HD Spec operator-(Spec a) { return {-a.v0, -a.v1, -a.v2, -a.v3}; }
AVR_HD Spec clamp_zero(Spec a) { return {fmaxf_(0.f, a.v0), fmaxf_(0.f, a.v1), fmaxf_(0.f, a.v2), fmaxf_(0.f, a.v3)}; }
AVR_HD Spec safe_div(Spec a, Spec b) {
    return {b.v0 != 0 ? a.v0 / b.v0 : 0.f, b.v1 != 0 ? a.v1 / b.v1 : 0.f, b.v2 != 0 ? a.v2 / b.v2 : 0.f,
            b.v3 != 0 ? a.v3 / b.v3 : 0.f};
}
AVR_HD Spec fast_exp(Spec a) { return {fast_exp(a.v0), fast_exp(a.v1), fast_exp(a.v2), fast_exp(a.v3)}; }

// Transcendentals: the canonical convention of avr_canon.h (f64 evaluation by a fixed IEEE
// op sequence, one rounding to float; the correctly rounded float except within ~1e-16 of a
// midpoint). pbrt's float libm calls are last-ulp platform-specific (glibc FMA/non-FMA
// variants, MSVC, CUDA); the oracle's "canonical" mode restates the same sequences, so a
// device sample replays the oracle's bit for bit. Used once per path (wavelengths), per
// scatter (phase direction) and per accepted free-flight candidate (log).
AVR_HD float cr_log(float x) { return canon::log_f(x); }
AVR_HD float cr_atanh(float x) { return canon::atanh_f(x); }
AVR_HD float cr_cosh(float x) { return canon::cosh_f(x); }
AVR_HD void cr_sincos(float x, float *s, float *c) { canon::sincos_f(x, s, c); }

// "fast" render mode (avr_set_render_mode 1; SURVEY §7: replay / fast): the hardware
// transcendentals (v_log_f32, v_exp_f32, v_sin/cos_f32 — about 1 ulp) replace the canonical
// f64 sequences and pbrt's CPU FastExp polynomial. The estimator is unchanged; sample paths
// differ in their last bits, so parity is statistical (tests/test_gpu_fast.py). The host
// versions exist only so that shared code compiles; fast mode is a device path.
#if defined(__HIP_DEVICE_COMPILE__)
AVR_HD float hw_log(float x) { return __builtin_amdgcn_logf(x) * 0.693147181f; }
AVR_HD float hw_exp(float x) { return __builtin_amdgcn_exp2f(x * 1.442695041f); }
AVR_HD float hw_rcp(float x) { return __builtin_amdgcn_rcpf(x); }
// sin / cos of 2*pi*t (the hardware takes its argument in turns)
AVR_HD void hw_sincos_turns(float t, float *s, float *c) {
    *s = __builtin_amdgcn_sinf(t);
    *c = __builtin_amdgcn_cosf(t);
}
#else   // host compilation pass (and host-side callers such as the C-ABI readback)
AVR_HD float hw_log(float x) { return logf(x); }
AVR_HD float hw_exp(float x) { return expf(x); }
AVR_HD float hw_rcp(float x) { return 1.f / x; }
AVR_HD void hw_sincos_turns(float t, float *s, float *c) {
    *s = sinf(6.28318531f * t);
    *c = cosf(6.28318531f * t);
}
#endif
// exponential free-flight distance -log(1 - u) / a (SampleExponential, sampling.h:222-225)
template <bool kFast> AVR_HD float m_exp_dist(float u, float a) {
    if (kFast) return -hw_log(1 - u) * hw_rcp(a);
    return -cr_log(1 - u) / a;
}

// Blackbody (spectrum.h:69-80) with FastExp, and BlackbodySpectrum's normalisation
// 1 / Blackbody(lambdaMax, T), lambdaMax = 2.8977721e-3 / T (spectrum.h:500-530)
AVR_HD float blackbody(float lambda, float T) {
    if (T <= 0) return 0;
    const float c = 299792458.f, h = 6.62606957e-34f, kb = 1.3806488e-23f;
    const float l = lambda * 1e-9f;
    const float l2 = l * l;
    return (2 * h * c * c) / (((l2 * l2) * l) * (fast_exp((h * c) / (l * kb * T)) - 1));
}
AVR_HD float blackbody_norm(float T) { return 1 / blackbody((2.8977721e-3f / T) * 1e9f, T); }

// Wavelength sampling — sampling.h:163-171, spectrum.h:334-347
AVR_HD float sample_visible_wavelength(float u) { return 538 - 138.888889f * cr_atanh(0.85691062f - 1.82750197f * u); }
// fast mode: atanh(x) = log((1 + x) / (1 - x)) / 2 with the hardware log
AVR_HD float sample_visible_wavelength_fast(float u) {
    const float x = 0.85691062f - 1.82750197f * u;
    return 538 - 138.888889f * (0.5f * hw_log((1 + x) / (1 - x)));
}
AVR_HD float visible_wavelength_pdf(float l) {
    if (l < 360 || l > 830) return 0;
    return 0.0039398042f / sqr(cr_cosh(0.0072f * (l - 538)));
}
// The camera stage's versions: the canonical tables read from a staged (LDS) copy and the
// four evaluations left unfenced, so their table reads overlap — same arithmetic, same bits
AVR_HD float sample_visible_wavelength(float u, const double *tabs) {
    return 538 - 138.888889f * canon::atanh_f(0.85691062f - 1.82750197f * u, tabs);
}
AVR_HD float visible_wavelength_pdf(float l, const double *tabs) {
    if (l < 360 || l > 830) return 0;
    return 0.0039398042f / sqr(canon::cosh_f(0.0072f * (l - 538), tabs));
}
struct Lambda { Spec l, pdf; };
// Device: the four f64 evaluations are kept apart (scheduling barriers) so their
// temporaries are not all live at once in the register-bound path kernel.
#if defined(__HIP_DEVICE_COMPILE__)
#define AVR_SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define AVR_SCHED_FENCE() ((void)0)
#endif
AVR_HD float visible_up(float u, int i) {
    float up = u + float(i) / 4;
    if (up > 1) up -= 1;
    return up;
}
AVR_HD Spec sample_visible_lambda_fast(float u) {
    return {sample_visible_wavelength_fast(visible_up(u, 0)), sample_visible_wavelength_fast(visible_up(u, 1)),
            sample_visible_wavelength_fast(visible_up(u, 2)), sample_visible_wavelength_fast(visible_up(u, 3))};
}
AVR_HD Spec sample_visible_lambda(float u) {
    Spec l;
    l.v0 = sample_visible_wavelength(visible_up(u, 0));
    AVR_SCHED_FENCE();
    l.v1 = sample_visible_wavelength(visible_up(u, 1));
    AVR_SCHED_FENCE();
    l.v2 = sample_visible_wavelength(visible_up(u, 2));
    AVR_SCHED_FENCE();
    l.v3 = sample_visible_wavelength(visible_up(u, 3));
    return l;
}
// SampledWavelengths::SampleUniform (spectrum.h:287-306): Lerp(u, min, max), then steps of
// (max - min) / 4 wrapped into the range; pdf 1 / (max - min)
AVR_HD Spec sample_visible_lambda(float u, const double *tabs) {
    return {sample_visible_wavelength(visible_up(u, 0), tabs), sample_visible_wavelength(visible_up(u, 1), tabs),
            sample_visible_wavelength(visible_up(u, 2), tabs), sample_visible_wavelength(visible_up(u, 3), tabs)};
}
AVR_HD Spec sample_uniform_lambda(float u, float lmin, float lmax) {
    Spec l;
    l.v0 = (1 - u) * lmin + u * lmax;
    const float delta = (lmax - lmin) / 4;
    l.v1 = l.v0 + delta;
    if (l.v1 > lmax) l.v1 = lmin + (l.v1 - lmax);
    l.v2 = l.v1 + delta;
    if (l.v2 > lmax) l.v2 = lmin + (l.v2 - lmax);
    l.v3 = l.v2 + delta;
    if (l.v3 > lmax) l.v3 = lmin + (l.v3 - lmax);
    return l;
}
AVR_HD Lambda sample_visible(float u) {
    Lambda w;
    w.l = sample_visible_lambda(u);
    w.pdf = {visible_wavelength_pdf(w.l.v0), visible_wavelength_pdf(w.l.v1), visible_wavelength_pdf(w.l.v2),
             visible_wavelength_pdf(w.l.v3)};
    return w;
}
// DenselySampledSpectrum::Sample — spectrum.h:390-400: table index lround(lambda) - 360
AVR_HD int lambda_offset(float l) { return (int)__builtin_lroundf(l) - kLambdaMin; }
AVR_HD float table_at(const float *t, int off) { return (off < 0 || off >= kNTable) ? 0.f : t[off]; }
struct LambdaIdx { int o0, o1, o2, o3; };
AVR_HD LambdaIdx lambda_index(const Spec &l) {
    return {lambda_offset(l.v0), lambda_offset(l.v1), lambda_offset(l.v2), lambda_offset(l.v3)};
}
AVR_HD Spec sample_table(const float *t, const LambdaIdx &i) {
    return {table_at(t, i.o0), table_at(t, i.o1), table_at(t, i.o2), table_at(t, i.o3)};
}

// sampling.h:222-225, 79-110
AVR_HD float sample_exponential(float u, float a) { return -cr_log(1 - u) / a; }
AVR_HD int sample_discrete3(float w0, float w1, float w2, float u) {
    float sum = ((0.f + w0) + w1) + w2;
    float up = u * sum;
    if (up == sum) up = next_down(up);
    if (0.f + w0 > up) return 0;
    float s = 0.f + w0;
    if (s + w1 > up) return 1;
    return 2;
}

// HG phase function — scattering.h:49-58, sampling.cpp:348-372, vecmath.h:1007-1013,1666-1672,1916
// Henyey-Greenstein's g-only terms, evaluated once per medium on the host with the same float
// operations hg_eval / hg_sample apply (so hg_eval_c / hg_sample_c return the same bits): the
// persistent kernel reads them as scalar kernel arguments instead of keeping hoisted copies in
// VGPRs. a = 1 + g^2, b = 2g, k = Inv4Pi (1 - g^2), c = 1 - g^2, m = -1 / (2g), d = 1 + g.
struct HgC {
    float g, a, b, k, c, m, d;
    int iso;   // |g| < 1e-3: uniform cosTheta
};
AVR_HD HgC hg_consts(float g) {
    HgC h;
    g = clampf(g, -.99f, .99f);
    h.g = g;
    h.a = 1 + sqr(g);
    h.b = 2 * g;
    h.c = 1 - sqr(g);
    h.k = kInv4Pi * h.c;
    h.m = -1 / (2 * g);
    h.d = 1 + g;
    h.iso = __builtin_fabsf(g) < 1e-3f ? 1 : 0;
    return h;
}
AVR_HD float hg_eval(float cosTheta, float g) {
    g = clampf(g, -.99f, .99f);
    float denom = 1 + sqr(g) + 2 * g * cosTheta;
    return kInv4Pi * (1 - sqr(g)) / (denom * __builtin_sqrtf(fmaxf_(0.f, denom)));
}
template <bool kFast = false>
AVR_HD V3 hg_sample(V3 wo, float g, float u0, float u1, float *pdf) {
    g = clampf(g, -.99f, .99f);
    float cosTheta;
    if (__builtin_fabsf(g) < 1e-3f) cosTheta = 1 - 2 * u0;
    else cosTheta = -1 / (2 * g) * (1 + sqr(g) - sqr((1 - sqr(g)) / (1 + g - 2 * g * u0)));
    float sinTheta = __builtin_sqrtf(fmaxf_(0.f, 1 - sqr(cosTheta)));
    float phi = 2 * kPi * u1;
    float sign = __builtin_copysignf(1.f, wo.z);
    float a = -1 / (sign + wo.z);
    float b = wo.x * wo.y * a;
    V3 fx = {1 + sign * sqr(wo.x) * a, sign * b, -sign * wo.x};
    V3 fy = {b, sign + sqr(wo.y) * a, -wo.y};
    float st = clampf(sinTheta, -1, 1);
    float sinPhi, cosPhi;
    if (kFast) hw_sincos_turns(u1, &sinPhi, &cosPhi);   // sin / cos of 2 pi u1 in hardware
    else cr_sincos(phi, &sinPhi, &cosPhi);
    V3 s = {st * cosPhi, st * sinPhi, clampf(cosTheta, -1, 1)};
    V3 wi = s.x * fx + s.y * fy + s.z * wo;
    *pdf = hg_eval(cosTheta, g);
    return wi;
}

// hg_eval / hg_sample from the precomputed terms (HgC): bit-identical results
AVR_HD float hg_eval_c(float cosTheta, const HgC &h) {
    float denom = h.a + h.b * cosTheta;
    return h.k / (denom * __builtin_sqrtf(fmaxf_(0.f, denom)));
}
template <bool kFast = false>
AVR_HD V3 hg_sample_c(V3 wo, const HgC &h, float u0, float u1, float *pdf) {
    float cosTheta;
    if (h.iso) cosTheta = 1 - 2 * u0;
    else cosTheta = h.m * (h.a - sqr(h.c / (h.d - h.b * u0)));
    float sinTheta = __builtin_sqrtf(fmaxf_(0.f, 1 - sqr(cosTheta)));
    float phi = 2 * kPi * u1;
    float sign = __builtin_copysignf(1.f, wo.z);
    float a = -1 / (sign + wo.z);
    float b = wo.x * wo.y * a;
    V3 fx = {1 + sign * sqr(wo.x) * a, sign * b, -sign * wo.x};
    V3 fy = {b, sign + sqr(wo.y) * a, -wo.y};
    float st = clampf(sinTheta, -1, 1);
    float sinPhi, cosPhi;
    if (kFast) hw_sincos_turns(u1, &sinPhi, &cosPhi);
    else cr_sincos(phi, &sinPhi, &cosPhi);
    V3 s = {st * cosPhi, st * sinPhi, clampf(cosTheta, -1, 1)};
    V3 wi = s.x * fx + s.y * fy + s.z * wo;
    *pdf = hg_eval_c(cosTheta, h);
    return wi;
}

// ---------------------------------------------------------------------------
// Affine transform rows (3x4, row-major) and pbrt's ray transforms with the
// interval-error origin offset — transform.h:136-179, 340-351, 391-433, transform.cpp:263-302
struct Xf { float m[12]; };
AVR_HD V3 xf_point_lr(const Xf &t, V3 p) {  // Transform::operator()(Point3<T>): left-to-right sums
    return {t.m[0] * p.x + t.m[1] * p.y + t.m[2] * p.z + t.m[3], t.m[4] * p.x + t.m[5] * p.y + t.m[6] * p.z + t.m[7],
            t.m[8] * p.x + t.m[9] * p.y + t.m[10] * p.z + t.m[11]};
}
AVR_HD V3 xf_point_pair(const Xf &t, V3 p) {  // ApplyInverse(Point3<T>) / Point3fi: pairwise grouping
    return {(t.m[0] * p.x + t.m[1] * p.y) + (t.m[2] * p.z + t.m[3]),
            (t.m[4] * p.x + t.m[5] * p.y) + (t.m[6] * p.z + t.m[7]),
            (t.m[8] * p.x + t.m[9] * p.y) + (t.m[10] * p.z + t.m[11])};
}
AVR_HD V3 xf_vector(const Xf &t, V3 v) {
    return {t.m[0] * v.x + t.m[1] * v.y + t.m[2] * v.z, t.m[4] * v.x + t.m[5] * v.y + t.m[6] * v.z,
            t.m[8] * v.x + t.m[9] * v.y + t.m[10] * v.z};
}
struct Ray { V3 o, d; };
// forward=true: Transform::operator()(Ray) (error includes |m[i][3]|); false: ApplyInverse(Ray)
AVR_HD Ray xf_ray(const Xf &t, Ray r, float *tMax, bool forward) {
    float v[3], lo[3], hi[3];
    const float g3 = gamma_n(3);
    _Pragma("unroll") for (int i = 0; i < 3; ++i) {
        const float *m = &t.m[4 * i];
        v[i] = (m[0] * r.o.x + m[1] * r.o.y) + (m[2] * r.o.z + m[3]);
        float e = __builtin_fabsf(m[0] * r.o.x) + __builtin_fabsf(m[1] * r.o.y) + __builtin_fabsf(m[2] * r.o.z);
        if (forward) e = e + __builtin_fabsf(m[3]);
        e = g3 * e;
        if (e == 0) { lo[i] = hi[i] = v[i]; }
        else { lo[i] = next_down(v[i] + -e); hi[i] = next_up(v[i] + e); }
    }
    V3 d = xf_vector(t, r.d);
    float lsq = length_sq(d);
    if (lsq > 0) {
        V3 oerr = {(hi[0] - lo[0]) / 2, (hi[1] - lo[1]) / 2, (hi[2] - lo[2]) / 2};
        float dt = dot({__builtin_fabsf(d.x), __builtin_fabsf(d.y), __builtin_fabsf(d.z)}, oerr) / lsq;
        V3 dd = d * dt;
        float ddv[3] = {dd.x, dd.y, dd.z};
        _Pragma("unroll") for (int i = 0; i < 3; ++i) {
            float a = next_down(lo[i] + ddv[i]), b = next_up(hi[i] + ddv[i]);
            lo[i] = fminf_(a, b); hi[i] = fmaxf_(a, b);
        }
        if (tMax) *tMax -= dt;
    }
    return {{(lo[0] + hi[0]) / 2, (lo[1] + hi[1]) / 2, (lo[2] + hi[2]) / 2}, d};
}

// Bounds3::IntersectP — vecmath.h:1547-1571
AVR_HD bool intersect_box(const float bmin[3], const float bmax[3], V3 o, V3 d, float tMax, float *h0, float *h1) {
    float t0 = 0, t1 = tMax;
    const float s = 1 + 2 * gamma_n(3);
    _Pragma("unroll") for (int i = 0; i < 3; ++i) {
        float inv = 1 / comp(d, i);
        float tNear = (bmin[i] - comp(o, i)) * inv;
        float tFar = (bmax[i] - comp(o, i)) * inv;
        if (tNear > tFar) { float tt = tNear; tNear = tFar; tFar = tt; }
        tFar *= s;
        t0 = tNear > t0 ? tNear : t0;
        t1 = tFar < t1 ? tFar : t1;
        if (t0 > t1) return false;
    }
    *h0 = t0; *h1 = t1;
    return true;
}
// Bounds3::Offset — vecmath.h:1323-1332
AVR_HD V3 box_offset(const float bmin[3], const float bmax[3], V3 p) {
    V3 o = {p.x - bmin[0], p.y - bmin[1], p.z - bmin[2]};
    if (bmax[0] > bmin[0]) o.x /= bmax[0] - bmin[0];
    if (bmax[1] > bmin[1]) o.y /= bmax[1] - bmin[1];
    if (bmax[2] > bmin[2]) o.z /= bmax[2] - bmin[2];
    return o;
}

}  // namespace avr

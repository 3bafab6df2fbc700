// volpath_oracle.cpp — ORACLE / TEST INFRASTRUCTURE. Never on the product path.
//
// A plain scalar C++ restatement of pbrt-v4's null-scattering volumetric path
// integrator (the AcceleratedVolRenderer reference, /root/reference) for the
// scene subset the MI355X path supports. Only tests/, __graft_entry__.smoke()
// and bench.py's cpu_baseline leg load it, as the checker / CPU baseline.
//
// Every function cites the reference file:line it restates (paths relative to
// /root/reference/src/pbrt). Float order of operations follows the reference
// exactly (compile with -ffp-contract=off, as pbrt's CMakeLists.txt:134-137 does),
// so per-sample radiance is reproducible bit for bit on the same libm.
// Pinned by tests/golden/ref_vectors.json, produced by the REAL reference code
// (oracle/ref/ref_harness.cpp built from the unmodified sources).
//
// Scene subset (see DESIGN.md "Scene model"):
//  * one GridMedium (media.h:265-352) whose bounds are also the scene's only
//    boundary (an "interface" box: rays enter/leave it without scattering,
//    interaction.cpp:91-97); camera outside, lights outside;
//  * DistantLight (lights.h:244-305) and UniformInfiniteLight (lights.cpp:950-972),
//    picked by the BVH light sampler's infinite-light branch (lightsamplers.h:266-277);
//  * orthographic / perspective pinhole cameras (cameras.cpp:284-306, 404-427);
//  * IndependentSampler (samplers.h:442-476), box filter (filters.h:48-77);
//  * RGBFilm + cie1931 PixelSensor (film.h:95-100, 232-316).
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <numeric>
#include <thread>
#include <unordered_map>
#include <vector>

namespace oracle {

// ---------------------------------------------------------------------------
// Float helpers — util/float.h:131-300
static inline uint32_t FloatToBits(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }
static inline float BitsToFloat(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }
static const float Infinity = std::numeric_limits<float>::infinity();
static const float OneMinusEpsilon = 0x1.fffffep-1f;  // util/math.h
static const float MachineEpsilon = std::numeric_limits<float>::epsilon() * 0.5f;
static const float Pi = 3.14159265358979323846f, Inv4Pi = 0.07957747154594766788f;
static const float ShadowEpsilon = 0.0001f;                    // util/math.h:42
static inline float gamma(int n) { return (n * MachineEpsilon) / (1 - n * MachineEpsilon); }

// util/float.h:164-193
static inline float NextFloatUp(float v) {
    if (std::isinf(v) && v > 0.f) return v;
    if (v == -0.f) v = 0.f;
    uint32_t ui = FloatToBits(v);
    if (v >= 0) ++ui; else --ui;
    return BitsToFloat(ui);
}
static inline float NextFloatDown(float v) {
    if (std::isinf(v) && v < 0.) return v;
    if (v == 0.f) v = -0.f;
    uint32_t ui = FloatToBits(v);
    if (v > 0) --ui; else ++ui;
    return BitsToFloat(ui);
}
// CPU branches of util/float.h:199-227
static inline float AddRoundUp(float a, float b) { return NextFloatUp(a + b); }
static inline float AddRoundDown(float a, float b) { return NextFloatDown(a + b); }
static inline float SubRoundUp(float a, float b) { return AddRoundUp(a, -b); }
static inline float SubRoundDown(float a, float b) { return AddRoundDown(a, -b); }

template <typename T, typename U, typename V>
static inline T Clamp(T val, U low, V high) {  // util/math.h:237-244
    if (val < low) return T(low);
    else if (val > high) return T(high);
    return val;
}
static inline float Lerp(float x, float a, float b) { return (1 - x) * a + x * b; }  // math.h:210
static inline float Sqr(float v) { return v * v; }
static inline float SafeSqrt(float x) { return std::sqrt(std::max(0.f, x)); }        // math.h:276

// FastExp, CPU branch — util/math.h:450-471 (EvaluatePolynomial uses std::fma, math.h:335)
static inline float FastExp(float x) {
    float xp = x * 1.442695041f;
    float fxp = std::floor(xp), f = xp - fxp;
    int i = (int)fxp;
    float twoToF = std::fma(f, std::fma(f, std::fma(f, 0.0781455737f, 0.226173572f), 0.695556856f), 1.f);
    int exponent = (int)(FloatToBits(twoToF) >> 23) - 127 + i;
    if (exponent < -126) return 0;
    if (exponent > 127) return Infinity;
    uint32_t bits = FloatToBits(twoToF);
    bits &= 0b10000000011111111111111111111111u;
    bits |= (uint32_t)(exponent + 127) << 23;
    return BitsToFloat(bits);
}

// ---------------------------------------------------------------------------
// Hash — util/hash.h:19-106
static inline uint64_t MurmurHash64A(const unsigned char *key, size_t len, uint64_t seed) {
    const uint64_t m = 0xc6a4a7935bd1e995ull;
    const int r = 47;
    uint64_t h = seed ^ (len * m);
    const unsigned char *end = key + 8 * (len / 8);
    while (key != end) {
        uint64_t k;
        std::memcpy(&k, key, 8);
        key += 8;
        k *= m; k ^= k >> r; k *= m;
        h ^= k; h *= m;
    }
    switch (len & 7) {
    case 7: h ^= uint64_t(key[6]) << 48; [[fallthrough]];
    case 6: h ^= uint64_t(key[5]) << 40; [[fallthrough]];
    case 5: h ^= uint64_t(key[4]) << 32; [[fallthrough]];
    case 4: h ^= uint64_t(key[3]) << 24; [[fallthrough]];
    case 3: h ^= uint64_t(key[2]) << 16; [[fallthrough]];
    case 2: h ^= uint64_t(key[1]) << 8; [[fallthrough]];
    case 1: h ^= uint64_t(key[0]); h *= m;
    }
    h ^= h >> r; h *= m; h ^= h >> r;
    return h;
}
static inline uint64_t MixBits(uint64_t v) {
    v ^= (v >> 31); v *= 0x7fb5d329728ea185; v ^= (v >> 27); v *= 0x81dadef4bc2dd44d; v ^= (v >> 33);
    return v;
}
static inline uint64_t HashBytes(const void *p, size_t n) { return MurmurHash64A((const unsigned char *)p, n, 0); }
static inline uint64_t HashFloat(float f) { return HashBytes(&f, 4); }
// Hash(int, int): the variadic Hash packs its arguments' bytes (util/hash.h:94-106)
static inline uint64_t HashInts2(int a, int b) {
    unsigned char buf[8];
    std::memcpy(buf, &a, 4);
    std::memcpy(buf + 4, &b, 4);
    return HashBytes(buf, 8);
}
static inline uint64_t HashPixelSeed(int x, int y, int seed) {
    int buf[3] = {x, y, seed};
    return HashBytes(buf, 12);
}

// ---------------------------------------------------------------------------
// RNG (PCG32) — util/rng.h:25-160
struct RNG {
    uint64_t state = 0x853c49e6748fea9bULL, inc = 0xda3e39cb94b95bdbULL;
    RNG() = default;
    RNG(uint64_t seq, uint64_t seed) { SetSequence(seq, seed); }
    void SetSequence(uint64_t seq, uint64_t seed) {
        state = 0u;
        inc = (seq << 1u) | 1u;
        U32();
        state += seed;
        U32();
    }
    void SetSequence(uint64_t seq) { SetSequence(seq, MixBits(seq)); }
    uint32_t U32() {
        uint64_t oldstate = state;
        state = oldstate * 0x5851f42d4c957f2dULL + inc;
        uint32_t xorshifted = (uint32_t)(((oldstate >> 18u) ^ oldstate) >> 27u);
        uint32_t rot = (uint32_t)(oldstate >> 59u);
        return (xorshifted >> rot) | (xorshifted << ((~rot + 1u) & 31));
    }
    float Uniform() { return std::min<float>(OneMinusEpsilon, U32() * 0x1p-32f); }
    void Advance(int64_t idelta) {
        uint64_t curMult = 0x5851f42d4c957f2dULL, curPlus = inc, accMult = 1u, accPlus = 0u;
        uint64_t delta = (uint64_t)idelta;
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
// Vectors — util/vecmath.h
struct V3 { float x, y, z; float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
            float &operator[](int i) { return i == 0 ? x : (i == 1 ? y : z); } };
static inline V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
static inline V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
static inline V3 operator*(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
static inline V3 operator*(float s, V3 a) { return {s * a.x, s * a.y, s * a.z}; }
static inline V3 operator/(V3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }      // vecmath.h:364-367
static inline V3 operator-(V3 a) { return {-a.x, -a.y, -a.z}; }
static inline float Dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }      // vecmath.h:963
static inline float LengthSquared(V3 v) { return Sqr(v.x) + Sqr(v.y) + Sqr(v.z); }     // vecmath.h:948
static inline float Length(V3 v) { return std::sqrt(LengthSquared(v)); }
static inline V3 Normalize(V3 v) { return v / Length(v); }
static inline V3 Abs(V3 v) { return {std::abs(v.x), std::abs(v.y), std::abs(v.z)}; }

// libm policy. pbrt calls the float overloads of std::log / sin / cos / atanh / cosh, whose
// last-ulp results are platform-specific: glibc 2.35 picks FMA or non-FMA variants at load
// time, and MSVC and CUDA's libdevice differ again. So pbrt's own sample streams differ
// across builds in ~1% of transcendental calls (then a path may take another, equally valid
// branch). Mode 0 ("platform", the default) calls them exactly as pbrt does; this is what
// the golden vectors of the reference harness built here pin. Mode 1 ("canonical") is the
// HIP path's convention: each function evaluated in f64 by a fixed sequence of IEEE ops
// (+ - * fma, table lookups), then rounded once to float, which is the correctly rounded
// float except within ~1e-15 of a midpoint. Restated here from the convention's definition
// (7-bit log table + degree-8 log1p, 2^(j/64) table + degree-6 exp for cosh, Cody-Waite
// sincos with 1/k! coefficients) independently of the device header
// acceleratedvolrenderer_amd/csrc/avr_canon.h; parity tests require the two to agree.
static int g_libm = 0;
namespace canon {
static const double kLn2Hi = 0x1.62e42fee00000p-1, kLn2Lo = 0x1.a39ef35793c76p-33;
static const double kPio2Hi = 0x1.921fb54400000p+0, kPio2Lo = 0x1.0b4611a626331p-34;
static const double kTwoOverPi = 0x1.45f306dc9c883p-1, kInvLn2 = 0x1.71547652b82fep+0;
static const double kSqrt2 = 0x1.6a09e667f3bcdp+0;
// 1/k!, k = 0..23, each the nearest double to the exact rational
static const double kInvFact[24] = {
    0x1.0000000000000p+0, 0x1.0000000000000p+0, 0x1.0000000000000p-1, 0x1.5555555555555p-3,
    0x1.5555555555555p-5, 0x1.1111111111111p-7, 0x1.6c16c16c16c17p-10, 0x1.a01a01a01a01ap-13,
    0x1.a01a01a01a01ap-16, 0x1.71de3a556c734p-19, 0x1.27e4fb7789f5cp-22, 0x1.ae64567f544e4p-26,
    0x1.1eed8eff8d898p-29, 0x1.6124613a86d09p-33, 0x1.93974a8c07c9dp-37, 0x1.ae7f3e733b81fp-41,
    0x1.ae7f3e733b81fp-45, 0x1.952c77030ad4ap-49, 0x1.6827863b97d97p-53, 0x1.2f49b46814157p-57,
    0x1.e542ba4020225p-62, 0x1.71b8ef6dcf572p-66, 0x1.0ce396db7f853p-70, 0x1.761b41316381ap-75,
};
static double InvFact(int k) { return kInvFact[k]; }
// Horner over c[0] (highest power) .. c[n-1] with fma
static double Horner(const double *c, int n, double z) {
    double p = c[0];
    for (int i = 1; i < n; ++i) p = std::fma(p, z, c[i]);
    return p;
}
struct Tables {
    double sinp[8], cosp[8];
    Tables() {
        for (int i = 0; i < 8; ++i) sinp[i] = ((7 - i) % 2 ? -1 : 1) * InvFact(15 - 2 * i);   // -1/15! .. 1
        for (int i = 0; i < 8; ++i) cosp[i] = ((7 - i) % 2 ? -1 : 1) * InvFact(16 - 2 * i);   // -1/16! .. 1/2
    }
};
static const Tables T;
// The path's log / atanh / cosh (the convention's table-driven forms; tables from
// tools/gen_canon_tables.py: each entry the double nearest to the exact value)
static const double kLogInvC[128] = {
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
};   // 1 / (1 + k/128)
static const double kLogC[128] = {
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
};   // log(1 + k/128)
static const double kExp2J64[64] = {
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
};   // 2^(j/64)
static const double kLn2_64Hi = 0x1.62e42fee00000p-7, kLn2_64Lo = 0x1.a39ef35793c76p-39;
static const double k64OverLn2 = 0x1.71547652b82fep+6;
// log1p(r) - r over r^2, degree 6 in r: -1/2 + r/3 - r^2/4 + ... - r^6/8 (coefficients 1/k
// rounded to double), highest first
static const double kLog1pQ[7] = {-1.0 / 8, 1.0 / 7, -1.0 / 6, 1.0 / 5, -1.0 / 4, 1.0 / 3, -1.0 / 2};
static double Log(double x) {
    if (!(x > 0)) return x == 0 ? -INFINITY : NAN;
    if (std::isinf(x)) return x;
    uint64_t b;
    std::memcpy(&b, &x, 8);
    int e = (int)((b >> 52) & 0x7ff) - 1023;
    const uint64_t frac = b & 0x000fffffffffffffull;
    int k = (int)((frac + (1ull << 44)) >> 45);   // the fraction rounded to 7 bits
    uint64_t mb = frac | 0x3ff0000000000000ull;
    double m;
    std::memcpy(&m, &mb, 8);
    if (k == 128) {   // m close to 2: use m / 2 next to c = 1
        m = m * 0.5;
        e += 1;
        k = 0;
    }
    const double c = 1.0 + k / 128.0;
    const double r = (m - c) * kLogInvC[k];
    const double l1 = std::fma(r * r, Horner(kLog1pQ, 7, r), r);
    return std::fma((double)e, kLn2Hi, std::fma((double)e, kLn2Lo, kLogC[k] + l1));
}
static double Atanh(double x) {
    if (std::fabs(x) < 0x1p-26) return x;
    return 0.5 * (Log(1.0 + x) - Log(1.0 - x));
}
// e^r to degree 6 (1/k! rounded), highest first
static const double kExpP6[7] = {0x1.6c16c16c16c17p-10, 0x1.1111111111111p-7, 0x1.5555555555555p-5,
                                  0x1.5555555555555p-3, 0.5, 1.0, 1.0};
static double Exp2N64(int n) {   // 2^(n/64)
    uint64_t sb = (uint64_t)((n >> 6) + 1023) << 52;
    double sc;
    std::memcpy(&sc, &sb, 8);
    return kExp2J64[n & 63] * sc;
}
static double Cosh(double x) {
    const double ax = std::fabs(x);
    const double nf = std::rint(ax * k64OverLn2);
    const double r = (ax - nf * kLn2_64Hi) - nf * kLn2_64Lo;
    const int n = (int)nf;
    const double ep = Horner(kExpP6, 7, r) * Exp2N64(n);
    const double em = Horner(kExpP6, 7, -r) * Exp2N64(-n);
    return 0.5 * (ep + em);
}
static void SinCos(double x, double *sn, double *cs) {
    double kf = std::rint(x * kTwoOverPi);
    double r = (x - kf * kPio2Hi) - kf * kPio2Lo;
    double z = r * r;
    double sr = r * Horner(T.sinp, 8, z);
    double cr = std::fma(-z, Horner(T.cosp, 8, z), 1.0);
    switch ((int)kf & 3) {
    case 0: *sn = sr; *cs = cr; break;
    case 1: *sn = cr; *cs = -sr; break;
    case 2: *sn = -sr; *cs = -cr; break;
    default: *sn = -cr; *cs = sr; break;
    }
}
}  // namespace canon
static inline float LmLog(float x) { return g_libm ? (float)canon::Log((double)x) : std::log(x); }
static inline float LmAtanh(float x) { return g_libm ? (float)canon::Atanh((double)x) : std::atanh(x); }
static inline float LmCosh(float x) { return g_libm ? (float)canon::Cosh((double)x) : std::cosh(x); }
static inline void LmSinCos(float x, float *s, float *c) {
    if (g_libm) {
        double sd, cd;
        canon::SinCos((double)x, &sd, &cd);
        *s = (float)sd;
        *c = (float)cd;
    } else {
        *s = std::sin(x);
        *c = std::cos(x);
    }
}

// CoordinateSystem / Frame::FromZ / FromLocal — vecmath.h:1007-1013, 1868-1916
static inline void CoordinateSystem(V3 v1, V3 *v2, V3 *v3) {
    float sign = std::copysign(1.f, v1.z);
    float a = -1 / (sign + v1.z);
    float b = v1.x * v1.y * a;
    *v2 = {1 + sign * Sqr(v1.x) * a, sign * b, -sign * v1.x};
    *v3 = {b, sign + Sqr(v1.y) * a, -v1.y};
}
static inline V3 SphericalDirection(float sinTheta, float cosTheta, float phi) {  // vecmath.h:1666
    float sinPhi, cosPhi;
    LmSinCos(phi, &sinPhi, &cosPhi);
    return {Clamp(sinTheta, -1, 1) * cosPhi, Clamp(sinTheta, -1, 1) * sinPhi,
            Clamp(cosTheta, -1, 1)};
}

// Interval arithmetic — util/math.h:818-1014 (CPU rounding branch)
struct Interval {
    float low, high;
    static Interval Exact(float v) { return {v, v}; }
    static Interval FromValueAndError(float v, float err) {
        if (err == 0) return {v, v};
        return {SubRoundDown(v, err), AddRoundUp(v, err)};
    }
    float Midpoint() const { return (low + high) / 2; }
    float Width() const { return high - low; }
};
static inline Interval IvAdd(Interval a, float f) {  // Interval + Interval(f)
    float lo = AddRoundDown(a.low, f), hi = AddRoundUp(a.high, f);
    return {std::min(lo, hi), std::max(lo, hi)};
}

// ---------------------------------------------------------------------------
// Transforms (affine, row-major m[4][4]) — util/transform.h / transform.cpp
struct Xform { float m[4][4], mInv[4][4]; };

// Transform::operator()(Point3<T>) — transform.h:313-322
static inline V3 XPoint(const float (&m)[4][4], V3 p) {
    float xp = m[0][0] * p.x + m[0][1] * p.y + m[0][2] * p.z + m[0][3];
    float yp = m[1][0] * p.x + m[1][1] * p.y + m[1][2] * p.z + m[1][3];
    float zp = m[2][0] * p.x + m[2][1] * p.y + m[2][2] * p.z + m[2][3];
    float wp = m[3][0] * p.x + m[3][1] * p.y + m[3][2] * p.z + m[3][3];
    if (wp == 1) return {xp, yp, zp};
    return V3{xp, yp, zp} / wp;
}
// Transform::operator()(Vector3<T>) / ApplyInverse(Vector3<T>) — transform.h:324-329, 405-410
static inline V3 XVector(const float (&m)[4][4], V3 v) {
    return {m[0][0] * v.x + m[0][1] * v.y + m[0][2] * v.z, m[1][0] * v.x + m[1][1] * v.y + m[1][2] * v.z,
            m[2][0] * v.x + m[2][1] * v.y + m[2][2] * v.z};
}
// Transform::ApplyInverse(Point3<T>) — transform.h:391-403 (note the pairwise grouping)
static inline V3 XInvPoint(const Xform &t, V3 p) {
    const auto &mi = t.mInv;
    float xp = (mi[0][0] * p.x + mi[0][1] * p.y) + (mi[0][2] * p.z + mi[0][3]);
    float yp = (mi[1][0] * p.x + mi[1][1] * p.y) + (mi[1][2] * p.z + mi[1][3]);
    float zp = (mi[2][0] * p.x + mi[2][1] * p.y) + (mi[2][2] * p.z + mi[2][3]);
    float wp = (mi[3][0] * p.x + mi[3][1] * p.y) + (mi[3][2] * p.z + mi[3][3]);
    if (wp == 1) return {xp, yp, zp};
    return V3{xp, yp, zp} / wp;
}
// Point3fi transform of an EXACT point: value + absolute error bound.
// forward: transform.h:136-179 (error includes |m[i][3]|); inverse: transform.cpp:263-302
// (error excludes |mInv[i][3]|). Affine transforms only (wp == 1).
static inline void XPointExactErr(const float (&m)[4][4], V3 p, bool inverse, V3 *v, V3 *err) {
    for (int i = 0; i < 3; ++i) {
        (*v)[i] = (m[i][0] * p.x + m[i][1] * p.y) + (m[i][2] * p.z + m[i][3]);
        float e = std::abs(m[i][0] * p.x) + std::abs(m[i][1] * p.y) + std::abs(m[i][2] * p.z);
        if (!inverse) e = e + std::abs(m[i][3]);
        (*err)[i] = gamma(3) * e;
    }
}
struct Ray { V3 o, d; };
// Transform::operator()(Ray, tMax) — transform.h:340-351 and ApplyInverse(Ray, tMax) — :420-433
static inline Ray XRay(const Xform &t, Ray r, float *tMax, bool inverse) {
    const auto &m = inverse ? t.mInv : t.m;
    V3 v, e;
    XPointExactErr(m, r.o, inverse, &v, &e);
    Interval o[3];
    for (int i = 0; i < 3; ++i) o[i] = Interval::FromValueAndError(v[i], e[i]);
    V3 d = XVector(m, r.d);
    float lengthSquared = LengthSquared(d);
    if (lengthSquared > 0) {
        V3 oErr = {o[0].Width() / 2, o[1].Width() / 2, o[2].Width() / 2};
        float dt = Dot(Abs(d), oErr) / lengthSquared;
        V3 dd = d * dt;
        for (int i = 0; i < 3; ++i) o[i] = IvAdd(o[i], dd[i]);
        if (tMax) *tMax -= dt;
    }
    return {{o[0].Midpoint(), o[1].Midpoint(), o[2].Midpoint()}, d};
}

// ---------------------------------------------------------------------------
// Bounds3f::IntersectP — vecmath.h:1547-1571; Offset — vecmath.h:1323-1332
struct Bounds { V3 pMin, pMax; };
static inline bool IntersectP(const Bounds &b, V3 o, V3 d, float tMax, float *hitt0, float *hitt1) {
    float t0 = 0, t1 = tMax;
    for (int i = 0; i < 3; ++i) {
        float invRayDir = 1 / d[i];
        float tNear = (b.pMin[i] - o[i]) * invRayDir;
        float tFar = (b.pMax[i] - o[i]) * invRayDir;
        if (tNear > tFar) std::swap(tNear, tFar);
        tFar *= 1 + 2 * gamma(3);
        t0 = tNear > t0 ? tNear : t0;
        t1 = tFar < t1 ? tFar : t1;
        if (t0 > t1) return false;
    }
    *hitt0 = t0; *hitt1 = t1;
    return true;
}
static inline V3 Offset(const Bounds &b, V3 p) {
    V3 o = p - b.pMin;
    if (b.pMax.x > b.pMin.x) o.x /= b.pMax.x - b.pMin.x;
    if (b.pMax.y > b.pMin.y) o.y /= b.pMax.y - b.pMin.y;
    if (b.pMax.z > b.pMin.z) o.z /= b.pMax.z - b.pMin.z;
    return o;
}

// ---------------------------------------------------------------------------
// Spectra — util/spectrum.h (NSpectrumSamples = 4)
static const int NS = 4;
struct Spec {
    float v[NS];
    static Spec Const(float c) { return {{c, c, c, c}}; }
    float operator[](int i) const { return v[i]; }
    float &operator[](int i) { return v[i]; }
    explicit operator bool() const { for (int i = 0; i < NS; ++i) if (v[i] != 0) return true; return false; }
    float Average() const { float s = v[0]; for (int i = 1; i < NS; ++i) s += v[i]; return s / NS; }
    float MaxComponentValue() const { float m = v[0]; for (int i = 1; i < NS; ++i) m = std::max(m, v[i]); return m; }
};
static inline Spec operator+(Spec a, const Spec &b) { for (int i = 0; i < NS; ++i) a.v[i] += b.v[i]; return a; }
static inline Spec operator-(Spec a, const Spec &b) { for (int i = 0; i < NS; ++i) a.v[i] -= b.v[i]; return a; }
static inline Spec operator*(Spec a, const Spec &b) { for (int i = 0; i < NS; ++i) a.v[i] *= b.v[i]; return a; }
static inline Spec operator/(Spec a, const Spec &b) { for (int i = 0; i < NS; ++i) a.v[i] /= b.v[i]; return a; }
static inline Spec operator*(Spec a, float s) { for (int i = 0; i < NS; ++i) a.v[i] *= s; return a; }
static inline Spec operator*(float s, Spec a) { return a * s; }
static inline Spec operator/(Spec a, float s) { for (int i = 0; i < NS; ++i) a.v[i] /= s; return a; }
static inline Spec operator-(Spec a) { for (int i = 0; i < NS; ++i) a.v[i] = -a.v[i]; return a; }
static inline Spec ClampZero(Spec a) { for (int i = 0; i < NS; ++i) a.v[i] = std::max<float>(0, a.v[i]); return a; }
static inline Spec SafeDiv(Spec a, Spec b) {  // spectrum.h:634-639
    Spec r; for (int i = 0; i < NS; ++i) r.v[i] = (b.v[i] != 0) ? a.v[i] / b.v[i] : 0.f; return r;
}
static inline Spec FastExpSpec(Spec a) { for (int i = 0; i < NS; ++i) a.v[i] = FastExp(a.v[i]); return a; }

struct Lambda { float lambda[NS], pdf[NS]; };
// SampleVisibleWavelengths / VisibleWavelengthsPDF — sampling.h:163-171;
// SampledWavelengths::SampleVisible — spectrum.h:334-347
static inline float SampleVisibleWavelengths(float u) { return 538 - 138.888889f * LmAtanh(0.85691062f - 1.82750197f * u); }
static inline float VisibleWavelengthsPDF(float l) {
    if (l < 360 || l > 830) return 0;
    return 0.0039398042f / Sqr(LmCosh(0.0072f * (l - 538)));
}
static inline Lambda SampleVisible(float u) {
    Lambda w;
    for (int i = 0; i < NS; ++i) {
        float up = u + float(i) / NS;
        if (up > 1) up -= 1;
        w.lambda[i] = SampleVisibleWavelengths(up);
        w.pdf[i] = VisibleWavelengthsPDF(w.lambda[i]);
    }
    return w;
}
// SampledWavelengths::SampleUniform — spectrum.h:287-306 (SpectralFilm::SampleWavelengths,
// film.h:408-410): Lerp(u, min, max) then steps of (max - min) / 4 wrapped into the range
static inline Lambda SampleUniform(float u, float lmin, float lmax) {
    Lambda w;
    w.lambda[0] = (1 - u) * lmin + u * lmax;   // Lerp, util/math.h
    const float delta = (lmax - lmin) / NS;
    for (int i = 1; i < NS; ++i) {
        w.lambda[i] = w.lambda[i - 1] + delta;
        if (w.lambda[i] > lmax) w.lambda[i] = lmin + (w.lambda[i] - lmax);
    }
    for (int i = 0; i < NS; ++i) w.pdf[i] = 1 / (lmax - lmin);
    return w;
}
// DenselySampledSpectrum::Sample — spectrum.h:390-400 (table over 360..830 nm)
static inline Spec SampleDense(const float *table, const Lambda &l) {
    Spec s;
    for (int i = 0; i < NS; ++i) {
        int offset = (int)std::lround(l.lambda[i]) - 360;
        s.v[i] = (offset < 0 || offset >= 471) ? 0.f : table[offset];
    }
    return s;
}

// ---------------------------------------------------------------------------
// Sampling — sampling.h:79-110, 222-225; sampling.cpp:348-372; scattering.h:49-58
static inline float SampleExponential(float u, float a) { return -LmLog(1 - u) / a; }
static inline int SampleDiscrete3(const float w[3], float u) {
    float sumWeights = 0;
    for (int i = 0; i < 3; ++i) sumWeights += w[i];
    float up = u * sumWeights;
    if (up == sumWeights) up = NextFloatDown(up);
    int offset = 0;
    float sum = 0;
    while (sum + w[offset] <= up) sum += w[offset++];
    return offset;
}
static inline float HenyeyGreenstein(float cosTheta, float g) {
    g = Clamp(g, -.99, .99);
    float denom = 1 + Sqr(g) + 2 * g * cosTheta;
    return Inv4Pi * (1 - Sqr(g)) / (denom * SafeSqrt(denom));
}
static inline V3 SampleHenyeyGreenstein(V3 wo, float g, float u0, float u1, float *pdf) {
    g = Clamp(g, -.99, .99);
    float cosTheta;
    if (std::abs(g) < 1e-3f)
        cosTheta = 1 - 2 * u0;
    else
        cosTheta = -1 / (2 * g) * (1 + Sqr(g) - Sqr((1 - Sqr(g)) / (1 + g - 2 * g * u0)));
    float sinTheta = SafeSqrt(1 - Sqr(cosTheta));
    float phi = 2 * Pi * u1;
    V3 x, y;
    CoordinateSystem(wo, &x, &y);
    V3 s = SphericalDirection(sinTheta, cosTheta, phi);
    V3 wi = s.x * x + s.y * y + s.z * wo;  // Frame::FromLocal, vecmath.h:1916
    *pdf = HenyeyGreenstein(cosTheta, g);
    return wi;
}

// ---------------------------------------------------------------------------
// SampledGrid<float> — util/containers.h:765-870
struct Grid {
    const float *values = nullptr;
    int nx = 1, ny = 1, nz = 1;
    float At(int x, int y, int z) const {
        if (x < 0 || x >= nx || y < 0 || y >= ny || z < 0 || z >= nz) return 0.f;
        return values[(z * ny + y) * nx + x];
    }
    float Lookup(V3 p) const {
        V3 ps = {p.x * nx - .5f, p.y * ny - .5f, p.z * nz - .5f};
        int ix = (int)std::floor(ps.x), iy = (int)std::floor(ps.y), iz = (int)std::floor(ps.z);
        V3 d = {ps.x - (float)ix, ps.y - (float)iy, ps.z - (float)iz};
        float d00 = Lerp(d.x, At(ix, iy, iz), At(ix + 1, iy, iz));
        float d10 = Lerp(d.x, At(ix, iy + 1, iz), At(ix + 1, iy + 1, iz));
        float d01 = Lerp(d.x, At(ix, iy, iz + 1), At(ix + 1, iy, iz + 1));
        float d11 = Lerp(d.x, At(ix, iy + 1, iz + 1), At(ix + 1, iy + 1, iz + 1));
        return Lerp(d.z, Lerp(d.y, d00, d10), Lerp(d.y, d01, d11));
    }
    float MaxValue(const Bounds &b) const {
        V3 ps0 = {b.pMin.x * nx - .5f, b.pMin.y * ny - .5f, b.pMin.z * nz - .5f};
        V3 ps1 = {b.pMax.x * nx - .5f, b.pMax.y * ny - .5f, b.pMax.z * nz - .5f};
        int lo[3] = {std::max((int)std::floor(ps0.x), 0), std::max((int)std::floor(ps0.y), 0),
                     std::max((int)std::floor(ps0.z), 0)};
        int hi[3] = {std::min((int)std::floor(ps1.x) + 1, nx - 1), std::min((int)std::floor(ps1.y) + 1, ny - 1),
                     std::min((int)std::floor(ps1.z) + 1, nz - 1)};
        float maxValue = At(lo[0], lo[1], lo[2]);
        for (int z = lo[2]; z <= hi[2]; ++z)
            for (int y = lo[1]; y <= hi[1]; ++y)
                for (int x = lo[0]; x <= hi[0]; ++x) maxValue = std::max(maxValue, At(x, y, z));
        return maxValue;
    }
};

// ---------------------------------------------------------------------------
// Perlin noise — util/noise.cpp (Ken Perlin's public reference permutation)
static const int NoisePerm[512] = {
    151, 160, 137, 91, 90, 15, 131, 13, 201, 95, 96, 53, 194, 233, 7, 225, 140, 36, 103, 30, 69, 142,
    8, 99, 37, 240, 21, 10, 23, 190, 6, 148, 247, 120, 234, 75, 0, 26, 197, 62, 94, 252, 219, 203, 117,
    35, 11, 32, 57, 177, 33, 88, 237, 149, 56, 87, 174, 20, 125, 136, 171, 168, 68, 175, 74, 165, 71,
    134, 139, 48, 27, 166, 77, 146, 158, 231, 83, 111, 229, 122, 60, 211, 133, 230, 220, 105, 92, 41,
    55, 46, 245, 40, 244, 102, 143, 54, 65, 25, 63, 161, 1, 216, 80, 73, 209, 76, 132, 187, 208, 89,
    18, 169, 200, 196, 135, 130, 116, 188, 159, 86, 164, 100, 109, 198, 173, 186, 3, 64, 52, 217, 226,
    250, 124, 123, 5, 202, 38, 147, 118, 126, 255, 82, 85, 212, 207, 206, 59, 227, 47, 16, 58, 17, 182,
    189, 28, 42, 223, 183, 170, 213, 119, 248, 152, 2, 44, 154, 163, 70, 221, 153, 101, 155, 167, 43,
    172, 9, 129, 22, 39, 253, 19, 98, 108, 110, 79, 113, 224, 232, 178, 185, 112, 104, 218, 246, 97,
    228, 251, 34, 242, 193, 238, 210, 144, 12, 191, 179, 162, 241, 81, 51, 145, 235, 249, 14, 239,
    107, 49, 192, 214, 31, 181, 199, 106, 157, 184, 84, 204, 176, 115, 121, 50, 45, 127, 4, 150, 254,
    138, 236, 205, 93, 222, 114, 67, 29, 24, 72, 243, 141, 128, 195, 78, 66, 215, 61, 156, 180,
    151, 160, 137, 91, 90, 15, 131, 13, 201, 95, 96, 53, 194, 233, 7, 225, 140, 36, 103, 30, 69, 142,
    8, 99, 37, 240, 21, 10, 23, 190, 6, 148, 247, 120, 234, 75, 0, 26, 197, 62, 94, 252, 219, 203, 117,
    35, 11, 32, 57, 177, 33, 88, 237, 149, 56, 87, 174, 20, 125, 136, 171, 168, 68, 175, 74, 165, 71,
    134, 139, 48, 27, 166, 77, 146, 158, 231, 83, 111, 229, 122, 60, 211, 133, 230, 220, 105, 92, 41,
    55, 46, 245, 40, 244, 102, 143, 54, 65, 25, 63, 161, 1, 216, 80, 73, 209, 76, 132, 187, 208, 89,
    18, 169, 200, 196, 135, 130, 116, 188, 159, 86, 164, 100, 109, 198, 173, 186, 3, 64, 52, 217, 226,
    250, 124, 123, 5, 202, 38, 147, 118, 126, 255, 82, 85, 212, 207, 206, 59, 227, 47, 16, 58, 17, 182,
    189, 28, 42, 223, 183, 170, 213, 119, 248, 152, 2, 44, 154, 163, 70, 221, 153, 101, 155, 167, 43,
    172, 9, 129, 22, 39, 253, 19, 98, 108, 110, 79, 113, 224, 232, 178, 185, 112, 104, 218, 246, 97,
    228, 251, 34, 242, 193, 238, 210, 144, 12, 191, 179, 162, 241, 81, 51, 145, 235, 249, 14, 239,
    107, 49, 192, 214, 31, 181, 199, 106, 157, 184, 84, 204, 176, 115, 121, 50, 45, 127, 4, 150, 254,
    138, 236, 205, 93, 222, 114, 67, 29, 24, 72, 243, 141, 128, 195, 78, 66, 215, 61, 156, 180};
static inline float Pow3(float v) { return (v * v) * v; }   // math.h:295-309 (Pow<n> by squaring)
static inline float Pow4(float v) { float n2 = v * v; return n2 * n2; }
static inline float Pow5(float v) { float n2 = v * v; return (n2 * n2) * v; }
static inline float Grad(int x, int y, int z, float dx, float dy, float dz) {
    int h = NoisePerm[NoisePerm[NoisePerm[x] + y] + z];
    h &= 15;
    float u = h < 8 || h == 12 || h == 13 ? dx : dy;
    float v = h < 4 || h == 12 || h == 13 ? dy : dz;
    return ((h & 1) ? -u : u) + ((h & 2) ? -v : v);
}
static inline float NoiseWeight(float t) { return 6 * Pow5(t) - 15 * Pow4(t) + 10 * Pow3(t); }
static float Noise(float x, float y, float z) {
    x = std::fmod(x, float(1 << 30)); y = std::fmod(y, float(1 << 30)); z = std::fmod(z, float(1 << 30));
    int ix = (int)std::floor(x), iy = (int)std::floor(y), iz = (int)std::floor(z);
    float dx = x - ix, dy = y - iy, dz = z - iz;
    ix &= 255; iy &= 255; iz &= 255;
    float w000 = Grad(ix, iy, iz, dx, dy, dz), w100 = Grad(ix + 1, iy, iz, dx - 1, dy, dz);
    float w010 = Grad(ix, iy + 1, iz, dx, dy - 1, dz), w110 = Grad(ix + 1, iy + 1, iz, dx - 1, dy - 1, dz);
    float w001 = Grad(ix, iy, iz + 1, dx, dy, dz - 1), w101 = Grad(ix + 1, iy, iz + 1, dx - 1, dy, dz - 1);
    float w011 = Grad(ix, iy + 1, iz + 1, dx, dy - 1, dz - 1);
    float w111 = Grad(ix + 1, iy + 1, iz + 1, dx - 1, dy - 1, dz - 1);
    float wx = NoiseWeight(dx), wy = NoiseWeight(dy), wz = NoiseWeight(dz);
    float x00 = Lerp(wx, w000, w100), x10 = Lerp(wx, w010, w110);
    float x01 = Lerp(wx, w001, w101), x11 = Lerp(wx, w011, w111);
    float y0 = Lerp(wy, x00, x10), y1 = Lerp(wy, x01, x11);
    return Lerp(wz, y0, y1);
}
static inline V3 DNoise(V3 p) {
    float delta = .01f;
    float n = Noise(p.x, p.y, p.z);
    V3 nd = {Noise(p.x + delta, p.y + 0.f, p.z + 0.f), Noise(p.x + 0.f, p.y + delta, p.z + 0.f),
             Noise(p.x + 0.f, p.y + 0.f, p.z + delta)};
    return (nd - V3{n, n, n}) / delta;
}
// CloudMedium::Density — media.h:496-520 (the synthetic-cloud generator)
static float CloudDensity(V3 p, float density, float wispiness, float frequency) {
    V3 pp = frequency * p;
    if (wispiness > 0) {
        float vomega = 0.05f * wispiness, vlambda = 10.f;
        for (int i = 0; i < 2; ++i) {
            pp = pp + vomega * DNoise(vlambda * pp);
            vomega *= 0.5f;
            vlambda *= 1.99f;
        }
    }
    float d = 0, omega = 0.5f, lambda = 1.f;
    for (int i = 0; i < 5; ++i) {
        V3 q = lambda * pp;
        d += omega * Noise(q.x, q.y, q.z);
        omega *= 0.5f;
        lambda *= 1.99f;
    }
    d = Clamp((1 - p.y) * 4.5f * density * d, 0, 1);
    d += 2 * std::max<float>(0, 0.5f - p.y);
    return Clamp(d, 0, 1);
}

// Blackbody — spectrum.h:69-80, BlackbodySpectrum spectrum.h:500-530
static inline float Blackbody(float lambda, float T) {
    if (T <= 0) return 0;
    const float c = 299792458.f, h = 6.62606957e-34f, kb = 1.3806488e-23f;
    float l = lambda * 1e-9f;
    return (2 * h * c * c) / (Pow5(l) * (FastExp((h * c) / (l * kb * T)) - 1));
}

// ---------------------------------------------------------------------------
// NanoVDB FloatGrid as NanoVDBMedium reads it (media.h:624-672). NanoVDB itself
// (openvdb @ 414bed84, feature/nanovdb) is an empty submodule here: its published
// semantics are restated — ReadAccessor::getValue (leaf value, else tile value, else
// background), Map::applyInverseMapF (InvMatF * (p - VecF) with fmaf rows),
// SampleFromVoxels<Tree, 1, false> (floor / fraction, 2x2x2 stencil, lerp a + w(b - a)
// along z, y, then x). PARITY UNPINNED: no reference test or asset exercises it.
// Storage here is a hash map from leaf origin to its 512 values (x-major), independent
// of the device's block-slot layout.
struct VdbTree {
    std::unordered_map<uint64_t, const float *> leaves;
    std::vector<float> leafStore;
    std::vector<int> tileBox;      // ox, oy, oz, size per tile
    std::vector<float> tileValue;
    // 8^3 tiles by origin (a dense grid's constant blocks: ~10^5 of them at 1024^3); larger
    // tiles (128^3 / 4096^3 internal-node tiles, few) are searched in tileBox order
    std::unordered_map<uint64_t, float> tile8;
    std::vector<int> bigTiles;     // indices into tileValue of tiles larger than 8^3
    float background = 0;
    int ibbox[6] = {0, 0, 0, -1, -1, -1};
    double matD[12] = {};          // index -> world (3x3 row-major, translation in column 3)
    float invF[9] = {}, vecF[3] = {};
    static uint64_t Key(int x, int y, int z) {
        return ((uint64_t)(uint32_t)(x >> 3) & 0x1fffff) | (((uint64_t)(uint32_t)(y >> 3) & 0x1fffff) << 21) |
               (((uint64_t)(uint32_t)(z >> 3) & 0x1fffff) << 42);
    }
    float GetValue(int x, int y, int z) const {
        auto it = leaves.find(Key(x, y, z));
        if (it != leaves.end()) return it->second[(x & 7) * 64 + (y & 7) * 8 + (z & 7)];
        // tiles do not overlap in a valid tree: at most one contains (x, y, z)
        auto t8 = tile8.find(Key(x, y, z));
        if (t8 != tile8.end()) return t8->second;
        for (int t : bigTiles) {
            const int *b = &tileBox[4 * t];
            if (x >= b[0] && x < b[0] + b[3] && y >= b[1] && y < b[1] + b[3] && z >= b[2] && z < b[2] + b[3])
                return tileValue[t];
        }
        return background;
    }
    V3 WorldToIndexF(V3 p) const {
        const float x = p.x - vecF[0], y = p.y - vecF[1], z = p.z - vecF[2];
        return {std::fmaf(x, invF[0], std::fmaf(y, invF[1], z * invF[2])),
                std::fmaf(x, invF[3], std::fmaf(y, invF[4], z * invF[5])),
                std::fmaf(x, invF[6], std::fmaf(y, invF[7], z * invF[8]))};
    }
    float Sample(V3 q) const {
        const float fl[3] = {std::floor(q.x), std::floor(q.y), std::floor(q.z)};
        const int i = (int)fl[0], j = (int)fl[1], k = (int)fl[2];
        const float u = q.x - fl[0], v = q.y - fl[1], w = q.z - fl[2];
        float c[2][2][2];
        for (int a = 0; a < 2; ++a)
            for (int b = 0; b < 2; ++b)
                for (int d = 0; d < 2; ++d) c[a][b][d] = GetValue(i + a, j + b, k + d);
        auto lerp = [](float a, float b, float t) { return a + t * (b - a); };
        const float x0 = lerp(lerp(c[0][0][0], c[0][0][1], w), lerp(c[0][1][0], c[0][1][1], w), v);
        const float x1 = lerp(lerp(c[1][0][0], c[1][0][1], w), lerp(c[1][1][0], c[1][1][1], w), v);
        return lerp(x0, x1, u);
    }
    // world bbox: the map of the corners of [min, max + 1] (f64, evaluated left to right)
    void WorldBBox(double lo[3], double hi[3]) const {
        for (int a = 0; a < 3; ++a) { lo[a] = HUGE_VAL; hi[a] = -HUGE_VAL; }
        for (int cx = 0; cx < 2; ++cx)
            for (int cy = 0; cy < 2; ++cy)
                for (int cz = 0; cz < 2; ++cz) {
                    const double x = cx ? ibbox[3] + 1.0 : ibbox[0];
                    const double y = cy ? ibbox[4] + 1.0 : ibbox[1];
                    const double z = cz ? ibbox[5] + 1.0 : ibbox[2];
                    for (int r = 0; r < 3; ++r) {
                        const double wv = matD[4 * r] * x + matD[4 * r + 1] * y + matD[4 * r + 2] * z + matD[4 * r + 3];
                        lo[r] = std::min(lo[r], wv);
                        hi[r] = std::max(hi[r], wv);
                    }
                }
    }
};

// NanoVDBMedium ctor's 64^3 majorant (media.cpp:556-613)
static void VdbMajorant(const VdbTree &g, const float b[6], int rx, int ry, int rz, float *out) {
    const int res[3] = {rx, ry, rz};
    // z-slices on the host's threads (cells are independent; the tree is read-only)
    std::atomic<int> nextZ{0};
    auto slice = [&]() {
    for (int z; (z = nextZ.fetch_add(1)) < rz;)
        for (int y = 0; y < ry; ++y)
            for (int x = 0; x < rx; ++x) {
                const int c[3] = {x, y, z};
                float p0[3], p1[3], lo[3], hi[3];
                for (int a = 0; a < 3; ++a) {   // bounds.Lerp (vecmath.h Bounds3::Lerp, math.h Lerp)
                    p0[a] = Lerp(float(c[a]) / res[a], b[a], b[3 + a]);
                    p1[a] = Lerp(float(c[a] + 1) / res[a], b[a], b[3 + a]);
                    lo[a] = std::min(p0[a], p1[a]);
                    hi[a] = std::max(p0[a], p1[a]);
                }
                const V3 i0 = g.WorldToIndexF({lo[0], lo[1], lo[2]}), i1 = g.WorldToIndexF({hi[0], hi[1], hi[2]});
                const float delta = 1.f;   // filter slop
                int n0[3], n1[3];
                for (int a = 0; a < 3; ++a) {
                    n0[a] = std::max(int((double)i0[a] - delta), g.ibbox[a]);
                    n1[a] = std::min(int((double)i1[a] + delta), g.ibbox[3 + a]);
                }
                float maxValue = 0;
                for (int nz = n0[2]; nz <= n1[2]; ++nz)
                    for (int ny = n0[1]; ny <= n1[1]; ++ny)
                        for (int nx = n0[0]; nx <= n1[0]; ++nx) maxValue = std::max(maxValue, g.GetValue(nx, ny, nz));
                out[x + rx * (y + ry * z)] = maxValue;
            }
    };
    const int nt = std::max(1, std::min(16, (int)std::thread::hardware_concurrency()));
    std::vector<std::thread> th;
    for (int i = 0; i < nt; ++i) th.emplace_back(slice);
    for (auto &t : th) t.join();
}

}  // namespace oracle

// ===========================================================================
// Scene and integrator
// ===========================================================================
using namespace oracle;

extern "C" {

// Must match acceleratedvolrenderer_amd/oracle_binding.py (ctypes) field for field.
typedef struct OracleScene {
    // GridMedium (media.h:265-352 / media.cpp:212-330)
    const float *density; int nx, ny, nz;
    float bounds[6];                  // p0.xyz, p1.xyz (medium space)
    float render_from_medium[16];     // row-major m
    float medium_from_render[16];     // row-major mInv
    const float *sigma_a;             // 471 (DenselySampled, x sigmaScale)
    const float *sigma_s;             // 471
    float g;
    int emissive;                     // GridMedium::isEmissive
    const float *Le;                  // 471
    const float *Lescale; int lnx, lny, lnz;  // LeScale grid (LeNorm folded in)
    const float *majorant; int mres[3];       // MajorantGrid voxels (x fastest)
    // lights (BVHLightSampler infinite-light branch; lightsamplers.h:266-277, 323-326)
    int nlights;
    int light_type[8];                // 0 = distant (delta), 1 = uniform infinite
    float light_w[8][3];              // distant: render-space unit vector towards the light
    const float *light_L[8];          // 471 each
    float light_scale[8];
    float scene_radius;               // Bounds3::BoundingSphere of the scene bounds
    // camera (cameras.cpp:284-306 ortho, 404-427 perspective)
    int camera_type;                  // 0 ortho, 1 perspective
    float camera_from_raster[16];
    float render_from_camera[16];
    // RGBFilm (film.h:232-316) + cie1931 PixelSensor (film.h:95-100)
    int width, height;
    float filter_radius[2];           // filter radius (box or gaussian)
    const float *sensor_xyz;          // 3 x 471: X, Y, Z matching functions
    float imaging_ratio;
    float output_from_sensor[9];      // colorSpace->RGBFromXYZ * XYZFromSensorRGB
    float max_component_value;
    // VolPathIntegrator (integrators.cpp:1401-1409) + sampler seed
    int max_depth;
    int seed;
    // sampler (samplers.h): 0 IndependentSampler, 1 ZSobolSampler (FastOwen); its
    // samplesPerPixel (ZSobol's Morton layout depends on it) — film full resolution = width x height
    int sampler_type;
    int samples_per_pixel;
    // pixel filter (filters.h): 0 BoxFilter, 1 GaussianFilter(radius = filter_radius, sigma)
    int filter_type;
    float filter_sigma;
    // medium type: 0 GridMedium, 1 HomogeneousMedium (media.h:217-262, filling the
    // interface box), 2 CloudMedium (media.h:430-528) with {density, wispiness, frequency}
    int medium_type;
    float cloud[3];
    // GridMedium temperature grid (media.h:299-316; null = Le spectrum), scale, offset
    const float *temperature;
    float temperature_scale, temperature_offset;
    // medium_type 3, NanoVDBMedium (media.h:602-685): oracle_vdb_create handles for the
    // density and (nullable) temperature grids, LeScale
    const void *vdb;
    const void *vdb_temperature;
    float vdb_lescale;
    // medium_type 4, RGBGridMedium (media.h:355-427): nx*ny*nz voxels of {c0, c1, c2, scale}
    // for sigma_a / sigma_s (RGBUnboundedSpectrum) and Le (RGBIlluminantSpectrum); nullable
    const float *rgb_sigma_a, *rgb_sigma_s, *rgb_Le;
    const float *rgb_illuminant;      // 471, the colour space's illuminant
    float rgb_sigma_scale, rgb_Le_scale;
    // light_type 2, ImageInfiniteLight (lights.h:552-640): res x res equal-area image as
    // per-pixel RGBIlluminantSpectrum {c0, c1, c2, scale}, GetSamplingDistribution (res*res),
    // renderFromLight / lightFromRender (3x3), the colour space's illuminant
    const float *light_img[8];
    int light_res[8];
    const float *light_dist[8];
    float light_rfl[8][9], light_lfr[8][9];
    const float *light_illuminant;
    // SpectralFilm (film.h:401-530): nbuckets > 0 selects it — uniform wavelengths over
    // [lambda_min, lambda_max] and per-pixel spectral buckets next to the RGB sums
    int film_nbuckets;
    float film_lambda_min, film_lambda_max;
    // medium interface: 0 the bounds box, 1 a sphere {cx, cy, cz, r} in render space,
    // 2 a convex polyhedron: n_planes half-spaces {nx, ny, nz, h}, inside n.p <= h
    int boundary;
    float sphere[4];
    int n_planes;
    const float *planes;
    // VolPath's "lightsampler": 0 bvh / uniform (identical for infinite lights), 1 power
    int light_sampler;
} OracleScene;

}  // extern "C"

namespace oracle {

// ---------------------------------------------------------------------------
// Samplers (samplers.h). IndependentSampler — samplers.h:442-476: Get2D = two Get1D.
// ZSobolSampler — samplers.h:225-330 with RandomizeStrategy::FastOwen (the default): the
// pixel's Morton index with the sample index appended, each base-4 digit permuted by a
// hash of the higher digits and the dimension, then a scrambled Sobol' point of
// dimension 0 (1D) or dimensions 0 and 1 (2D) — lowdiscrepancy.h:168-180, 220-237.

// Sobol' generator matrices of dimensions 0 and 1 (sobolmatrices.cpp, first two rows),
// from their definition: dimension 0 is the van der Corput radical inverse (column i =
// bit 31-i); dimension 1 is the Pascal matrix mod 2 (direction numbers of x + 1):
// column i = column i-1 XOR (column i-1 >> 1). The tables hold SobolMatrixSize = 52
// columns (sobolmatrices.h:16): dimension 0's columns 32..51 are zero, dimension 1's
// repeat columns 0..19 (the Pascal pattern has period 32 in 32 bits).
static uint32_t SobolColumn(int dim, int i) {
    if (dim == 0) return i < 32 ? 1u << (31 - i) : 0u;
    uint32_t v = 0x80000000u;
    for (int k = 1; k <= (i & 31); ++k) v ^= v >> 1;
    return v;
}
static uint32_t SobolBits(uint64_t a, int dim) {
    uint32_t v = 0;
    for (int i = 0; a != 0; a >>= 1, ++i)
        if (a & 1) v ^= SobolColumn(dim, i);
    return v;
}
static inline uint32_t ReverseBits32(uint32_t n) {   // util/math.h:56-66
    n = (n << 16) | (n >> 16);
    n = ((n & 0x00ff00ffu) << 8) | ((n & 0xff00ff00u) >> 8);
    n = ((n & 0x0f0f0f0fu) << 4) | ((n & 0xf0f0f0f0u) >> 4);
    n = ((n & 0x33333333u) << 2) | ((n & 0xccccccccu) >> 2);
    n = ((n & 0x55555555u) << 1) | ((n & 0xaaaaaaaau) >> 1);
    return n;
}
static inline uint32_t FastOwen(uint32_t v, uint32_t seed) {   // lowdiscrepancy.h:220-237
    v = ReverseBits32(v);
    v ^= v * 0x3d20adeau;
    v += seed;
    v *= (seed >> 16) | 1;
    v ^= v * 0x05526c56u;
    v ^= v * 0x53a22864u;
    return ReverseBits32(v);
}
static inline float SobolSampleFastOwen(uint64_t a, int dim, uint32_t seed) {   // :168-180
    uint32_t v = FastOwen(SobolBits(a, dim), seed);
    return std::min(v * 0x1p-32f, 0x1.fffffep-1f);
}
static inline uint64_t LeftShift2(uint64_t x) {   // util/math.h:83-91
    x &= 0xffffffff;
    x = (x ^ (x << 16)) & 0x0000ffff0000ffffull;
    x = (x ^ (x << 8)) & 0x00ff00ff00ff00ffull;
    x = (x ^ (x << 4)) & 0x0f0f0f0f0f0f0f0full;
    x = (x ^ (x << 2)) & 0x3333333333333333ull;
    x = (x ^ (x << 1)) & 0x5555555555555555ull;
    return x;
}
static inline uint64_t EncodeMorton2(uint32_t x, uint32_t y) { return (LeftShift2(y) << 1) | LeftShift2(x); }
static inline int Log2Int(uint32_t v) { return 31 - __builtin_clz(v); }
static inline uint32_t RoundUpPow2(uint32_t v) {
    v--; v |= v >> 1; v |= v >> 2; v |= v >> 4; v |= v >> 8; v |= v >> 16; return v + 1;
}
// the 24 permutations of a base-4 digit, in ZSobolSampler::GetSampleIndex's order
static const uint8_t kZPerm[24][4] = {
    {0, 1, 2, 3}, {0, 1, 3, 2}, {0, 2, 1, 3}, {0, 2, 3, 1}, {0, 3, 2, 1}, {0, 3, 1, 2},
    {1, 0, 2, 3}, {1, 0, 3, 2}, {1, 2, 0, 3}, {1, 2, 3, 0}, {1, 3, 2, 0}, {1, 3, 0, 2},
    {2, 1, 0, 3}, {2, 1, 3, 0}, {2, 0, 1, 3}, {2, 0, 3, 1}, {2, 3, 0, 1}, {2, 3, 1, 0},
    {3, 1, 2, 0}, {3, 1, 0, 2}, {3, 2, 1, 0}, {3, 2, 0, 1}, {3, 0, 2, 1}, {3, 0, 1, 2}};

struct Sampler {
    // IndependentSampler
    RNG rng;
    // ZSobolSampler
    int type = 0, seed = 0, log2spp = 0, nBase4Digits = 0, dimension = 0;
    uint64_t mortonIndex = 0;

    void Start(const OracleScene &s, int px, int py, int sampleIndex) {
        type = s.sampler_type;
        seed = s.seed;
        if (type == 0) {   // samplers.h:457-460
            rng.SetSequence(HashPixelSeed(px, py, s.seed));
            rng.Advance((int64_t)(sampleIndex * 65536ull + 0));
            return;
        }
        // ZSobolSampler ctor (samplers.h:228-238) + StartPixelSample (:250-254)
        log2spp = Log2Int((uint32_t)s.samples_per_pixel);
        int res = (int)RoundUpPow2((uint32_t)std::max(s.width, s.height));
        int log4spp = (log2spp + 1) / 2;
        nBase4Digits = Log2Int((uint32_t)res) + log4spp;
        dimension = 0;
        mortonIndex = (EncodeMorton2((uint32_t)px, (uint32_t)py) << log2spp) | (uint64_t)sampleIndex;
    }
    uint64_t SampleIndex() const {   // samplers.h:296-355
        uint64_t sampleIndex = 0;
        bool pow2Samples = log2spp & 1;
        int lastDigit = pow2Samples ? 1 : 0;
        for (int i = nBase4Digits - 1; i >= lastDigit; --i) {
            int digitShift = 2 * i - (pow2Samples ? 1 : 0);
            int digit = (mortonIndex >> digitShift) & 3;
            uint64_t higherDigits = mortonIndex >> (digitShift + 2);
            int p = (MixBits(higherDigits ^ (0x55555555u * (uint32_t)dimension)) >> 24) % 24;
            digit = kZPerm[p][digit];
            sampleIndex |= uint64_t(digit) << digitShift;
        }
        if (pow2Samples) {
            int digit = mortonIndex & 1;
            sampleIndex |= digit ^ (MixBits((mortonIndex >> 1) ^ (0x55555555u * (uint32_t)dimension)) & 1);
        }
        return sampleIndex;
    }
    float Get1D() {
        if (type == 0) return rng.Uniform();
        uint64_t sampleIndex = SampleIndex();
        ++dimension;
        uint32_t sampleHash = (uint32_t)HashInts2(dimension, seed);
        return SobolSampleFastOwen(sampleIndex, 0, sampleHash);
    }
    void Get2D(float *u0, float *u1) {
        if (type == 0) {   // {Uniform, Uniform}, left to right
            *u0 = rng.Uniform();
            *u1 = rng.Uniform();
            return;
        }
        uint64_t sampleIndex = SampleIndex();
        dimension += 2;
        uint64_t bits = HashInts2(dimension, seed);
        *u0 = SobolSampleFastOwen(sampleIndex, 0, (uint32_t)bits);
        *u1 = SobolSampleFastOwen(sampleIndex, 1, (uint32_t)(bits >> 32));
    }
};

// ---------------------------------------------------------------------------
// GaussianFilter sampling — filters.h:80-118 via FilterSampler (filters.h:26-45,
// filters.cpp:133-147): the filter tabulated at 32 x radius cells per axis over
// [-radius, radius], sampled with PiecewiseConstant2D (sampling.h:603-770), weight =
// f[cell] / pdf.
static inline float GaussianF(float x, float mu, float sigma) {   // util/math.h:477-480
    return 1 / std::sqrt(2 * Pi * sigma * sigma) * FastExp(-Sqr(x - mu) / (2 * sigma * sigma));
}
struct PC1D {   // PiecewiseConstant1D
    std::vector<float> func, cdf;
    float min = 0, max = 1, funcInt = 0;
    void Build(const float *f, int n, float mn, float mx) {
        func.assign(f, f + n);
        cdf.assign(n + 1, 0.f);
        min = mn; max = mx;
        for (float &v : func) v = std::abs(v);
        cdf[0] = 0;
        for (int i = 1; i < n + 1; ++i) cdf[i] = cdf[i - 1] + func[i - 1] * (max - min) / n;
        funcInt = cdf[n];
        if (funcInt == 0)
            for (int i = 1; i < n + 1; ++i) cdf[i] = float(i) / float(n);
        else
            for (int i = 1; i < n + 1; ++i) cdf[i] /= funcInt;
    }
    float Sample(float u, float *pdf, int *offset) const {
        // FindInterval (util/math.h:508-519) over cdf[index] <= u
        long size = (long)cdf.size() - 2, first = 1;
        while (size > 0) {
            long half = size >> 1, middle = first + half;
            bool pr = cdf[middle] <= u;
            first = pr ? middle + 1 : first;
            size = pr ? size - (half + 1) : half;
        }
        int o = (int)std::clamp<long>(first - 1, 0, (long)cdf.size() - 2);
        *offset = o;
        float du = u - cdf[o];
        if (cdf[o + 1] - cdf[o] > 0) du /= cdf[o + 1] - cdf[o];
        *pdf = (funcInt > 0) ? func[o] / funcInt : 0;
        return Lerp((o + du) / (float)func.size(), min, max);
    }
};
struct GaussianSampler {
    int nx = 0, ny = 0;
    std::vector<float> f;            // nx * ny, x fastest (Array2D)
    std::vector<PC1D> cond;          // per row
    PC1D marginal;
    void Build(float rx, float ry, float sigma) {
        float expX = GaussianF(rx, 0, sigma), expY = GaussianF(ry, 0, sigma);
        nx = int(32 * rx);
        ny = int(32 * ry);
        f.assign((size_t)nx * ny, 0.f);
        for (int y = 0; y < ny; ++y)
            for (int x = 0; x < nx; ++x) {
                // Bounds2f::Lerp (vecmath.h:1228-1231) of ((x+0.5)/nx, (y+0.5)/ny) over [-r, r]
                float px = Lerp((x + 0.5f) / nx, -rx, rx), py = Lerp((y + 0.5f) / ny, -ry, ry);
                f[(size_t)y * nx + x] = std::max<float>(0, GaussianF(px, 0, sigma) - expX) *
                                        std::max<float>(0, GaussianF(py, 0, sigma) - expY);
            }
        cond.resize(ny);
        std::vector<float> marg(ny);
        for (int y = 0; y < ny; ++y) {
            cond[y].Build(&f[(size_t)y * nx], nx, -rx, rx);
            marg[y] = cond[y].funcInt;
        }
        marginal.Build(marg.data(), ny, -ry, ry);
    }
    void Sample(float u0, float u1, float *p0, float *p1, float *weight) const {
        float pdf1, pdf0;
        int v, uo;
        *p1 = marginal.Sample(u1, &pdf1, &v);
        *p0 = cond[v].Sample(u0, &pdf0, &uo);
        *weight = f[(size_t)v * nx + uo] / (pdf0 * pdf1);
    }
};

// ---------------------------------------------------------------------------
// RGBSigmoidPolynomial (util/color.h:332-365) and the RGB*Spectrum grids of RGBGridMedium
struct Rsp {
    float c0, c1, c2;
    static float S(float x) {   // color.h:356-360
        if (std::isinf(x)) return x > 0 ? 1 : 0;
        return .5f + x / (2 * std::sqrt(1 + Sqr(x)));
    }
    float operator()(float lambda) const { return S(std::fma(lambda, std::fma(lambda, c0, c1), c2)); }   // EvaluatePolynomial(lambda, c2, c1, c0)
    float MaxValue() const {
        float result = std::max((*this)(360), (*this)(830));
        float lambda = -c1 / (2 * c0);
        if (lambda >= 360 && lambda <= 830) result = std::max(result, (*this)(lambda));
        return result;
    }
};
// SampledGrid<RGBUnboundedSpectrum / RGBIlluminantSpectrum> (containers.h:785-857)
struct RgbGrid {
    const float *v;   // 4 per voxel: c0, c1, c2, scale
    int nx, ny, nz;
    const float *illuminant;   // non-null: RGBIlluminantSpectrum
    bool Inside(int x, int y, int z) const { return x >= 0 && x < nx && y >= 0 && y < ny && z >= 0 && z < nz; }
    Spec Convert(int x, int y, int z, const Lambda &l) const {
        Spec s = Spec::Const(0.f);
        if (!Inside(x, y, z)) return s;   // convert(T{}) = 0 (an illuminant spectrum without illuminant)
        const float *c = v + 4 * ((size_t)(z * ny + y) * nx + x);
        Rsp rsp{c[0], c[1], c[2]};
        for (int i = 0; i < NS; ++i) s.v[i] = c[3] * rsp(l.lambda[i]);
        if (illuminant) s = s * SampleDense(illuminant, l);
        return s;
    }
    static Spec LerpS(float t, const Spec &a, const Spec &b) { return (1 - t) * a + t * b; }
    Spec Lookup(V3 p, const Lambda &l) const {
        float px = p.x * nx - .5f, py = p.y * ny - .5f, pz = p.z * nz - .5f;
        int ix = (int)std::floor(px), iy = (int)std::floor(py), iz = (int)std::floor(pz);
        float dx = px - ix, dy = py - iy, dz = pz - iz;
        Spec d00 = LerpS(dx, Convert(ix, iy, iz, l), Convert(ix + 1, iy, iz, l));
        Spec d10 = LerpS(dx, Convert(ix, iy + 1, iz, l), Convert(ix + 1, iy + 1, iz, l));
        Spec d01 = LerpS(dx, Convert(ix, iy, iz + 1, l), Convert(ix + 1, iy, iz + 1, l));
        Spec d11 = LerpS(dx, Convert(ix, iy + 1, iz + 1, l), Convert(ix + 1, iy + 1, iz + 1, l));
        return LerpS(dz, LerpS(dy, d00, d10), LerpS(dy, d01, d11));
    }
    float MaxAt(int x, int y, int z) const {   // RGBUnboundedSpectrum::MaxValue
        const float *c = v + 4 * ((size_t)(z * ny + y) * nx + x);
        return c[3] * Rsp{c[0], c[1], c[2]}.MaxValue();
    }
    float MaxValue(const Bounds &b) const {   // SampledGrid::MaxValue(bounds, convert)
        float ps0[3] = {b.pMin.x * nx - .5f, b.pMin.y * ny - .5f, b.pMin.z * nz - .5f};
        float ps1[3] = {b.pMax.x * nx - .5f, b.pMax.y * ny - .5f, b.pMax.z * nz - .5f};
        const int n[3] = {nx, ny, nz};
        int lo[3], hi[3];
        for (int a = 0; a < 3; ++a) {
            lo[a] = std::max((int)std::floor(ps0[a]), 0);
            hi[a] = std::min((int)std::floor(ps1[a]) + 1, n[a] - 1);
        }
        float m = MaxAt(lo[0], lo[1], lo[2]);
        for (int z = lo[2]; z <= hi[2]; ++z)
            for (int y = lo[1]; y <= hi[1]; ++y)
                for (int x = lo[0]; x <= hi[0]; ++x) m = std::max(m, MaxAt(x, y, z));
        return m;
    }
};


// ImageInfiniteLight support (lights.h:552-640, lights.cpp:1007-1052)
static V3 EqualAreaSquareToSphere(float px, float py) {   // util/math.cpp:292-315
    float u = 2 * px - 1, v = 2 * py - 1;
    float up = std::abs(u), vp = std::abs(v);
    float signedDistance = 1 - (up + vp);
    float d = std::abs(signedDistance);
    float r = 1 - d;
    float phi = (r == 0 ? 1 : (vp - up) / r + 1) * Pi / 4;
    float z = std::copysign(1 - Sqr(r), signedDistance);
    float sn, cs;
    LmSinCos(phi, &sn, &cs);
    float cosPhi = std::copysign(cs, u), sinPhi = std::copysign(sn, v);
    return {cosPhi * r * SafeSqrt(2 - Sqr(r)), sinPhi * r * SafeSqrt(2 - Sqr(r)), z};
}
static void EqualAreaSphereToSquare(V3 d, float *ou, float *ov) {   // util/math.cpp:317-361
    float x = std::abs(d.x), y = std::abs(d.y), z = std::abs(d.z);
    float r = SafeSqrt(1 - z);
    float a = std::max(x, y), b = std::min(x, y);
    b = a == 0 ? 0 : b / a;
    const float t1 = 0.406758566246788489601959989e-5;
    const float t2 = 0.636226545274016134946890922156;
    const float t3 = 0.61572017898280213493197203466e-2;
    const float t4 = -0.247333733281268944196501420480;
    const float t5 = 0.881770664775316294736387951347e-1;
    const float t6 = 0.419038818029165735901852432784e-1;
    const float t7 = -0.251390972343483509333252996350e-1;
    // EvaluatePolynomial(b, t1, ..., t7): FMA(b, EvaluatePolynomial(b, t2, ...), t1)
    const float c[7] = {t1, t2, t3, t4, t5, t6, t7};
    float phi = c[6];
    for (int i = 5; i >= 0; --i) phi = std::fma(b, phi, c[i]);
    if (x < y) phi = 1 - phi;
    float v = phi * r;
    float u = r - v;
    if (d.z < 0) {
        std::swap(u, v);
        u = 1 - u;
        v = 1 - v;
    }
    u = std::copysign(u, d.x);
    v = std::copysign(v, d.y);
    *ou = 0.5f * (u + 1);
    *ov = 0.5f * (v + 1);
}
// RemapPixelCoords with WrapMode::OctahedralSphere (util/image.h:96-123)
static void RemapOctahedral(int *x, int *y, int res) {
    int &p0 = *x, &p1 = *y;
    if (p0 < 0) { p0 = -p0; p1 = res - 1 - p1; }
    else if (p0 >= res) { p0 = 2 * res - 1 - p0; p1 = res - 1 - p1; }
    if (p1 < 0) { p0 = res - 1 - p0; p1 = -p1; }
    else if (p1 >= res) { p0 = res - 1 - p0; p1 = 2 * res - 1 - p1; }
    if (res == 1) p0 = p1 = 0;
}
// Image::LookupNearestChannel(uv, c, OctahedralSphere): Point2i(p.x * res, p.y * res), remapped
static int OctahedralPixel(float u, float v, int res) {
    int p0 = (int)(u * res), p1 = (int)(v * res);
    RemapOctahedral(&p0, &p1, res);
    return p1 * res + p0;
}
struct PC2D {   // PiecewiseConstant2D over [0,1]^2 (util/sampling.h:698-779)
    std::vector<PC1D> cond;
    PC1D marg;
    int nu = 0, nv = 0;
    void Build(const float *d, int nu_, int nv_) {
        nu = nu_; nv = nv_;
        cond.resize(nv);
        std::vector<float> mf(nv);
        for (int v = 0; v < nv; ++v) {
            cond[v].Build(d + (size_t)v * nu, nu, 0, 1);
            mf[v] = cond[v].funcInt;
        }
        marg.Build(mf.data(), nv, 0, 1);
    }
    void Sample(float u0, float u1, float *su, float *sv, float *pdf) const {
        float p0, p1;
        int ov, ou;
        *sv = marg.Sample(u1, &p1, &ov);
        *su = cond[ov].Sample(u0, &p0, &ou);
        *pdf = p0 * p1;
    }
    float PDF(float u, float v) const {
        int iu = std::clamp(int(u * nu), 0, nu - 1), iv = std::clamp(int(v * nv), 0, nv - 1);
        return cond[iv].func[iu] / marg.funcInt;
    }
};
struct ImageLight {
    const float *img = nullptr;
    int res = 0;
    PC2D compensated;
    const float *rfl = nullptr, *lfr = nullptr;
    void Build(const float *image, int r, const float *dist, const float *rfl_, const float *lfr_) {
        img = image; res = r; rfl = rfl_; lfr = lfr_;
        const size_t n = (size_t)r * r;
        std::vector<float> d(dist, dist + n);
        float average = std::accumulate(d.begin(), d.end(), 0.) / d.size();   // lights.cpp:1031
        for (float &v : d) v = std::max<float>(v - average, 0);
        if (std::all_of(d.begin(), d.end(), [](float v) { return v == 0; })) std::fill(d.begin(), d.end(), 1.f);
        compensated.Build(d.data(), r, r);
    }
    static V3 Mul(const float *m, V3 v) {   // Transform::operator()(Vector3f)
        return {m[0] * v.x + m[1] * v.y + m[2] * v.z, m[3] * v.x + m[4] * v.y + m[5] * v.z,
                m[6] * v.x + m[7] * v.y + m[8] * v.z};
    }
    Spec ImageLe(float u, float v, const Lambda &l, const float *illum, float scale) const {   // lights.h:620-627
        const float *c = img + 4 * (size_t)OctahedralPixel(u, v, res);
        Rsp rsp{c[0], c[1], c[2]};
        Spec s;
        for (int i = 0; i < NS; ++i) s.v[i] = c[3] * rsp(l.lambda[i]);
        s = s * SampleDense(illum, l);
        return scale * s;
    }
};

// PowerLightSampler (lightsamplers.h:63-99, lightsamplers.cpp:76-96) over the infinite lights:
// each light's weight Average(SafeDiv(Phi(lambda), lambda.PDF())) at SampleVisible(0.5), then
// AliasTable (util/sampling.cpp:563-645).
struct PowerSampler {
    float q[8] = {}, p[8] = {};
    int alias[8] = {};
    static float Weight(const OracleScene &s, const ImageLight *img, int i) {
        const Lambda l = SampleVisible(0.5f);
        const float R2 = Sqr(s.scene_radius);
        Spec phi;
        if (s.light_type[i] == 0) {          // DistantLight::Phi, lights.cpp:216-218
            phi = s.light_scale[i] * SampleDense(s.light_L[i], l) * Pi * R2;
        } else if (s.light_type[i] == 1) {   // UniformInfiniteLight::Phi, lights.cpp:974-976
            phi = 4 * Pi * Pi * R2 * s.light_scale[i] * SampleDense(s.light_L[i], l);
        } else {                             // ImageInfiniteLight::Phi, lights.cpp:1042-1060
            const int res = img[i].res;
            Spec sumL = Spec::Const(0.f);
            for (int v = 0; v < res; ++v)
                for (int u = 0; u < res; ++u) {
                    const float *c = img[i].img + 4 * ((size_t)v * res + u);
                    Rsp rsp{c[0], c[1], c[2]};
                    Spec e;
                    for (int k = 0; k < NS; ++k) e.v[k] = c[3] * rsp(l.lambda[k]);
                    sumL = sumL + e * SampleDense(s.light_illuminant, l);
                }
            phi = 4 * Pi * Pi * R2 * s.light_scale[i] * sumL;
            for (int k = 0; k < NS; ++k) phi.v[k] /= (float)(res * res);
        }
        Spec w;
        for (int k = 0; k < NS; ++k) w.v[k] = l.pdf[k] != 0 ? phi.v[k] / l.pdf[k] : 0;   // SafeDiv
        return w.Average();
    }
    void Build(const OracleScene &s, const ImageLight *img) {
        const int n = s.nlights;
        std::vector<float> w(n);
        for (int i = 0; i < n; ++i) w[i] = Weight(s, img, i);
        if (std::accumulate(w.begin(), w.end(), 0.f) == 0.f) std::fill(w.begin(), w.end(), 1.f);
        const float sum = std::accumulate(w.begin(), w.end(), 0.);
        for (int i = 0; i < n; ++i) p[i] = w[i] / sum;
        struct Outcome { float pHat; size_t index; };
        std::vector<Outcome> under, over;
        for (int i = 0; i < n; ++i) {
            const float pHat = p[i] * (size_t)n;
            if (pHat < 1) under.push_back({pHat, (size_t)i});
            else over.push_back({pHat, (size_t)i});
        }
        while (!under.empty() && !over.empty()) {
            Outcome un = under.back(), ov = over.back();
            under.pop_back();
            over.pop_back();
            q[un.index] = un.pHat;
            alias[un.index] = (int)ov.index;
            const float pExcess = un.pHat + ov.pHat - 1;
            if (pExcess < 1) under.push_back({pExcess, ov.index});
            else over.push_back({pExcess, ov.index});
        }
        while (!over.empty()) { q[over.back().index] = 1; alias[over.back().index] = -1; over.pop_back(); }
        while (!under.empty()) { q[under.back().index] = 1; alias[under.back().index] = -1; under.pop_back(); }
    }
    int Sample(int n, float u, float *pmf) const {   // AliasTable::Sample
        int offset = std::min<int>(u * (size_t)n, n - 1);
        float up = std::min<float>(u * (size_t)n - offset, OneMinusEpsilon);
        if (up < q[offset]) { *pmf = p[offset]; return offset; }
        *pmf = p[alias[offset]];
        return alias[offset];
    }
};

struct SceneView {
    const OracleScene &s;
    Xform mediumX, cameraX, rasterX;
    Bounds bounds;
    Grid density, lescale, majorant, temperature;
    GaussianSampler gauss;
    ImageLight img[8];
    PowerSampler power;
    explicit SceneView(const OracleScene &sc) : s(sc) {
        if (sc.filter_type == 1) gauss.Build(sc.filter_radius[0], sc.filter_radius[1], sc.filter_sigma);
        for (int i = 0; i < sc.nlights; ++i)
            if (sc.light_type[i] == 2)
                img[i].Build(sc.light_img[i], sc.light_res[i], sc.light_dist[i], sc.light_rfl[i], sc.light_lfr[i]);
        if (sc.light_sampler == 1 && sc.nlights > 0) power.Build(sc, img);
        for (int i = 0; i < 16; ++i) {
            mediumX.m[i / 4][i % 4] = sc.render_from_medium[i];
            mediumX.mInv[i / 4][i % 4] = sc.medium_from_render[i];
            cameraX.m[i / 4][i % 4] = sc.render_from_camera[i];
            cameraX.mInv[i / 4][i % 4] = 0;
            rasterX.m[i / 4][i % 4] = sc.camera_from_raster[i];
            rasterX.mInv[i / 4][i % 4] = 0;
        }
        bounds = {{sc.bounds[0], sc.bounds[1], sc.bounds[2]}, {sc.bounds[3], sc.bounds[4], sc.bounds[5]}};
        density = {sc.density, sc.nx, sc.ny, sc.nz};
        temperature = {sc.temperature, sc.nx, sc.ny, sc.nz};
        lescale = {sc.Lescale, sc.lnx, sc.lny, sc.lnz};
        majorant = {sc.majorant, sc.mres[0], sc.mres[1], sc.mres[2]};
    }
};

// MediumProperties for GridMedium::SamplePoint — media.h:287-319 (no temperature grid)
struct MediumProps { Spec sigma_a, sigma_s, Le; };
static inline MediumProps SamplePoint(const SceneView &sv, V3 p, const Lambda &l) {
    MediumProps mp;
    mp.sigma_a = SampleDense(sv.s.sigma_a, l);
    mp.sigma_s = SampleDense(sv.s.sigma_s, l);
    mp.Le = Spec::Const(0.f);
    if (sv.s.medium_type == 1) {   // HomogeneousMedium::SamplePoint (media.h:241-247)
        if (sv.s.emissive) mp.Le = SampleDense(sv.s.Le, l);
        return mp;
    }
    p = XInvPoint(sv.mediumX, p);
    if (sv.s.medium_type == 4) {   // RGBGridMedium::SamplePoint (media.h:377-403)
        p = Offset(sv.bounds, p);
        const OracleScene &s = sv.s;
        Spec sa = s.rgb_sigma_a ? RgbGrid{s.rgb_sigma_a, s.nx, s.ny, s.nz, nullptr}.Lookup(p, l) : Spec::Const(1.f);
        Spec ss = s.rgb_sigma_s ? RgbGrid{s.rgb_sigma_s, s.nx, s.ny, s.nz, nullptr}.Lookup(p, l) : Spec::Const(1.f);
        mp.sigma_a = s.rgb_sigma_scale * sa;
        mp.sigma_s = s.rgb_sigma_scale * ss;
        if (s.rgb_Le && s.rgb_Le_scale > 0)
            mp.Le = s.rgb_Le_scale * RgbGrid{s.rgb_Le, s.nx, s.ny, s.nz, s.rgb_illuminant}.Lookup(p, l);
        return mp;
    }
    if (sv.s.medium_type == 3) {   // NanoVDBMedium::SamplePoint (media.h:624-637)
        const VdbTree &dg = *(const VdbTree *)sv.s.vdb;
        const float d = dg.Sample(dg.WorldToIndexF(p));
        mp.sigma_a = mp.sigma_a * d;
        mp.sigma_s = mp.sigma_s * d;
        if (sv.s.vdb_temperature) {   // NanoVDBMedium::Le (media.h:660-672)
            const VdbTree &tg = *(const VdbTree *)sv.s.vdb_temperature;
            float temp = tg.Sample(tg.WorldToIndexF(p));
            temp = (temp - sv.s.temperature_offset) * sv.s.temperature_scale;
            if (temp > 100.f) {
                float lambdaMax = 2.8977721e-3f / temp;
                float normalizationFactor = 1 / Blackbody(lambdaMax * 1e9f, temp);
                Spec b;
                for (int i = 0; i < NS; ++i) b.v[i] = Blackbody(l.lambda[i], temp) * normalizationFactor;
                mp.Le = sv.s.vdb_lescale * b;
            }
        }
        return mp;
    }
    if (sv.s.medium_type == 2) {   // CloudMedium::SamplePoint (media.h:456-465)
        float d = CloudDensity(p, sv.s.cloud[0], sv.s.cloud[1], sv.s.cloud[2]);
        mp.sigma_a = d * mp.sigma_a;
        mp.sigma_s = d * mp.sigma_s;
        return mp;
    }
    p = Offset(sv.bounds, p);
    float d = sv.density.Lookup(p);
    mp.sigma_a = mp.sigma_a * d;
    mp.sigma_s = mp.sigma_s * d;
    mp.Le = Spec::Const(0.f);
    if (sv.s.emissive) {
        float scale = sv.lescale.Lookup(p);
        if (scale > 0) {
            if (sv.s.temperature) {   // media.h:304-312
                float temp = sv.temperature.Lookup(p);
                temp = (temp - sv.s.temperature_offset) * sv.s.temperature_scale;
                if (temp > 100.f) {
                    // BlackbodySpectrum(temp).Sample(lambda) (spectrum.h:500-521)
                    float lambdaMax = 2.8977721e-3f / temp;
                    float normalizationFactor = 1 / Blackbody(lambdaMax * 1e9f, temp);
                    Spec b;
                    for (int i = 0; i < NS; ++i) b.v[i] = Blackbody(l.lambda[i], temp) * normalizationFactor;
                    mp.Le = scale * b;
                }
            } else {
                mp.Le = scale * SampleDense(sv.s.Le, l);
            }
        }
    }
    return mp;
}

// DDAMajorantIterator — media.h:136-214
struct DDA {
    Spec sigma_t;
    float tMin = Infinity, tMax = -Infinity;
    const Grid *grid = nullptr;
    float nextCrossingT[3], deltaT[3];
    int step[3], voxelLimit[3], voxel[3];
    bool valid = false;
    bool single = false, called = false;   // HomogeneousMajorantIterator (media.h:80-102)
    void InitSingle(float tMin_, float tMax_, Spec st) {
        tMin = tMin_; tMax = tMax_; sigma_t = st; valid = true; single = true;
    }
    void Init(Ray ray, float tMin_, float tMax_, const Grid *g, const Bounds &gb, Spec st) {
        tMin = tMin_; tMax = tMax_; grid = g; sigma_t = st; valid = true;
        V3 diag = gb.pMax - gb.pMin;
        Ray rg = {Offset(gb, ray.o), {ray.d.x / diag.x, ray.d.y / diag.y, ray.d.z / diag.z}};
        V3 gi = rg.o + rg.d * tMin;
        const int res[3] = {g->nx, g->ny, g->nz};
        for (int axis = 0; axis < 3; ++axis) {
            voxel[axis] = (int)Clamp(gi[axis] * res[axis], 0, res[axis] - 1);
            deltaT[axis] = 1 / (std::abs(rg.d[axis]) * res[axis]);
            if (rg.d[axis] == -0.f) rg.d[axis] = 0.f;
            if (rg.d[axis] >= 0) {
                float nextVoxelPos = float(voxel[axis] + 1) / res[axis];
                nextCrossingT[axis] = tMin + (nextVoxelPos - gi[axis]) / rg.d[axis];
                step[axis] = 1;
                voxelLimit[axis] = res[axis];
            } else {
                float nextVoxelPos = float(voxel[axis]) / res[axis];
                nextCrossingT[axis] = tMin + (nextVoxelPos - gi[axis]) / rg.d[axis];
                step[axis] = -1;
                voxelLimit[axis] = -1;
            }
        }
    }
    // returns false when exhausted
    bool Next(float *segMin, float *segMax, Spec *sigma_maj) {
        if (single) {
            if (!valid || called) return false;
            called = true;
            *segMin = tMin; *segMax = tMax; *sigma_maj = sigma_t;
            return true;
        }
        if (!valid || tMin >= tMax) return false;
        int bits = ((nextCrossingT[0] < nextCrossingT[1]) << 2) + ((nextCrossingT[0] < nextCrossingT[2]) << 1) +
                   ((nextCrossingT[1] < nextCrossingT[2]));
        static const int cmpToAxis[8] = {2, 1, 2, 1, 2, 2, 0, 0};
        int stepAxis = cmpToAxis[bits];
        float tVoxelExit = std::min(tMax, nextCrossingT[stepAxis]);
        *sigma_maj = sigma_t * grid->values[voxel[0] + grid->nx * (voxel[1] + grid->ny * voxel[2])];
        *segMin = tMin;
        *segMax = tVoxelExit;
        tMin = tVoxelExit;
        if (nextCrossingT[stepAxis] > tMax) tMin = tMax;
        voxel[stepAxis] += step[stepAxis];
        if (voxel[stepAxis] == voxelLimit[stepAxis]) tMin = tMax;
        nextCrossingT[stepAxis] += deltaT[stepAxis];
        return true;
    }
};

// GridMedium::SampleRay — media.h:322-337
static inline DDA SampleRay(const SceneView &sv, Ray ray, float raytMax, const Lambda &l) {
    DDA it;
    ray = XRay(sv.mediumX, ray, &raytMax, /*inverse=*/true);
    float tMin, tMax;
    if (!IntersectP(sv.bounds, ray.o, ray.d, raytMax, &tMin, &tMax)) return it;
    Spec sigma_t = SampleDense(sv.s.sigma_a, l) + SampleDense(sv.s.sigma_s, l);
    if (sv.s.medium_type == 1 || sv.s.medium_type == 2) {   // CloudMedium::SampleRay (media.h:467-484); homogeneous: the box crossing
        it.InitSingle(tMin, tMax, sigma_t);
        return it;
    }
    it.Init(ray, tMin, tMax, &sv.majorant, sv.bounds, sigma_t);
    return it;
}

// SampleT_maj<GridMedium> — media.h:741-806
template <typename F>
static Spec SampleT_maj(const SceneView &sv, Ray ray, float tMax, float u, RNG &rng, const Lambda &l,
                        F callback) {
    tMax *= Length(ray.d);
    ray.d = Normalize(ray.d);
    DDA iter = SampleRay(sv, ray, tMax, l);
    Spec T_maj = Spec::Const(1.f);
    bool done = false;
    while (!done) {
        float segMin, segMax;
        Spec sigma_maj;
        if (!iter.Next(&segMin, &segMax, &sigma_maj)) return T_maj;
        if (sigma_maj[0] == 0) {
            float dt = segMax - segMin;
            if (std::isinf(dt)) dt = std::numeric_limits<float>::max();
            T_maj = T_maj * FastExpSpec(-dt * sigma_maj);
            continue;
        }
        float tMin = segMin;
        while (true) {
            float t = tMin + SampleExponential(u, sigma_maj[0]);
            u = rng.Uniform();
            if (t < segMax) {
                T_maj = T_maj * FastExpSpec(-(t - tMin) * sigma_maj);
                V3 p = ray.o + ray.d * t;
                MediumProps mp = SamplePoint(sv, p, l);
                if (!callback(p, mp, sigma_maj, T_maj)) { done = true; break; }
                T_maj = Spec::Const(1.f);
                tMin = t;
            } else {
                float dt = segMax - tMin;
                if (std::isinf(dt)) dt = std::numeric_limits<float>::max();
                T_maj = T_maj * FastExpSpec(-dt * sigma_maj);
                break;
            }
        }
    }
    return Spec::Const(1.f);
}

// Interface sphere (OracleScene::boundary 1; defined after the graph section's SphereHits).
// The medium is inside the sphere (a shape without material whose MediumInterface is
// (inside = medium, outside = none)): a camera ray moves to its entry point before its first
// medium segment — pbrt samples no medium before it and calls SkipIntersection there
// (integrators.cpp:1118-1122) — and every segment / shadow ray ends at the sphere exit seen
// from its own origin (pbrt re-intersects from the spawned point). Origins are not offset by
// the intersection's error bounds (the same model as the device).
static float InterfaceExit(const OracleScene &s, V3 o, V3 d);
static V3 InterfaceEntry(const OracleScene &s, V3 o, V3 d);

// VolPathIntegrator::SampleLd for a medium interaction — integrators.cpp:1282-1399
static Spec SampleLd(const SceneView &sv, V3 p, V3 wo, const Lambda &l, Sampler &sampler, Spec beta, Spec r_p) {
    const OracleScene &s = sv.s;
    // lightSampler.Sample (BVH, infinite lights only) — lightsamplers.h:266-277
    float u = sampler.Get1D();
    float uL0, uL1;
    sampler.Get2D(&uL0, &uL1);   // uLight (unused by distant lights)
    if (s.nlights == 0) return Spec::Const(0.f);
    int index;
    float pmf;
    if (s.light_sampler == 1) {   // PowerLightSampler::Sample (lightsamplers.h:69-75)
        index = sv.power.Sample(s.nlights, u, &pmf);
    } else {
        float pInfinite = float(s.nlights) / float(s.nlights + 0);
        if (!(u < pInfinite)) return Spec::Const(0.f);
        u /= pInfinite;
        index = std::min<int>(u * s.nlights, s.nlights - 1);
        pmf = pInfinite / s.nlights;
    }
    if (s.light_type[index] == 1) return Spec::Const(0.f);  // UniformInfiniteLight::SampleLi with allowIncompletePDF
    V3 wi;
    Spec Ls;
    float lsPdf = 1;
    const bool delta = s.light_type[index] == 0;
    if (delta) {   // DistantLight::SampleLi — lights.h:284-291
        wi = {s.light_w[index][0], s.light_w[index][1], s.light_w[index][2]};
        Ls = s.light_scale[index] * SampleDense(s.light_L[index], l);
    } else {       // ImageInfiniteLight::SampleLi(allowIncompletePDF = true) — lights.h:588-613
        const ImageLight &il = sv.img[index];
        float su, sv_, mapPDF = 0;
        il.compensated.Sample(uL0, uL1, &su, &sv_, &mapPDF);
        if (mapPDF == 0) return Spec::Const(0.f);
        V3 wLight = EqualAreaSquareToSphere(su, sv_);
        wi = ImageLight::Mul(il.rfl, wLight);
        lsPdf = mapPDF / (4 * Pi);
        Ls = il.ImageLe(su, sv_, l, s.light_illuminant, s.light_scale[index]);
    }
    V3 pOutside = p + wi * (2 * s.scene_radius);
    if (!Ls || lsPdf == 0) return Spec::Const(0.f);
    float p_l = pmf * lsPdf;
    // phase function
    float fval = HenyeyGreenstein(Dot(wo, wi), s.g);
    Spec f_hat = Spec::Const(fval);
    float scatterPDF = fval;
    if (!f_hat) return Spec::Const(0.f);
    // SpawnRayTo from a medium interaction (ray.h:75-108: zero error, zero normal)
    Ray lightRay = {p, pOutside - p};
    Spec T_ray = Spec::Const(1.f), r_l = Spec::Const(1.f), r_u = Spec::Const(1.f);
    RNG rng(HashBytes(&lightRay.o, 12), HashBytes(&lightRay.d, 12));
    // The box boundary only toggles the medium; SampleT_maj clips to the same bounds. An
    // interface sphere ends the medium part at its exit (Intersect(lightRay, 1 - eps)->tHit).
    float tMax = 1 - ShadowEpsilon;
    if (s.boundary) tMax = std::min<float>(tMax, InterfaceExit(s, lightRay.o, lightRay.d));
    float uu = rng.Uniform();
    Spec T_maj = SampleT_maj(sv, lightRay, tMax, uu, rng, l, [&](V3, const MediumProps &mp, Spec sigma_maj, Spec Tm) {
        Spec sigma_n = ClampZero(sigma_maj - mp.sigma_a - mp.sigma_s);
        float pdf = Tm[0] * sigma_maj[0];
        T_ray = T_ray * (Tm * sigma_n / pdf);
        r_l = r_l * (Tm * sigma_maj / pdf);
        r_u = r_u * (Tm * sigma_n / pdf);
        Spec Tr = T_ray / (r_l + r_u).Average();
        if (Tr.MaxComponentValue() < 0.05f) {
            float q = 0.75f;
            if (rng.Uniform() < q) T_ray = Spec::Const(0.);
            else T_ray = T_ray / (1 - q);
        }
        if (!T_ray) return false;
        return true;
    });
    T_ray = T_ray * (T_maj / T_maj[0]);
    r_l = r_l * (T_maj / T_maj[0]);
    r_u = r_u * (T_maj / T_maj[0]);
    if (!T_ray) return Spec::Const(0.f);
    r_l = r_l * (r_p * p_l);
    r_u = r_u * (r_p * scatterPDF);
    if (delta) return beta * f_hat * T_ray * Ls / r_l.Average();
    return beta * f_hat * T_ray * Ls / (r_l + r_u).Average();
}

// VolPathIntegrator::Li — integrators.cpp:962-1280, restricted to the interface-box scene.
static Spec Li(const SceneView &sv, Ray ray, Lambda &l, Sampler &sampler, int *nEvents) {
    const OracleScene &s = sv.s;
    Spec L = Spec::Const(0.f), beta = Spec::Const(1.f), r_u = Spec::Const(1.f), r_l = Spec::Const(1.f);
    bool specularBounce = false;
    int depth = 0;
    const int maxDepth = s.max_depth;
    if (s.boundary) ray.o = InterfaceEntry(s, ray.o, ray.d);
    while (true) {
        // ray.medium is the grid medium (see header: the interface box only toggles it)
        bool scattered = false, terminated = false;
        float tMax = s.boundary ? InterfaceExit(s, ray.o, ray.d) : Infinity;
        uint64_t hash0 = HashFloat(sampler.Get1D());
        uint64_t hash1 = HashFloat(sampler.Get1D());
        RNG rng(hash0, hash1);
        float u0 = sampler.Get1D();
        Ray segRay = ray;
        Spec T_maj = SampleT_maj(sv, segRay, tMax, u0, rng, l,
            [&](V3 p, const MediumProps &mp, Spec sigma_maj, Spec Tm) -> bool {
                if (nEvents) ++*nEvents;
                if (!beta) { terminated = true; return false; }
                if (depth < maxDepth && mp.Le) {
                    float pdf = sigma_maj[0] * Tm[0];
                    Spec betap = beta * Tm / pdf;
                    Spec r_e = r_u * sigma_maj * Tm / pdf;
                    if (r_e) L = L + betap * mp.sigma_a * mp.Le / r_e.Average();
                }
                float pAbsorb = mp.sigma_a[0] / sigma_maj[0];
                float pScatter = mp.sigma_s[0] / sigma_maj[0];
                float pNull = std::max<float>(0, 1 - pAbsorb - pScatter);
                float um = rng.Uniform();
                const float w[3] = {pAbsorb, pScatter, pNull};
                int mode = SampleDiscrete3(w, um);
                if (mode == 0) { terminated = true; return false; }
                if (mode == 1) {
                    if (depth++ >= maxDepth) { terminated = true; return false; }
                    float pdf = Tm[0] * mp.sigma_s[0];
                    beta = beta * (Tm * mp.sigma_s / pdf);
                    r_u = r_u * (Tm * mp.sigma_s / pdf);
                    if (beta && r_u) {
                        V3 wo = -ray.d;
                        L = L + SampleLd(sv, p, wo, l, sampler, beta, r_u);
                        float uph0, uph1;
                        sampler.Get2D(&uph0, &uph1);
                        float phPdf;
                        V3 wi = SampleHenyeyGreenstein(wo, s.g, uph0, uph1, &phPdf);
                        if (phPdf == 0) terminated = true;
                        else {
                            beta = beta * (phPdf / phPdf);
                            r_l = r_u / phPdf;
                            scattered = true;
                            ray.o = p;
                            ray.d = wi;
                            specularBounce = false;
                        }
                    }
                    return false;
                }
                Spec sigma_n = ClampZero(sigma_maj - mp.sigma_a - mp.sigma_s);
                float pdf = Tm[0] * sigma_n[0];
                beta = beta * (Tm * sigma_n / pdf);
                if (pdf == 0) beta = Spec::Const(0.f);
                r_u = r_u * (Tm * sigma_n / pdf);
                r_l = r_l * (Tm * sigma_maj / pdf);
                return (bool)beta && (bool)r_u;
            });
        if (terminated || !beta || !r_u) return L;
        if (scattered) continue;
        beta = beta * (T_maj / T_maj[0]);
        r_u = r_u * (T_maj / T_maj[0]);
        r_l = r_l * (T_maj / T_maj[0]);
        // Escaped: infinite lights (integrators.cpp:1090-1107)
        for (int i = 0; i < s.nlights; ++i) {
            if (s.light_type[i] == 0) continue;
            Spec Le;
            if (s.light_type[i] == 1) {
                Le = s.light_scale[i] * SampleDense(s.light_L[i], l);
            } else {   // ImageInfiniteLight::Le (lights.h:581-585)
                const ImageLight &il = sv.img[i];
                V3 wl = Normalize(ImageLight::Mul(il.lfr, ray.d));
                float eu, ev;
                EqualAreaSphereToSquare(wl, &eu, &ev);
                Le = il.ImageLe(eu, ev, l, s.light_illuminant, s.light_scale[i]);
            }
            if (!Le) continue;
            if (depth == 0 || specularBounce)
                L = L + beta * Le / r_u.Average();
            else {
                // lightSampler.PMF * PDF_Li(prevIntrContext, ray.d, allowIncompletePDF = true)
                float pdfLi = 0;
                if (s.light_type[i] == 2) {   // lights.cpp:1042-1052 (wLight not normalised)
                    const ImageLight &il = sv.img[i];
                    float eu, ev;
                    EqualAreaSphereToSquare(ImageLight::Mul(il.lfr, ray.d), &eu, &ev);
                    pdfLi = il.compensated.PDF(eu, ev) / (4 * Pi);
                }
                float p_l = (s.light_sampler == 1 ? sv.power.p[i] : 1.f / (s.nlights + 0)) * pdfLi;
                r_l = r_l * p_l;
                L = L + beta * Le / (r_u + r_l).Average();
            }
        }
        break;
    }
    return L;
}

// RayIntegrator::EvaluatePixelSample — integrators.cpp:235-298 (+ GetCameraSample samplers.h:797-815)
struct SampleResult { Spec L; Lambda l; float weight; };
static SampleResult EvaluatePixelSample(const SceneView &sv, int px, int py, int sampleIndex, int *nEvents) {
    const OracleScene &s = sv.s;
    Sampler sampler;
    sampler.Start(s, px, py, sampleIndex);
    float lu = sampler.Get1D();
    // Film::SampleWavelengths: RGBFilm SampleVisible, SpectralFilm SampleUniform
    Lambda l = s.film_nbuckets > 0 ? SampleUniform(lu, s.film_lambda_min, s.film_lambda_max) : SampleVisible(lu);
    float fu0, fu1;
    sampler.Get2D(&fu0, &fu1);            // GetPixel2D
    float fpx, fpy, filterWeight = 1;
    if (s.filter_type == 0) {             // BoxFilter::Sample — filters.h:67-70
        fpx = Lerp(fu0, -s.filter_radius[0], s.filter_radius[0]);
        fpy = Lerp(fu1, -s.filter_radius[1], s.filter_radius[1]);
    } else {
        sv.gauss.Sample(fu0, fu1, &fpx, &fpy, &filterWeight);
    }
    float pFilmX = ((float)px + fpx) + 0.5f, pFilmY = ((float)py + fpy) + 0.5f;
    sampler.Get1D();                      // time
    float ul0, ul1;
    sampler.Get2D(&ul0, &ul1);            // lens
    // Camera ray (GenerateRayDifferential main ray, then RenderFromCamera)
    V3 pCamera = XPoint(sv.rasterX.m, V3{pFilmX, pFilmY, 0.f});
    Ray ray;
    if (s.camera_type == 0) ray = {pCamera, {0.f, 0.f, 1.f}};
    else ray = {{0.f, 0.f, 0.f}, Normalize(pCamera)};
    ray = XRay(sv.cameraX, ray, nullptr, /*inverse=*/false);
    Spec L = Spec::Const(1.f) * Li(sv, ray, l, sampler, nEvents);
    bool bad = false;
    for (int i = 0; i < NS; ++i) if (std::isnan(L.v[i])) bad = true;
    if (!bad) {
        // IsInf(L.y(lambda)) — spectrum.cpp SampledSpectrum::y
        Spec Ys = SampleDense(s.sensor_xyz + 471, l);
        Spec pdf; for (int i = 0; i < NS; ++i) pdf.v[i] = l.pdf[i];
        float y = SafeDiv(Ys * L, pdf).Average() / 106.856895f;
        if (std::isinf(y)) bad = true;
    }
    if (bad) L = Spec::Const(0.f);
    return {L, l, filterWeight};
}

// RGBFilm::AddSample — film.h:239-255 with PixelSensor::ToSensorRGB film.h:95-100
static inline void AddSample(const OracleScene &s, double *rgbSum, double *wSum, const Spec &Lin, const Lambda &l,
                             float weight) {
    Spec pdf; for (int i = 0; i < NS; ++i) pdf.v[i] = l.pdf[i];
    Spec L = SafeDiv(Lin, pdf);
    float rgb[3];
    for (int c = 0; c < 3; ++c) rgb[c] = s.imaging_ratio * (SampleDense(s.sensor_xyz + 471 * c, l) * L).Average();
    float m = std::max({rgb[0], rgb[1], rgb[2]});
    if (m > s.max_component_value)
        for (int c = 0; c < 3; ++c) rgb[c] *= s.max_component_value / m;
    for (int c = 0; c < 3; ++c) rgbSum[c] += weight * rgb[c];
    *wSum += weight;
}

// SpectralFilm::AddSample — film.h:413-455: the RGB part as RGBFilm's, then L clamped by
// its max component, scaled by weight * CIE_Y_integral, and added into the bucket of each
// wavelength (LambdaToBucket, film.h:500-504) with the weight
static inline void AddSampleSpectral(const OracleScene &s, double *rgbSum, double *wSum, double *bucketSums,
                                     double *weightSums, const Spec &Lin, const Lambda &l, float weight) {
    AddSample(s, rgbSum, wSum, Lin, l, weight);
    Spec L = Lin;
    float lm = L.v[0];
    for (int i = 1; i < NS; ++i) lm = std::max(lm, L.v[i]);
    if (lm > s.max_component_value)
        for (int i = 0; i < NS; ++i) L.v[i] *= s.max_component_value / lm;
    const float k = weight * 106.856895f;   // CIE_Y_integral
    for (int i = 0; i < NS; ++i) L.v[i] *= k;
    const int nb = s.film_nbuckets;
    for (int i = 0; i < NS; ++i) {
        int b = nb * (l.lambda[i] - s.film_lambda_min) / (s.film_lambda_max - s.film_lambda_min);
        b = std::min(std::max(b, 0), nb - 1);
        bucketSums[b] += L.v[i];
        weightSums[b] += weight;
    }
}

}  // namespace oracle

// ===========================================================================
// C API (ctypes)
// ===========================================================================
extern "C" {
// 0 = platform float libm (pbrt as built on this host), 1 = correctly rounded (HIP convention)
void oracle_set_libm(int mode) { g_libm = mode ? 1 : 0; }
int oracle_get_libm() { return g_libm; }
// the canonical convention's float functions (tests)
float oracle_canon_log(float x) { return (float)canon::Log((double)x); }
float oracle_canon_atanh(float x) { return (float)canon::Atanh((double)x); }
float oracle_canon_cosh(float x) { return (float)canon::Cosh((double)x); }
void oracle_canon_sincos(float x, float *s, float *c) {
    double sd, cd;
    canon::SinCos((double)x, &sd, &cd);
    *s = (float)sd;
    *c = (float)cd;
}


// ImageInfiniteLight pieces (test infrastructure)
void oracle_equal_area_square_to_sphere(float u, float v, float *out) {
    V3 w = EqualAreaSquareToSphere(u, v);
    out[0] = w.x; out[1] = w.y; out[2] = w.z;
}
void oracle_equal_area_sphere_to_square(float x, float y, float z, float *out) {
    EqualAreaSphereToSquare({x, y, z}, out, out + 1);
}
void oracle_remap_octahedral(int x, int y, int res, int *out) {
    RemapOctahedral(&x, &y, res);
    out[0] = x; out[1] = y;
}
// PiecewiseConstant2D over [0,1]^2 of func (nu x nv): n samples (u0, u1) -> (x, y, pdf, PDF(x, y))
void oracle_pc2d(const float *func, int nu, int nv, int n, const float *u, float *out) {
    PC2D d;
    d.Build(func, nu, nv);
    for (int i = 0; i < n; ++i) {
        float x, y, pdf;
        d.Sample(u[2 * i], u[2 * i + 1], &x, &y, &pdf);
        out[4 * i] = x; out[4 * i + 1] = y; out[4 * i + 2] = pdf; out[4 * i + 3] = d.PDF(x, y);
    }
}

// RGBGridMedium (test infrastructure)
float oracle_rsp_eval(float c0, float c1, float c2, float lambda) { return Rsp{c0, c1, c2}(lambda); }
float oracle_rsp_max(float c0, float c1, float c2) { return Rsp{c0, c1, c2}.MaxValue(); }
// ctor's 16^3 majorant (media.cpp:364-377) over MajorantGrid::VoxelBounds
void oracle_rgb_majorant(const float *sa, const float *ss, int nx, int ny, int nz, float sigmaScale, int rx, int ry,
                         int rz, float *out) {
    // cells are independent (media.cpp:364-377 builds them in a ParallelFor too): threads over
    // cells, each cell's max in pbrt's voxel order
    const int ncell = rx * ry * rz;
    auto cell = [&](int c) {
        const int x = c % rx, y = (c / rx) % ry, z = c / (rx * ry);
        Bounds b{{float(x) / rx, float(y) / ry, float(z) / rz}, {float(x + 1) / rx, float(y + 1) / ry, float(z + 1) / rz}};
        float maxSigma_t = (sa ? RgbGrid{sa, nx, ny, nz, nullptr}.MaxValue(b) : 1) +
                           (ss ? RgbGrid{ss, nx, ny, nz, nullptr}.MaxValue(b) : 1);
        out[c] = sigmaScale * maxSigma_t;
    };
    const int nt = std::max(1, std::min(16, std::min(ncell, (int)std::thread::hardware_concurrency())));
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t)
        th.emplace_back([&, t] {
            for (int c = t; c < ncell; c += nt) cell(c);
        });
    for (auto &x : th) x.join();
}

// NanoVDB grids (test infrastructure handles; see VdbTree)
void *oracle_vdb_create(int nLeaves, const int *leafOrigin, const float *leafValues, int nTiles, const int *tileOrigin,
                        const int *tileSize, const float *tileValue, float background, const int ibbox[6],
                        const double indexToWorld[12], const double worldToIndex[9]) {
    auto *g = new VdbTree();
    g->leafStore.assign(leafValues, leafValues + (size_t)nLeaves * 512);
    for (int l = 0; l < nLeaves; ++l) {
        const int *o = leafOrigin + 3 * l;
        g->leaves[VdbTree::Key(o[0], o[1], o[2])] = g->leafStore.data() + (size_t)l * 512;
    }
    for (int t = 0; t < nTiles; ++t) {
        for (int a = 0; a < 3; ++a) g->tileBox.push_back(tileOrigin[3 * t + a]);
        g->tileBox.push_back(tileSize[t]);
        g->tileValue.push_back(tileValue[t]);
        const int *o = tileOrigin + 3 * t;
        // the hash lookup keys a voxel by (x >> 3, y >> 3, z >> 3): only an 8-aligned 8^3 tile
        // covers exactly its key's block; any other tile goes to the box search
        if (tileSize[t] == 8 && ((o[0] | o[1] | o[2]) & 7) == 0) {
            g->tile8[VdbTree::Key(o[0], o[1], o[2])] = tileValue[t];
        } else {
            g->bigTiles.push_back(t);
        }
    }
    g->background = background;
    for (int a = 0; a < 6; ++a) g->ibbox[a] = ibbox[a];
    for (int a = 0; a < 12; ++a) g->matD[a] = indexToWorld[a];
    for (int a = 0; a < 9; ++a) g->invF[a] = (float)worldToIndex[a];   // Map::set: mInvMatF = float(mInvMatD)
    for (int a = 0; a < 3; ++a) g->vecF[a] = (float)indexToWorld[4 * a + 3];
    return g;
}
void oracle_vdb_free(void *g) { delete (VdbTree *)g; }
float oracle_vdb_value(const void *g, int x, int y, int z) { return ((const VdbTree *)g)->GetValue(x, y, z); }
float oracle_vdb_sample_world(const void *g, float x, float y, float z) {
    const VdbTree &t = *(const VdbTree *)g;
    return t.Sample(t.WorldToIndexF({x, y, z}));
}
// NanoVDBMedium bounds: density world bbox, Union with the temperature grid's (media.cpp:531-549)
void oracle_vdb_bounds(const void *density, const void *temperature, float out[6]) {
    double lo[3], hi[3];
    ((const VdbTree *)density)->WorldBBox(lo, hi);
    for (int a = 0; a < 3; ++a) { out[a] = (float)lo[a]; out[3 + a] = (float)hi[a]; }
    if (temperature) {
        ((const VdbTree *)temperature)->WorldBBox(lo, hi);
        for (int a = 0; a < 3; ++a) {
            out[a] = std::min(out[a], (float)lo[a]);
            out[3 + a] = std::max(out[3 + a], (float)hi[a]);
        }
    }
}
void oracle_vdb_majorant(const void *density, const float bounds[6], int rx, int ry, int rz, float *out) {
    VdbMajorant(*(const VdbTree *)density, bounds, rx, ry, rz, out);
}

// MajorantGrid build — media.cpp:229,241-246 with MajorantGrid::VoxelBounds media.h:123-127
void oracle_build_majorant(const float *density, int nx, int ny, int nz, int rx, int ry, int rz, float *out) {
    Grid g{density, nx, ny, nz};
    for (int z = 0; z < rz; ++z)
        for (int y = 0; y < ry; ++y)
            for (int x = 0; x < rx; ++x) {
                Bounds b{{float(x) / rx, float(y) / ry, float(z) / rz},
                         {float(x + 1) / rx, float(y + 1) / ry, float(z + 1) / rz}};
                out[x + rx * (y + ry * z)] = g.MaxValue(b);
            }
}

// One pixel sample: L (4), lambda (4), pdf (4); returns number of tentative collisions.
int oracle_pixel_sample(const OracleScene *s, int px, int py, int sampleIndex, float *L, float *lambda, float *pdf,
                        float *weight) {
    SceneView sv(*s);
    int nEvents = 0;
    SampleResult r = EvaluatePixelSample(sv, px, py, sampleIndex, &nEvents);
    for (int i = 0; i < NS; ++i) { L[i] = r.L.v[i]; lambda[i] = r.l.lambda[i]; pdf[i] = r.l.pdf[i]; }
    if (weight) *weight = r.weight;
    return nEvents;
}

// Film accumulation for samples [spp0, spp1) of every pixel; rgbSum[W*H*3], wSum[W*H] (fp64).
// Tiles of <=32x32 pixels handed to nthreads workers (util/parallel.cpp:307-328); per pixel
// the samples are added in sampleIndex order, as ImageTileIntegrator::Render does.
long long oracle_render(const OracleScene *s, int spp0, int spp1, int nthreads, double *rgbSum, double *wSum) {
    SceneView sv(*s);
    const int W = s->width, H = s->height, tile = 32;
    const int ntx = (W + tile - 1) / tile, nty = (H + tile - 1) / tile;
    std::atomic<int> next{0};
    std::atomic<long long> events{0};
    auto worker = [&]() {
        long long ev = 0;
        while (true) {
            int t = next.fetch_add(1);
            if (t >= ntx * nty) break;
            int tx = t % ntx, ty = t / ntx;
            for (int py = ty * tile; py < std::min(H, (ty + 1) * tile); ++py)
                for (int px = tx * tile; px < std::min(W, (tx + 1) * tile); ++px)
                    for (int si = spp0; si < spp1; ++si) {
                        int ne = 0;
                        SampleResult r = EvaluatePixelSample(sv, px, py, si, &ne);
                        ev += ne;
                        size_t pi = (size_t)py * W + px;
                        AddSample(*s, rgbSum + 3 * pi, wSum + pi, r.L, r.l, r.weight);
                    }
        }
        events += ev;
    };
    if (nthreads <= 1) worker();
    else {
        std::vector<std::thread> th;
        for (int i = 0; i < nthreads; ++i) th.emplace_back(worker);
        for (auto &t : th) t.join();
    }
    return events.load();
}

// Same, for an explicit pixel list (the bounded CPU-baseline sample of bench.py):
// pixels[i] = linear pixel index; film sums written per list entry.
long long oracle_render_list(const OracleScene *s, const int *pixels, int n, int spp0, int spp1, int nthreads,
                             double *rgbSum, double *wSum) {
    SceneView sv(*s);
    std::atomic<int> next{0};
    std::atomic<long long> events{0};
    auto worker = [&]() {
        long long ev = 0;
        while (true) {
            int i = next.fetch_add(1);
            if (i >= n) break;
            int px = pixels[i] % s->width, py = pixels[i] / s->width;
            for (int si = spp0; si < spp1; ++si) {
                int ne = 0;
                SampleResult r = EvaluatePixelSample(sv, px, py, si, &ne);
                ev += ne;
                AddSample(*s, rgbSum + 3 * (size_t)i, wSum + i, r.L, r.l, r.weight);
            }
        }
        events += ev;
    };
    if (nthreads <= 1) worker();
    else {
        std::vector<std::thread> th;
        for (int i = 0; i < nthreads; ++i) th.emplace_back(worker);
        for (auto &t : th) t.join();
    }
    return events.load();
}

// RGBFilm::GetPixelRGB — film.h:258-274 (no splats).
void oracle_film_resolve(const OracleScene *s, const double *rgbSum, const double *wSum, float *rgbOut) {
    const size_t n = (size_t)s->width * s->height;
    for (size_t i = 0; i < n; ++i) {
        float rgb[3] = {(float)rgbSum[3 * i], (float)rgbSum[3 * i + 1], (float)rgbSum[3 * i + 2]};
        float w = (float)wSum[i];
        if (w != 0) for (int c = 0; c < 3; ++c) rgb[c] /= w;
        const float *m = s->output_from_sensor;
        for (int r = 0; r < 3; ++r) rgbOut[3 * i + r] = m[3 * r] * rgb[0] + m[3 * r + 1] * rgb[1] + m[3 * r + 2] * rgb[2];
    }
}

// Integrator::Tr (integrators.cpp:324-374): ratio-tracking transmittance between
// medium points p0 -> p1 (no surfaces inside the interface box), n segments; writes Tr[0].
// Used for the analytic Beer-Lambert known-answer tests.
void oracle_transmittance(const OracleScene *s, int n, const float *p0, const float *p1, float lambda_u, float *trOut) {
    SceneView sv(*s);
    Lambda l = SampleVisible(lambda_u);
    for (int i = 0; i < n; ++i) {
        V3 a = {p0[3 * i], p0[3 * i + 1], p0[3 * i + 2]}, b = {p1[3 * i], p1[3 * i + 1], p1[3 * i + 2]};
        RNG rng(HashBytes(&a, 12), HashBytes(&b, 12));
        Ray ray = {a, b - a};  // SpawnRayTo from a medium interaction (ray.h:103-108)
        Spec Tr = Spec::Const(1.f), inv_w = Spec::Const(1.f);
        if (LengthSquared(ray.d) == 0) { trOut[i] = 1.f; continue; }
        V3 pExit = ray.o + ray.d * (1 - ShadowEpsilon);
        ray.d = pExit - ray.o;
        float u = rng.Uniform();
        Spec T_maj = SampleT_maj(sv, ray, 1.f, u, rng, l,
            [&](V3, const MediumProps &mp, Spec sigma_maj, Spec Tm) {
                Spec sigma_n = ClampZero(sigma_maj - mp.sigma_a - mp.sigma_s);
                float pr = Tm[0] * sigma_maj[0];
                Tr = Tr * (Tm * sigma_n / pr);
                inv_w = inv_w * (Tm * sigma_maj / pr);
                if (!Tr || !inv_w) return false;
                return true;
            });
        Tr = Tr * (T_maj / T_maj[0]);
        inv_w = inv_w * (T_maj / T_maj[0]);
        trOut[i] = (Tr / inv_w.Average())[0];
    }
}

// Integrator::Tr at explicit wavelengths (4 per query), all four components.
void oracle_transmittance4(const OracleScene *s, int n, const float *p0, const float *p1, const float *lambdas,
                           float *trOut) {
    SceneView sv(*s);
    for (int i = 0; i < n; ++i) {
        Lambda l;
        for (int k = 0; k < NS; ++k) { l.lambda[k] = lambdas[4 * i + k]; l.pdf[k] = VisibleWavelengthsPDF(l.lambda[k]); }
        V3 a = {p0[3 * i], p0[3 * i + 1], p0[3 * i + 2]}, b = {p1[3 * i], p1[3 * i + 1], p1[3 * i + 2]};
        RNG rng(HashBytes(&a, 12), HashBytes(&b, 12));
        Ray ray = {a, b - a};
        Spec Tr = Spec::Const(1.f), inv_w = Spec::Const(1.f);
        if (LengthSquared(ray.d) != 0) {
            V3 pExit = ray.o + ray.d * (1 - ShadowEpsilon);
            ray.d = pExit - ray.o;
            float u = rng.Uniform();
            Spec T_maj = SampleT_maj(sv, ray, 1.f, u, rng, l,
                [&](V3, const MediumProps &mp, Spec sigma_maj, Spec Tm) {
                    Spec sigma_n = ClampZero(sigma_maj - mp.sigma_a - mp.sigma_s);
                    float pr = Tm[0] * sigma_maj[0];
                    Tr = Tr * (Tm * sigma_n / pr);
                    inv_w = inv_w * (Tm * sigma_maj / pr);
                    if (!Tr || !inv_w) return false;
                    return true;
                });
            Tr = Tr * (T_maj / T_maj[0]);
            inv_w = inv_w * (T_maj / T_maj[0]);
            Tr = Tr / inv_w.Average();
        }
        for (int k = 0; k < NS; ++k) trOut[4 * i + k] = Tr.v[k];
    }
}

// Majorant DDA segments of one ray (for tests): returns count, writes (tMin, tMax, sigma_maj[0]).
int oracle_dda_segments(const OracleScene *s, const float *o, const float *d, float tMax, float lambda_u, int maxSegs,
                        float *out) {
    SceneView sv(*s);
    Lambda l = SampleVisible(lambda_u);
    Ray ray = {{o[0], o[1], o[2]}, {d[0], d[1], d[2]}};
    tMax *= Length(ray.d);
    ray.d = Normalize(ray.d);
    DDA it = SampleRay(sv, ray, tMax, l);
    int n = 0;
    float a, b; Spec sm;
    while (n < maxSegs && it.Next(&a, &b, &sm)) { out[3 * n] = a; out[3 * n + 1] = b; out[3 * n + 2] = sm[0]; ++n; }
    return n;
}

// ---- primitive exports pinned by tests/golden/ref_vectors.json ------------
void oracle_rng(uint64_t seq, uint64_t seed, int n, uint32_t *u32, int64_t advance, uint32_t *after, int nAfter) {
    RNG r(seq, seed);
    for (int i = 0; i < n; ++i) u32[i] = r.U32();
    r.Advance(advance);
    for (int i = 0; i < nAfter; ++i) after[i] = r.U32();
}
void oracle_rng_uniform(uint64_t seq, uint64_t seed, int skip, int n, float *out) {
    RNG r(seq, seed);
    for (int i = 0; i < skip; ++i) r.U32();
    for (int i = 0; i < n; ++i) out[i] = r.Uniform();
}
void oracle_rng_single(uint64_t seq, int n, uint32_t *out) {
    RNG r; r.SetSequence(seq);
    for (int i = 0; i < n; ++i) out[i] = r.U32();
}
uint64_t oracle_hash_float(float f) { return HashFloat(f); }
uint64_t oracle_hash_pixel_seed(int x, int y, int seed) { return HashPixelSeed(x, y, seed); }
uint64_t oracle_hash_point3f(float x, float y, float z) { float b[3] = {x, y, z}; return HashBytes(b, 12); }
uint64_t oracle_mixbits(uint64_t v) { return MixBits(v); }
float oracle_fastexp(float x) { return FastExp(x); }
float oracle_sample_exponential(float u, float a) { return SampleExponential(u, a); }
int oracle_sample_discrete3(const float *w, float u) { return SampleDiscrete3(w, u); }
void oracle_sample_uniform(float u, float lmin, float lmax, float *lambda, float *pdf) {
    Lambda l = SampleUniform(u, lmin, lmax);
    for (int i = 0; i < NS; ++i) { lambda[i] = l.lambda[i]; pdf[i] = l.pdf[i]; }
}
// SpectralFilm render: like oracle_render, plus bucketSums / weightSums [W*H*nbuckets]
long long oracle_render_spectral(const OracleScene *s, int spp0, int spp1, int nthreads, double *rgbSum,
                                 double *wSum, double *bucketSums, double *weightSums) {
    SceneView sv(*s);
    const int W = s->width, H = s->height, nb = s->film_nbuckets;
    std::atomic<int> next{0};
    std::atomic<long long> events{0};
    auto worker = [&]() {
        long long ev = 0;
        while (true) {
            int py = next.fetch_add(1);
            if (py >= H) break;
            for (int px = 0; px < W; ++px)
                for (int si = spp0; si < spp1; ++si) {
                    int ne = 0;
                    SampleResult r = EvaluatePixelSample(sv, px, py, si, &ne);
                    ev += ne;
                    size_t pi = (size_t)py * W + px;
                    AddSampleSpectral(*s, rgbSum + 3 * pi, wSum + pi, bucketSums + pi * nb, weightSums + pi * nb, r.L,
                                      r.l, r.weight);
                }
        }
        events += ev;
    };
    if (nthreads <= 1) worker();
    else {
        std::vector<std::thread> th;
        for (int i = 0; i < nthreads; ++i) th.emplace_back(worker);
        for (auto &t : th) t.join();
    }
    return events.load();
}
void oracle_sample_visible(float u, float *lambda, float *pdf) {
    Lambda l = SampleVisible(u);
    for (int i = 0; i < NS; ++i) { lambda[i] = l.lambda[i]; pdf[i] = l.pdf[i]; }
}
float oracle_hg_eval(float c, float g) { return HenyeyGreenstein(c, g); }
void oracle_hg_sample(const float *wo, float g, float u0, float u1, float *wi, float *pdf) {
    V3 w = SampleHenyeyGreenstein(V3{wo[0], wo[1], wo[2]}, g, u0, u1, pdf);
    wi[0] = w.x; wi[1] = w.y; wi[2] = w.z;
}
float oracle_grid_lookup(const float *v, int nx, int ny, int nz, float x, float y, float z) {
    Grid g{v, nx, ny, nz}; return g.Lookup(V3{x, y, z});
}
float oracle_grid_maxvalue(const float *v, int nx, int ny, int nz, const float *b6) {
    Grid g{v, nx, ny, nz};
    return g.MaxValue(Bounds{{b6[0], b6[1], b6[2]}, {b6[3], b6[4], b6[5]}});
}
int oracle_intersectp(const float *b6, const float *o, const float *d, float tMax, float *t01) {
    Bounds b{{b6[0], b6[1], b6[2]}, {b6[3], b6[4], b6[5]}};
    return IntersectP(b, V3{o[0], o[1], o[2]}, V3{d[0], d[1], d[2]}, tMax, &t01[0], &t01[1]) ? 1 : 0;
}
void oracle_transform_ray(const float *m16, const float *minv16, const float *o, const float *d, int inverse,
                          float *out7) {
    Xform t;
    for (int i = 0; i < 16; ++i) { t.m[i / 4][i % 4] = m16[i]; t.mInv[i / 4][i % 4] = minv16[i]; }
    float tMax = 10.f;
    Ray r = XRay(t, Ray{{o[0], o[1], o[2]}, {d[0], d[1], d[2]}}, &tMax, inverse != 0);
    out7[0] = r.o.x; out7[1] = r.o.y; out7[2] = r.o.z; out7[3] = r.d.x; out7[4] = r.d.y; out7[5] = r.d.z;
    out7[6] = tMax;
}
void oracle_independent_sampler(int px, int py, int sampleIndex, int seed, int dim0, int n, float *out) {
    RNG r;
    r.SetSequence(HashPixelSeed(px, py, seed));
    r.Advance((int64_t)(sampleIndex * 65536ull + dim0));
    for (int i = 0; i < n; ++i) out[i] = r.Uniform();
}
// ZSobolSampler stream for one (pixel, sample): pattern of '1' (Get1D) / '2' (Get2D) calls
void oracle_zsobol(int spp, int resx, int resy, int px, int py, int sampleIndex, int seed, const char *pattern,
                   float *out) {
    OracleScene sc{};
    sc.sampler_type = 1;
    sc.samples_per_pixel = spp;
    sc.width = resx;
    sc.height = resy;
    sc.seed = seed;
    Sampler smp;
    smp.Start(sc, px, py, sampleIndex);
    for (const char *q = pattern; *q; ++q) {
        if (*q == '1') *out++ = smp.Get1D();
        else { smp.Get2D(out, out + 1); out += 2; }
    }
}
float oracle_sobol_fastowen(unsigned long long a, int dim, unsigned int seed) { return SobolSampleFastOwen(a, dim, seed); }
float oracle_sobol_plain(unsigned long long a, int dim) { return std::min(SobolBits(a, dim) * 0x1p-32f, 0x1.fffffep-1f); }
// GaussianFilter::Sample(u): out = {p.x, p.y, weight}
void oracle_gaussian_filter_sample(float rx, float ry, float sigma, int n, const float *u, float *out) {
    GaussianSampler g;
    g.Build(rx, ry, sigma);
    for (int i = 0; i < n; ++i) g.Sample(u[2 * i], u[2 * i + 1], out + 3 * i, out + 3 * i + 1, out + 3 * i + 2);
}
float oracle_noise(float x, float y, float z, float *dnoise3) {
    V3 dn = DNoise(V3{x, y, z});
    dnoise3[0] = dn.x; dnoise3[1] = dn.y; dnoise3[2] = dn.z;
    return Noise(x, y, z);
}
float oracle_blackbody(float lambda, float T) { return Blackbody(lambda, T); }
float oracle_cloud_density(float x, float y, float z, float density, float wispiness, float frequency) {
    return CloudDensity(V3{x, y, z}, density, wispiness, frequency);
}

// ===========================================================================
// Lighting graph (src/graph/): the fork's own SampleT_maj callers.
//
// Geometry model: the medium's boundary primitive is its bounds box, hit
// by a slab test in medium space (the ray mapped by medium_from_render without error
// offsets; Bounds3::IntersectP, vecmath.h:1547-1571), so GetHits(primitive)
// (graph/util.h:419-458) yields OutsideTwoHits {t0, t1} for an origin outside and
// InsideOneHit {t1} for one inside; SkipIntersection moves the origin to ray(t) with no
// surface offset. Spheres (util.h:280-300, 460-463) use Sphere::BasicIntersect's interval
// solve (shapes.h:152-200) once: both roots come from one quadratic, where pbrt re-intersects
// from the spawned exit-side point (t1 differs by round-off; t0 is pbrt's bit for bit).
namespace graphm {
enum { OutsideTwoHits = 0, OutsideOneHit = 1, OutsideZeroHits = 2, InsideOneHit = 3 };
struct Hits { int type; float t[2]; };

static Hits BoxHits(const SceneView &sv, V3 o, V3 d) {
    V3 om = XPoint(sv.mediumX.mInv, o), dm = XVector(sv.mediumX.mInv, d);
    float t0, t1;
    if (!IntersectP(sv.bounds, om, dm, Infinity, &t0, &t1)) return {OutsideZeroHits, {0, 0}};
    if (t0 > 0) return {OutsideTwoHits, {t0, t1}};
    return {InsideOneHit, {t1, 0}};
}
// Primitive::Intersect(ray, Infinity)->tHit in the same model: the first crossing
static bool BoxFirstHit(const SceneView &sv, V3 o, V3 d, float *tHit) {
    Hits h = BoxHits(sv, o, d);
    if (h.type == OutsideZeroHits) return false;
    *tHit = h.t[0];
    return true;
}

// Interval ops of util/math.h:818-1070 (CPU rounding: NextFloatUp/Down of the float op)
static inline float MulRoundUp(float a, float b) { return NextFloatUp(a * b); }
static inline float MulRoundDown(float a, float b) { return NextFloatDown(a * b); }
static inline float DivRoundUp(float a, float b) { return NextFloatUp(a / b); }
static inline float DivRoundDown(float a, float b) { return NextFloatDown(a / b); }
static inline Interval Iv(float lo, float hi) { return {std::min(lo, hi), std::max(lo, hi)}; }
static inline Interval IAdd(Interval a, Interval b) { return Iv(AddRoundDown(a.low, b.low), AddRoundUp(a.high, b.high)); }
static inline Interval ISub(Interval a, Interval b) { return Iv(SubRoundDown(a.low, b.high), SubRoundUp(a.high, b.low)); }
static inline Interval IMul(Interval a, Interval b) {
    float lp[4] = {MulRoundDown(a.low, b.low), MulRoundDown(a.high, b.low), MulRoundDown(a.low, b.high),
                   MulRoundDown(a.high, b.high)};
    float hp[4] = {MulRoundUp(a.low, b.low), MulRoundUp(a.high, b.low), MulRoundUp(a.low, b.high),
                   MulRoundUp(a.high, b.high)};
    return Iv(std::min({lp[0], lp[1], lp[2], lp[3]}), std::max({hp[0], hp[1], hp[2], hp[3]}));
}
static inline bool InRange0(Interval i) { return 0 >= i.low && 0 <= i.high; }
static inline Interval IDiv(Interval a, Interval b) {
    if (InRange0(b)) return Iv(-Infinity, Infinity);
    float lq[4] = {DivRoundDown(a.low, b.low), DivRoundDown(a.high, b.low), DivRoundDown(a.low, b.high),
                   DivRoundDown(a.high, b.high)};
    float hq[4] = {DivRoundUp(a.low, b.low), DivRoundUp(a.high, b.low), DivRoundUp(a.low, b.high),
                   DivRoundUp(a.high, b.high)};
    return Iv(std::min({lq[0], lq[1], lq[2], lq[3]}), std::max({hq[0], hq[1], hq[2], hq[3]}));
}
static inline Interval IScale(float f, Interval i) {   // Float * Interval (math.h:1007-1012)
    if (f > 0) return Iv(MulRoundDown(f, i.low), MulRoundUp(f, i.high));
    return Iv(MulRoundDown(f, i.high), MulRoundUp(f, i.low));
}
static inline Interval ISqr(Interval i) {              // Sqr(Interval), math.h:988-995
    float alow = std::abs(i.low), ahigh = std::abs(i.high);
    if (alow > ahigh) std::swap(alow, ahigh);
    if (InRange0(i)) return Iv(0, MulRoundUp(ahigh, ahigh));
    return Iv(MulRoundDown(alow, alow), MulRoundUp(ahigh, ahigh));
}
static inline Interval ISqrt(Interval i) {             // Sqrt(Interval), math.h:1069-1071
    return Iv(std::max<float>(0, NextFloatDown(std::sqrt(i.low))), NextFloatUp(std::sqrt(i.high)));
}

// Sphere of radius r at c: objectFromRender = Inverse(Translate(c)) (util.h:289-291), the ray
// mapped as exact Point3fi / Vector3fi (transform.h:136-180, 276-310), then the quadric
// solve of Sphere::BasicIntersect (shapes.h:152-191) with tMax = Infinity. A full sphere
// never clips. Returns hit-type and (Float) midpoints of the roots.
static Hits SphereHits(V3 c, float r, V3 o, V3 d) {
    const float m[3][4] = {{1, 0, 0, -c.x}, {0, 1, 0, -c.y}, {0, 0, 1, -c.z}};
    Interval oi[3], di[3];
    const float ov[3] = {o.x, o.y, o.z}, dv[3] = {d.x, d.y, d.z};
    for (int k = 0; k < 3; ++k) {
        float xp = (m[k][0] * ov[0] + m[k][1] * ov[1]) + (m[k][2] * ov[2] + m[k][3]);
        float e = gamma(3) * (std::abs(m[k][0] * ov[0]) + std::abs(m[k][1] * ov[1]) + std::abs(m[k][2] * ov[2]) +
                              std::abs(m[k][3]));
        oi[k] = Interval::FromValueAndError(xp, e);
        float vp = m[k][0] * dv[0] + m[k][1] * dv[1] + m[k][2] * dv[2];
        float ve = gamma(3) * (std::abs(m[k][0] * dv[0]) + std::abs(m[k][1] * dv[1]) + std::abs(m[k][2] * dv[2]));
        di[k] = Interval::FromValueAndError(vp, ve);
    }
    Interval a = IAdd(IAdd(ISqr(di[0]), ISqr(di[1])), ISqr(di[2]));
    Interval b = IScale(2, IAdd(IAdd(IMul(di[0], oi[0]), IMul(di[1], oi[1])), IMul(di[2], oi[2])));
    Interval R = Interval::Exact(r);
    Interval cc = ISub(IAdd(IAdd(ISqr(oi[0]), ISqr(oi[1])), ISqr(oi[2])), ISqr(R));
    Interval bq = IDiv(b, IScale(2, a));
    Interval v[3];
    for (int k = 0; k < 3; ++k) v[k] = ISub(oi[k], IMul(bq, di[k]));   // bq * di = {bq * di.x, ..} (vecmath.h:351-353, 387-389)
    Interval len = ISqrt(IAdd(IAdd(ISqr(v[0]), ISqr(v[1])), ISqr(v[2])));
    Interval discrim = IMul(IMul(IScale(4, a), IAdd(R, len)), ISub(R, len));
    if (discrim.low < 0) return {OutsideZeroHits, {0, 0}};
    Interval rootDiscrim = ISqrt(discrim);
    Interval q = (b.Midpoint() < 0) ? IScale(-.5f, ISub(b, rootDiscrim)) : IScale(-.5f, IAdd(b, rootDiscrim));
    Interval t0 = IDiv(q, a), t1 = IDiv(cc, q);
    if (t0.low > t1.low) std::swap(t0, t1);
    if (t0.high > Infinity || t1.low <= 0) return {OutsideZeroHits, {0, 0}};
    if (t0.low <= 0) return {InsideOneHit, {t1.Midpoint(), 0}};
    return {OutsideTwoHits, {t0.Midpoint(), t1.Midpoint()}};
}

// util::GetDiskPoints — graph/util.h:179-204
static void DiskPoints(V3 center, float radius, int n, V3 dir, std::vector<V3> &out) {
    out.clear();
    if (n == 0) { out.push_back(center); return; }
    V3 xv, yv;
    CoordinateSystem(dir, &xv, &yv);
    float step = radius / (float)(n + 1);
    xv = xv * step;
    yv = yv * step;
    for (int x = -n; x <= n; ++x)
        for (int y = -n; y <= n; ++y) {
            V3 p = (center + (float)x * xv) + (float)y * yv;
            if (Length(p - center) <= radius) out.push_back(p);
        }
}

// util::StartEndT / GetStartEndT — util.h:469-503
struct StartEnd { float startT, endT, startScatterT, endScatterT; bool notInMedium; };
static StartEnd GetStartEnd(const Hits &mh, const Hits &sh) {
    float mEntry = mh.type == OutsideTwoHits ? mh.t[0] : 0, sEntry = sh.type == OutsideTwoHits ? sh.t[0] : 0;
    float mExit = mh.type == OutsideTwoHits ? mh.t[1] : mh.t[0], sExit = sh.type == OutsideTwoHits ? sh.t[1] : sh.t[0];
    StartEnd se;
    se.startT = mEntry;
    se.endT = std::min(mExit, sExit);
    se.startScatterT = std::max(mEntry, sEntry);
    se.endScatterT = se.endT;
    se.notInMedium = se.endT < se.startScatterT || se.endScatterT < se.startT;
    return se;
}

// Pixel of a graph sampling index (util.h:816-817): samplingResolution.x wide rows
static inline void IndexPixel(uint64_t index, int resX, int *px, int *py) {
    *py = (int)(index / (uint64_t)resX);
    *px = (int)(index - (uint64_t)*py * (uint64_t)resX);
}

// util::SampleTransmittance — util.h:344-366: single-channel ratio tracking. The RNG's
// two constructor arguments are unsequenced in the reference (`RNG rng(Hash(Get1D()),
// Hash(Get1D()))`); GCC — the compiler oracle/ref builds the reference with — evaluates
// them right to left, so the FIRST draw seeds the offset and the SECOND the sequence.
static float SampleTransmittance(const SceneView &sv, Ray ray, float tMax, Sampler &smp, const OracleScene &s,
                                 const Lambda &l) {
    float uOff = smp.Get1D();
    float uSeq = smp.Get1D();
    RNG rng(HashFloat(uSeq), HashFloat(uOff));
    float Tr = 1;
    float u = smp.Get1D();
    SampleT_maj(sv, ray, tMax, u, rng, l, [&](V3, const MediumProps &mp, Spec sigma_maj, Spec) {
        Spec sigma_n = ClampZero(sigma_maj - mp.sigma_a - mp.sigma_s);
        Tr *= sigma_n[0] / sigma_maj[0];
        return Tr != 0;
    });
    (void)s;
    return Tr;
}

// util::Averager::GetAverage (util.h:545-565) with unit weights
static inline float Average(const std::vector<float> &v) {
    if (v.empty()) return 0;
    float avg = 0, w = 0;
    for (float x : v) { avg += x * 1; w += 1; }
    return avg / w;
}
}  // namespace graphm


// LightingCalculator::GetLightVector (lighting_calculator.cpp:84-155) with
// ComputeRaysToSphere(rayInSphere = nullopt) (util.h:814-840): per vertex (list index =
// vertex id), disk points around vertex - inDir * maxDistToCenter * 2, a ray along inDir
// from each; rays that cross both the medium box and the vertex's sphere average
// `iterations` ratio-tracking estimates to a uniform point of the sphere chord; the light is
// that average over disk points times Inv4Pi. Sampler = the scene's (s->sampler_type, seed,
// samples_per_pixel, width x height), StartPixelSample(pixel(index), i).
void oracle_graph_light(const OracleScene *s, int nv, const float *verts, const float *inDir, float radius,
                        int pointsOnRadius, int iterations, int resX, float maxDistToCenter, float *out) {
    using namespace graphm;
    SceneView sv(*s);
    Lambda l = SampleVisible(0.f);
    V3 dir = {inDir[0], inDir[1], inDir[2]};
    std::vector<V3> disk;
    Sampler smp;
    for (int v = 0; v < nv; ++v) {
        V3 c = {verts[3 * v], verts[3 * v + 1], verts[3 * v + 2]};
        V3 origin = c - (dir * maxDistToCenter) * 2.f;
        DiskPoints(origin, radius, pointsOnRadius, dir, disk);
        std::vector<float> perPoint;
        uint64_t startIndex = (uint64_t)v * disk.size();
        for (size_t k = 0; k < disk.size(); ++k) {
            uint64_t curIndex = startIndex + k;
            Hits mh = BoxHits(sv, disk[k], dir), sh = SphereHits(c, radius, disk[k], dir);
            if (mh.type != OutsideTwoHits || sh.type != OutsideTwoHits) continue;
            StartEnd se = GetStartEnd(mh, sh);
            if (se.notInMedium) continue;
            Ray ray = {disk[k] + dir * se.startT, dir};   // SkipIntersection (model: no offset)
            float st = se.startT;
            se.startT -= st; se.endT -= st; se.startScatterT -= st; se.endScatterT -= st;
            int px, py;
            IndexPixel(curIndex, resX, &px, &py);
            float distInSphere = se.endScatterT - se.startScatterT;
            std::vector<float> trs;
            for (int i = 0; i < iterations; ++i) {
                smp.Start(*s, px, py, i);
                float curDist = distInSphere * smp.Get1D();
                float curT = se.startScatterT + curDist;
                trs.push_back(SampleTransmittance(sv, ray, curT, smp, *s, l));
            }
            perPoint.push_back(Average(trs));
        }
        out[v] = Average(perPoint) * Inv4Pi;
    }
}

// FreeGraphBuilder::TracePath (free/free_graph_builder.cpp:19-141), its medium part: from
// each ray, `iterations` walks (path index ray * iterations + i, sampling index index0[ray]
// + i, StartPixelSample(pixel, sampleIndex)). Per segment: two sampler draws hash into the
// segment RNG (sequenced: RNG(hash0, hash1)), one draw is the first free-flight u; delta
// tracking with absorb / scatter / null choice; the first segment ends at tFirst, later ones
// at the box crossing; a real scatter records its point and, below maxDepth, samples the HG
// phase function (Get2D) for the next direction. Writes up to maxDepth points per walk.
// skipDims: sampler dimensions drawn after StartPixelSample before TracePath (the
// reinforcement rays' phase sample, free_graph_builder.cpp:448-451)
void oracle_graph_walks(const OracleScene *s, int nrays, const float *o, const float *d, const float *tFirst,
                        const long long *index0, int iterations, int sampleIndex, int skipDims, int resX,
                        int maxDepth, float *points, int *counts) {
    using namespace graphm;
    SceneView sv(*s);
    Lambda l = SampleVisible(0.f);
    Sampler smp;
    for (int r = 0; r < nrays; ++r)
        for (int i = 0; i < iterations; ++i) {
            long long path = (long long)r * iterations + i;
            int px, py;
            IndexPixel((uint64_t)(index0[r] + i), resX, &px, &py);
            smp.Start(*s, px, py, sampleIndex);
            for (int k = 0; k < skipDims; ++k) (void)smp.Get1D();
            V3 ro = {o[3 * r], o[3 * r + 1], o[3 * r + 2]}, rd = {d[3 * r], d[3 * r + 1], d[3 * r + 2]};
            bool usedTHit = false;
            int k = 0;
            while (k < maxDepth) {
                float h0 = smp.Get1D();
                float h1 = smp.Get1D();
                RNG rng(HashFloat(h0), HashFloat(h1));
                float tMax;
                if (!usedTHit) { tMax = tFirst[r]; usedTHit = true; }
                else if (!BoxFirstHit(sv, ro, rd, &tMax)) break;
                bool scattered = false;
                V3 pScatter = {0, 0, 0};
                float u = smp.Get1D();
                SampleT_maj(sv, Ray{ro, rd}, tMax, u, rng, l, [&](V3 p, const MediumProps &mp, Spec sigma_maj, Spec) {
                    float pAbsorb = mp.sigma_a[0] / sigma_maj[0];
                    float pScat = mp.sigma_s[0] / sigma_maj[0];
                    float w[3] = {pAbsorb, pScat, std::max<float>(0, 1 - pAbsorb - pScat)};
                    float um = rng.Uniform();
                    int mode = SampleDiscrete3(w, um);
                    if (mode == 0) return false;
                    if (mode == 1) { scattered = true; pScatter = p; return false; }
                    return true;
                });
                if (!scattered) break;
                float *dst = points + 3 * (path * maxDepth + k);
                dst[0] = pScatter.x; dst[1] = pScatter.y; dst[2] = pScatter.z;
                ++k;
                if (k == maxDepth) break;
                float u0, u1, pdf;
                smp.Get2D(&u0, &u1);
                V3 wi = SampleHenyeyGreenstein(-rd, s->g, u0, u1, &pdf);
                ro = pScatter;
                rd = wi;
            }
            counts[path] = k;
        }
}

// FreeGraphBuilder::ReinforceSparseVertices' rays (free_graph_builder.cpp:434-475):
// `sampler.StartPixelSample(Point2i(0, 0), cycle)`, then GetSphereVolumePointsRandom
// (util.h:238-252) on the sampler copy it receives: Point3f((Get1D() - 0.5) * 2 * radius, x3)
// in double arithmetic, the constructor's arguments evaluated right to left by GCC (the first
// draw is z), kept when Length < radius, plus the center; then for each point
// StartPixelSample(pixel(vertexId * nRays + p), cycle), the medium's phase
// Sample_p(Vector3f(1, 0, 0), Get2D()), GetHits(primitive) and SkipIntersection.
void oracle_graph_reinforce_rays(const OracleScene *s, int n, const int *ids, const float *pts, float radius, int nRays,
                                 int cycle, int resX, float *o, float *d, float *tFirst, int *valid) {
    using namespace graphm;
    SceneView sv(*s);
    for (int v = 0; v < n; ++v) {
        Sampler cube;
        cube.Start(*s, 0, 0, cycle);
        const V3 c = {pts[3 * v], pts[3 * v + 1], pts[3 * v + 2]};
        std::vector<V3> sp;
        while ((int)sp.size() < nRays) {
            const double uz = cube.Get1D(), uy = cube.Get1D(), ux = cube.Get1D();
            const V3 q = {(float)((ux - 0.5) * 2 * radius), (float)((uy - 0.5) * 2 * radius),
                          (float)((uz - 0.5) * 2 * radius)};
            if (Length(q) < radius) sp.push_back(q + c);
        }
        for (int k = 0; k < nRays; ++k) {
            const long long ray = (long long)v * nRays + k;
            int px, py;
            IndexPixel((uint64_t)ids[v] * (uint64_t)nRays + (uint64_t)k, resX, &px, &py);
            Sampler smp;
            smp.Start(*s, px, py, cycle);
            float u0, u1, pdf;
            smp.Get2D(&u0, &u1);
            const V3 dir = SampleHenyeyGreenstein(V3{1.f, 0.f, 0.f}, s->g, u0, u1, &pdf);
            const Hits h = BoxHits(sv, sp[k], dir);
            V3 og = sp[k];
            float t = 0.f;
            int ok = 0;
            if (h.type == OutsideTwoHits) { og = sp[k] + dir * h.t[0]; t = h.t[1] - h.t[0]; ok = 1; }
            else if (h.type == InsideOneHit) { t = h.t[0]; ok = 1; }
            o[3 * ray] = og.x; o[3 * ray + 1] = og.y; o[3 * ray + 2] = og.z;
            d[3 * ray] = dir.x; d[3 * ray + 1] = dir.y; d[3 * ray + 2] = dir.z;
            tFirst[ray] = t;
            valid[ray] = ok;
        }
    }
}

// LightingCalculator::ComputeFinalLight (lighting_calculator.cpp:23-59) with Eigen's
// SparseMatrix<float> (column-major) x SparseVector product (the conservative sparse-sparse
// product: row i accumulates T(i,k) * x(k) over k ascending, starting from the first
// product) and SparseVector +=. Dense restatement: with nonnegative finite entries the
// terms Eigen skips (unstored x(k)) add +0. CSR rows must hold ascending columns.
// Returns the iterations completed (a NaN/Inf in the new vector stops before adding it).
int oracle_graph_propagate(int n, const int *rowptr, const int *col, const float *val, const float *light, int bounces,
                           float *total) {
    std::vector<float> cur(light, light + n), next(n);
    for (int i = 0; i < n; ++i) total[i] = light[i];
    int it = 0;
    for (; it < bounces; ++it) {
        bool bad = false;
        for (int i = 0; i < n; ++i) {
            float acc = 0;
            for (int e = rowptr[i]; e < rowptr[i + 1]; ++e) acc = (e == rowptr[i]) ? val[e] * cur[col[e]] : acc + val[e] * cur[col[e]];
            next[i] = acc;
            if (std::isnan(acc) || std::isinf(acc)) bad = true;
        }
        if (bad) break;
        for (int i = 0; i < n; ++i) total[i] += next[i];
        cur.swap(next);
    }
    return it;
}
// Sphere hits / disk points of the model (tests)
int oracle_graph_sphere_hits(float cx, float cy, float cz, float r, const float *o, const float *d, float *t) {
    graphm::Hits h = graphm::SphereHits(V3{cx, cy, cz}, r, V3{o[0], o[1], o[2]}, V3{d[0], d[1], d[2]});
    t[0] = h.t[0]; t[1] = h.t[1];
    return h.type;
}
int oracle_graph_box_hits(const OracleScene *s, const float *o, const float *d, float *t) {
    SceneView sv(*s);
    graphm::Hits h = graphm::BoxHits(sv, V3{o[0], o[1], o[2]}, V3{d[0], d[1], d[2]});
    t[0] = h.t[0]; t[1] = h.t[1];
    return h.type;
}
int oracle_graph_disk_points(const float *center, float radius, int n, const float *dir, float *out, int cap) {
    std::vector<V3> pts;
    graphm::DiskPoints(V3{center[0], center[1], center[2]}, radius, n, V3{dir[0], dir[1], dir[2]}, pts);
    for (size_t i = 0; i < pts.size() && (int)i < cap; ++i) { out[3 * i] = pts[i].x; out[3 * i + 1] = pts[i].y; out[3 * i + 2] = pts[i].z; }
    return (int)pts.size();
}

// Fill an n^3 grid with CloudMedium::Density at voxel centres (i+0.5)/n (BASELINE.md S-cloud).
void oracle_cloud_grid(int n, int z0, int z1, float *out) {
    for (int z = z0; z < z1; ++z)
        for (int y = 0; y < n; ++y)
            for (int x = 0; x < n; ++x)
                out[((size_t)(z - z0) * n + y) * n + x] =
                    CloudDensity(V3{(x + 0.5f) / n, (y + 0.5f) / n, (z + 0.5f) / n}, 1.f, 1.f, 5.f);
}

}  // extern "C"

// Interface sphere helpers (declared before SampleLd / Li), C++ linkage
namespace oracle {
// Convex polyhedron = intersection of half-spaces n.p <= h: the parametric slab clip of
// Bounds3::IntersectP (vecmath.h:1547-1571) over arbitrary planes; dot products left to right.
static graphm::Hits ConvexHits(const float *pl, int n, V3 o, V3 d) {
    float t0 = -Infinity, t1 = Infinity;
    for (int i = 0; i < n; ++i) {
        const float nx = pl[4 * i], ny = pl[4 * i + 1], nz = pl[4 * i + 2], h = pl[4 * i + 3];
        const float denom = (nx * d.x + ny * d.y) + nz * d.z;
        const float num = h - ((nx * o.x + ny * o.y) + nz * o.z);
        if (denom == 0.f) {
            if (num < 0.f) return {graphm::OutsideZeroHits, {0, 0}};
        } else {
            const float t = num / denom;
            if (denom > 0.f) t1 = std::min(t1, t);
            else t0 = std::max(t0, t);
        }
    }
    if (!(t0 <= t1) || t1 <= 0.f) return {graphm::OutsideZeroHits, {0, 0}};
    if (t0 <= 0.f) return {graphm::InsideOneHit, {t1, 0}};
    return {graphm::OutsideTwoHits, {t0, t1}};
}
static graphm::Hits InterfaceHits(const OracleScene &s, V3 o, V3 d) {
    if (s.boundary == 2) return ConvexHits(s.planes, s.n_planes, o, d);
    return graphm::SphereHits(V3{s.sphere[0], s.sphere[1], s.sphere[2]}, s.sphere[3], o, d);
}
static float InterfaceExit(const OracleScene &s, V3 o, V3 d) {
    const graphm::Hits h = InterfaceHits(s, o, d);
    return h.type == graphm::InsideOneHit ? h.t[0] : (h.type == graphm::OutsideTwoHits ? h.t[1] : 0.f);
}
static V3 InterfaceEntry(const OracleScene &s, V3 o, V3 d) {
    const graphm::Hits h = InterfaceHits(s, o, d);
    return h.type == graphm::OutsideTwoHits ? o + d * h.t[0] : o;
}
}  // namespace oracle

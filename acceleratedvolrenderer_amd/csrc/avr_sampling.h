// Pixel-sample generation shared by the device kernels and the host side of the C-ABI:
// ZSobolSampler (samplers.h:225-330, FastOwen randomisation) and the tabulated
// FilterSampler of GaussianFilter (filters.h:26-118, filters.cpp:133-147, PiecewiseConstant
// 1D/2D sampling.h:603-770). Standalone (no HIP headers) so the host tests can compile it
// with g++ and pin it against the reference goldens; device and oracle agree bit for bit.
#pragma once

#include <cstddef>
#include <cstdint>

#ifndef AVR_HD
#define AVR_HD __host__ __device__ __forceinline__
#endif

namespace avr {
namespace smp {

AVR_HD uint32_t bitrev32(uint32_t n) {
#if defined(__clang__)
    return __builtin_bitreverse32(n);
#else
    n = (n << 16) | (n >> 16);
    n = ((n & 0x00ff00ffu) << 8) | ((n & 0xff00ff00u) >> 8);
    n = ((n & 0x0f0f0f0fu) << 4) | ((n & 0xf0f0f0f0u) >> 4);
    n = ((n & 0x33333333u) << 2) | ((n & 0xccccccccu) >> 2);
    n = ((n & 0x55555555u) << 1) | ((n & 0xaaaaaaaau) >> 1);
    return n;
#endif
}

AVR_HD uint64_t mix64(uint64_t v) {   // MixBits, util/hash.h:84-92
    v ^= (v >> 31);
    v *= 0x7fb5d329728ea185ull;
    v ^= (v >> 27);
    v *= 0x81dadef4bc2dd44dull;
    v ^= (v >> 33);
    return v;
}

// MurmurHash64A of an 8-byte key (util/hash.h:19-66): Hash(int a, int b)
AVR_HD uint64_t hash_2u32(uint32_t a, uint32_t b) {
    const uint64_t m = 0xc6a4a7935bd1e995ull;
    uint64_t h = 8ull * m;
    uint64_t k = (uint64_t)a | ((uint64_t)b << 32);
    k *= m;
    k ^= k >> 47;
    k *= m;
    h ^= k;
    h *= m;
    h ^= h >> 47;
    h *= m;
    h ^= h >> 47;
    return h;
}

AVR_HD uint64_t left_shift2(uint64_t x) {   // util/math.h:83-91
    x &= 0xffffffff;
    x = (x ^ (x << 16)) & 0x0000ffff0000ffffull;
    x = (x ^ (x << 8)) & 0x00ff00ff00ff00ffull;
    x = (x ^ (x << 4)) & 0x0f0f0f0f0f0f0f0full;
    x = (x ^ (x << 2)) & 0x3333333333333333ull;
    x = (x ^ (x << 1)) & 0x5555555555555555ull;
    return x;
}
AVR_HD uint64_t encode_morton2(uint32_t x, uint32_t y) { return (left_shift2(y) << 1) | left_shift2(x); }

// Sobol' dimension 0 (van der Corput: column i = bit 31-i) and dimension 1 (Pascal
// matrix mod 2: column i has bit 31-k set iff k is a bit-subset of i) for an index < 2^32:
// dim 0 is the bit reversal; dim 1 is the superset-parity transform of the index bits
// (out_k = XOR of a_i over i ⊇ k), bit-reversed. Equal to the SobolMatrices32 products
// (tests/test_sampling_header.py against the reference's SobolSample).
AVR_HD uint32_t sobol_bits(uint32_t a, int dim) {
    if (dim == 0) return bitrev32(a);
    uint32_t w = a;
    w ^= (w >> 1) & 0x55555555u;
    w ^= (w >> 2) & 0x33333333u;
    w ^= (w >> 4) & 0x0f0f0f0fu;
    w ^= (w >> 8) & 0x00ff00ffu;
    w ^= (w >> 16) & 0x0000ffffu;
    return bitrev32(w);
}
AVR_HD uint32_t fast_owen(uint32_t v, uint32_t seed) {   // lowdiscrepancy.h:220-237
    v = bitrev32(v);
    v ^= v * 0x3d20adeau;
    v += seed;
    v *= (seed >> 16) | 1;
    v ^= v * 0x05526c56u;
    v ^= v * 0x53a22864u;
    return bitrev32(v);
}
AVR_HD float u32_to_unit(uint32_t v) {   // min(v * 2^-32, OneMinusEpsilon)
    // (never NaN: the hardware minimum, one v_min_f32, gives the select's value)
    return __builtin_fminf((float)v * 0x1p-32f, 0x1.fffffep-1f);
}

// The 24 permutations of a base-4 digit in ZSobolSampler::GetSampleIndex's table order,
// each packed into one byte (2 bits per entry), 8 per word.
constexpr uint64_t kZPermW0 = 0xb1e19c6c78d8b4e4ull;   // {0,1,2,3} .. {1,0,3,2}
constexpr uint64_t kZPermW1 = 0x72d236c68d2d39c9ull;   // {1,2,0,3} .. {2,0,3,1}
constexpr uint64_t kZPermW2 = 0x93634b1b87271e4eull;   // {2,3,0,1} .. {3,0,1,2}

struct ZSobolParams {
    int log2spp, nBase4Digits, seed;
    // Optional table of the pixel-only part of GetSampleIndex (zsobol_upper) for the first
    // `dmax` dimensions, row (Morton(pixel) * dmax + dimension); null = computed per call
    const uint32_t *upper;
    int dmax;
    // Optional per-pass table (zsobol_pass_entry) for the first `pdims` dimensions, row
    // (Morton(pixel) * pdims + dimension): valid only for sample indices that agree with the
    // pass's above their low `plo` bits (the host builds it per pass; null = not used)
    const uint64_t *ptab;
    int pdims, plo;
    // Optional compact copy of the pass table's entries the camera stage reads (dimensions 0, 1
    // and 6..9, in that order, 48 B per pixel in scanline order) so its loads stream instead of
    // gathering 48 B from each pixel's row (null = read the rows)
    const uint64_t *ctab;
};
// the fixed-prefix bits of a pass-table entry (below its perm-fixed digit's permutation)
AVR_HD uint64_t pass_prefix_mask(const ZSobolParams &) { return 0x00ffffffffffffffull; }

// Morton(pixel) << log2(spp) | sampleIndex fits 32 bits (nBase4Digits <= 16: e.g. 1024 spp
// at 1080p); beyond it (4096 spp at 720p ...) the index and the digit prefixes are 64-bit.
AVR_HD bool zsobol_wide(const ZSobolParams &zp) { return zp.nBase4Digits > 16; }

// (MixBits(x) >> 24) % 24 (util/hash.h:84-92) with the 40-bit quotient split into 32-bit
// pieces: 2^32 = 16 (mod 24). M = 32-bit: x zero-extended, so v ^= v >> 31 is done in 32 bits.
template <typename M, bool kNarrow = true>
AVR_HD uint32_t mix_perm24(M x) {
    // a 64-bit prefix below 2^32 mixes exactly as its 32-bit value (x >> 31 < 2 either way): the
    // sample digits of indices up to 34 bits (e.g. 4096 spp at 720p) keep the 32-bit multiplies
    // (kNarrow false: always the 64-bit sequence — for lanes of one wave that would split between
    // the two, where the branch runs both)
    if (kNarrow && sizeof(M) == 8 && ((uint64_t)x >> 32) == 0) return mix_perm24<uint32_t>((uint32_t)x);
    uint64_t v = sizeof(M) == 4 ? (uint64_t)(uint32_t)(x ^ (x >> 31)) : ((uint64_t)x ^ ((uint64_t)x >> 31));
    v *= 0x7fb5d329728ea185ull;
    v ^= v >> 27;
    v *= 0x81dadef4bc2dd44dull;
    v ^= v >> 33;
    return ((uint32_t)(v >> 56) * 16u + (uint32_t)(v >> 24) % 24u) % 24u;
}
AVR_HD uint32_t zperm(uint32_t p, uint32_t digit) {
    const uint64_t w = p < 8 ? kZPermW0 : (p < 16 ? kZPermW1 : kZPermW2);
    return (uint32_t)(w >> ((p & 7) * 8 + 2 * digit)) & 3u;
}
// zperm from the 24 permutations staged as bytes (zpt[p] = byte p of kZPermW0..2, e.g. in LDS),
// or from the 64-bit words when zpt is null
AVR_HD uint32_t zperm_t(const uint8_t *zpt, uint32_t p, uint32_t digit) {
    return zpt ? ((uint32_t)zpt[p] >> (2 * digit)) & 3u : zperm(p, digit);
}

// ZSobolSampler::GetSampleIndex (samplers.h:296-355), digits i in [iLo, iHi] (most
// significant first) of the current dimension. M is uint32_t when the whole index fits 32
// bits (the reference's uint64_t values then have zero upper halves), uint64_t otherwise.
// 0x55555555u * dimension is a 32-bit product, zero-extended by the XOR.
template <typename M>
AVR_HD M zsobol_digits(M morton, uint32_t dimension, const ZSobolParams &zp, int iHi, int iLo) {
    M sampleIndex = 0;
    const bool pow2 = zp.log2spp & 1;
    const uint32_t dmix = 0x55555555u * dimension;
    constexpr int kBits = 8 * (int)sizeof(M);
    for (int i = iHi; i >= iLo; --i) {
        const int shift = 2 * i - (pow2 ? 1 : 0);
        const uint32_t digit = (uint32_t)(morton >> shift) & 3u;
        const M higher = shift + 2 >= kBits ? M(0) : M(morton >> (shift + 2));
        const uint32_t p = mix_perm24<M>((M)(higher ^ (M)dmix));
        sampleIndex |= (M)zperm(p, digit) << shift;
    }
    return sampleIndex;
}

// First digit whose bits (and all higher bits) lie in Morton(pixel): shift = 2i - pow2 >= log2spp.
AVR_HD int zsobol_split(const ZSobolParams &zp) { return (zp.log2spp + (zp.log2spp & 1)) / 2; }

// The digits that depend on the pixel only (not on the sample index): a function of
// (Morton(pixel), dimension), shared by every sample of the pixel. Returned shifted down by
// log2(spp) (the lowest of them sits at bit log2spp), so it fits 32 bits for any resolution
// up to 65536^2; pm = Morton(pixel).
AVR_HD uint32_t zsobol_upper(uint32_t pm, uint32_t dimension, const ZSobolParams &zp) {
    if (zsobol_wide(zp)) {
        const uint64_t m = (uint64_t)pm << zp.log2spp;
        return (uint32_t)(zsobol_digits<uint64_t>(m, dimension, zp, zp.nBase4Digits - 1, zsobol_split(zp)) >>
                          zp.log2spp);
    }
    const uint32_t m = pm << zp.log2spp;
    return zsobol_digits<uint32_t>(m, dimension, zp, zp.nBase4Digits - 1, zsobol_split(zp)) >> zp.log2spp;
}

// The remaining digits and the final base-2 digit of an odd log2(spp)
template <typename M>
AVR_HD uint32_t zsobol_lower(M morton, uint32_t dimension, const ZSobolParams &zp) {
    const bool pow2 = zp.log2spp & 1;
    uint32_t sampleIndex = (uint32_t)zsobol_digits<M>(morton, dimension, zp, zsobol_split(zp) - 1, pow2 ? 1 : 0);
    if (pow2) {
        const uint32_t dmix = 0x55555555u * dimension;
        const uint32_t digit = (uint32_t)morton & 1u;
        const M x = (M)(morton >> 1) ^ (M)dmix;
        uint64_t v = (uint64_t)x;
        v ^= v >> 31;
        v *= 0x7fb5d329728ea185ull;
        v ^= v >> 27;
        v *= 0x81dadef4bc2dd44dull;
        v ^= v >> 33;
        sampleIndex |= digit ^ (uint32_t)(v & 1);
    }
    return sampleIndex;
}

// The part of GetSampleIndex shared by a PASS of sample indices that differ only in their low
// `plo` bits (plo <= log2spp), for one (pixel, dimension): digit i (shift s = 2i - pw) is
//   fixed      when s >= plo      — its value bits and its permutation (MixBits of the bits
//                                   above s + 2 and the dimension) lie above plo;
//   perm-fixed when s < plo <= s + 2 — its permutation reads bits >= plo only, its value varies;
//   varying    when s + 2 < plo   — the permutation reads varying bits: computed per draw.
// Returns the fixed digits' permuted bits shifted down by plo (bits 0..55; < 2^52 since the
// index is) and the perm-fixed digit's permutation (0..23) in bits 56..63, 0xFF if none.
// `morton`: the index of any sample of the pass; `up`: zsobol_upper of the pixel (the
// digits above log2spp). A pass of S consecutive indices from `base` has plo = the lowest
// bit count at which base and base + S - 1 agree.
template <typename M>
AVR_HD uint64_t zsobol_pass_entry(M morton, uint32_t dimension, const ZSobolParams &zp, int plo, uint32_t up) {
    const int pw = zp.log2spp & 1;
    const uint32_t dmix = 0x55555555u * dimension;
    constexpr int kBits = 8 * (int)sizeof(M);
    uint64_t fixed = (uint64_t)up << zp.log2spp;
    uint32_t perm = 0xFFu;
    for (int i = zsobol_split(zp) - 1; i >= pw; --i) {
        const int shift = 2 * i - pw;
        if (shift + 2 < plo) break;   // this and every lower digit: varying
        const M higher = shift + 2 >= kBits ? M(0) : M(morton >> (shift + 2));
        const uint32_t p = mix_perm24<M>((M)(higher ^ (M)dmix));
        if (shift >= plo) fixed |= (uint64_t)zperm(p, (uint32_t)(morton >> shift) & 3u) << shift;
        else perm = p;
    }
    return (fixed >> plo) | ((uint64_t)perm << 56);
}

// The entry for `plo` from the entry eA the same pixel, dimension and pass prefix have for
// plo + 2 (plo + 2 <= log2spp): eA's fixed digits, its perm-fixed digit — whose value bits now
// lie at or above plo, so it is fixed too — and the permutation of the digit under plo (one
// MixBits instead of the log2(spp)/2 - plo/2 + 1 a fresh entry takes). A pass of 64 indices
// shares eA with the three passes after it (bits >= plo + 2 agree), so eA is built once per
// four passes.
template <typename M>
AVR_HD uint64_t zsobol_pass_entry_from(M morton, uint32_t dimension, const ZSobolParams &zp, int plo, uint64_t eA) {
    const int pw = zp.log2spp & 1;
    const int ploA = plo + 2;
    constexpr int kBits = 8 * (int)sizeof(M);
    uint64_t fixed = (eA & 0x00ffffffffffffffull) << ploA;
    const uint32_t permA = (uint32_t)(eA >> 56);
    const int iTopA = (ploA + pw - 1) >> 1;
    if (permA != 0xFFu) {
        const int sh = 2 * iTopA - pw;
        fixed |= (uint64_t)zperm(permA, (uint32_t)(morton >> sh) & 3u) << sh;
    }
    uint32_t perm = 0xFFu;
    const int iTop = iTopA - 1;   // (plo + pw - 1) >> 1
    if (iTop >= pw) {
        const int shift = 2 * iTop - pw;
        const M higher = shift + 2 >= kBits ? M(0) : M(morton >> (shift + 2));
        perm = mix_perm24<M>((M)(higher ^ (M)(0x55555555u * dimension)));
    }
    return (fixed >> plo) | ((uint64_t)perm << 56);
}

// GetSampleIndex of (morton, dimension) from the sample's pass entry e: the varying digits
// computed, the perm-fixed digit from e's permutation, the rest from e; an odd log2(spp)'s
// final base-2 digit as zsobol_lower. Bit-identical to zsobol_index without tables.
template <typename M>
AVR_HD M zsobol_index_pass(M morton, uint32_t dimension, const ZSobolParams &zp, uint64_t e, const uint8_t *zpt = nullptr) {
    const int pw = zp.log2spp & 1, plo = zp.plo;
    const uint32_t dmix = 0x55555555u * dimension;
    constexpr int kBits = 8 * (int)sizeof(M);
    M idx = (M)((e & pass_prefix_mask(zp)) << plo);
    const uint32_t perm = (uint32_t)(e >> 56);
    const int iTop = (plo + pw - 1) >> 1;
    for (int i = iTop; i >= pw; --i) {   // digits with shift < plo
        const int shift = 2 * i - pw;
        uint32_t p = perm;
        if (shift + 2 < plo) {
            const M higher = shift + 2 >= kBits ? M(0) : M(morton >> (shift + 2));
            p = mix_perm24<M>((M)(higher ^ (M)dmix));
        }
        idx |= (M)zperm_t(zpt, p, (uint32_t)(morton >> shift) & 3u) << shift;
    }
    if (pw) {
        const uint32_t digit = (uint32_t)morton & 1u;
        const M x = (M)(morton >> 1) ^ (M)dmix;
        uint64_t v = (uint64_t)x;
        v ^= v >> 31;
        v *= 0x7fb5d329728ea185ull;
        v ^= v >> 27;
        v *= 0x81dadef4bc2dd44dull;
        v ^= v >> 33;
        idx |= (M)(digit ^ (uint32_t)(v & 1));
    }
    return idx;
}

// GetSampleIndex of (morton, dimension): from the pass table, else the upper digits from the
// pixel table when present
template <typename M>
AVR_HD M zsobol_index(M morton, uint32_t dimension, const ZSobolParams &zp, const uint8_t *zpt = nullptr) {
    if (zp.ptab && (int)dimension < zp.pdims) {
        const uint32_t pm = (uint32_t)(morton >> zp.log2spp);
        return zsobol_index_pass<M>(morton, dimension, zp, zp.ptab[(size_t)pm * (size_t)zp.pdims + dimension], zpt);
    }
    uint32_t up;
    const uint32_t pm = (uint32_t)(morton >> zp.log2spp);
    if (zp.upper && (int)dimension < zp.dmax)
        up = zp.upper[(size_t)pm * (size_t)zp.dmax + dimension];
    else
        up = zsobol_upper(pm, dimension, zp);
    return ((M)up << zp.log2spp) | (M)zsobol_lower<M>(morton, dimension, zp);
}

// SobolSample bits (lowdiscrepancy.h:168-180) of a 64-bit index: dimension 0's columns
// 32..51 are zero; dimension 1's repeat columns 0..19 (the Pascal matrix mod 2 has period
// 32 in 32 bits; sobolmatrices.cpp rows 0 and 1), so its bits XOR over the two halves.
AVR_HD uint32_t sobol_bits64(uint32_t lo, uint32_t hi, int dim) {
    return dim == 0 ? sobol_bits(lo, 0) : (sobol_bits(lo, 1) ^ sobol_bits(hi, 1));
}

// ZSobolSampler state of one pixel sample: the Morton index with the sample index appended
// (hi = its upper 32 bits, zero unless zsobol_wide) and the dimension
struct ZSobol {
    uint32_t morton;
    uint32_t hi;
    uint32_t dimension;
    AVR_HD void start(int px, int py, int sampleIndex, const ZSobolParams &zp) {
        const uint64_t m = (encode_morton2((uint32_t)px, (uint32_t)py) << zp.log2spp) | (uint64_t)(uint32_t)sampleIndex;
        morton = (uint32_t)m;
        hi = (uint32_t)(m >> 32);
        dimension = 0;
    }
    // kW: 0 = index width decided at run time, 1 = 32-bit (Morton(pixel) << log2 spp fits 32
    // bits; the caller guarantees !zsobol_wide), 2 = 64-bit (the caller guarantees zsobol_wide).
    // The fixed widths let a kernel instantiation carry one code path only.
    template <int kW = 0>
    AVR_HD void index(const ZSobolParams &zp, uint32_t *alo, uint32_t *ahi, const uint8_t *zpt = nullptr) const {
        if (kW == 2 || (kW == 0 && zsobol_wide(zp))) {
            const uint64_t a = zsobol_index<uint64_t>(((uint64_t)hi << 32) | morton, dimension, zp, zpt);
            *alo = (uint32_t)a;
            *ahi = (uint32_t)(a >> 32);
        } else {
            *alo = zsobol_index<uint32_t>(morton, dimension, zp, zpt);
            *ahi = 0;
        }
    }
    template <int kW = 0>
    AVR_HD float get1d(const ZSobolParams &zp) {
        uint32_t a, ah;
        index<kW>(zp, &a, &ah);   // dimension 0 reads the low 32 bits only
        ++dimension;
        const uint32_t h = (uint32_t)hash_2u32(dimension, (uint32_t)zp.seed);
        return u32_to_unit(fast_owen(sobol_bits(a, 0), h));
    }
    template <int kW = 0>
    AVR_HD void get2d(const ZSobolParams &zp, float *u0, float *u1) {
        uint32_t a, ah;
        index<kW>(zp, &a, &ah);
        dimension += 2;
        const uint64_t h = hash_2u32(dimension, (uint32_t)zp.seed);
        *u0 = u32_to_unit(fast_owen(sobol_bits(a, 0), (uint32_t)h));
        *u1 = u32_to_unit(fast_owen(sobol_bits64(a, ah, 1), (uint32_t)(h >> 32)));
    }
    // The draw get1d (two = false: *u0) or get2d (two = true: *u0, *u1) would return with
    // the state's dimension at `dim`, without touching the state: a pure function of
    // (morton, hi, dim), so any lane can evaluate it for another.
    // `dhash`: optional table of Hash(d, seed) for d < dhash_n (the draw's scramble seeds)
    template <int kW = 0>
    AVR_HD void draw_at(const ZSobolParams &zp, uint32_t dim, bool two, float *u0, float *u1,
                        const uint64_t *dhash = nullptr, uint32_t dhash_n = 0, const uint8_t *zpt = nullptr) const {
        ZSobol s = *this;
        s.dimension = dim;
        uint32_t a, ah;
        s.index<kW>(zp, &a, &ah, zpt);
        const uint32_t hd = dim + (two ? 2u : 1u);
        const uint64_t h = hd < dhash_n ? dhash[hd] : hash_2u32(hd, (uint32_t)zp.seed);
        *u0 = u32_to_unit(fast_owen(sobol_bits(a, 0), (uint32_t)h));
        *u1 = u32_to_unit(fast_owen(sobol_bits64(a, ah, 1), (uint32_t)(h >> 32)));
    }
};

// ZSobolSampler constructor parameters (samplers.h:228-238)
inline int ilog2(uint32_t v) { return 31 - __builtin_clz(v); }
inline uint32_t round_up_pow2(uint32_t v) {
    v--; v |= v >> 1; v |= v >> 2; v |= v >> 4; v |= v >> 8; v |= v >> 16;
    return v + 1;
}
inline ZSobolParams zsobol_params(int spp, int width, int height, int seed) {
    ZSobolParams zp;
    zp.log2spp = ilog2((uint32_t)spp);
    const int res = (int)round_up_pow2((uint32_t)(width > height ? width : height));
    zp.nBase4Digits = ilog2((uint32_t)res) + (zp.log2spp + 1) / 2;
    zp.seed = seed;
    zp.upper = nullptr;
    zp.dmax = 0;
    zp.ptab = nullptr;
    zp.pdims = 0;
    zp.plo = 0;
    zp.ctab = nullptr;
    return zp;
}

// ---------------------------------------------------------------------------
// FilterSampler tables of a GaussianFilter: nx = int(32 rx) by ny = int(32 ry) cells.
// Layout (floats): f[ny*nx] | ccdf[ny*(nx+1)] | cint[ny] | mcdf[ny+1] | {mint}
// Optional guide (null = none): for each of the ny conditional CDFs and then the marginal one,
// kFilterGuideK + 1 bytes g[k] = FindInterval's answer at u = k / K (filter_guide_build), so a
// search for u starts from [g[k], g[k + 1]] with k = floor(u K) instead of the whole CDF.
constexpr int kFilterGuideK = 128;
struct FilterTables {
    int nx, ny;
    float rx, ry;
    const float *f, *ccdf, *cint, *mcdf;
    float mint;
    const uint8_t *guide;
    // Optional (null = none): the sample weight of every cell, f / (pdf0 * pdf1) evaluated on
    // the host with the same float operations (filter_cell_weight), so a sample reads it
    // instead of dividing three times
    const float *wt;
};
AVR_HD int filter_table_floats(int nx, int ny) { return nx * ny + ny * (nx + 1) + ny + (ny + 1) + 1; }
AVR_HD int filter_guide_bytes(int ny) { return (ny + 1) * (kFilterGuideK + 1); }
AVR_HD int filter_guide_floats(int ny) { return (filter_guide_bytes(ny) + 3) / 4; }
// tables | guide bytes (padded to a float) | cell weights, in floats
AVR_HD int filter_blob_floats(int nx, int ny) { return filter_table_floats(nx, ny) + filter_guide_floats(ny) + nx * ny; }
// GaussianFilter::Sample's weight for cell (v, u): f / (pdf0 * pdf1) with pdf1 = cint[v] / mint
// and pdf0 = f / cint[v] (0 where the integral is 0), as pc1d_sample computes them
AVR_HD float filter_cell_weight(const float *f, const float *cint, float mint, int nx, int v, int u) {
    const float fv = f[(std::size_t)v * nx + u];
    const float pdf1 = (mint > 0) ? cint[v] / mint : 0;
    const float pdf0 = (cint[v] > 0) ? fv / cint[v] : 0;
    return fv / (pdf0 * pdf1);
}

// FindInterval(n + 1, cdf[i] <= u), util/math.h:508-519, clamped to [0, n - 1] as pc1d_sample
// uses it: for a non-decreasing cdf, the number of i in [1, n - 1] with cdf[i] <= u
AVR_HD int find_interval(const float *cdf, int n, float u) {
    int size = (n + 1) - 2, first = 1;
    while (size > 0) {
        const int half = size >> 1, middle = first + half;
        const bool pr = cdf[middle] <= u;
        first = pr ? middle + 1 : first;
        size = pr ? size - (half + 1) : half;
    }
    const int o = first - 1;
    return o < 0 ? 0 : (o > n - 1 ? n - 1 : o);
}
// The same answer from a guide row g (K + 1 entries, g[k] = find_interval(cdf, n, k / K)): the
// count is monotone in u, so for k / K <= u < (k + 1) / K (u K is exact: K is a power of two)
// it lies in [g[k], g[k + 1]], and the indices there are searched for the last cdf[i] <= u.
// n <= 256 (the guide's entries are bytes); u outside [0, 1) takes the full search.
AVR_HD int find_interval_guided(const float *cdf, int n, const uint8_t *g, float u) {
    if (!(u >= 0.f && u < 1.f)) return find_interval(cdf, n, u);
    const int k = (int)(u * (float)kFilterGuideK);
    int lo = g[k], hi = g[k + 1];
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        const bool pr = cdf[mid] <= u;
        lo = pr ? mid : lo;
        hi = pr ? hi : mid - 1;
    }
    return lo;
}
// the guide row of one CDF (host side of the build)
inline void filter_guide_build(const float *cdf, int n, uint8_t *g) {
    for (int k = 0; k <= kFilterGuideK; ++k) g[k] = (uint8_t)find_interval(cdf, n, (float)k / (float)kFilterGuideK);
}

// The sample point of one PiecewiseConstant1D (cdf[n+1]) over [mn, mx] and its interval
// (guide: the CDF's guide row, or null)
AVR_HD float pc1d_point(const float *cdf, int n, float mn, float mx, float u, int *off, const uint8_t *guide = nullptr) {
    const int o = guide ? find_interval_guided(cdf, n, guide, u) : find_interval(cdf, n, u);
    *off = o;
    float du = u - cdf[o];
    if (cdf[o + 1] - cdf[o] > 0) du /= cdf[o + 1] - cdf[o];
    const float t = (o + du) / (float)n;
    return (1 - t) * mn + t * mx;   // Lerp
}
// Sample one PiecewiseConstant1D given as (cdf[n+1], func[n], funcInt) over [mn, mx]
AVR_HD float pc1d_sample(const float *cdf, const float *func, int n, float funcInt, float mn, float mx, float u,
                         float *pdf, int *off, const uint8_t *guide = nullptr) {
    const float x = pc1d_point(cdf, n, mn, mx, u, off, guide);
    *pdf = (funcInt > 0) ? func[*off] / funcInt : 0;
    return x;
}

// GaussianFilter::Sample(u) -> (p, weight = f[cell] / pdf)
AVR_HD void gaussian_filter_sample(const FilterTables &T, float u0, float u1, float *px, float *py, float *weight) {
    float pdf1, pdf0;
    int v, uo;
    if (T.wt) {   // the cell's weight from the table (a NaN entry: recomputed, its bits are the device's)
        const uint8_t *gm = T.guide ? T.guide + (std::size_t)T.ny * (kFilterGuideK + 1) : nullptr;
        *py = pc1d_point(T.mcdf, T.ny, -T.ry, T.ry, u1, &v, gm);
        const uint8_t *gc = T.guide ? T.guide + (std::size_t)v * (kFilterGuideK + 1) : nullptr;
        *px = pc1d_point(T.ccdf + (std::size_t)v * (T.nx + 1), T.nx, -T.rx, T.rx, u0, &uo, gc);
        const float w = T.wt[(std::size_t)v * T.nx + uo];
        *weight = w == w ? w : filter_cell_weight(T.f, T.cint, T.mint, T.nx, v, uo);
        return;
    }
    const uint8_t *gm = T.guide ? T.guide + (std::size_t)T.ny * (kFilterGuideK + 1) : nullptr;
    *py = pc1d_sample(T.mcdf, T.cint, T.ny, T.mint, -T.ry, T.ry, u1, &pdf1, &v, gm);
    const uint8_t *gc = T.guide ? T.guide + (std::size_t)v * (kFilterGuideK + 1) : nullptr;
    *px = pc1d_sample(T.ccdf + (std::size_t)v * (T.nx + 1), T.f + (std::size_t)v * T.nx, T.nx, T.cint[v], -T.rx, T.rx, u0,
                      &pdf0, &uo, gc);
    *weight = T.f[(std::size_t)v * T.nx + uo] / (pdf0 * pdf1);
}

}  // namespace smp
}  // namespace avr

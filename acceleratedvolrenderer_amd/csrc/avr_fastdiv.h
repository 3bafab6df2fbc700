// Integer division by a run-time divisor as a multiply and a shift (shared by the device
// kernels and the host side; standalone so the host tests compile it with g++).
#pragma once

#include <cstdint>

#ifndef AVR_HD
#define AVR_HD __host__ __device__ __forceinline__
#endif

namespace avr {

// Division of a non-negative int (< 2^31) by a run-time divisor d >= 1 as one 32 x 32 -> 64
// multiply and a shift (Granlund-Montgomery): m = ceil(2^p / d), p = 31 + ceil(log2 d); the
// error n (m - 2^p / d) / 2^p < 2^-ceil(log2 d) <= 1 / d keeps floor exact for every n < 2^31
// (tests/test_fastdiv.py). Replaces the ~20-instruction integer division sequences of the
// per-sample index -> (slot, sample) and pixel -> (x, y) splits.
struct FastDiv {
    uint32_t d, m;
    int p;
};
inline FastDiv fastdiv_make(uint32_t d) {
    FastDiv f;
    f.d = d;
    int l = 0;
    while ((1ull << l) < d) ++l;
    f.p = 31 + l;
    f.m = (uint32_t)(((1ull << f.p) + d - 1) / d);
    return f;
}
AVR_HD int fdiv(int n, const FastDiv &f) { return (int)(((uint64_t)(uint32_t)n * f.m) >> f.p); }
AVR_HD int fmod_(int n, int q, const FastDiv &f) { return n - q * (int)f.d; }

}  // namespace avr

// Sparse float grids with NanoVDB value semantics for NanoVDBMedium (media.h:602-685,
// media.cpp:511-616). NanoVDB (openvdb @ 414bed84, feature/nanovdb, an un-vendored
// submodule of the reference) is absent here; what pbrt uses of it is restated:
//   * Grid::worldToIndexF (Map::applyInverseMapF): index = InvMatF * (xyz - VecF), each row
//     fmaf(x, m0, fmaf(y, m1, z * m2));
//   * ReadAccessor::getValue(ijk): the value stored for ijk in a leaf or a tile, else the
//     grid's background;
//   * SampleFromVoxels<Tree, 1, false>(xyz): ijk = floor(xyz), uvw = xyz - ijk, the 2x2x2
//     stencil of getValue, lerp(a, b, w) = a + w * (b - a) along z, then y, then x
//     (TrilinearSampler::sample).
// Storage: the base layout (Grid) is one int per 8^3 block of the grid's leaf-aligned extent
// (a leaf index, a tile, or background) and 512 floats per leaf, x-major
// ((x&7) << 6 | (y&7) << 3 | z&7) as NanoVDB's LeafNode; the kernels sample the apron layout
// (Apron, below) built from it. Standalone (no HIP headers) for the host-compiled tests.
#pragma once

#include <cstdint>
#include <cstddef>
#include <vector>

#ifndef AVR_HD
#define AVR_HD __host__ __device__ __forceinline__
#endif

namespace avr {
namespace vdb {

constexpr int kBackgroundSlot = INT32_MIN;   // block holds no leaf and no tile

struct Grid {
    const int *slot;          // lnx*lny*lnz: >= 0 leaf index, -(t+1) tile t, kBackgroundSlot
    const float *leaves;      // 512 per leaf
    const float *tiles;       // tile values
    int ox, oy, oz;           // index of the first block's voxel (multiples of 8)
    int lnx, lny, lnz;        // blocks per axis
    float background;
    float inv[9];             // Map::mInvMatF (row-major)
    float vec[3];             // Map::mVecF
};

AVR_HD float get_value(const Grid &g, int x, int y, int z) {
    const int rx = x - g.ox, ry = y - g.oy, rz = z - g.oz;
    if (rx < 0 || ry < 0 || rz < 0) return g.background;
    const int bx = rx >> 3, by = ry >> 3, bz = rz >> 3;
    if (bx >= g.lnx || by >= g.lny || bz >= g.lnz) return g.background;
    const int s = g.slot[((long long)bz * g.lny + by) * g.lnx + bx];
    if (s >= 0) return g.leaves[(long long)s * 512 + (((rx & 7) << 6) | ((ry & 7) << 3) | (rz & 7))];
    if (s == kBackgroundSlot) return g.background;
    return g.tiles[-s - 1];
}

template <typename G>
AVR_HD void world_to_index(const G &g, float x, float y, float z, float *ix, float *iy, float *iz) {
    const float dx = x - g.vec[0], dy = y - g.vec[1], dz = z - g.vec[2];
    *ix = __builtin_fmaf(dx, g.inv[0], __builtin_fmaf(dy, g.inv[1], dz * g.inv[2]));
    *iy = __builtin_fmaf(dx, g.inv[3], __builtin_fmaf(dy, g.inv[4], dz * g.inv[5]));
    *iz = __builtin_fmaf(dx, g.inv[6], __builtin_fmaf(dy, g.inv[7], dz * g.inv[8]));
}

AVR_HD float lerp_vdb(float a, float b, float w) { return a + w * (b - a); }

// One axis of the 2-voxel stencil: block index, in-leaf offset and validity of voxels r, r+1
struct StencilAxis {
    int b0, b1, l0, l1;
    bool v0, v1;
};
AVR_HD StencilAxis stencil_axis(int r, int nblocks, int shift) {
    StencilAxis a;
    a.b0 = r >> 3;
    a.b1 = (r + 1) >> 3;
    a.l0 = (r & 7) << shift;
    a.l1 = ((r + 1) & 7) << shift;
    a.v0 = r >= 0 && a.b0 < nblocks;
    a.v1 = r + 1 >= 0 && a.b1 < nblocks;
    return a;
}
// getValue for one stencil tap from the shared per-axis terms (same value as get_value)
AVR_HD float stencil_value(const Grid &g, bool valid, int bx, int by, int bz, int off) {
    if (!valid) return g.background;
    const int s = g.slot[((long long)bz * g.lny + by) * g.lnx + bx];
    if (s >= 0) return g.leaves[(long long)s * 512 + off];
    if (s == kBackgroundSlot) return g.background;
    return g.tiles[-s - 1];
}

// SampleFromVoxels<Tree, 1, false> at index-space xyz. The eight getValue calls share their
// per-axis block / offset / bounds terms (the stencil crosses a block face on an axis only
// when the voxel's local coordinate is 7); every tap reads the value get_value would.
AVR_HD float sample_trilinear(const Grid &g, float x, float y, float z) {
    const float fx = __builtin_floorf(x), fy = __builtin_floorf(y), fz = __builtin_floorf(z);
    const int i = (int)fx, j = (int)fy, k = (int)fz;
    const float u = x - fx, v = y - fy, w = z - fz;
    const StencilAxis ax = stencil_axis(i - g.ox, g.lnx, 6), ay = stencil_axis(j - g.oy, g.lny, 3),
                      az = stencil_axis(k - g.oz, g.lnz, 0);
    const float v000 = stencil_value(g, ax.v0 && ay.v0 && az.v0, ax.b0, ay.b0, az.b0, ax.l0 | ay.l0 | az.l0);
    const float v001 = stencil_value(g, ax.v0 && ay.v0 && az.v1, ax.b0, ay.b0, az.b1, ax.l0 | ay.l0 | az.l1);
    const float v010 = stencil_value(g, ax.v0 && ay.v1 && az.v0, ax.b0, ay.b1, az.b0, ax.l0 | ay.l1 | az.l0);
    const float v011 = stencil_value(g, ax.v0 && ay.v1 && az.v1, ax.b0, ay.b1, az.b1, ax.l0 | ay.l1 | az.l1);
    const float v100 = stencil_value(g, ax.v1 && ay.v0 && az.v0, ax.b1, ay.b0, az.b0, ax.l1 | ay.l0 | az.l0);
    const float v101 = stencil_value(g, ax.v1 && ay.v0 && az.v1, ax.b1, ay.b0, az.b1, ax.l1 | ay.l0 | az.l1);
    const float v110 = stencil_value(g, ax.v1 && ay.v1 && az.v0, ax.b1, ay.b1, az.b0, ax.l1 | ay.l1 | az.l0);
    const float v111 = stencil_value(g, ax.v1 && ay.v1 && az.v1, ax.b1, ay.b1, az.b1, ax.l1 | ay.l1 | az.l1);
    return lerp_vdb(lerp_vdb(lerp_vdb(v000, v001, w), lerp_vdb(v010, v011, w), v),
                    lerp_vdb(lerp_vdb(v100, v101, w), lerp_vdb(v110, v111, w), v), u);
}

// Grid::worldToIndexF(p) then the sampler (NanoVDBMedium::SamplePoint, media.h:627-636)
AVR_HD float sample_world(const Grid &g, float x, float y, float z) {
    float ix, iy, iz;
    world_to_index(g, x, y, z, &ix, &iy, &iz);
    return sample_trilinear(g, ix, iy, iz);
}

// ---------------------------------------------------------------------------
// Apron layout — what the kernels sample. The trilinear stencil of base voxel r spans r and
// r + 1 per axis, so it leaves r's 8^3 block only through that block's +1 faces. Each block
// b of the extended range [-1, ln - 1] per axis whose 9^3 neighbourhood [8b, 8b + 8]^3 is not
// one constant stores that neighbourhood (getValue of every voxel: its own leaf values, the
// first voxels of the +x/+y/+z neighbours, tiles, background) as an apron block of 729
// floats; a constant neighbourhood stores only its value. A lookup then reads ONE slot and
// eight values of ONE apron block (one dependent round trip instead of the base layout's 8
// slot reads followed by 8 leaf reads), and every tap is the value getValue returns, so the
// sampler's result is bit-identical.
constexpr int kApron = 9;                       // voxels per axis of an apron block
constexpr int kApronVals = kApron * kApron * kApron;

struct Apron {
    const int *slot;          // (lnx+1)*(lny+1)*(lnz+1), extended block e = b + 1: >= 0 apron
                              //   block, < 0: constant consts[-s-1]
    const float *blocks;      // 729 per apron block, x-major: x * 81 + y * 9 + z
    const float *consts;      // constant neighbourhood values (tiles, the background)
    int ox, oy, oz;           // index of base block 0's first voxel
    int lnx, lny, lnz;        // base blocks per axis
    float background;
    float inv[9];
    float vec[3];
    // optional "fat" copy (the density grid's, like GridMedium's): per apron block, for each of
    // its 8^3 base voxels the eight stencil taps as 32 contiguous bytes (8 floats in
    // apron_fat_entry's order), so a lookup after the slot read is ONE 32-B access
    const float *fat;
};

// The fat entry of base voxel k = (x*8 + y)*8 + z of apron block i: the stencil taps
// v000 v001 v010 v011 | v100 v101 v110 v111 (digits = x, y, z offsets), as sample_trilinear
// reads them from the 9^3 block
AVR_HD void apron_fat_entry(const float *blocks, long long i, int k, float out[8]) {
    const float *b = blocks + i * kApronVals + (k >> 6) * (kApron * kApron) + ((k >> 3) & 7) * kApron + (k & 7);
    out[0] = b[0];
    out[1] = b[1];
    out[2] = b[kApron];
    out[3] = b[kApron + 1];
    out[4] = b[kApron * kApron];
    out[5] = b[kApron * kApron + 1];
    out[6] = b[kApron * kApron + kApron];
    out[7] = b[kApron * kApron + kApron + 1];
}

// getValue(x, y, z) from the apron layout (every voxel of the base extent lies in its own
// block's apron; outside the extended range: background)
AVR_HD float get_value(const Apron &g, int x, int y, int z) {
    const int rx = x - g.ox, ry = y - g.oy, rz = z - g.oz;
    const int ex = (rx >> 3) + 1, ey = (ry >> 3) + 1, ez = (rz >> 3) + 1;
    if (ex < 0 || ey < 0 || ez < 0 || ex > g.lnx || ey > g.lny || ez > g.lnz) return g.background;
    const int s = g.slot[((long long)ez * (g.lny + 1) + ey) * (g.lnx + 1) + ex];
    if (s < 0) return g.consts[-s - 1];
    return g.blocks[(long long)s * kApronVals + (rx & 7) * (kApron * kApron) + (ry & 7) * kApron + (rz & 7)];
}

// SampleFromVoxels<Tree, 1, false> at index-space xyz from the apron layout: the same eight
// getValue taps and the same lerps as sample_trilinear
AVR_HD float sample_trilinear(const Apron &g, float x, float y, float z) {
    const float fx = __builtin_floorf(x), fy = __builtin_floorf(y), fz = __builtin_floorf(z);
    const int i = (int)fx, j = (int)fy, k = (int)fz;
    const float u = x - fx, v = y - fy, w = z - fz;
    const int rx = i - g.ox, ry = j - g.oy, rz = k - g.oz;
    const int ex = (rx >> 3) + 1, ey = (ry >> 3) + 1, ez = (rz >> 3) + 1;
    float v000, v001, v010, v011, v100, v101, v110, v111;
    if (ex < 0 || ey < 0 || ez < 0 || ex > g.lnx || ey > g.lny || ez > g.lnz) {
        v000 = v001 = v010 = v011 = v100 = v101 = v110 = v111 = g.background;
    } else {
        const int s = g.slot[((long long)ez * (g.lny + 1) + ey) * (g.lnx + 1) + ex];
        if (s < 0) {
            v000 = v001 = v010 = v011 = v100 = v101 = v110 = v111 = g.consts[-s - 1];
        } else if (g.fat) {
            const float *f = g.fat + ((long long)s * 512 + ((rx & 7) << 6) + ((ry & 7) << 3) + (rz & 7)) * 8;
#if defined(__HIP_DEVICE_COMPILE__)
            const float4 lo = *reinterpret_cast<const float4 *>(f), hi = *reinterpret_cast<const float4 *>(f + 4);
            v000 = lo.x; v001 = lo.y; v010 = lo.z; v011 = lo.w;
            v100 = hi.x; v101 = hi.y; v110 = hi.z; v111 = hi.w;
#else
            v000 = f[0]; v001 = f[1]; v010 = f[2]; v011 = f[3];
            v100 = f[4]; v101 = f[5]; v110 = f[6]; v111 = f[7];
#endif
        } else {
            const float *b = g.blocks + (long long)s * kApronVals + (rx & 7) * (kApron * kApron) + (ry & 7) * kApron +
                             (rz & 7);
            v000 = b[0];
            v001 = b[1];
            v010 = b[kApron];
            v011 = b[kApron + 1];
            v100 = b[kApron * kApron];
            v101 = b[kApron * kApron + 1];
            v110 = b[kApron * kApron + kApron];
            v111 = b[kApron * kApron + kApron + 1];
        }
    }
    return lerp_vdb(lerp_vdb(lerp_vdb(v000, v001, w), lerp_vdb(v010, v011, w), v),
                    lerp_vdb(lerp_vdb(v100, v101, w), lerp_vdb(v110, v111, w), v), u);
}
AVR_HD float sample_world(const Apron &g, float x, float y, float z) {
    float ix, iy, iz;
    world_to_index(g, x, y, z, &ix, &iy, &iz);
    return sample_trilinear(g, ix, iy, iz);
}

// Apron slot of extended block (ex, ey, ez) from the base layout's slots (host side of the
// build): -1 when the 9^3 neighbourhood touches a leaf (an apron block is needed), else the
// base slot whose constant fills all of it (a tile -(t+1) or kBackgroundSlot), or -2 when the
// constant blocks around it disagree (an apron block is needed as well).
inline int apron_classify(const int *slot, int lnx, int lny, int lnz, const float *tiles, float background, int ex,
                          int ey, int ez) {
    int first = 0;
    float c0 = 0.f;
    for (int d = 0; d < 8; ++d) {
        const int bx = ex - 1 + (d & 1), by = ey - 1 + ((d >> 1) & 1), bz = ez - 1 + (d >> 2);
        int s = kBackgroundSlot;
        if (bx >= 0 && by >= 0 && bz >= 0 && bx < lnx && by < lny && bz < lnz)
            s = slot[((long long)bz * lny + by) * lnx + bx];
        if (s >= 0) return -1;
        const float c = s == kBackgroundSlot ? background : tiles[-s - 1];
        if (d == 0) {
            first = s;
            c0 = c;
        } else if (__builtin_memcmp(&c, &c0, sizeof(float)) != 0) {
            return -2;
        }
    }
    return first;
}

// The apron slots of a base layout (host): aslot[(ez * (lny+1) + ey) * (lnx+1) + ex] is the
// apron block index (blocks listed in `list` by extended linear index) or -(c+1) with c the
// constant's index in consts = {tile values..., background} (c = ntiles: the background).
inline void build_apron_slots(const int *slot, int lnx, int lny, int lnz, const float *tiles, int ntiles, float background,
                              std::vector<int> &aslot, std::vector<long long> &list) {
    const long long ne = (long long)(lnx + 1) * (lny + 1) * (lnz + 1);
    aslot.assign((std::size_t)ne, 0);
    list.clear();
    for (int ez = 0; ez <= lnz; ++ez)
        for (int ey = 0; ey <= lny; ++ey)
            for (int ex = 0; ex <= lnx; ++ex) {
                const long long e = ((long long)ez * (lny + 1) + ey) * (lnx + 1) + ex;
                const int k = apron_classify(slot, lnx, lny, lnz, tiles, background, ex, ey, ez);
                if (k == -1 || k == -2) {
                    aslot[(std::size_t)e] = (int)list.size();
                    list.push_back(e);
                } else {
                    aslot[(std::size_t)e] = k == kBackgroundSlot ? -(ntiles + 1) : k;   // tile t: -(t+1)
                }
            }
}

// Values of apron block (ex, ey, ez): getValue over [8b, 8b + 8]^3, b = e - 1, x-major
AVR_HD float apron_value(const Grid &base, int ex, int ey, int ez, int k) {
    const int a = k / (kApron * kApron), bb = (k / kApron) % kApron, c = k % kApron;
    return get_value(base, base.ox + 8 * (ex - 1) + a, base.oy + 8 * (ey - 1) + bb, base.oz + 8 * (ez - 1) + c);
}

}  // namespace vdb
}  // namespace avr

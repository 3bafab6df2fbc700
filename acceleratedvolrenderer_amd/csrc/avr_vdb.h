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
// Storage: one int per 8^3 block of the grid's leaf-aligned extent (a leaf index, a tile,
// or background) and 512 floats per leaf, x-major ((x&7) << 6 | (y&7) << 3 | z&7) as
// NanoVDB's LeafNode. Standalone (no HIP headers) for the host-compiled tests.
#pragma once

#include <cstdint>

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

AVR_HD void world_to_index(const Grid &g, float x, float y, float z, float *ix, float *iy, float *iz) {
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

}  // namespace vdb
}  // namespace avr

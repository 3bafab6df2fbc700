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

// SampleFromVoxels<Tree, 1, false> at index-space xyz
AVR_HD float sample_trilinear(const Grid &g, float x, float y, float z) {
    const float fx = __builtin_floorf(x), fy = __builtin_floorf(y), fz = __builtin_floorf(z);
    const int i = (int)fx, j = (int)fy, k = (int)fz;
    const float u = x - fx, v = y - fy, w = z - fz;
    const float v000 = get_value(g, i, j, k), v001 = get_value(g, i, j, k + 1);
    const float v010 = get_value(g, i, j + 1, k), v011 = get_value(g, i, j + 1, k + 1);
    const float v100 = get_value(g, i + 1, j, k), v101 = get_value(g, i + 1, j, k + 1);
    const float v110 = get_value(g, i + 1, j + 1, k), v111 = get_value(g, i + 1, j + 1, k + 1);
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

// avr_kernels.hip — MI355X (gfx950) wavefront kernels of the volumetric path integrator.
//
// Replaces, for the GPU, pbrt-v4's VolPathIntegrator::Li/SampleLd
// (cpu/integrators.cpp:962-1399), SampleT_maj + DDAMajorantIterator (media.h:136-214,
// 730-806), GridMedium sampling (media.h:265-352), the wavefront work queues
// (wavefront/workqueue.h:41-172) and RGBFilm accumulation (film.h:232-316).
// Paths relative to /root/reference/src/pbrt.
//
// Decomposition (one pass = P pixels x S sample indices, path id = s*P + pixel):
//   k_camera   : sampler start, wavelengths, box-filter camera sample, camera ray
//   k_medium   : delta tracking over the majorant DDA (majorant grid staged in LDS),
//                absorption / real / null events, medium emission, NEE light pick +
//                shadow-ray spawn, HG phase sampling, escaped-ray infinite lights.
//                Survivors and shadow rays are pushed with one atomic per wave
//                (__ballot + __popcll + mbcnt prefix) — stream compaction between events.
//   k_shadow   : ratio-tracking transmittance with Russian roulette along shadow rays
//   k_film     : per pixel, samples added in sampleIndex order into fp64 sums
//                (bit-identical order to ImageTileIntegrator::Render's per-pixel loop).
#include "avr_numerics.h"
#include "avr_sampling.h"
#include "avr_vdb.h"
#include "avr_envmap.h"
#include "avr_flip.h"
#include "avr_boundary.h"

#include <type_traits>

namespace avr {

constexpr int kOccWords = 4096;   // majorant occupancy words k_paths stages (64^3 cells in pairs)

struct DevMedium {
    const float *density;
    int nx, ny, nz;
    float bmin[3], bmax[3];
    Xf render_from_medium, medium_from_render;
    const float *sigma_a, *sigma_s;   // 471-entry densely sampled tables (sigmaScale folded in)
    float g;
    HgC hg;                             // g's Henyey-Greenstein terms (hg_consts(g)), host-computed
    // float(nx, ny, nz) and float(mres), float(mres - 1): host-converted, so the persistent
    // kernel takes them from scalar kernel arguments (each the exact int -> float conversion)
    float fn[3], fres[3], fresm1[3];
    float gray_sigma_a, gray_sigma_s;   // sigma_a[0], sigma_s[0]: the whole tables when the medium is gray
    int emissive;
    const float *Le;                  // 471
    const float *lescale;
    int lnx, lny, lnz;
    const float *majorant;            // mres cells + one trailing 0 (the empty-cell read target)
    int mres[3];
    // coarse occupancy level of the majorant (NanoVDB's 64^3 grid, k_paths): bit b of word w is
    // set unless linear cells 64w+2b and 64w+2b+1 both have majorant 0; null when the grid has
    // more than 64 * kOccWords cells. Staged in LDS by k_paths (16 KiB at 64^3).
    const unsigned *occ;
    // "fat" copy of the density grid (the trilinear footprint of every lookup stored
    // contiguously): entry (ix,iy,iz), ix in [-1, nx-1], holds the 8 taps
    // v(ix..ix+1, iy..iy+1, iz..iz+1) (zero outside the grid) as two float4 = 32 B, so a
    // lookup is ONE 32-B-aligned access inside one cache line instead of 8 scattered taps
    // in 2-4 lines. 8x the grid's memory ((n+1)^3 x 32 B; 34 GB at 1024^3 of the 288 GB).
    const float4 *fat;
    // bricked copy (avr_set_grid_layout 2): 8^3 base voxels per brick with a
    // +1 apron, i.e. the 9^3 values v(8b-1 .. 8b+7) per axis (zero outside the grid) stored x
    // fastest in kBrickFloats floats, bricks in x-fastest order over (nb[0], nb[1], nb[2]) =
    // ceil((n + 1) / 8): every trilinear footprint lies inside ONE brick (offsets 0, 1, 9, 10,
    // 81, 82, 90, 91 floats from its base tap). 1.42x the grid instead of the fat copy's 8x.
    const float *brick;
    int nb[3];
    // medium interface (f3): 0 = the bounds box (the default scene model), 1 = a sphere
    // {cx, cy, cz, r} in render space, 2 = a convex polyhedron (n_planes half-spaces
    // {nx, ny, nz, h}: n.p <= h inside; a convex triangle mesh's face planes) — shapes with no
    // material and MediumInterface(inside = this medium, outside = none): interaction.cpp:91-97
    int boundary;
    float sph[4];
    const float4 *planes;
    int n_planes;
    // optional lookup trace of the wavefront kernels' GridMedium density fetches (unit-box
    // point, in fetch order), for the standalone density-fetch measurement (avr_record_lookups)
    float4 *trace;
    unsigned long long *trace_count;
    long long trace_cap;
    int unit_box;          // bounds extent exactly 1 on every axis: Offset's divisions are by 1.0f
    // medium type: 0 GridMedium (media.h:265-352), 1 HomogeneousMedium (media.h:217-262),
    // 2 CloudMedium (media.h:430-528). Types 1 and 2 have one majorant segment (the
    // HomogeneousMajorantIterator over the bounds crossing, sigma_maj = sigma_t): a 1^3
    // majorant of 1.0 whose DDA never crosses a cell face.
    int type;
    float cloud_density, cloud_wispiness, cloud_frequency;
    // GridMedium temperature grid (media.h:299-316): Le = LeScale * Blackbody(T) normalised,
    // T = (temperature - offset) * scale, emission only where T > 100 K; null = Le spectrum
    const float *temperature;
    float temp_scale, temp_offset;
    // 3 NanoVDBMedium (media.h:602-685): density and optional temperature as sparse grids
    // sampled in index space (avr_vdb.h); Le = LeScale * Blackbody(T) where T > 100 K,
    // emissive iff a temperature grid is present (the integrator tests mp.Le itself)
    vdb::Apron vdb, vdb_temp;
    float vdb_lescale;
    // 4 RGBGridMedium (media.h:355-427): per-voxel RGBUnboundedSpectrum sigma_a / sigma_s and
    // RGBIlluminantSpectrum Le as {c0, c1, c2, scale} (nx*ny*nz each, null = absent), the
    // colour space's illuminant table, sigmaScale and LeScale; sigma tables are {1, 0} so
    // the majorant segments carry SampleRay's sigma_t = 1
    const float4 *rgb_a, *rgb_s, *rgb_le;
    const float *illuminant;
    float rgb_sigma_scale, rgb_le_scale;
};


constexpr int kMaxLights = 8;
struct DevLight {
    int type;                         // 0 distant (delta), 1 uniform infinite, 2 image infinite
    float w[3];                       // render-space direction towards a distant light
    float scale;
    const float *L;                   // 471-entry table
    // type 2, ImageInfiniteLight (lights.h:552-640): res x res equal-area image, per pixel the
    // RGBIlluminantSpectrum {c0, c1, c2, scale}; the colour space's illuminant; the
    // compensated sampling distribution; renderFromLight and its inverse (3x3)
    const float4 *img;
    int res;
    const float *illum;
    env::Distrib2D dist;
    float rfl[9], lfr[9];
    // PowerLightSampler (lightsamplers.h:63-99): this light's AliasTable bin {q, p, alias}
    // (util/sampling.h:822-826) over the lights' Phi; p is the light's PMF
    float aq, ap;
    int alias;
};
struct DevLights {
    int n;
    const DevLight *list;             // device array (indexed by the sampled light)
    float scene_radius;
    int power;                        // 1: PowerLightSampler; 0: BVH / uniform (infinite lights)
};

// VolPath's light pick among infinite lights: BVHLightSampler's infinite branch and
// UniformLightSampler (lightsamplers.h:266-277, 35-50): index min(u / pInf * n, n - 1), PMF
// pInf / n; PowerLightSampler (lightsamplers.h:69-75): AliasTable::Sample
// (util/sampling.cpp:620-645) over the light list's bins. Returns -1 when no light is picked.
// kGeneral: the power branch is compiled in (the wavefront kernels and k_paths' kImage
// instantiation, which the host selects for power renders); k_paths' other instantiations
// keep the BVH pick alone — the branch cost 1.2 % on the headline.
template <bool kGeneral>
__device__ __forceinline__ int light_pick(const DevLights &ls, float u, float *pmf) {
    const int nl = ls.n;
    if (kGeneral && ls.power) {
        int offset = (int)(u * nl);
        offset = offset < nl - 1 ? offset : nl - 1;
        const float up = fminf_(u * nl - offset, kOneMinusEpsilon);
        const DevLight &b = ls.list[offset];
        const int idx = up < b.aq ? offset : b.alias;
        *pmf = ls.list[idx].ap;
        return idx;
    }
    const float pInf = float(nl) / float(nl + 0);
    if (!(u < pInf)) return -1;
    int idx = (int)(u / pInf * nl);
    idx = idx < nl - 1 ? idx : nl - 1;
    *pmf = pInf / nl;
    return idx;
}
// the sampler's PMF of light k (PowerLightSampler::PMF, lightsamplers.h:78-82; BVH: pInf / n)
template <bool kGeneral>
__device__ __forceinline__ float light_pmf(const DevLights &ls, int k) {
    if (kGeneral && ls.power) return ls.list[k].ap;
    return float(ls.n) / float(ls.n + 0) / ls.n;
}

struct DevCamera {
    int type;                         // 0 orthographic, 1 perspective
    float raster[16];                 // cameraFromRaster (full 4x4; perspective is projective)
    Xf render_from_camera;
};

struct DevFilm {
    int width, height;
    float filter_rx, filter_ry;
    int filter_type;                  // 0 BoxFilter, 1 GaussianFilter (FilterSampler tables below)
    smp::FilterTables gauss;
    const float *xyz;                 // 3 x 471
    float imaging_ratio;
    float max_component;
    double *rgb_sum;                  // W*H*3
    double *w_sum;                    // W*H
    // SpectralFilm (film.h:401-530): nbuckets > 0 — uniform wavelengths over [lmin, lmax] and
    // per-pixel bucket sums next to the RGB sums (pixel-major: [pixel * nbuckets + b])
    int nbuckets;
    float lmin, lmax;
    double *bucket_sum, *bucket_w;
};
// Film::SampleWavelengths: RGBFilm SampleVisible (spectrum.h:334-347), SpectralFilm
// SampleUniform (spectrum.h:287-306)
__device__ __forceinline__ Spec film_sample_lambda(const DevFilm &f, float u) {
    return f.nbuckets > 0 ? sample_uniform_lambda(u, f.lmin, f.lmax) : sample_visible_lambda(u);
}
// fast render mode: the visible-wavelength inversion with the hardware log (same u -> same
// wavelengths in k_paths and k_film, both on the device)
__device__ __forceinline__ Spec film_sample_lambda_fast(const DevFilm &f, float u) {
    return f.nbuckets > 0 ? sample_uniform_lambda(u, f.lmin, f.lmax) : sample_visible_lambda_fast(u);
}
__device__ __forceinline__ float film_lambda_pdf(const DevFilm &f, float l) {
    return f.nbuckets > 0 ? 1 / (f.lmax - f.lmin) : visible_wavelength_pdf(l);
}
// the camera stage's: canonical tables staged in LDS (canon::kCanonTabDoubles at `tabs`)
__device__ __forceinline__ Spec film_sample_lambda(const DevFilm &f, float u, const double *tabs) {
    return f.nbuckets > 0 ? sample_uniform_lambda(u, f.lmin, f.lmax) : sample_visible_lambda(u, tabs);
}
__device__ __forceinline__ float film_lambda_pdf(const DevFilm &f, float l, const double *tabs) {
    return f.nbuckets > 0 ? 1 / (f.lmax - f.lmin) : visible_wavelength_pdf(l, tabs);
}

// Interface sphere (DevMedium::boundary 1). Model, shared with the oracle: the medium lives
// inside the sphere; a camera ray that crosses it starts its first medium segment at the
// entry point o + t0 d (pbrt: no medium outside, so no SampleT_maj before the entry and
// SkipIntersection there, integrators.cpp:1118-1122); every medium segment and shadow ray
// ends at the sphere exit computed from its own origin (pbrt re-intersects from the spawned
// point); a ray that does not cross the sphere sees no medium. Sphere::BasicIntersect's
// interval quadric (avr_boundary.h); origins are not offset by intersection error bounds,
// so paths match pbrt's statistically, the oracle's bit for bit.
__device__ __forceinline__ shape::Hits interface_hits(const DevMedium &m, V3 o, V3 d) {
    if (m.boundary == 2) return shape::convex_hits(m.planes, m.n_planes, o, d);
    return shape::sphere_hits(V3{m.sph[0], m.sph[1], m.sph[2]}, m.sph[3], o, d);
}
__device__ __forceinline__ float interface_exit(const DevMedium &m, V3 o, V3 d) {
    const shape::Hits h = interface_hits(m, o, d);
    return h.type == shape::kInsideOneHit ? h.t0 : (h.type == shape::kOutsideTwoHits ? h.t1 : 0.f);
}
__device__ __forceinline__ V3 interface_entry(const DevMedium &m, V3 o, V3 d) {
    const shape::Hits h = interface_hits(m, o, d);
    return h.type == shape::kOutsideTwoHits ? o + d * h.t0 : o;
}

struct PathSoA {
    float4 *o, *d, *lambda, *pdf, *beta, *r_u, *r_l, *L;
    uint64_t *smp_state, *smp_inc;
    int *depth;
    float *weight;                    // per-sample filter weight (GaussianFilter only)
    // k_paths' per-sample record: L (16 B at id), written once at path end
    float4 *rec;
    // k_paths' camera stage (k_paths_camera, one lane per sample of the pass), read by the
    // refill and by k_film: cam0 {o, u}, cam1 {d, ZSobol: the first light-pick draw /
    // independent: the filter weight}, cam2 lambda, cam3 the first segment's RNG SetSequence
    // arguments {seqA, seqB} (u64 each), cam4 the wavelength pdfs, cam5 the IndependentSampler's
    // PCG32 {state, inc} after the camera draws (unused with ZSobol), camw the filter weight
    // (k_film's 4-B read)
    float4 *cam0, *cam1, *cam2, *cam4;
    uint4 *cam3, *cam5;
    float *camw;
};
struct ShadowSoA {
    int *path;
    float4 *o, *d, *bf, *Ls, *rp;     // rp: the path's r_u at the scatter (SampleLd's r_p)
    float2 *pdfs;                     // {p_l, scatterPDF}; scatterPDF < 0 marks a delta light
};

// Per-launch work counters (u64): [0] lookups k_medium, [1] items in k_medium,
// [2] items out k_medium (survivors + shadow pushes), [3] lookups k_shadow, [4] items k_shadow,
// [5] DDA steps k_medium, [6] DDA steps k_shadow; k_paths: [6] loop iterations (per wave),
// [7] sum over iterations of active lanes (SIMD utilisation = [7] / (64 * [6]))
constexpr int kNumStats = 10;   // 0-6 wavefront/shared work counters, 8-9 k_paths wave loop

struct Params {
    DevMedium med;
    DevLights lights;
    DevCamera cam;
    DevFilm film;
    PathSoA ps;
    ShadowSoA sh;
    int max_depth;
    int seed;
    int pass_pixels;                  // P
    int pass_samples;                 // S
    int sample_base;                  // first sampleIndex of the pass
    const int *queue_in;              // nullptr: identity (first depth)
    const int *count_in;
    int *queue_out;
    int *count_out;
    int *shadow_count;
    unsigned long long *stats;
    int *heads;                       // k_paths: 8 per-XCD work counters (zeroed per pass by the
                                      //   camera stage) + [8] the pass generation it last zeroed them for
    int pass_gen;                     // this pass's generation (k_paths runs only after its camera stage)
    const uint64_t *advance;          // k_paths: per pass sample s, {A, H}: Advance(sIdx*65536) ==
                                      //   state' = A*state + inc*H (PCG32 advance is linear in inc)
    int sampler_kind;                 // 0 IndependentSampler, 1 ZSobolSampler (kernels templated on it)
    smp::ZSobolParams zs;
    int refill_min;                   // k_paths: refill a wave once this many lanes are idle
    int dda_budget;                   // k_paths: majorant cells a lane may cross per tracking
                                      //   iteration before yielding (bounds DDA divergence)
    int rec_mode;                     // k_film: 1 = read k_paths' records (ps.rec), 0 = wavefront SoA
    const int *sh_perm;               // k_shadow: processing order of the shadow queue (ray binning), or null
    int fast;                         // render mode: 0 replay (canonical math), 1 fast (hardware math)
    int cam_quad;                     // k_paths_camera: ZSobol quads (pass aligned to 4 sample indices)
    // k_paths' pixel order (avr_set_pixel_order; null = scanline): pass-local slot j of a sample
    // index holds pixel pix_order[j]; pix_slot is the inverse (pixel -> slot, read by k_film)
    const int *pix_order;
    const int *pix_slot;
    FastDiv div_pixels;               // by pass_pixels
    FastDiv div_width;                // by film.width
};

// Kernel arguments re-read where they are used: k_paths' event handlers and collision block and
// the camera stage's sample loop take the Params through the kernarg segment pointer passed
// through an empty asm, so the compiler reloads the fields they use with scalar loads right
// there instead of keeping them live in SGPRs across the kernels' loops. At the SGPR limit those
// long-lived values were spilled to VGPR lanes: in k_paths' headline instantiation 180 SGPR
// spills and 1095 v_readlane VALU instructions (771 in the tracking loop); reloaded, it has 2
// v_readlane, 8572 instead of 9829 instructions and 107 instead of 126 VGPRs (+3.7 % grid,
// +1.6 % NanoVDB, profiles/r06_ab_walk.json); in the camera stage 858 v_readlane and 175
// v_writelane go. The segment pointer, not the by-value argument's address: taking that would
// make the compiler copy the argument to scratch. Only for kernels whose (first and only)
// argument is a Params by value (k_paths, k_paths_camera).
__device__ __forceinline__ const Params &fresh_params() {
    typedef const __attribute__((address_space(4))) Params *KP;
    KP p = (KP)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return *(const Params *)p;
}

__device__ __forceinline__ int lane_id() { return __lane_id(); }

// Wave-aggregated queue push: one atomic per wave, lane offset from the ballot prefix.
__device__ __forceinline__ int wave_push(int *counter, bool pred) {
    const uint64_t mask = __ballot(pred);
    if (mask == 0) return -1;
    const int leader = __ffsll((long long)mask) - 1;
    int base = 0;
    if (lane_id() == leader) base = atomicAdd(counter, __popcll(mask));
    base = __shfl(base, leader);
    const uint64_t lt = (lane_id() == 0) ? 0ull : (mask & ((~0ull) >> (64 - lane_id())));
    return pred ? base + __popcll(lt) : -1;
}

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}
__device__ __forceinline__ void flush_stat(unsigned long long *stats, int idx, unsigned long long v) {
    v = wave_sum_u64(v);
    if (lane_id() == 0 && v) atomicAdd(stats + idx, v);
}

// ---------------------------------------------------------------------------
// GridMedium density fetch — SampledGrid<float>::Lookup (util/containers.h:804-835)
__device__ __forceinline__ float grid_at(const float *__restrict__ v, int nx, int ny, int nz, int x, int y, int z) {
    if (x < 0 || x >= nx || y < 0 || y >= ny || z < 0 || z >= nz) return 0.f;
    return v[(z * ny + y) * nx + x];
}
// fn: float(nx, ny, nz) when the caller has them (the same value as the int -> float conversion)
__device__ __forceinline__ float grid_lookup(const float *__restrict__ v, int nx, int ny, int nz, V3 p,
                                             const float *fn = nullptr) {
    const float fx = fn ? fn[0] : (float)nx, fy = fn ? fn[1] : (float)ny, fz = fn ? fn[2] : (float)nz;
    float psx = p.x * fx - .5f, psy = p.y * fy - .5f, psz = p.z * fz - .5f;
    int ix = (int)__builtin_floorf(psx), iy = (int)__builtin_floorf(psy), iz = (int)__builtin_floorf(psz);
    float dx = psx - (float)ix, dy = psy - (float)iy, dz = psz - (float)iz;
    float d00 = lerp(dx, grid_at(v, nx, ny, nz, ix, iy, iz), grid_at(v, nx, ny, nz, ix + 1, iy, iz));
    float d10 = lerp(dx, grid_at(v, nx, ny, nz, ix, iy + 1, iz), grid_at(v, nx, ny, nz, ix + 1, iy + 1, iz));
    float d01 = lerp(dx, grid_at(v, nx, ny, nz, ix, iy, iz + 1), grid_at(v, nx, ny, nz, ix + 1, iy, iz + 1));
    float d11 = lerp(dx, grid_at(v, nx, ny, nz, ix, iy + 1, iz + 1), grid_at(v, nx, ny, nz, ix + 1, iy + 1, iz + 1));
    return lerp(dz, lerp(dy, d00, d10), lerp(dy, d01, d11));
}

// Same value as grid_lookup() bit for bit (same taps, same lerp order) from the fat layout,
// in two halves so a caller can issue the gather early and combine it later (k_paths issues
// it before the DDA walk and consumes it after, hiding the HBM latency behind the walk).
// fat_issue: false when p's footprint lies outside the fat copy (grid_lookup applies).
__device__ __forceinline__ bool fat_issue(const float4 *__restrict__ fat, int nx, int ny, int nz, V3 p, float4 &a,
                                          float4 &b, float &dx, float &dy, float &dz, const float *fn = nullptr) {
    const float fx = fn ? fn[0] : (float)nx, fy = fn ? fn[1] : (float)ny, fz = fn ? fn[2] : (float)nz;
    float psx = p.x * fx - .5f, psy = p.y * fy - .5f, psz = p.z * fz - .5f;
    int ix = (int)__builtin_floorf(psx), iy = (int)__builtin_floorf(psy), iz = (int)__builtin_floorf(psz);
    if (ix < -1 || ix >= nx || iy < -1 || iy >= ny || iz < -1 || iz >= nz) return false;
    dx = psx - (float)ix, dy = psy - (float)iy, dz = psz - (float)iz;
    // entry index in 32 bits with 24-bit multiplies when the copy has < 2^31 entries (grids to
    // 1290^3; the condition is wave-uniform): (iz + 1)(ny + 1) + iy + 1 < 1291^2 < 2^24
    const uint32_t ex = (uint32_t)nx + 1, ey = (uint32_t)ny + 1;
    size_t e;
    if ((uint64_t)ex * ey * ((uint64_t)nz + 1) < (1ull << 31))
        e = (size_t)(__umul24(__umul24((uint32_t)(iz + 1), ey) + (uint32_t)(iy + 1), ex) + (uint32_t)(ix + 1)) * 2;
    else
        e = (((size_t)(iz + 1) * ey + (iy + 1)) * ex + (ix + 1)) * 2;
    a = fat[e], b = fat[e + 1];
    return true;
}
__device__ __forceinline__ float fat_lerp(float4 a, float4 b, float dx, float dy, float dz) {
    float d00 = lerp(dx, a.x, a.y);
    float d10 = lerp(dx, a.z, a.w);
    float d01 = lerp(dx, b.x, b.y);
    float d11 = lerp(dx, b.z, b.w);
    return lerp(dz, lerp(dy, d00, d10), lerp(dy, d01, d11));
}
// Same value as grid_lookup() bit for bit from the bricked layout (DevMedium::brick).
constexpr int kBrickFloats = 736;   // 9^3 = 729 apron values, padded to 23 x 128-B lines
__device__ __forceinline__ float brick_lookup(const float *__restrict__ brick, const int nb[3],
                                              const float *__restrict__ v, int nx, int ny, int nz, V3 p,
                                              const float *fn = nullptr) {
    const float fx = fn ? fn[0] : (float)nx, fy = fn ? fn[1] : (float)ny, fz = fn ? fn[2] : (float)nz;
    float psx = p.x * fx - .5f, psy = p.y * fy - .5f, psz = p.z * fz - .5f;
    int ix = (int)__builtin_floorf(psx), iy = (int)__builtin_floorf(psy), iz = (int)__builtin_floorf(psz);
    if (ix < -1 || ix >= nx || iy < -1 || iy >= ny || iz < -1 || iz >= nz) return grid_lookup(v, nx, ny, nz, p, fn);
    float dx = psx - (float)ix, dy = psy - (float)iy, dz = psz - (float)iz;
    const int ux = ix + 1, uy = iy + 1, uz = iz + 1;   // 0 .. n: brick u >> 3, apron-local u & 7
    const size_t b = ((size_t)(uz >> 3) * nb[1] + (uy >> 3)) * nb[0] + (ux >> 3);
    const float *q = brick + b * kBrickFloats + ((uz & 7) * 9 + (uy & 7)) * 9 + (ux & 7);
    float d00 = lerp(dx, q[0], q[1]);
    float d10 = lerp(dx, q[9], q[10]);
    float d01 = lerp(dx, q[81], q[82]);
    float d11 = lerp(dx, q[90], q[91]);
    return lerp(dz, lerp(dy, d00, d10), lerp(dy, d01, d11));
}
// GridMedium density in the medium's layout: fat, bricked, or pbrt's linear SampledGrid
__device__ __forceinline__ float grid_density(const DevMedium &m, V3 p);

__device__ __forceinline__ float fat_lookup(const float4 *__restrict__ fat, const float *__restrict__ v, int nx, int ny,
                                            int nz, V3 p, const float *fn = nullptr) {
    float4 a, b;
    float dx, dy, dz;
    if (!fat_issue(fat, nx, ny, nz, p, a, b, dx, dy, dz, fn)) return grid_lookup(v, nx, ny, nz, p, fn);
    return fat_lerp(a, b, dx, dy, dz);
}

__device__ __forceinline__ float grid_density(const DevMedium &m, V3 p) {
    if (m.fat) return fat_lookup(m.fat, m.density, m.nx, m.ny, m.nz, p, m.fn);
    if (m.brick) return brick_lookup(m.brick, m.nb, m.density, m.nx, m.ny, m.nz, p, m.fn);
    return grid_lookup(m.density, m.nx, m.ny, m.nz, p, m.fn);
}

#ifndef AVR_KPATHS_TU   // host-launched kernels: compiled in the C-ABI translation unit only
// the bricked copy (DevMedium::brick): one thread per stored float (pad floats zero)
__global__ void __launch_bounds__(256) k_brickify(const float *__restrict__ v, int nx, int ny, int nz, int nbx, int nby,
                                                  long long nbricks, float *brick) {
    const long long n = nbricks * kBrickFloats;
    for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
        const long long b = e / kBrickFloats;
        const int l = (int)(e - b * kBrickFloats);
        float val = 0.f;
        if (l < 729) {
            const int lx = l % 9, ly = (l / 9) % 9, lz = l / 81;
            const int bx = (int)(b % nbx), by = (int)((b / nbx) % nby), bz = (int)(b / ((long long)nbx * nby));
            val = grid_at(v, nx, ny, nz, 8 * bx + lx - 1, 8 * by + ly - 1, 8 * bz + lz - 1);
        }
        brick[e] = val;
    }
}
__global__ void __launch_bounds__(256) k_fatten(const float *__restrict__ v, int nx, int ny, int nz, float4 *fat) {
    const size_t n = (size_t)(nx + 1) * (ny + 1) * (nz + 1);
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x) {
        const int ix = (int)(e % (nx + 1)) - 1, iy = (int)((e / (nx + 1)) % (ny + 1)) - 1,
                  iz = (int)(e / ((size_t)(nx + 1) * (ny + 1))) - 1;
        fat[2 * e] = make_float4(grid_at(v, nx, ny, nz, ix, iy, iz), grid_at(v, nx, ny, nz, ix + 1, iy, iz),
                                 grid_at(v, nx, ny, nz, ix, iy + 1, iz), grid_at(v, nx, ny, nz, ix + 1, iy + 1, iz));
        fat[2 * e + 1] = make_float4(grid_at(v, nx, ny, nz, ix, iy, iz + 1), grid_at(v, nx, ny, nz, ix + 1, iy, iz + 1),
                                     grid_at(v, nx, ny, nz, ix, iy + 1, iz + 1),
                                     grid_at(v, nx, ny, nz, ix + 1, iy + 1, iz + 1));
    }
}

#endif

// ---------------------------------------------------------------------------
// CloudMedium::Density — the procedural medium (medium type 2) and the generator of the
// synthetic heterogeneous grid (BASELINE.md S-cloud; k_cloud below): CloudMedium::Density
// (media.h:496-520; density 1, wispiness 1, frequency 5) at voxel centres, with
// pbrt's Perlin Noise/DNoise (util/noise.cpp). Only +,-,*,floor,fmod: bit-exact vs CPU.
static __constant__ int c_perm[512] = {
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

__device__ __forceinline__ float noise_grad(int x, int y, int z, float dx, float dy, float dz) {
    int h = c_perm[c_perm[c_perm[x] + y] + z] & 15;
    float u = h < 8 || h == 12 || h == 13 ? dx : dy;
    float v = h < 4 || h == 12 || h == 13 ? dy : dz;
    return ((h & 1) ? -u : u) + ((h & 2) ? -v : v);
}
__device__ __forceinline__ float noise_weight(float t) {
    float t2 = t * t;
    return 6 * ((t2 * t2) * t) - 15 * (t2 * t2) + 10 * (t2 * t);
}
__device__ float perlin(float x, float y, float z) {
    x = fmodf(x, float(1 << 30)); y = fmodf(y, float(1 << 30)); z = fmodf(z, float(1 << 30));
    int ix = (int)__builtin_floorf(x), iy = (int)__builtin_floorf(y), iz = (int)__builtin_floorf(z);
    float dx = x - ix, dy = y - iy, dz = z - iz;
    ix &= 255; iy &= 255; iz &= 255;
    float w000 = noise_grad(ix, iy, iz, dx, dy, dz), w100 = noise_grad(ix + 1, iy, iz, dx - 1, dy, dz);
    float w010 = noise_grad(ix, iy + 1, iz, dx, dy - 1, dz), w110 = noise_grad(ix + 1, iy + 1, iz, dx - 1, dy - 1, dz);
    float w001 = noise_grad(ix, iy, iz + 1, dx, dy, dz - 1), w101 = noise_grad(ix + 1, iy, iz + 1, dx - 1, dy, dz - 1);
    float w011 = noise_grad(ix, iy + 1, iz + 1, dx, dy - 1, dz - 1);
    float w111 = noise_grad(ix + 1, iy + 1, iz + 1, dx - 1, dy - 1, dz - 1);
    float wx = noise_weight(dx), wy = noise_weight(dy), wz = noise_weight(dz);
    float x00 = lerp(wx, w000, w100), x10 = lerp(wx, w010, w110), x01 = lerp(wx, w001, w101), x11 = lerp(wx, w011, w111);
    return lerp(wz, lerp(wy, x00, x10), lerp(wy, x01, x11));
}
__device__ float cloud_density(V3 p, float density, float wispiness, float frequency) {
    V3 pp = frequency * p;
    if (wispiness > 0) {
        float vomega = 0.05f * wispiness, vlambda = 10.f;
        for (int i = 0; i < 2; ++i) {
            V3 q = vlambda * pp;
            const float delta = .01f;
            float n = perlin(q.x, q.y, q.z);
            V3 nd = {perlin(q.x + delta, q.y + 0.f, q.z + 0.f), perlin(q.x + 0.f, q.y + delta, q.z + 0.f),
                     perlin(q.x + 0.f, q.y + 0.f, q.z + delta)};
            V3 dn = (nd - V3{n, n, n}) / delta;
            pp = pp + vomega * dn;
            vomega *= 0.5f;
            vlambda *= 1.99f;
        }
    }
    float d = 0, omega = 0.5f, lam = 1.f;
    for (int i = 0; i < 5; ++i) {
        V3 q = lam * pp;
        d += omega * perlin(q.x, q.y, q.z);
        omega *= 0.5f;
        lam *= 1.99f;
    }
    d = clampf((1 - p.y) * 4.5f * density * d, 0, 1);
    d += 2 * fmaxf_(0.f, 0.5f - p.y);
    return clampf(d, 0, 1);
}

// RGBSigmoidPolynomial (util/color.h:332-365): s(EvaluatePolynomial(lambda, c2, c1, c0))
__device__ __forceinline__ float rsp_eval(float c0, float c1, float c2, float lambda) {
    const float x = __builtin_fmaf(lambda, __builtin_fmaf(lambda, c0, c1), c2);
    if (__builtin_isinf(x)) return x > 0 ? 1.f : 0.f;
    return .5f + x / (2 * __builtin_sqrtf(1 + x * x));
}
__device__ __forceinline__ float rsp_max(float c0, float c1, float c2) {
    const float a = rsp_eval(c0, c1, c2, 360), b = rsp_eval(c0, c1, c2, 830);
    float result = a < b ? b : a;
    const float lambda = -c1 / (2 * c0);
    if (lambda >= 360 && lambda <= 830) {
        const float v = rsp_eval(c0, c1, c2, lambda);
        result = result < v ? v : result;
    }
    return result;
}
// SampledGrid<RGB*Spectrum>::Lookup(p, convert) (containers.h:785-800): the 8 taps are
// converted to sampled spectra (scale * rsp(lambda_i), times the illuminant for Le) and
// lerped per wavelength; taps outside the grid convert T{} = 0
__device__ __forceinline__ Spec rgb_tap(const float4 *__restrict__ g, int nx, int ny, int nz, int x, int y, int z,
                                        const Spec &lam, const Spec &illum, bool illuminant) {
    if (x < 0 || x >= nx || y < 0 || y >= ny || z < 0 || z >= nz) return Spec::c(0.f);
    const float4 c = g[(z * ny + y) * nx + x];
    Spec s{c.w * rsp_eval(c.x, c.y, c.z, lam.v0), c.w * rsp_eval(c.x, c.y, c.z, lam.v1),
           c.w * rsp_eval(c.x, c.y, c.z, lam.v2), c.w * rsp_eval(c.x, c.y, c.z, lam.v3)};
    return illuminant ? s * illum : s;
}
__device__ __forceinline__ Spec spec_lerp(float t, const Spec &a, const Spec &b) { return a * (1 - t) + b * t; }
__device__ Spec rgb_lookup(const float4 *__restrict__ g, int nx, int ny, int nz, V3 p, const Spec &lam,
                           const Spec &illum, bool illuminant) {
    const float psx = p.x * nx - .5f, psy = p.y * ny - .5f, psz = p.z * nz - .5f;
    const int ix = (int)__builtin_floorf(psx), iy = (int)__builtin_floorf(psy), iz = (int)__builtin_floorf(psz);
    const float dx = psx - (float)ix, dy = psy - (float)iy, dz = psz - (float)iz;
    auto T = [&](int a, int b, int c) { return rgb_tap(g, nx, ny, nz, ix + a, iy + b, iz + c, lam, illum, illuminant); };
    const Spec d00 = spec_lerp(dx, T(0, 0, 0), T(1, 0, 0));
    const Spec d10 = spec_lerp(dx, T(0, 1, 0), T(1, 1, 0));
    const Spec d01 = spec_lerp(dx, T(0, 0, 1), T(1, 0, 1));
    const Spec d11 = spec_lerp(dx, T(0, 1, 1), T(1, 1, 1));
    return spec_lerp(dz, spec_lerp(dy, d00, d10), spec_lerp(dy, d01, d11));
}

// GridMedium emission at medium point p (box-offset, media.h:299-316): LeScale lookup, then
// the temperature grid's blackbody or the Le spectrum
__device__ __forceinline__ Spec grid_emission(const DevMedium &m, V3 p, const Spec &lam, const Spec &Le_l) {
    Spec Le = Spec::c(0.f);
    const float scale = grid_lookup(m.lescale, m.lnx, m.lny, m.lnz, p);
    if (scale > 0) {
        if (m.temperature) {
            float temp = grid_lookup(m.temperature, m.nx, m.ny, m.nz, p);
            temp = (temp - m.temp_offset) * m.temp_scale;
            if (temp > 100.f) {
                const float nf = blackbody_norm(temp);
                Le = Spec{blackbody(lam.v0, temp) * nf, blackbody(lam.v1, temp) * nf, blackbody(lam.v2, temp) * nf,
                          blackbody(lam.v3, temp) * nf} * scale;
            }
        } else {
            Le = Le_l * scale;
        }
    }
    return Le;
}

// NanoVDBMedium emission at medium point p (media.h:660-672): LeScale * normalised blackbody
// of the temperature grid where T > 100 K
__device__ __forceinline__ Spec vdb_emission(const DevMedium &m, V3 p, const Spec &lam) {
    float temp = vdb::sample_world(m.vdb_temp, p.x, p.y, p.z);
    temp = (temp - m.temp_offset) * m.temp_scale;
    if (!(temp > 100.f)) return Spec::c(0.f);
    const float nf = blackbody_norm(temp);
    return Spec{m.vdb_lescale * (blackbody(lam.v0, temp) * nf), m.vdb_lescale * (blackbody(lam.v1, temp) * nf),
                m.vdb_lescale * (blackbody(lam.v2, temp) * nf), m.vdb_lescale * (blackbody(lam.v3, temp) * nf)};
}

// ImageInfiniteLight::ImageLe (lights.h:620-627): nearest pixel (octahedral wrap), its
// RGBIlluminantSpectrum sampled at lambda, times the light scale
__device__ __forceinline__ Spec image_le(const DevLight &lt, float u, float v, const Spec &lam) {
    const float4 c = lt.img[env::octahedral_pixel(u, v, lt.res)];
    const Spec il = sample_table(lt.illum, lambda_index(lam));
    const Spec s{c.w * rsp_eval(c.x, c.y, c.z, lam.v0), c.w * rsp_eval(c.x, c.y, c.z, lam.v1),
                 c.w * rsp_eval(c.x, c.y, c.z, lam.v2), c.w * rsp_eval(c.x, c.y, c.z, lam.v3)};
    return s * il * lt.scale;
}
// Transform::operator()(Vector3f) with a 3x3 (row-major): ((m0 x + m1 y) + m2 z)
__device__ __forceinline__ V3 xf_vec3(const float *m, V3 v) {
    return {(m[0] * v.x + m[1] * v.y) + m[2] * v.z, (m[3] * v.x + m[4] * v.y) + m[5] * v.z,
            (m[6] * v.x + m[7] * v.y) + m[8] * v.z};
}
// ImageInfiniteLight::Le(ray) (lights.h:581-585): Le and the equal-area (u, v) of direction d
__device__ __forceinline__ Spec image_le_dir(const DevLight &lt, V3 d, const Spec &lam, float *u, float *v) {
    const V3 wl = normalize(xf_vec3(lt.lfr, d));
    env::sphere_to_square(wl.x, wl.y, wl.z, u, v);
    return image_le(lt, *u, *v, lam);
}
// PDF_Li(ctx, w, allowIncompletePDF = true) (lights.cpp:1042-1052): wLight not normalised
__device__ __forceinline__ float image_pdf_li(const DevLight &lt, V3 w) {
    const V3 wl = xf_vec3(lt.lfr, w);
    float u, v;
    env::sphere_to_square(wl.x, wl.y, wl.z, &u, &v);
    return env::distrib_pdf(lt.dist, u, v) / (4 * kPi);
}

struct MediumSample { Spec sigma_a, sigma_s, Le; };

// GridMedium::SamplePoint — media.h:287-319 (no temperature grid); sig_a/sig_s pre-sampled at lambda
__device__ __forceinline__ MediumSample sample_point(const DevMedium &m, V3 p, const Spec &sig_a, const Spec &sig_s,
                                                     const Spec &Le_l, const Spec &lam, bool emissive = true) {
    MediumSample ms;
    p = xf_point_pair(m.medium_from_render, p);
    ms.Le = Spec::c(0.f);
    if (m.type == 1) {             // HomogeneousMedium::SamplePoint: constant properties
        ms.sigma_a = sig_a;
        ms.sigma_s = sig_s;
        if (emissive && m.emissive) ms.Le = Le_l;
        return ms;
    }
    if (m.type == 2) {             // CloudMedium::SamplePoint: density * sigma at the medium-space point
        const float d = cloud_density(p, m.cloud_density, m.cloud_wispiness, m.cloud_frequency);
        ms.sigma_a = sig_a * d;
        ms.sigma_s = sig_s * d;
        return ms;
    }
    if (m.type == 4) {             // RGBGridMedium::SamplePoint (media.h:377-403)
        p = m.unit_box ? V3{p.x - m.bmin[0], p.y - m.bmin[1], p.z - m.bmin[2]} : box_offset(m.bmin, m.bmax, p);
        const Spec none = Spec::c(0.f);
        const Spec sa = m.rgb_a ? rgb_lookup(m.rgb_a, m.nx, m.ny, m.nz, p, lam, none, false) : Spec::c(1.f);
        const Spec ss = m.rgb_s ? rgb_lookup(m.rgb_s, m.nx, m.ny, m.nz, p, lam, none, false) : Spec::c(1.f);
        ms.sigma_a = sa * m.rgb_sigma_scale;
        ms.sigma_s = ss * m.rgb_sigma_scale;
        if (emissive && m.emissive) {
            const Spec il = sample_table(m.illuminant, lambda_index(lam));
            ms.Le = rgb_lookup(m.rgb_le, m.nx, m.ny, m.nz, p, lam, il, true) * m.rgb_le_scale;
        }
        return ms;
    }
    if (m.type == 3) {             // NanoVDBMedium::SamplePoint (media.h:624-637) and Le (media.h:660-672)
        const float d = vdb::sample_world(m.vdb, p.x, p.y, p.z);
        ms.sigma_a = sig_a * d;
        ms.sigma_s = sig_s * d;
        if (emissive && m.emissive) ms.Le = vdb_emission(m, p, lam);
        return ms;
    }
    // Bounds3::Offset (vecmath.h:1323-1332); x / 1.0f == x exactly, so a unit box skips it
    p = m.unit_box ? V3{p.x - m.bmin[0], p.y - m.bmin[1], p.z - m.bmin[2]} : box_offset(m.bmin, m.bmax, p);
    if (m.trace) {
        const unsigned long long k = atomicAdd(m.trace_count, 1ull);
        if ((long long)k < m.trace_cap) m.trace[k] = make_float4(p.x, p.y, p.z, 0.f);
    }
    float d = grid_density(m, p);
    ms.sigma_a = sig_a * d;
    ms.sigma_s = sig_s * d;
    if (emissive && m.emissive) ms.Le = grid_emission(m, p, lam, Le_l);
    return ms;
}

// DDAMajorantIterator — media.h:136-214. Per-axis state in named scalars (no arrays),
// so the iterator lives in VGPRs: an indexed array here is demoted to scratch.
struct Dda {
    float tMin, tMax;
    float nx, ny, nz;      // nextCrossingT
    float dx, dy, dz;      // deltaT
    int vx, vy, vz;        // voxel
    int sx, sy, sz;        // step (+1/-1); voxelLimit = step > 0 ? res : -1
};
// res: the axis' majorant resolution as a float (exact), resm1 = float(res - 1)
__device__ __forceinline__ void dda_axis(float gia, float gda, float res, float resm1, float tMin, int &voxel, float &next,
                                         float &delta, int &step) {
    voxel = (int)clampf(gia * res, 0.f, resm1);
    delta = 1 / (__builtin_fabsf(gda) * res);
    if (gda == -0.f) gda = 0.f;
    if (gda >= 0) {
        float nextPos = float(voxel + 1) / res;
        next = tMin + (nextPos - gia) / gda;
        step = 1;
    } else {
        float nextPos = float(voxel) / res;
        next = tMin + (nextPos - gia) / gda;
        step = -1;
    }
}
__device__ __forceinline__ bool dda_init(Dda &it, const DevMedium &m, Ray ray, float raytMax) {
    // GridMedium::SampleRay — media.h:322-337
    ray = xf_ray(m.medium_from_render, ray, &raytMax, /*forward=*/false);
    float tMin, tMax;
    if (!intersect_box(m.bmin, m.bmax, ray.o, ray.d, raytMax, &tMin, &tMax)) {
        it.tMin = kInf; it.tMax = -kInf;
        return false;
    }
    it.tMin = tMin; it.tMax = tMax;
    // Bounds3::Offset and d / Diagonal(): divisions by exactly 1.0f for a unit box (x / 1 == x)
    V3 go, gd;
    if (m.unit_box) {
        go = {ray.o.x - m.bmin[0], ray.o.y - m.bmin[1], ray.o.z - m.bmin[2]};
        gd = ray.d;
    } else {
        const float diag0 = m.bmax[0] - m.bmin[0], diag1 = m.bmax[1] - m.bmin[1], diag2 = m.bmax[2] - m.bmin[2];
        go = box_offset(m.bmin, m.bmax, ray.o);
        gd = {ray.d.x / diag0, ray.d.y / diag1, ray.d.z / diag2};
    }
    V3 gi = go + gd * tMin;
    dda_axis(gi.x, gd.x, m.fres[0], m.fresm1[0], tMin, it.vx, it.nx, it.dx, it.sx);
    dda_axis(gi.y, gd.y, m.fres[1], m.fresm1[1], tMin, it.vy, it.ny, it.dy, it.sy);
    dda_axis(gi.z, gd.z, m.fres[2], m.fresm1[2], tMin, it.vz, it.nz, it.dz, it.sz);
    if (m.type == 1 || m.type == 2) {   // HomogeneousMajorantIterator(tMin, tMax, sigma_t): one segment
        it.vx = it.vy = it.vz = 0;
        it.nx = it.ny = it.nz = kInf;
    }
    return true;
}
// Returns false when exhausted; majorant values read through `maj` (LDS-staged when it fits)
__device__ __forceinline__ bool dda_next(Dda &it, const float *maj, const int *res, float *s0, float *s1, float *mval) {
    if (it.tMin >= it.tMax) return false;
    const int bits = ((it.nx < it.ny) << 2) + ((it.nx < it.nz) << 1) + ((it.ny < it.nz));
    // cmpToAxis = {2, 1, 2, 1, 2, 2, 0, 0}
    const int ax = (bits >= 6) ? 0 : ((bits == 1 || bits == 3) ? 1 : 2);
    const float nextA = ax == 0 ? it.nx : (ax == 1 ? it.ny : it.nz);
    const float tExit = nextA < it.tMax ? nextA : it.tMax;   // std::min(tMax, next), NaN -> tMax
    *mval = maj[it.vx + res[0] * (it.vy + res[1] * it.vz)];
    *s0 = it.tMin;
    *s1 = tExit;
    it.tMin = tExit;
    if (nextA > it.tMax) it.tMin = it.tMax;
    if (ax == 0) {
        it.vx += it.sx;
        if (it.vx == (it.sx > 0 ? res[0] : -1)) it.tMin = it.tMax;
        it.nx += it.dx;
    } else if (ax == 1) {
        it.vy += it.sy;
        if (it.vy == (it.sy > 0 ? res[1] : -1)) it.tMin = it.tMax;
        it.ny += it.dy;
    } else {
        it.vz += it.sz;
        if (it.vz == (it.sz > 0 ? res[2] : -1)) it.tMin = it.tMax;
        it.nz += it.dz;
    }
    return true;
}

// SampleT_maj<GridMedium> — media.h:741-806. `cb(p, ms, sigma_maj, T_maj)` returns false to stop.
template <typename F>
__device__ __forceinline__ Spec sample_t_maj(const DevMedium &m, const float *maj, Ray ray, float tMax, float u,
                                            Pcg32 &rng, const Spec &sig_a, const Spec &sig_s, const Spec &Le_l,
                                            const Spec &lam, unsigned long long &nLookup, unsigned long long &nSteps,
                                            F &&cb) {
    tMax *= length(ray.d);
    ray.d = normalize(ray.d);
    Dda it;
    dda_init(it, m, ray, tMax);
    const Spec sigma_t = sig_a + sig_s;
    Spec T_maj = Spec::c(1.f);
    while (true) {
        float segMin, segMax, mv;
        if (!dda_next(it, maj, m.mres, &segMin, &segMax, &mv)) return T_maj;
        ++nSteps;
        const Spec sigma_maj = sigma_t * mv;
        if (sigma_maj.v0 == 0) {
            float dt = segMax - segMin;
            if (__builtin_isinf(dt)) dt = kFloatMax;
            T_maj = T_maj * fast_exp(-(sigma_maj * dt));
            continue;
        }
        float tMin = segMin;
        while (true) {
            float t = tMin + sample_exponential(u, sigma_maj.v0);
            u = rng.uniform();
            if (t < segMax) {
                T_maj = T_maj * fast_exp(-(sigma_maj * (t - tMin)));
                V3 p = ray.o + ray.d * t;
                ++nLookup;
                MediumSample ms = sample_point(m, p, sig_a, sig_s, Le_l, lam);
                if (!cb(p, ms, sigma_maj, T_maj)) return Spec::c(1.f);
                T_maj = Spec::c(1.f);
                tMin = t;
            } else {
                float dt = segMax - tMin;
                if (__builtin_isinf(dt)) dt = kFloatMax;
                T_maj = T_maj * fast_exp(-(sigma_maj * dt));
                break;
            }
        }
    }
}

// Per-path sampler state. IndependentSampler — samplers.h:442-476: PCG32 stream
// SetSequence(Hash(p, seed)) (the one-argument SetSequence seeds with MixBits(seq),
// rng.h:43-45) advanced by sampleIndex * 65536; Get2D = two Get1D, left to right.
// ZSobolSampler — samplers.h:225-330 (avr_sampling.h). In the wavefront SoA the state
// lives in smp_state / smp_inc (PCG state / increment, or Morton index / dimension).
// PathSampler<K>: K = 0 IndependentSampler; K = 1 ZSobolSampler (index width decided per
// call); K = 2 / 3 ZSobolSampler with a 32-bit / 64-bit sample index fixed at compile time
// (k_paths instantiations: one code path per kernel; the host picks by zsobol_wide).
template <int K> struct PathSampler;
template <> struct PathSampler<0> {
    Pcg32 rng;
    __device__ __forceinline__ void start(const Params &P, int px, int py, int sampleIndex) {
        const uint64_t seq = hash_3u32((uint32_t)px, (uint32_t)py, (uint32_t)P.seed);
        rng.set_sequence(seq, mix_bits(seq));
        rng.advance((uint64_t)sampleIndex * 65536ull);
    }
    __device__ __forceinline__ float get1d(const Params &) { return rng.uniform(); }
    __device__ __forceinline__ void get2d(const Params &, float *u0, float *u1) {
        *u0 = rng.uniform();
        *u1 = rng.uniform();
    }
    __device__ __forceinline__ void load(const Params &P, int i) { rng.state = P.ps.smp_state[i]; rng.inc = P.ps.smp_inc[i]; }
    __device__ __forceinline__ void save(const Params &P, int i) { P.ps.smp_state[i] = rng.state; P.ps.smp_inc[i] = rng.inc; }
};
template <int K> struct PathSampler {
    static_assert(K >= 1 && K <= 3, "ZSobol sampler variants");
    static constexpr int kW = K - 1;   // 0 run-time width, 1 32-bit, 2 64-bit
    smp::ZSobol z;
    __device__ __forceinline__ void start(const Params &P, int px, int py, int sampleIndex) {
        z.start(px, py, sampleIndex, P.zs);
    }
    __device__ __forceinline__ float get1d(const Params &P) { return z.template get1d<kW>(P.zs); }
    __device__ __forceinline__ void get2d(const Params &P, float *u0, float *u1) {
        z.template get2d<kW>(P.zs, u0, u1);
    }
    __device__ __forceinline__ void load(const Params &P, int i) {
        const uint64_t st = P.ps.smp_state[i];
        z.morton = (uint32_t)st;
        z.hi = (uint32_t)(st >> 32);
        z.dimension = (uint32_t)P.ps.smp_inc[i];
    }
    __device__ __forceinline__ void save(const Params &P, int i) {
        P.ps.smp_state[i] = ((uint64_t)z.hi << 32) | z.morton;
        P.ps.smp_inc[i] = z.dimension;
    }
};

// The pixel sample of GetCameraSample (samplers.h:797-815) from its 2D draw (fu0, fu1): the
// film's filter (BoxFilter::Sample filters.h:67-70 or GaussianFilter's FilterSampler);
// returns pFilm and the filter weight.
__device__ __forceinline__ void camera_filter(const Params &P, int px, int py, float fu0, float fu1, float *pFilmX,
                                              float *pFilmY, float *weight, const smp::FilterTables *ft) {
    float fpx, fpy;
    *weight = 1.f;
    if (P.film.filter_type == 0) {
        fpx = lerp(fu0, -P.film.filter_rx, P.film.filter_rx);
        fpy = lerp(fu1, -P.film.filter_ry, P.film.filter_ry);
    } else {
        ::avr::smp::gaussian_filter_sample(ft ? *ft : P.film.gauss, fu0, fu1, &fpx, &fpy, weight);
    }
    *pFilmX = ((float)px + fpx) + 0.5f;
    *pFilmY = ((float)py + fpy) + 0.5f;
}
// GetCameraSample after the wavelength draw: pixel 2D through the filter, time (1D) and
// lens (2D).
template <typename Smp>
__device__ __forceinline__ void camera_sample(const Params &P, Smp &smp, int px, int py, float *pFilmX, float *pFilmY,
                                              float *weight, const smp::FilterTables *ft = nullptr) {
    float fu0, fu1;
    smp.get2d(P, &fu0, &fu1);
    camera_filter(P, px, py, fu0, fu1, pFilmX, pFilmY, weight, ft);
    smp.get1d(P);                 // time
    float l0, l1;
    smp.get2d(P, &l0, &l1);       // lens
}

// Cooperative ZSobol draws in k_paths' service rounds. Each lane with `req` needs N draws at
// its dimension + off[j] (a 2D draw where two[j]); the wave's N * popc(req) draws are spread
// over all 64 lanes — busy lanes included, which wait through the handler anyway — so a
// round evaluates the sampler ceil(N * popc / 64) times instead of N times. The lane that
// evaluates draw j of requester rank r writes it to s_res[r * K + slot[j]] (a 2D draw's second
// value after it), so no requester holds N results in VGPRs through the evaluation loop;
// returns the calling lane's rank (its record is s_res + rank * K). Results are bit-identical
// to the sequential get1d / get2d calls (ZSobol::draw_at: a pure function of sample and
// dimension); the requesters' dimension then advances by `adv`. s_st: this wave's 64 LDS entries.
constexpr int kDimHash = 128;   // Hash(d, seed) of the first dimensions, staged in LDS by k_paths (paths deeper than ~15 bounces hash per draw)
template <int kW, int N, int K>
__device__ __forceinline__ int coop_draws_lds(smp::ZSobol &z, const smp::ZSobolParams &zp, bool req, const int (&off)[N],
                                              const bool (&two)[N], const int (&slot)[N], int adv, float *s_res,
                                              uint3 *s_st, const uint64_t *dhash = nullptr, const uint8_t *zpt = nullptr) {
    const uint64_t mask = __ballot(req);
    const int lane = lane_id();
    const int rank = __popcll(mask & ((1ull << lane) - 1ull));
    if (req) s_st[rank] = make_uint3(z.morton, z.hi, z.dimension);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int total = __popcll(mask) * N;
    for (int c = 0; c < total; c += 64) {
        const int t = c + lane;
        if (t < total) {
            const int r = t / N, j = t - r * N;
            int o = off[0], sl = slot[0];
            bool tw = two[0];
            _Pragma("unroll") for (int jj = 1; jj < N; ++jj) {
                o = j == jj ? off[jj] : o;
                sl = j == jj ? slot[jj] : sl;
                tw = j == jj ? two[jj] : tw;
            }
            const uint3 st = s_st[r];
            smp::ZSobol q;
            q.morton = st.x;
            q.hi = st.y;
            q.dimension = 0;
            float v0, v1;
            q.template draw_at<kW>(zp, st.z + (uint32_t)o, tw, &v0, &v1, dhash, dhash ? kDimHash : 0, zpt);
            s_res[r * K + sl] = v0;
            if (tw) s_res[r * K + sl + 1] = v1;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (req) z.dimension += (uint32_t)adv;
    return rank;
}

__device__ __forceinline__ const float *base_of(const smp::FilterTables &t) { return t.f; }
__device__ __forceinline__ float4 to4(V3 v) { return make_float4(v.x, v.y, v.z, 0.f); }
__device__ __forceinline__ V3 from4(float4 v) { return {v.x, v.y, v.z}; }
__device__ __forceinline__ float4 to4(Spec s) { return make_float4(s.v0, s.v1, s.v2, s.v3); }
__device__ __forceinline__ Spec spec4(float4 v) { return {v.x, v.y, v.z, v.w}; }

__device__ __forceinline__ const float *stage_majorant(const DevMedium &m, float *lds) {
    const int n = m.mres[0] * m.mres[1] * m.mres[2];
    if (n > 4096) return m.majorant;
    for (int i = threadIdx.x; i < n; i += blockDim.x) lds[i] = m.majorant[i];
    __syncthreads();
    return lds;
}

// GaussianFilter's FilterSampler tables (pbrt's default radius 1.5: the 48 x 48 CDFs, ~9.6 KB,
// their 6.3 KB of search guides and 9.2 KB of cell weights) staged in LDS when they fit, so the
// camera sample's two guided searches run on LDS. The function table f (another 9.2 KB) stays in
// global memory: with the cell weights it is read only for a cell whose weight entry is NaN.
// 25.6 KB instead of 34.8 lets five camera blocks share a CU's LDS instead of four (with the
// 16384-block grid: camera stage 2.71 -> 2.41 ms, profiles/r06_ab_camera_grid.json). Returns
// (after a block barrier) whether they were staged; filter_lds_tables then describes the copy.
// The descriptor is built in registers from the kernel arguments, not read back from LDS: its
// pointers then stay LDS-typed (ds_read, not flat loads) and the first table read does not wait
// for a descriptor read.
constexpr int kFiltLds = 6400;
__device__ __forceinline__ bool stage_filter(const Params &P, float *s_filt) {
    bool staged = false;
    if (P.film.filter_type != 0) {
        const smp::FilterTables &g = P.film.gauss;
        const int nf = smp::filter_blob_floats(g.nx, g.ny) - g.nx * g.ny;   // the blob after f
        if (g.guide && g.wt && nf <= kFiltLds) {
            const float *base = g.f + g.nx * g.ny;
            for (int i = threadIdx.x; i < nf; i += blockDim.x) s_filt[i] = base[i];
            staged = true;
        }
    }
    __syncthreads();
    return staged;
}
__device__ __forceinline__ smp::FilterTables filter_lds_tables(const smp::FilterTables &g, const float *s_filt) {
    smp::FilterTables t = g;   // (t.f stays g.f, in global memory)
    t.ccdf = s_filt;
    t.cint = t.ccdf + g.ny * (g.nx + 1);
    t.mcdf = t.cint + g.ny;
    const int tabs = smp::filter_table_floats(g.nx, g.ny) - g.nx * g.ny;
    t.guide = reinterpret_cast<const uint8_t *>(s_filt + tabs);
    t.wt = s_filt + tabs + smp::filter_guide_floats(g.ny);
    return t;
}

// ZSobol draws shared by a QUAD of lanes holding samples 4m .. 4m+3 of one pixel (the camera
// stage's layout): their Morton indices differ only in bits 0-1, so every base-4 digit's
// permutation — MixBits of the index bits above the digit and the dimension, one 64-bit
// multiply chain each — is the same for the four lanes. Lane q of the quad computes the
// permutations of lower digits q and q + 4 only and the quad exchanges them by DPP quad_perm
// broadcasts (no LDS); each lane applies them to its own digits. Same index, bit for bit, as
// zsobol_lower (an odd log2(spp)'s base-2 digit depends on bit 1 and stays per lane).
template <int J>
__device__ __forceinline__ uint32_t quad_bcast(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, J * 0x55, 0xf, 0xf, false);
}
template <int J, typename M>
__device__ __forceinline__ void quad_digit(M morton, const uint32_t (&mine)[2], int iLo, int iHi, int pw, uint32_t &idx) {
    const int i = iLo + J;
    const uint32_t p = quad_bcast<J & 3>(mine[J >> 2]);   // every lane of the quad executes it
    if (i <= iHi) {
        const int shift = 2 * i - pw;
        idx |= smp::zperm(p, (uint32_t)(morton >> shift) & 3u) << shift;
    }
}
// digits iLo..iHi (at most 8, log2 spp <= 16) and an odd log2(spp)'s final base-2 digit
template <typename M>
__device__ __forceinline__ uint32_t zsobol_lower_quad(M morton, uint32_t dimension, const smp::ZSobolParams &zp,
                                                      int iLo, int iHi) {
    constexpr int kBits = 8 * (int)sizeof(M);
    const int pw = zp.log2spp & 1;
    const int q = lane_id() & 3;
    const uint32_t dmix = 0x55555555u * dimension;
    uint32_t mine[2] = {0, 0};
    _Pragma("unroll") for (int r = 0; r < 2; ++r) {
        const int i = iLo + q + 4 * r;
        if (i <= iHi) {
            const int shift = 2 * i - pw;
            const M higher = shift + 2 >= kBits ? M(0) : M(morton >> (shift + 2));
            mine[r] = smp::mix_perm24<M>((M)(higher ^ (M)dmix));
        }
    }
    uint32_t idx = 0;
    quad_digit<0>(morton, mine, iLo, iHi, pw, idx);
    quad_digit<1>(morton, mine, iLo, iHi, pw, idx);
    quad_digit<2>(morton, mine, iLo, iHi, pw, idx);
    quad_digit<3>(morton, mine, iLo, iHi, pw, idx);
    if (iHi - iLo >= 4) {
        quad_digit<4>(morton, mine, iLo, iHi, pw, idx);
        quad_digit<5>(morton, mine, iLo, iHi, pw, idx);
        quad_digit<6>(morton, mine, iLo, iHi, pw, idx);
        quad_digit<7>(morton, mine, iLo, iHi, pw, idx);
    }
    if (pw) {   // the final base-2 digit (as zsobol_lower)
        const uint32_t digit = (uint32_t)morton & 1u;
        const M x = (M)(morton >> 1) ^ (M)dmix;
        uint64_t v = (uint64_t)x;
        v ^= v >> 31;
        v *= 0x7fb5d329728ea185ull;
        v ^= v >> 27;
        v *= 0x81dadef4bc2dd44dull;
        v ^= v >> 33;
        idx |= digit ^ (uint32_t)(v & 1);
    }
    return idx;
}
// Two GetSampleIndex values of a quad's samples, at dimensions dA and dB, from their pass-table
// entries, for passes with at most two varying base-4 digits (a 64-index pass: digits 0 and 1):
// lane q of the quad evaluates the MixBits of digit pw + (q & 1) for dA (q < 2) or dB (q >= 2),
// so one round of MixBits serves both draws (zsobol_draw_quad spends a round per draw with two
// of its four lanes busy). Same bits as zsobol_index_pass / zsobol_index.
template <typename M>
__device__ __forceinline__ void zsobol_index_quad_pair(M morton, const smp::ZSobolParams &zp, uint32_t dA, uint64_t eA,
                                                       uint32_t dB, uint64_t eB, M *ia, M *ib,
                                                       const uint8_t *zpt = nullptr) {
    // zpt: the 24 permutations as bytes (4 x 2 bits, smp::zperm's table) staged in LDS — one
    // byte read and a bit-field extract per digit instead of selecting among three 64-bit words
    auto zp_ = [&](uint32_t p, uint32_t digit) -> uint32_t {
        return zpt ? ((uint32_t)zpt[p] >> (2 * digit)) & 3u : smp::zperm(p, digit);
    };
    constexpr int kBits = 8 * (int)sizeof(M);
    const int pw = zp.log2spp & 1, plo = zp.plo;
    const int iTop = (plo + pw - 1) >> 1;   // the perm-fixed digit (when >= pw); digits below it vary
    const int q = lane_id() & 3;
    const int i = pw + (q & 1);
    uint32_t p = 0;
    if (i < iTop) {
        const int shift = 2 * i - pw;
        const M higher = shift + 2 >= kBits ? M(0) : M(morton >> (shift + 2));
        // (the quad's lanes mix digits pw and pw + 1, whose prefixes straddle 2^32 for wide indices:
        // one 64-bit sequence for all instead of both branches of the narrow fast path)
        p = smp::mix_perm24<M, false>((M)(higher ^ (M)(0x55555555u * (q < 2 ? dA : dB))));
    }
    const uint32_t pA0 = quad_bcast<0>(p), pA1 = quad_bcast<1>(p), pB0 = quad_bcast<2>(p), pB1 = quad_bcast<3>(p);
    auto assemble = [&](uint64_t e, uint32_t d, uint32_t p0, uint32_t p1) -> M {
        M idx = (M)((e & smp::pass_prefix_mask(zp)) << plo);
        if (iTop >= pw) {
            const int sh = 2 * iTop - pw;
            idx |= (M)zp_((uint32_t)(e >> 56), (uint32_t)(morton >> sh) & 3u) << sh;
        }
        if (pw < iTop) idx |= (M)zp_(p0, (uint32_t)(morton >> pw) & 3u) << pw;
        if (pw + 1 < iTop) idx |= (M)zp_(p1, (uint32_t)(morton >> (pw + 2)) & 3u) << (pw + 2);
        if (pw) {   // the final base-2 digit (as zsobol_lower)
            const M x = (M)(morton >> 1) ^ (M)(0x55555555u * d);
            uint64_t v = (uint64_t)x;
            v ^= v >> 31;
            v *= 0x7fb5d329728ea185ull;
            v ^= v >> 27;
            v *= 0x81dadef4bc2dd44dull;
            v ^= v >> 33;
            idx |= (M)(((uint32_t)morton & 1u) ^ (uint32_t)(v & 1));
        }
        return idx;
    };
    *ia = assemble(eA, dA, pA0, pA1);
    *ib = assemble(eB, dB, pB0, pB1);
}
// A ZSobol draw from its index (ZSobol::get1d / get2d after GetSampleIndex): `dnext` = the
// dimension after the draw (the FastOwen seed is Hash(dnext, seed))
template <typename M>
__device__ __forceinline__ void zsobol_finish(M idx, uint32_t dnext, const smp::ZSobolParams &zp, bool two, float *u0,
                                              float *u1, const uint64_t *dh) {
    const uint64_t h = (dh && dnext < 16) ? dh[dnext] : smp::hash_2u32(dnext, (uint32_t)zp.seed);
    const uint32_t a = (uint32_t)idx, ah = sizeof(M) == 8 ? (uint32_t)((uint64_t)idx >> 32) : 0u;
    *u0 = smp::u32_to_unit(smp::fast_owen(smp::sobol_bits(a, 0), (uint32_t)h));
    if (two) *u1 = smp::u32_to_unit(smp::fast_owen(smp::sobol_bits64(a, ah, 1), (uint32_t)(h >> 32)));
}
// ZSobol::get1d / get2d with the quad-shared lower digits (kW: 1 32-bit, 2 64-bit index)
constexpr uint32_t kCamDimHash = 16;   // the camera stage's draws end at dimension 10
template <int kW>
// pe: the dimension's pass-table entry when the caller loaded it ahead (pe_ok), else it is read here
__device__ __forceinline__ void zsobol_draw_quad(smp::ZSobol &z, const smp::ZSobolParams &zp, bool two, float *u0,
                                                 float *u1, const uint64_t *dh = nullptr, uint64_t pe = 0,
                                                 bool pe_ok = false) {
    uint32_t a, ah = 0;
    const uint32_t pm = kW == 2 ? (uint32_t)((((uint64_t)z.hi << 32) | z.morton) >> zp.log2spp) : z.morton >> zp.log2spp;
    const int pw = zp.log2spp & 1;
    if (pe_ok || (zp.ptab && (int)z.dimension < zp.pdims)) {
        // the pass table (zsobol_pass_entry): the quad computes the varying digits only (those
        // below the perm-fixed digit iTop, the highest one under the pass's plo bits)
        const uint64_t e = pe_ok ? pe : zp.ptab[(size_t)pm * (size_t)zp.pdims + z.dimension];
        const int iTop = (zp.plo + pw - 1) >> 1;
        const uint32_t perm = (uint32_t)(e >> 56);
        const uint64_t fx = (e & smp::pass_prefix_mask(zp)) << zp.plo;
        if constexpr (kW == 2) {
            const uint64_t m = ((uint64_t)z.hi << 32) | z.morton;
            uint64_t idx = fx | zsobol_lower_quad<uint64_t>(m, z.dimension, zp, pw, iTop - 1);
            if (iTop >= pw) {
                const int sh = 2 * iTop - pw;
                idx |= (uint64_t)smp::zperm(perm, (uint32_t)(m >> sh) & 3u) << sh;
            }
            a = (uint32_t)idx;
            ah = (uint32_t)(idx >> 32);
        } else {
            a = (uint32_t)fx | zsobol_lower_quad<uint32_t>(z.morton, z.dimension, zp, pw, iTop - 1);
            if (iTop >= pw) {
                const int sh = 2 * iTop - pw;
                a |= smp::zperm(perm, (z.morton >> sh) & 3u) << sh;
            }
        }
    } else {
        const uint32_t up = (zp.upper && (int)z.dimension < zp.dmax) ? zp.upper[(size_t)pm * (size_t)zp.dmax + z.dimension]
                                                                       : smp::zsobol_upper(pm, z.dimension, zp);
        const int iHi = smp::zsobol_split(zp) - 1;
        if constexpr (kW == 2) {
            const uint64_t m = ((uint64_t)z.hi << 32) | z.morton;
            const uint64_t idx = ((uint64_t)up << zp.log2spp) | zsobol_lower_quad<uint64_t>(m, z.dimension, zp, pw, iHi);
            a = (uint32_t)idx;
            ah = (uint32_t)(idx >> 32);
        } else {
            a = (up << zp.log2spp) | zsobol_lower_quad<uint32_t>(z.morton, z.dimension, zp, pw, iHi);
        }
    }
    z.dimension += two ? 2 : 1;
    // Hash(dimension, seed): from the caller's staged table when it covers the dimension
    const uint64_t h = (dh && z.dimension < kCamDimHash) ? dh[z.dimension] : smp::hash_2u32(z.dimension, (uint32_t)zp.seed);
    *u0 = smp::u32_to_unit(smp::fast_owen(smp::sobol_bits(a, 0), (uint32_t)h));
    if (two) *u1 = smp::u32_to_unit(smp::fast_owen(smp::sobol_bits64(a, ah, 1), (uint32_t)(h >> 32)));
}

#ifndef AVR_KPATHS_TU
// k_paths' camera stage — everything a path needs before its first medium segment, with one
// lane per (pixel, sample) of the pass: the sampler's camera draws (wavelength 1D at dimension
// 0, pixel 2D at 1, time and lens at 3..5 unused, the first segment's three 1D draws at 6..8:
// RNG(Hash(u0), Hash(u1)) and the first free-flight u, integrators.cpp:984-989), the
// wavelengths and their pdfs (canonical f64 sequences, or the hardware log in fast mode), the
// filter sample (BoxFilter / GaussianFilter's FilterSampler), the camera ray
// (cameras.cpp:284-306, 404-427) and its medium-interface entry. k_paths' refill then loads
// 64 B per new path instead of running this per service round with most lanes idle, and
// k_film reads the wavelengths, pdfs and filter weight instead of re-deriving them.
// kSmp: 0 IndependentSampler, 2 / 3 ZSobolSampler with 32- / 64-bit indices.
// The camera stage's ZSobol draws read Hash(dimension, seed) and its wavelength math the
// canonical tables from LDS. The wavelength pdfs are evaluated by k_film from the wavelengths
// (the same canonical function on the same floats, so the same bits) instead of being carried
// from here: 16 B less written and read per sample, and the four f64 cosh move from this
// VALU-bound stage to the HBM-bound film kernel.
#ifndef AVR_CAM_WAVES
#define AVR_CAM_WAVES 1   // minimum waves per SIMD asked of k_paths_camera (1: the compiler's choice)
#endif
template <int kSmp, bool kFast>
__global__ void __launch_bounds__(256, AVR_CAM_WAVES) k_paths_camera(Params Pk) {
    const Params &P = Pk;
    __shared__ float s_filt[kFiltLds];
    __shared__ double s_canon[canon::kCanonTabDoubles];
    for (int i = threadIdx.x; i < canon::kCanonTabDoubles; i += blockDim.x)   // (fast mode too: k_film's pdfs stay canonical)
        s_canon[i] = i < 128 ? canon::kLogInvC[i] : (i < 256 ? canon::kLogC[i - 128] : canon::kExp2J64[i - 256]);
    __shared__ uint64_t s_cdh[kCamDimHash];
    __shared__ uint8_t s_zpt[24];   // smp::zperm's 24 permutations, one byte each
    if (threadIdx.x < 24) {
        const uint64_t w = threadIdx.x < 8 ? smp::kZPermW0 : (threadIdx.x < 16 ? smp::kZPermW1 : smp::kZPermW2);
        s_zpt[threadIdx.x] = (uint8_t)(w >> ((threadIdx.x & 7) * 8));
    }
    if constexpr (kSmp != 0)
        if (threadIdx.x < kCamDimHash) s_cdh[threadIdx.x] = smp::hash_2u32(threadIdx.x, (uint32_t)P.zs.seed);
    // the pass's per-XCD work counters of k_paths, zeroed here (stream order: after the previous
    // pass's k_paths, before this pass's) instead of by a separate fill
    if (blockIdx.x == 0 && threadIdx.x < 9) P.heads[threadIdx.x] = threadIdx.x < 8 ? 0 : P.pass_gen;
    const bool ftab_lds = stage_filter(P, s_filt);   // (its barrier covers s_canon and s_cdh)
    const int npix = P.pass_pixels;
    const long long n = (long long)npix * P.pass_samples;
    // ZSobol quads (zsobol_draw_quad): lanes 4a .. 4a+3 take samples 4m .. 4m+3 of one pixel
    // when the pass is quad-aligned (sample_base and pass_samples multiples of 4, log2 spp <=
    // 16; the host sets P.cam_quad), so each store still writes 16 consecutive pixels per wave
    const bool quad = kSmp != 0 && P.cam_quad;
    // (n < 2^31: the host bounds a pass by max_paths; 32-bit index arithmetic, FastDiv splits)
    for (uint32_t tu = blockIdx.x * blockDim.x + threadIdx.x; tu < (uint32_t)n; tu += gridDim.x * blockDim.x) {
        // the kernel arguments re-read per sample with scalar loads (fresh_params) instead of
        // living across the loop in SGPRs that spill to VGPR lanes
        const Params &P = fresh_params();
        const int t = (int)tu;
        int slot, s;
        if (quad) {
            const int qd = t >> 2, qs = fdiv(qd, P.div_pixels);
            slot = fmod_(qd, qs, P.div_pixels);
            s = qs * 4 + (t & 3);
        } else {
            s = fdiv(t, P.div_pixels);
            slot = fmod_(t, s, P.div_pixels);
        }
        // the camera stage and k_paths walk the pass in slot order; slot -> pixel by pix_order
        const int id = s * npix + slot;
        const int pix = P.pix_order ? P.pix_order[slot] : slot;
        const int py = fdiv(pix, P.div_width), px = fmod_(pix, py, P.div_width);
        PathSampler<kSmp> smp;
        if constexpr (kSmp == 0) {
            const uint64_t seq = hash_3u32((uint32_t)px, (uint32_t)py, (uint32_t)P.seed);
            smp.rng.set_sequence(seq, mix_bits(seq));
            // == rng.Advance((sample_base + s) * 65536) (rng.h:132-146), precomputed (k_advance)
            smp.rng.state = P.advance[2 * s] * smp.rng.state + smp.rng.inc * P.advance[2 * s + 1];
        } else {
            smp.start(P, px, py, P.sample_base + s);
        }
        // ZSobol with the pass table: the entries of the stage's six draws (dimensions 0, 1 and
        // 6..9) loaded up front by three 16-B loads of the pixel's row, so the draws wait for
        // one memory round trip instead of six in sequence
        [[maybe_unused]] uint64_t pe0 = 0, pe1 = 0, pe6 = 0, pe7 = 0, pe8 = 0, pe9 = 0;
        [[maybe_unused]] bool pe_ok = false;
        if constexpr (kSmp != 0) {
            if (quad && P.zs.ptab && P.zs.pdims >= 10) {
                const uint32_t pmk = PathSampler<kSmp>::kW == 2
                                         ? (uint32_t)((((uint64_t)smp.z.hi << 32) | smp.z.morton) >> P.zs.log2spp)
                                         : smp.z.morton >> P.zs.log2spp;
                // the pixel's compact copy (48 B, pixels consecutive along the wave) when built,
                // else its pass-table row
                const ulonglong2 *row = P.zs.ctab ? reinterpret_cast<const ulonglong2 *>(P.zs.ctab + 6 * (size_t)pix)
                                                  : reinterpret_cast<const ulonglong2 *>(P.zs.ptab + (size_t)pmk * (size_t)P.zs.pdims);
                const ulonglong2 r01 = row[0], r67 = row[P.zs.ctab ? 1 : 3], r89 = row[P.zs.ctab ? 2 : 4];
                pe0 = r01.x; pe1 = r01.y; pe6 = r67.x; pe7 = r67.y; pe8 = r89.x; pe9 = r89.y;
                pe_ok = true;
            }
        }
        // the sampler's draws: a ZSobol quad shares its digit permutations
        // pe: the draw's preloaded pass-table entry (used when pe_ok)
        auto get1 = [&](uint64_t pe) -> float {
            if constexpr (kSmp != 0) {
                if (quad) {
                    float a, b;
                    zsobol_draw_quad<PathSampler<kSmp>::kW>(smp.z, P.zs, false, &a, &b, s_cdh, pe, pe_ok);
                    return a;
                }
            }
            return smp.get1d(P);
        };
        // ZSobol quads whose pass varies at most two base-4 digits: the six draws as three pairs
        // of indices (zsobol_index_quad_pair), each pair one round of MixBits for the quad
        [[maybe_unused]] float pu[7] = {};   // ulam, fu0, fu1, h0, h1, u, ulight
        bool paired = false;
        if constexpr (kSmp != 0) {
            if (pe_ok && ((P.zs.plo + (P.zs.log2spp & 1) - 1) >> 1) - (P.zs.log2spp & 1) <= 2) {
                using M = typename std::conditional<PathSampler<kSmp>::kW == 2, uint64_t, uint32_t>::type;
                const M m = PathSampler<kSmp>::kW == 2 ? (M)(((uint64_t)smp.z.hi << 32) | smp.z.morton) : (M)smp.z.morton;
                const uint64_t *dh = s_cdh;
                M i0, i1, i6, i7, i8, i9;
                zsobol_index_quad_pair<M>(m, P.zs, 0, pe0, 1, pe1, &i0, &i1, s_zpt);
                zsobol_index_quad_pair<M>(m, P.zs, 6, pe6, 7, pe7, &i6, &i7, s_zpt);
                zsobol_index_quad_pair<M>(m, P.zs, 8, pe8, 9, pe9, &i8, &i9, s_zpt);
                float dummy;
                zsobol_finish<M>(i0, 1, P.zs, false, &pu[0], &dummy, dh);
                zsobol_finish<M>(i1, 3, P.zs, true, &pu[1], &pu[2], dh);
                zsobol_finish<M>(i6, 7, P.zs, false, &pu[3], &dummy, dh);
                zsobol_finish<M>(i7, 8, P.zs, false, &pu[4], &dummy, dh);
                zsobol_finish<M>(i8, 9, P.zs, false, &pu[5], &dummy, dh);
                zsobol_finish<M>(i9, 10, P.zs, false, &pu[6], &dummy, dh);
                smp.z.dimension = 10;
                paired = true;
            }
        }
        const float ulam = paired ? pu[0] : get1(pe0);
        const Spec lam = kFast ? film_sample_lambda_fast(P.film, ulam) : film_sample_lambda(P.film, ulam, s_canon);
        float pFilmX, pFilmY, fweight;
        if constexpr (kSmp != 0) {
            float fu0, fu1;
            if (paired) {
                fu0 = pu[1];
                fu1 = pu[2];
            } else if (quad) {
                zsobol_draw_quad<PathSampler<kSmp>::kW>(smp.z, P.zs, true, &fu0, &fu1, s_cdh, pe1, pe_ok);
            } else {
                smp.get2d(P, &fu0, &fu1);
            }
            if (ftab_lds) {
                const smp::FilterTables ft = filter_lds_tables(P.film.gauss, s_filt);
                camera_filter(P, px, py, fu0, fu1, &pFilmX, &pFilmY, &fweight, &ft);
            } else {
                camera_filter(P, px, py, fu0, fu1, &pFilmX, &pFilmY, &fweight, nullptr);
            }
            if (!paired) smp.z.dimension += 3;   // time (1D) and lens (2D): drawn by pbrt, unused by pinholes
        } else {
            if (ftab_lds) {
                const smp::FilterTables ft = filter_lds_tables(P.film.gauss, s_filt);
                camera_sample(P, smp, px, py, &pFilmX, &pFilmY, &fweight, &ft);
            } else {
                camera_sample(P, smp, px, py, &pFilmX, &pFilmY, &fweight, nullptr);
            }
        }
        const float *r = P.cam.raster;
        V3 pCam = {r[0] * pFilmX + r[1] * pFilmY + r[2] * 0.f + r[3], r[4] * pFilmX + r[5] * pFilmY + r[6] * 0.f + r[7],
                   r[8] * pFilmX + r[9] * pFilmY + r[10] * 0.f + r[11]};
        const float wp = r[12] * pFilmX + r[13] * pFilmY + r[14] * 0.f + r[15];
        if (wp != 1) pCam = pCam / wp;
        Ray ray;
        if (P.cam.type == 0) ray = {pCam, {0.f, 0.f, 1.f}};
        else ray = {{0.f, 0.f, 0.f}, normalize(pCam)};
        ray = xf_ray(P.cam.render_from_camera, ray, nullptr, /*forward=*/true);
        const V3 o = P.med.boundary ? interface_entry(P.med, ray.o, ray.d) : ray.o;
        // first medium segment: RNG from two sampler dims, u from a third (984-989)
        const float h0 = paired ? pu[3] : get1(pe6);
        const float h1 = paired ? pu[4] : get1(pe7);
        const float u = paired ? pu[5] : get1(pe8);
        const uint64_t seqA = hash_u32(f2u(h0)), seqB = hash_u32(f2u(h1));
        // ZSobol: the first scatter's light-pick draw (dimension 9) ahead of time (k_paths' NEE
        // handler reads it instead of evaluating the sampler for its lanes)
        const float ulight = kSmp != 0 ? (paired ? pu[6] : get1(pe9)) : 0.f;
        P.ps.cam0[id] = make_float4(o.x, o.y, o.z, u);
        // ZSobol: the first light pick rides in cam1.w (k_paths' refill reads 4 x 16 B, no 4-B gather)
        P.ps.cam1[id] = make_float4(ray.d.x, ray.d.y, ray.d.z, kSmp != 0 ? ulight : fweight);
        P.ps.cam2[id] = to4(lam);
        P.ps.cam3[id] = make_uint4((uint32_t)seqA, (uint32_t)(seqA >> 32), (uint32_t)seqB, (uint32_t)(seqB >> 32));
        P.ps.camw[id] = fweight;
        if constexpr (kSmp == 0)
            P.ps.cam5[id] = make_uint4((uint32_t)smp.rng.state, (uint32_t)(smp.rng.state >> 32), (uint32_t)smp.rng.inc,
                                       (uint32_t)(smp.rng.inc >> 32));
    }
}
#endif

// ---------------------------------------------------------------------------
// Camera rays — RayIntegrator::EvaluatePixelSample (cpu/integrators.cpp:235-268),
// GetCameraSample (samplers.h:797-815), BoxFilter::Sample (filters.h:67-70),
// Orthographic/PerspectiveCamera::GenerateRay (cameras.cpp:284-306, 404-427)
template <bool kZSobol>
__global__ void __launch_bounds__(256) k_camera(Params P) {
    const int n = P.pass_pixels * P.pass_samples;
    for (int id = blockIdx.x * blockDim.x + threadIdx.x; id < n; id += gridDim.x * blockDim.x) {
        const int pix = id % P.pass_pixels, s = id / P.pass_pixels;
        const int px = pix % P.film.width, py = pix / P.film.width;
        const int sampleIndex = P.sample_base + s;
        PathSampler<kZSobol> smp;
        smp.start(P, px, py, sampleIndex);
        const float lu = smp.get1d(P);
        Lambda lam;
        lam.l = film_sample_lambda(P.film, lu);
        lam.pdf = {film_lambda_pdf(P.film, lam.l.v0), film_lambda_pdf(P.film, lam.l.v1),
                   film_lambda_pdf(P.film, lam.l.v2), film_lambda_pdf(P.film, lam.l.v3)};
        float pFilmX, pFilmY, fweight;
        camera_sample(P, smp, px, py, &pFilmX, &pFilmY, &fweight);
        if (P.film.filter_type != 0) P.ps.weight[id] = fweight;
        const float *r = P.cam.raster;
        float xp = r[0] * pFilmX + r[1] * pFilmY + r[2] * 0.f + r[3];
        float yp = r[4] * pFilmX + r[5] * pFilmY + r[6] * 0.f + r[7];
        float zp = r[8] * pFilmX + r[9] * pFilmY + r[10] * 0.f + r[11];
        float wp = r[12] * pFilmX + r[13] * pFilmY + r[14] * 0.f + r[15];
        V3 pCam = {xp, yp, zp};
        if (wp != 1) pCam = pCam / wp;
        Ray ray;
        if (P.cam.type == 0) ray = {pCam, {0.f, 0.f, 1.f}};
        else ray = {{0.f, 0.f, 0.f}, normalize(pCam)};
        ray = xf_ray(P.cam.render_from_camera, ray, nullptr, /*forward=*/true);
        if (P.med.boundary) ray.o = interface_entry(P.med, ray.o, ray.d);
        P.ps.o[id] = to4(ray.o);
        P.ps.d[id] = to4(ray.d);
        P.ps.lambda[id] = to4(lam.l);
        P.ps.pdf[id] = to4(lam.pdf);
        P.ps.beta[id] = make_float4(1.f, 1.f, 1.f, 1.f);
        P.ps.r_u[id] = make_float4(1.f, 1.f, 1.f, 1.f);
        P.ps.r_l[id] = make_float4(1.f, 1.f, 1.f, 1.f);
        P.ps.L[id] = make_float4(0.f, 0.f, 0.f, 0.f);
        smp.save(P, id);
        P.ps.depth[id] = 0;
    }
}

// ---------------------------------------------------------------------------
// Delta tracking — VolPathIntegrator::Li's medium branch (cpu/integrators.cpp:981-1088),
// SampleLd's light pick and shadow-ray spawn (1282-1338), escaped rays (1090-1107).
template <bool kZSobol>
__global__ void __launch_bounds__(256) k_medium(Params P) {
    __shared__ float s_maj[4096];
    const float *maj = stage_majorant(P.med, s_maj);
    const int count = *P.count_in;
    unsigned long long nLookup = 0, nIn = 0, nOut = 0, nSteps = 0;
    const int stride = gridDim.x * blockDim.x;
    // Every lane of a wave runs the same number of outer iterations so the wave-wide
    // queue pushes below see all 64 lanes.
    const int nIter = (count + stride - 1) / stride;
    for (int it = 0; it < nIter; ++it) {
        const int i = it * stride + blockIdx.x * blockDim.x + threadIdx.x;
        const bool valid = i < count;
        bool pushActive = false, pushShadow = false;
        int path = 0;
        V3 newO{}, newD{};
        float4 shO{}, shD{}, shBF{}, shLs{}, shRP{};
        float2 shPdfs{};
        if (valid) {
            ++nIn;
            path = P.queue_in ? P.queue_in[i] : i;
            const V3 o = from4(P.ps.o[path]);
            const V3 d = from4(P.ps.d[path]);
            const Spec lamv = spec4(P.ps.lambda[path]);
            Spec beta = spec4(P.ps.beta[path]), r_u = spec4(P.ps.r_u[path]), r_l = spec4(P.ps.r_l[path]);
            Spec L = spec4(P.ps.L[path]);
            PathSampler<kZSobol> smp;
            smp.load(P, path);
            int depth = P.ps.depth[path];
            const LambdaIdx li = lambda_index(lamv);
            const Spec sig_a = sample_table(P.med.sigma_a, li);
            const Spec sig_s = sample_table(P.med.sigma_s, li);
            const Spec Le_l = P.med.emissive ? sample_table(P.med.Le, li) : Spec::c(0.f);
            const int maxDepth = P.max_depth;
            bool scattered = false, terminated = false;
            const float h0 = smp.get1d(P);
            const float h1 = smp.get1d(P);
            Pcg32 rng;
            rng.set_sequence(hash_u32(f2u(h0)), hash_u32(f2u(h1)));
            const float u0 = smp.get1d(P);
            V3 pScatter{};
            auto cb = [&](V3 p, const MediumSample &ms, const Spec &sigma_maj, const Spec &T_maj) -> bool {
                if (!beta.nonzero()) { terminated = true; return false; }
                if (depth < maxDepth && ms.Le.nonzero()) {
                    float pdf = sigma_maj.v0 * T_maj.v0;
                    Spec betap = beta * T_maj / pdf;
                    Spec r_e = r_u * sigma_maj * T_maj / pdf;
                    if (r_e.nonzero()) L = L + betap * ms.sigma_a * ms.Le / r_e.avg();
                }
                float pAbsorb = ms.sigma_a.v0 / sigma_maj.v0;
                float pScat = ms.sigma_s.v0 / sigma_maj.v0;
                float pNull = fmaxf_(0.f, 1 - pAbsorb - pScat);
                float um = rng.uniform();
                int mode = sample_discrete3(pAbsorb, pScat, pNull, um);
                if (mode == 0) { terminated = true; return false; }
                if (mode == 1) {
                    if (depth++ >= maxDepth) { terminated = true; return false; }
                    float pdf = T_maj.v0 * ms.sigma_s.v0;
                    beta = beta * (T_maj * ms.sigma_s / pdf);
                    r_u = r_u * (T_maj * ms.sigma_s / pdf);
                    if (beta.nonzero() && r_u.nonzero()) {
                        scattered = true;   // resolved below (NEE + phase sampling)
                        pScatter = p;
                    }
                    return false;
                }
                Spec sigma_n = clamp_zero(sigma_maj - ms.sigma_a - ms.sigma_s);
                float pdf = T_maj.v0 * sigma_n.v0;
                beta = beta * (T_maj * sigma_n / pdf);
                if (pdf == 0) beta = Spec::c(0.f);
                r_u = r_u * (T_maj * sigma_n / pdf);
                r_l = r_l * (T_maj * sigma_maj / pdf);
                return beta.nonzero() && r_u.nonzero();
            };
            const float tMax = P.med.boundary ? interface_exit(P.med, o, d) : kInf;
            Spec T_maj = sample_t_maj(P.med, maj, Ray{o, d}, tMax, u0, rng, sig_a, sig_s, Le_l, lamv, nLookup, nSteps, cb);

            if (scattered) {
                // ---- SampleLd for the medium interaction (integrators.cpp:1282-1338) ----
                const V3 wo = -d;
                const float ul = smp.get1d(P);
                float uL0, uL1;
                smp.get2d(P, &uL0, &uL1);   // uLight (unused by distant lights)
                bool shadowSpawned = false;
                const int nl = P.lights.n;
                if (nl > 0) {
                    float pmf = 0.f;
                    const int idx = light_pick<true>(P.lights, ul, &pmf);
                    if (idx >= 0) {
                        const DevLight &lt = P.lights.list[idx];
                        if (lt.type == 0 || lt.type == 2) {
                            V3 wi = {lt.w[0], lt.w[1], lt.w[2]};
                            Spec Ls;
                            float lsPdf = 1.f;
                            if (lt.type == 0) {
                                Ls = sample_table(lt.L, li) * lt.scale;
                            } else {   // ImageInfiniteLight::SampleLi, compensated distribution (lights.h:588-613)
                                float su, sv;
                                env::distrib_sample(lt.dist, uL0, uL1, &su, &sv, &lsPdf);
                                if (lsPdf != 0) {
                                    V3 wl;
                                    env::square_to_sphere(su, sv, &wl.x, &wl.y, &wl.z);
                                    wi = xf_vec3(lt.rfl, wl);
                                    lsPdf = lsPdf / (4 * kPi);
                                    Ls = image_le(lt, su, sv, lamv);
                                } else {
                                    Ls = Spec::c(0.f);
                                }
                            }
                            if (Ls.nonzero() && lsPdf != 0) {
                                const V3 pOut = pScatter + wi * (2 * P.lights.scene_radius);
                                const float p_l = pmf * lsPdf;
                                const float fval = hg_eval(dot(wo, wi), P.med.g);
                                const Spec f_hat = Spec::c(fval);
                                if (f_hat.nonzero()) {
                                    shO = to4(pScatter);
                                    shD = to4(pOut - pScatter);
                                    shBF = to4(beta * f_hat);
                                    shLs = to4(Ls);
                                    shRP = to4(r_u);
                                    shPdfs = make_float2(p_l, lt.type == 0 ? -1.f : fval);
                                    shadowSpawned = true;
                                }
                            }
                        }
                    }
                }
                if (!shadowSpawned) L = L + Spec::c(0.f);   // L += SampleLd(...) == 0
                pushShadow = shadowSpawned;
                // ---- phase-function sampling (integrators.cpp:1046-1061) ----
                float up0, up1;
                smp.get2d(P, &up0, &up1);
                float phPdf;
                const V3 wi = hg_sample(wo, P.med.g, up0, up1, &phPdf);
                if (phPdf == 0) {
                    terminated = true;
                } else {
                    beta = beta * (phPdf / phPdf);
                    r_l = r_u / phPdf;
                    newO = pScatter;
                    newD = wi;
                    pushActive = true;
                }
            } else if (!terminated && beta.nonzero() && r_u.nonzero()) {
                beta = beta * (T_maj / T_maj.v0);
                r_u = r_u * (T_maj / T_maj.v0);
                r_l = r_l * (T_maj / T_maj.v0);
                // escaped: infinite lights (integrators.cpp:1090-1107)
                for (int k = 0; k < P.lights.n; ++k) {
                    const DevLight &lt = P.lights.list[k];
                    if (lt.type == 0) continue;
                    float eu = 0, ev = 0;
                    const Spec Le = lt.type == 1 ? sample_table(lt.L, li) * lt.scale : image_le_dir(lt, d, lamv, &eu, &ev);
                    if (!Le.nonzero()) continue;
                    if (depth == 0) L = L + beta * Le / r_u.avg();
                    else {
                        // lightSampler.PMF * PDF_Li(prevIntrContext, ray.d, true): 0 for the uniform light
                        float p_l = light_pmf<true>(P.lights, k) * (lt.type == 1 ? 0.f : image_pdf_li(lt, d));
                        r_l = r_l * p_l;
                        L = L + beta * Le / (r_u + r_l).avg();
                    }
                }
            }
            P.ps.L[path] = to4(L);
            if (pushActive) {
                P.ps.o[path] = to4(newO);
                P.ps.d[path] = to4(newD);
                P.ps.beta[path] = to4(beta);
                P.ps.r_u[path] = to4(r_u);
                P.ps.r_l[path] = to4(r_l);
                smp.save(P, path);
                P.ps.depth[path] = depth;
            }
        }
        const int slot = wave_push(P.count_out, pushActive);
        if (pushActive) { P.queue_out[slot] = path; ++nOut; }
        const int sslot = wave_push(P.shadow_count, pushShadow);
        if (pushShadow) {
            ++nOut;
            P.sh.path[sslot] = path;
            P.sh.o[sslot] = shO;
            P.sh.d[sslot] = shD;
            P.sh.bf[sslot] = shBF;
            P.sh.Ls[sslot] = shLs;
            P.sh.rp[sslot] = shRP;
            P.sh.pdfs[sslot] = shPdfs;
        }
    }
    flush_stat(P.stats, 0, nLookup);
    flush_stat(P.stats, 1, nIn);
    flush_stat(P.stats, 2, nOut);
    flush_stat(P.stats, 5, nSteps);
}

// ---------------------------------------------------------------------------
// Ratio tracking along shadow rays — SampleLd's transmittance loop
// (cpu/integrators.cpp:1339-1398), incl. Russian roulette at Tr < 0.05, q = 0.75.
#ifndef AVR_KPATHS_TU
__global__ void __launch_bounds__(256) k_shadow(Params P) {
    __shared__ float s_maj[4096];
    const float *maj = stage_majorant(P.med, s_maj);
    const int count = *P.shadow_count;
    unsigned long long nLookup = 0, nIn = 0, nSteps = 0;
    for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < count; k += gridDim.x * blockDim.x) {
        ++nIn;
        const int i = P.sh_perm ? P.sh_perm[k] : k;   // binned order (avr_set_ray_binning)
        const int path = P.sh.path[i];
        const V3 o = from4(P.sh.o[i]);
        const V3 d = from4(P.sh.d[i]);
        const Spec lamv = spec4(P.ps.lambda[path]);
        const LambdaIdx li = lambda_index(lamv);
        const Spec sig_a = sample_table(P.med.sigma_a, li);
        const Spec sig_s = sample_table(P.med.sigma_s, li);
        const Spec Le_l = P.med.emissive ? sample_table(P.med.Le, li) : Spec::c(0.f);
        Spec T_ray = Spec::c(1.f), r_l = Spec::c(1.f), r_u = Spec::c(1.f);
        Pcg32 rng;
        rng.set_sequence(hash_3u32(f2u(o.x), f2u(o.y), f2u(o.z)), hash_3u32(f2u(d.x), f2u(d.y), f2u(d.z)));
        const float u = rng.uniform();
        auto cb = [&](V3, const MediumSample &ms, const Spec &sigma_maj, const Spec &T_maj) -> bool {
            Spec sigma_n = clamp_zero(sigma_maj - ms.sigma_a - ms.sigma_s);
            float pdf = T_maj.v0 * sigma_maj.v0;
            T_ray = T_ray * (T_maj * sigma_n / pdf);
            r_l = r_l * (T_maj * sigma_maj / pdf);
            r_u = r_u * (T_maj * sigma_n / pdf);
            Spec Tr = T_ray / (r_l + r_u).avg();
            if (Tr.maxc() < 0.05f) {
                float q = 0.75f;
                if (rng.uniform() < q) T_ray = Spec::c(0.f);
                else T_ray = T_ray / (1 - q);
            }
            return T_ray.nonzero();
        };
        const float tMax = P.med.boundary ? fminf_(1 - kShadowEpsilon, interface_exit(P.med, o, d)) : 1 - kShadowEpsilon;
        Spec T_maj = sample_t_maj(P.med, maj, Ray{o, d}, tMax, u, rng, sig_a, sig_s, Le_l, lamv,
                                  nLookup, nSteps, cb);
        T_ray = T_ray * (T_maj / T_maj.v0);
        r_l = r_l * (T_maj / T_maj.v0);
        r_u = r_u * (T_maj / T_maj.v0);
        Spec contrib = Spec::c(0.f);
        if (T_ray.nonzero()) {
            // r_l *= r_p * p_l; r_u *= r_p * scatterPDF (integrators.cpp:1391-1398)
            const Spec rp = spec4(P.sh.rp[i]);
            const float2 pd = P.sh.pdfs[i];
            r_l = r_l * (rp * pd.x);
            if (pd.y < 0) {
                contrib = spec4(P.sh.bf[i]) * T_ray * spec4(P.sh.Ls[i]) / r_l.avg();
            } else {
                r_u = r_u * (rp * pd.y);
                contrib = spec4(P.sh.bf[i]) * T_ray * spec4(P.sh.Ls[i]) / (r_l + r_u).avg();
            }
        }
        P.ps.L[path] = to4(spec4(P.ps.L[path]) + contrib);
    }
    flush_stat(P.stats, 3, nLookup);
    flush_stat(P.stats, 4, nIn);
    flush_stat(P.stats, 6, nSteps);
}
#endif

// ---------------------------------------------------------------------------
// k_paths — persistent-wave megakernel (the default path).
//
// The same VolPath estimator as k_camera + k_medium + k_shadow, restructured for CDNA4:
// every lane keeps its whole path state in VGPRs and runs a flat state machine
// {fetch, medium segment, shadow segment}; one loop iteration advances each lane to its
// next tentative collision (majorant DDA in LDS), does the density fetch for all lanes
// that reached one together, and applies that lane's event. Lanes whose path ended are
// refilled from the pass's sample range with one atomic per wave (__ballot/__popcll/
// mbcnt prefix) on per-XCD work counters, so waves stay full until the pass drains and no
// per-bounce state goes through HBM. Per-sample L and lambda are written at path end and
// k_film adds them to the film in sampleIndex order (deterministic, as before).
// Float operation order per path is identical to the wavefront kernels and to the CPU
// oracle (cpu/integrators.cpp:962-1399, media.h:741-806).
enum : int { M_FETCH = 0, M_MEDIUM = 1, M_SHADOW = 2, M_DONE = 3 };

__device__ __forceinline__ int xcc_id() {
    unsigned v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
    return (int)(v & 7);
}

// Start SampleT_maj (media.h:744-749): normalise, transform to medium space, clip, DDA.
__device__ __forceinline__ void seg_begin(const DevMedium &m, V3 o, V3 d, float tMax, V3 &sd, Dda &it,
                                          Spec &T_maj, bool &needNext) {
    tMax *= length(d);
    d = normalize(d);
    sd = d;
    dda_init(it, m, Ray{o, d}, tMax);
    T_maj = Spec::c(1.f);
    needNext = true;
}

// k_paths' DDA: DDAMajorantIterator (media.h:141-214) restated for the persistent kernel.
// Same segments, bit for bit; the state is laid out for a branch-free step:
//   voxel (x,y,z)           -> one linear index into the LDS majorant (x-fastest, media.h:112-115)
//   step[] / voxelLimit[]   -> the sign bit of deltaT[] and a packed count of the cells left
//                              before the exit face (8 bits per axis; majorant res <= 255)
struct DdaL {
    float tMin, tMax;
    float nx, ny, nz;      // nextCrossingT
    float dx, dy, dz;      // deltaT, negated when the step along that axis is -1
    int vidx;              // x + rx * (y + ry * z)
    int rem;               // cells left: x bits 0-7, y 8-15, z 16-23
    int pidx;              // cell whose majorant mcur holds (vidx, clamped into the grid)
    float mcur;            // majorant of cell pidx, loaded one step ahead (software pipelining):
                           // the caller reloads it (ddal_prefetch) unconditionally every iteration
};
__device__ __forceinline__ void ddal_init(DdaL &q, const DevMedium &m, Ray ray, float raytMax, const float *maj) {
    Dda it;
    if (!dda_init(it, m, ray, raytMax)) {
        q.tMin = kInf; q.tMax = -kInf;
        q.nx = q.ny = q.nz = q.dx = q.dy = q.dz = 0; q.vidx = 0; q.rem = 0; q.pidx = 0; q.mcur = 0;
        return;
    }
    q.tMin = it.tMin; q.tMax = it.tMax;
    q.nx = it.nx; q.ny = it.ny; q.nz = it.nz;
    q.dx = it.sx > 0 ? it.dx : -it.dx;
    q.dy = it.sy > 0 ? it.dy : -it.dy;
    q.dz = it.sz > 0 ? it.dz : -it.dz;
    q.vidx = it.vx + m.mres[0] * (it.vy + m.mres[1] * it.vz);
    const int cx = it.sx > 0 ? m.mres[0] - 1 - it.vx : it.vx;
    const int cy = it.sy > 0 ? m.mres[1] - 1 - it.vy : it.vy;
    const int cz = it.sz > 0 ? m.mres[2] - 1 - it.vz : it.vz;
    q.rem = cx | (cy << 8) | (cz << 16);
    q.pidx = q.vidx;
    q.mcur = maj[q.vidx];
}
// Reload mcur from pidx: one load per loop iteration into the loop-carried register, so the
// wait for it lands at the next ddal_next (a load inside ddal_next's predicated block is
// followed by a phi copy that waits right away).
__device__ __forceinline__ void ddal_prefetch(DdaL &q, const float *maj) { q.mcur = maj[q.pidx]; }
// The global (NanoVDB) majorant through a buffer resource over its ncells + 1 floats: the
// hardware bounds check returns 0 for an index past either end, so the walk's one-step-ahead
// prefetch needs no clamp (the value past the last cell is never used: the next Next() ends)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t maj_rsrc(const float *maj, int ncells) {
    return __builtin_amdgcn_make_buffer_rsrc((void *)maj, (short)0, (ncells + 1) * 4, 0x00020000);
}
__device__ __forceinline__ float maj_load(__amdgpu_buffer_rsrc_t r, int idx) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, idx * 4, 0, 0));
}
__device__ __forceinline__ void ddal_prefetch_buf(DdaL &q, __amdgpu_buffer_rsrc_t r) { q.mcur = maj_load(r, q.pidx); }
// With the coarse occupancy level in LDS: a cell whose pair bit is clear has majorant 0, and
// its lane reads the trailing zero cell maj[ncells] instead (one cached line shared by every
// such lane) — the L2 read of the 1 MiB grid is left to the occupied cells. Same value either way.
__device__ __forceinline__ void ddal_prefetch_occ_buf(DdaL &q, __amdgpu_buffer_rsrc_t r, const unsigned *occ, int ncells) {
    const int p = q.pidx;
    const unsigned w = occ[p >> 6];   // (LDS: an out-of-range index cannot fault; the bit is then moot)
    q.mcur = maj_load(r, ((w >> ((p >> 1) & 31)) & 1u) ? p : ncells);
}
// Next(): false when exhausted. `maj` is the LDS copy; sy/sz the linear strides of y and z.
// The next cell's index (pidx) is left unclamped: the caller's prefetch reads LDS, where an
// out-of-range index cannot fault, or a bounds-checked buffer (maj_load)
__device__ __forceinline__ bool ddal_next(DdaL &q, const float *maj, int sy, int sz, float *s0, float *s1,
                                          float *mval) {
    // fields are copied to values first: a select between struct members invites the
    // compiler to turn the struct into a scratch array indexed by the axis
    const float tMin = q.tMin, tMax = q.tMax, nx = q.nx, ny = q.ny, nz = q.nz;
    const float dx = q.dx, dy = q.dy, dz = q.dz;
    const int rem = q.rem, vidx = q.vidx;
    if (tMin >= tMax) return false;
    // cmpToAxis = {2, 1, 2, 1, 2, 2, 0, 0} over bits (nx<ny, nx<nz, ny<nz)
    const bool xy = nx < ny, xz = nx < nz, yz = ny < nz;
    const bool ax0 = xy && xz, ax1 = !xy && yz;
    const float nextA = ax0 ? nx : (ax1 ? ny : nz);
    const float dA = ax0 ? dx : (ax1 ? dy : dz);
    const int shift = ax0 ? 0 : (ax1 ? 8 : 16);
    const int stride = ax0 ? 1 : (ax1 ? sy : sz);
    *mval = q.mcur;
    *s0 = tMin;
    // tVoxelExit = std::min(tMax, next) — (next < tMax) ? next : tMax, so a NaN crossing gives
    // tMax as in pbrt; and with it pbrt's "next > tMax -> tMin = tMax" is already tExit
    const float tExit = nextA < tMax ? nextA : tMax;
    *s1 = tExit;
    const bool last = ((rem >> shift) & 0xff) == 0;   // voxel + step == voxelLimit
    q.tMin = last ? tMax : tExit;
    q.rem = rem - (1 << shift);
    // step +-1 along the axis: the sign of deltaT as +-1 times the axis' linear stride
    const int nv = vidx + __mul24(stride, (__float_as_int(dA) >> 31) | 1);
    q.vidx = nv;
    // the next cell's majorant is loaded by ddal_prefetch so its latency (L2 for NanoVDB's
    // 64^3 grid) hides behind this step's work; past the last cell the index is left as it is
    // (its value is never used: the next call returns false)
    q.pidx = nv;
    const float nn = nextA + __builtin_fabsf(dA);
    q.nx = ax0 ? nn : nx;
    q.ny = ax1 ? nn : ny;
    q.nz = (ax0 || ax1) ? nz : nn;
    return true;
}

// PCG32 Advance(s * 65536) of sample index s (IndependentSampler::StartPixelSample,
// samplers.h:457-460; rng.h:132-146) as an affine map state' = A * state + inc * H: every
// step of the log-time loop is linear in inc, so H is the loop's accPlus run with inc = 1.
// One entry per sample index of a pass; k_paths applies it to each pixel's stream.
#ifndef AVR_KPATHS_TU
__global__ void k_advance(uint64_t *adv, long long base, int S) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= S) return;
    uint64_t delta = (uint64_t)(base + s) * 65536ull;
    uint64_t curMult = 0x5851f42d4c957f2dULL, curPlus = 1, accMult = 1, accPlus = 0;
    while (delta > 0) {
        if (delta & 1) {
            accMult *= curMult;
            accPlus = accPlus * curMult + curPlus;
        }
        curPlus = (curMult + 1) * curPlus;
        curMult *= curMult;
        delta /= 2;
    }
    adv[2 * s] = accMult;
    adv[2 * s + 1] = accPlus;
}
#endif

// ---------------------------------------------------------------------------
// Ray binning for the wavefront organisation (north star: "density-grid fetches coalesced
// along sorted ray packets"): before a k_medium / k_shadow launch the
// queue is counting-sorted by key = (majorant cell of the ray origin, direction octant), so
// the 64 lanes of a wave start in the same majorant cell heading the same way and their
// trilinear gathers share cache lines. Order only: every path's result is unchanged.
#ifndef AVR_KPATHS_TU
__device__ __forceinline__ int ray_bin(const DevMedium &m, V3 o, V3 d) {
    const V3 pm = xf_point_lr(m.medium_from_render, o);
    int c[3];
    const float pv[3] = {pm.x, pm.y, pm.z};
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float u = (pv[a] - m.bmin[a]) / (m.bmax[a] - m.bmin[a]);
        int k = (int)(u * (float)m.mres[a]);
        c[a] = k < 0 ? 0 : (k >= m.mres[a] ? m.mres[a] - 1 : k);
    }
    const int oct = (d.x < 0 ? 1 : 0) | (d.y < 0 ? 2 : 0) | (d.z < 0 ? 4 : 0);
    return ((c[2] * m.mres[1] + c[1]) * m.mres[0] + c[0]) * 8 + oct;
}
// pass 1: key per item (queue entry or identity) and the bin histogram
__global__ void __launch_bounds__(256) k_bin_count(DevMedium m, const int *__restrict__ queue, const int *count_p,
                                                   const float4 *__restrict__ o, const float4 *__restrict__ d,
                                                   int *__restrict__ keys, int *__restrict__ hist) {
    const int count = *count_p;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < count; i += gridDim.x * blockDim.x) {
        const int j = queue ? queue[i] : i;
        const int k = ray_bin(m, from4(o[j]), from4(d[j]));
        keys[i] = k;
        atomicAdd(hist + k, 1);
    }
}
// pass 2: exclusive scan of the histogram in place (one workgroup; nbins <= 8 * 4096)
__global__ void __launch_bounds__(1024) k_bin_scan(int *hist, int nbins) {
    __shared__ int s_part[1024];
    const int per = (nbins + 1023) / 1024;
    const int lo = threadIdx.x * per, hi = lo + per < nbins ? lo + per : nbins;
    int sum = 0;
    for (int i = lo; i < hi; ++i) sum += hist[i];
    s_part[threadIdx.x] = sum;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {   // Hillis-Steele inclusive scan of the parts
        const int v = threadIdx.x >= off ? s_part[threadIdx.x - off] : 0;
        __syncthreads();
        s_part[threadIdx.x] += v;
        __syncthreads();
    }
    int run = s_part[threadIdx.x] - sum;
    for (int i = lo; i < hi; ++i) {
        const int h = hist[i];
        hist[i] = run;
        run += h;
    }
}
// pass 3: scatter the items (queue entries or indices) to their bins
__global__ void __launch_bounds__(256) k_bin_scatter(const int *__restrict__ queue, const int *count_p,
                                                     const int *__restrict__ keys, int *__restrict__ offs,
                                                     int *__restrict__ out) {
    const int count = *count_p;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < count; i += gridDim.x * blockDim.x)
        out[atomicAdd(offs + keys[i], 1)] = queue ? queue[i] : i;
}
#endif

#ifndef AVR_PATHS_WAVES_GRAY
#define AVR_PATHS_WAVES_GRAY 4   // <= 128 VGPRs: with the k_paths units' -disable-machine-licm and the host-computed constants, 126 (ZSobol-64 GridMedium) / 127 (NanoVDB) and no scratch (tools/kres.py on the -Rpass-analysis log)
#endif
#ifndef AVR_PATHS_WAVES_SPEC
#define AVR_PATHS_WAVES_SPEC 2   // 4-wavelength state: ~220 VGPRs without scratch
#endif
// Lane events, deferred and handled in batches: a lane that reaches an event parks until
// enough lanes of its wave need service, so each event handler runs once per batch
// instead of once per tracking iteration (SQ_INSTS_VALU showed the per-iteration union
// of all branches, ~8k wave-instructions, dominating an eager state machine).
// (Phase requests and NEE spawns pooled across the block's four waves through LDS were measured
// 4-18 % slower and removed: DESIGN §6, profiles/r05_ab_pooled_handlers.json.)
enum : int { EV_NONE = 0, EV_SCATTER = 1, EV_SHADOW_DONE = 2, EV_PHASE = 3, EV_ESCAPE = 4, EV_END = 5 };


// Spectral-state type of k_paths: Spec (4 wavelengths) in general; float for a GRAY medium
// (sigma_a and sigma_s tables constant over 360..830 nm, decided on the host). In a gray
// medium beta, r_u, r_l, T_maj and the shadow ratios have four equal components at every
// step (they start at 1 and only ever multiply/divide by gray factors), so one scalar op
// yields exactly the bits each component would get: the overloads below restate Spec's
// operations on one component (Spec::avg of four equal values is (((x+x)+x)+x)/4, NOT x).
__device__ __forceinline__ float sv0(float x) { return x; }
// x / x as IEEE division computes it: exactly 1 for a finite nonzero x, NaN for 0, inf or NaN.
// pbrt's ratios T_maj / T_maj[0] and T_maj * sigma / (T_maj[0] * sigma[0]) are such quotients in
// a gray medium (the same float products on both sides); the division itself runs only when a
// lane of the wave has a special x, so the result (NaN bits included) is the division's.
__device__ __forceinline__ float unit_quot(float x) {
    const bool plain = __builtin_isfinite(x) && x != 0.f;
    if (__ballot(!plain) == 0) return 1.f;
    return plain ? 1.f : x / x;
}
__device__ __forceinline__ float sv0(const Spec &x) { return x.v0; }
__device__ __forceinline__ bool snz(float x) { return x != 0; }
__device__ __forceinline__ bool snz(const Spec &x) { return x.nonzero(); }
__device__ __forceinline__ float savg(float x) { return (((x + x) + x) + x) / 4; }
__device__ __forceinline__ float savg(const Spec &x) { return x.avg(); }
__device__ __forceinline__ float smaxc(float x) { return x; }
__device__ __forceinline__ float smaxc(const Spec &x) { return x.maxc(); }
__device__ __forceinline__ float sclamp0(float x) { return fmaxf_(0.f, x); }
__device__ __forceinline__ Spec sclamp0(const Spec &x) { return clamp_zero(x); }
__device__ __forceinline__ float sexp(float x) { return fast_exp(x); }
__device__ __forceinline__ Spec sexp(const Spec &x) { return fast_exp(x); }
// FastExp (replay) or the hardware exp (fast mode)
template <bool kFast> __device__ __forceinline__ float sexpm(float x) { return kFast ? hw_exp(x) : fast_exp(x); }
template <bool kFast> __device__ __forceinline__ Spec sexpm(const Spec &x) {
    return kFast ? Spec{hw_exp(x.v0), hw_exp(x.v1), hw_exp(x.v2), hw_exp(x.v3)} : fast_exp(x);
}
template <typename S> __device__ __forceinline__ S sconst(float a);
template <> __device__ __forceinline__ float sconst<float>(float a) { return a; }
template <> __device__ __forceinline__ Spec sconst<Spec>(float a) { return Spec::c(a); }
__device__ __forceinline__ Spec to_spec(float x) { return Spec::c(x); }
__device__ __forceinline__ Spec to_spec(const Spec &x) { return x; }
template <typename S> __device__ __forceinline__ S sfrom(const Spec &x);
template <> __device__ __forceinline__ float sfrom<float>(const Spec &x) { return x.v0; }
template <> __device__ __forceinline__ Spec sfrom<Spec>(const Spec &x) { return x; }
// spectrum (light / emission) times path state: component-wise products commute exactly
__device__ __forceinline__ Spec smul(const Spec &a, float b) { return a * b; }
__device__ __forceinline__ Spec smul(const Spec &a, const Spec &b) { return a * b; }

// Section profiling (variant builds with -DAVR_PROFILE_SECTIONS only; tools/section_profile.py):
// per wave, s_memtime cycles spent in {event handlers, refill, segment starts, DDA walk,
// collision (exact candidate, fetch, callback)} summed into the context's section counters.
#ifdef AVR_PROFILE_SECTIONS
// the cycles land in stats[kNumStats .. kNumStats + 4] (the context allocates kNumStats + 8
// counters): one buffer shared by every k_paths translation unit, unlike a __device__ global
// (each separately compiled unit would hold its own copy)
struct SecProf {
    // 0 NEE spawn, 1 refill, 2 segment starts, 3 DDA walk, 4 collision, 5 shadow done,
    // 6 phase sampling, 7 escape + path end
    unsigned long long acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long last = 0;
    int cur = 0;
    __device__ __forceinline__ void mark(int next) {
        const unsigned long long t = clock64();
        const unsigned long long d = t - last;
        if (cur == 0) acc[0] += d; else if (cur == 1) acc[1] += d; else if (cur == 2) acc[2] += d;
        else if (cur == 3) acc[3] += d; else if (cur == 4) acc[4] += d; else if (cur == 5) acc[5] += d;
        else if (cur == 6) acc[6] += d; else acc[7] += d;
        last = t;
        cur = next;
    }
    __device__ __forceinline__ void flush(unsigned long long *stats) {
        mark(0);
        if (lane_id() == 0)
            for (int i = 0; i < 8; ++i) atomicAdd(&stats[kNumStats + i], acc[i]);
    }
};
#define AVR_SEC_INIT SecProf secp; secp.last = clock64();
#define AVR_SEC(i) secp.mark(i);
#define AVR_SEC_FLUSH secp.flush(P.stats);
#else
#define AVR_SEC_INIT
#define AVR_SEC(i)
#define AVR_SEC_FLUSH
#endif

// Walk / gather probes (variant builds with -DAVR_PROBE_STATS only; tools/probe_stats.py): wave
// counters of the DDA walk's lane occupancy and of how many distinct cache lines the lanes of one
// collision round gather from (the coalescing an in-wave sort of the lookups could exploit, N1),
// summed into stats[kNumStats + 0..7] like the section profile. Results unchanged.
#ifdef AVR_PROBE_STATS
struct ProbeStats {
    // 0 walk trips, 1 walking lanes summed over trips, 2 collision rounds, 3 collision lanes,
    // 4 distinct 128-B lines, 5 distinct 64-B lines (fat entries), 6 zero-majorant lane steps,
    // 7 walks ended by the DDA budget with lanes still walking. Per wave in LDS: the first
    // active lane adds (values are wave-uniform; inactive lanes of a divergent region skip it)
    unsigned long long *c;
    __device__ __forceinline__ void add(int k, unsigned long long v) {
        const uint64_t am = __ballot(1);
        if (lane_id() == __ffsll((long long)am) - 1) atomicAdd(c + k, v);
    }
    // distinct keys among the active lanes (wave-uniform result)
    __device__ __forceinline__ static unsigned distinct(long long key) {
        uint64_t rem = __ballot(1);
        unsigned n = 0;
        while (rem) {
            const int l = __ffsll((long long)rem) - 1;
            const long long k0 = __shfl(key, l);
            rem &= ~__ballot(key == k0);
            ++n;
        }
        return n;
    }
    __device__ __forceinline__ void flush(unsigned long long *stats) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (lane_id() < 8 && c[lane_id()]) atomicAdd(&stats[kNumStats + lane_id()], c[lane_id()]);
    }
};
#define AVR_PROBE(k, v) probe.add(k, v);
#else
#define AVR_PROBE(k, v)
#endif

// NanoVDBMedium (kVdb, media.h:602-685): the same loop over the sparse tree. Its 64^3
// majorant (1 MiB) does not fit LDS and is read through L2 (per-XCD 4 MiB); the density
// fetch is NanoVDB's index-space trilinear sampler (avr_vdb.h) and emission comes from the
// temperature grid. GridMedium (!kVdb) keeps its 16^3 majorant in LDS.
// RGBGridMedium (kMed 4, media.h:355-427): per-voxel RGB spectra (never gray), 16^3 majorant
// in LDS, sigma and Le from GridMedium-style trilinear sigmoid lookups (sample_point).
// kImage: the scene holds an ImageInfiniteLight (non-delta NEE with MIS, MIS-weighted
// escapes); a separate instantiation so the other kernels keep their register budget.
// kFast: the "fast" render mode (hardware transcendentals, statistical parity); replay otherwise.
template <bool kEmissive, bool kGray, int kSmp, int kMed, bool kImage, bool kFast>
__global__ void __launch_bounds__(256, kGray ? (kMed == 1 ? 3 : AVR_PATHS_WAVES_GRAY) : AVR_PATHS_WAVES_SPEC) k_paths(Params Pk) {
    const Params &P = Pk;
    // kMed 1: HomogeneousMedium or CloudMedium — dda_init gives their single
    // HomogeneousMajorantIterator segment over a 1^3 majorant of 1.0; properties from sample_point
    constexpr bool kVdb = kMed == 3, kRgb = kMed == 4, kAnalytic = kMed == 1;
    static_assert(!(kRgb && kGray), "RGB grids carry per-voxel spectra");
    // the work heads are valid only after this pass's camera stage zeroed them (it stamps the
    // pass generation): otherwise render nothing and flag stats[7], which the host reports
    if (__builtin_amdgcn_readfirstlane(__hip_atomic_load(P.heads + 8, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) !=
        P.pass_gen) {
        if (threadIdx.x == 0) atomicAdd(P.stats + 7, 1ull);
        return;
    }
    using S = typename std::conditional<kGray, float, Spec>::type;
    // LDS: majorant grid (16 KiB at pbrt's 16^3) + the 471-entry spectral tables the path
    // samples at path start, NEE and escape (sigma_a, sigma_s, up to 4 light spectra).
    __shared__ float s_maj[kVdb ? 1 : 4096];
    // (a gray medium's sigma_a / sigma_s are one value each: the kernel takes them as scalars)
    constexpr int kSigTabs = kGray ? 0 : 2;
    constexpr int kLdsLights = 4;
    __shared__ float s_tab[(kSigTabs + kLdsLights) * kNTable];
    // ImageInfiniteLight shadow rays (non-delta NEE): the sampled (u, v), p_l and the phase
    // value per lane, parked here while the lane traces its shadow ray (off the VGPR budget)
    __shared__ float4 s_img[kImage ? 256 : 1];
    // ZSobol: the requesters' sampler state for the cooperative draws (coop_draws_lds), 64 per wave
    __shared__ uint3 s_zst[kSmp != 0 ? 256 : 1];
    // NEE toward a delta light: the light's spectrum at the path's wavelengths and the phase
    // value f_hat, computed when the shadow ray is spawned and read back when it finishes
    // (SampleLd evaluates them once, integrators.cpp:1311-1331)
    __shared__ float4 s_ls[256];
    __shared__ float s_fhat[256];
    // ZSobol: Hash(d, seed) of the first kDimHash dimensions — each draw's FastOwen seeds,
    // read by the cooperative draws instead of a MurmurHash64A per draw
    __shared__ uint64_t s_dh[kSmp != 0 ? kDimHash : 1];
    if constexpr (kSmp != 0)
        for (int i = threadIdx.x; i < kDimHash; i += blockDim.x) s_dh[i] = smp::hash_2u32((uint32_t)i, (uint32_t)P.zs.seed);
    // ZSobol: smp::zperm's 24 permutations as bytes (the cooperative draws' digit permutations;
    // not for NanoVDB, whose kernel measured 2.4 % slower with them: profiles/r05_ab_zperm_lds.json)
    constexpr bool kZpt = kSmp != 0 && !kVdb;
    __shared__ uint8_t s_zpt[kZpt ? 24 : 1];
    if constexpr (kZpt)
        if (threadIdx.x < 24) {
            const uint64_t w = threadIdx.x < 8 ? smp::kZPermW0 : (threadIdx.x < 16 ? smp::kZPermW1 : smp::kZPermW2);
            s_zpt[threadIdx.x] = (uint8_t)(w >> ((threadIdx.x & 7) * 8));
        }
    // ZSobol: each lane's next light-pick draw (SampleLd's 1D, integrators.cpp:1302), evaluated
    // ahead with the previous bounce's cooperative phase draws (or by the camera stage)
    __shared__ float s_ul[kSmp != 0 ? 256 : 1];
    // the host routes GridMedium majorant grids of more than 4096 cells to the wavefront kernels
    if constexpr (!kVdb) stage_majorant(P.med, s_maj);
    const float *__restrict__ majp = kVdb ? P.med.majorant : s_maj;
    // NanoVDB: the majorant's coarse occupancy level (one bit per cell pair, 16 KiB at 64^3;
    // 33 + 16 KiB per block keeps three blocks of 256 lanes per CU)
    __shared__ unsigned s_occ[kVdb ? kOccWords : 1];
    const bool useOcc = kVdb && P.med.occ != nullptr;
    if (useOcc) {
        const int nw = (P.med.mres[0] * P.med.mres[1] * P.med.mres[2] + 63) >> 6;
        for (int i = threadIdx.x; i < nw; i += blockDim.x) s_occ[i] = P.med.occ[i];
    }
    const int nlds = P.lights.n < kLdsLights ? P.lights.n : kLdsLights;
    for (int i = threadIdx.x; i < kNTable; i += blockDim.x) {
        if constexpr (!kGray) {
            s_tab[i] = P.med.sigma_a[i];
            s_tab[kNTable + i] = P.med.sigma_s[i];
        }
        for (int k = 0; k < nlds; ++k)
            if (P.lights.list[k].type != 2) s_tab[(kSigTabs + k) * kNTable + i] = P.lights.list[k].L[i];
    }
    __syncthreads();
    const float *tab_sa = s_tab, *tab_ss = s_tab + kNTable;
    auto light_table = [&](int k) -> const float * {
        return k < kLdsLights ? s_tab + (kSigTabs + k) * kNTable : P.lights.list[k].L;
    };
    const DevMedium &m = P.med;
    const int npix = P.pass_pixels;
    const long long N = (long long)npix * P.pass_samples;
    const int lane = lane_id();
    const int xcc = xcc_id();
    // work counters off the VGPR budget: per wave in LDS, one ds_add by the first active lane
    // of each event batch (wave_count); DDA steps as a wave-uniform (scalar) sum of ballots;
    // the wave-loop counters wave-uniform (scalar registers)
    __shared__ unsigned s_cnt[4][6];
    if (threadIdx.x < 24) (&s_cnt[0][0])[threadIdx.x] = 0;
    __syncthreads();
    unsigned *const wcnt = s_cnt[threadIdx.x >> 6];
    auto wave_count = [&](int k) {
        const uint64_t am = __ballot(1);
        if (lane_id() == __ffsll((long long)am) - 1) atomicAdd(wcnt + k, (unsigned)__popcll(am));
    };
    unsigned long long nStepsW = 0;
#define AVR_COUNT(var, k) wave_count(k)
    unsigned long long nIter = 0, nActive = 0;

    int mode = M_FETCH, ev = EV_NONE;
    int g = 0;
    const int maj_sy = m.mres[0], maj_sz = m.mres[0] * m.mres[1], maj_n = maj_sz * m.mres[2];
    [[maybe_unused]] const __amdgpu_buffer_rsrc_t majr = maj_rsrc(P.med.majorant, maj_n);
    // path state (Li, integrators.cpp:966-971)
    Spec L{}, lam{}, Le_l{};
    S beta{}, r_u{}, r_l{}, sig_a{}, sig_s{};
    // gray: the same sigma_a and sigma_s at every wavelength, for every path (host-checked)
    if constexpr (kGray) {
        sig_a = P.med.gray_sigma_a;
        sig_s = P.med.gray_sigma_s;
    }
    constexpr bool kZSobol = kSmp != 0;   // kSmp: 0 Independent, 2 / 3 ZSobol with 32 / 64-bit index
    // ZSobol: the phase handler's draws evaluated cooperatively by the whole wave with their
    // results in LDS (coop_draws_lds), including the next light-pick draw (s_ul)
    constexpr bool kCoopLds = kZSobol;
    __shared__ float s_res[kCoopLds ? 256 * 6 : 1];
    PathSampler<kSmp> smp{};
    int depth = 0;
    V3 po{}, pd{};         // segment origin (== the path vertex) and the path's ray direction
    // segment state (SampleT_maj)
    Pcg32 rng{};
    float u = 0, tMin = 0, segMax = 0, mv = 0;
    DdaL it{};
    V3 sd{};               // normalised segment direction
    S T_maj{};
    bool needNext = true, shadowStopped = false;
    bool segPending = false;      // a segment start is queued for the shared block below
    uint64_t seqA = 0, seqB = 0;  // its RNG SetSequence arguments
    // shadow state (SampleLd, integrators.cpp:1339-1391)
    int light = 0;
    S T_ray{}, sr_l{}, sr_u{};

    auto seg_start = [&](const DevMedium &md, V3 o, V3 d, float tMax) {
        // SampleT_maj prologue (media.h:744-749): normalise, medium-space ray, clip, DDA
        tMax *= length(d);
        d = normalize(d);
        sd = d;
        ddal_init(it, md, Ray{o, d}, tMax, majp);
        T_maj = sconst<S>(1.f);
        needNext = true;
    };

    AVR_SEC_INIT
#ifdef AVR_PROBE_STATS
    __shared__ unsigned long long s_probe[4][8];
    if (threadIdx.x < 32) (&s_probe[0][0])[threadIdx.x] = 0;
    __syncthreads();
    ProbeStats probe{s_probe[threadIdx.x >> 6]};
#endif
    while (true) {
        AVR_SEC(0)
        // =================== batched event handlers (each runs once per batch) ===========
        if (__ballot(ev == EV_SCATTER)) {
            [[maybe_unused]] const Params &P = fresh_params();
            [[maybe_unused]] const DevMedium &m = P.med;
            if (ev == EV_SCATTER) {
                // SampleLd: light pick (BVH infinite-light branch) + shadow-ray spawn (1282-1338)
                const V3 wo = -pd;
                float ul;
                if constexpr (kZSobol) {
                    ul = s_ul[threadIdx.x];   // drawn ahead (same sampler dimension)
                    smp.z.dimension += 1;
                } else {
                    ul = smp.get1d(P);
                }
                float uL0 = 0.f, uL1 = 0.f;
                // uLight: read by the image light only; the other instantiations just step the
                // ZSobol dimension past it (the independent sampler's PCG32 still draws twice)
                if constexpr (kImage || !kZSobol) smp.get2d(P, &uL0, &uL1);
                else smp.z.dimension += 2;
                ev = EV_PHASE;                       // unless a shadow ray is spawned
                L = L + Spec::c(0.f);                // L += SampleLd(...) == 0 if nothing spawns
                const int nl = P.lights.n;
                if (nl > 0) {
                    float pmf = 0.f;
                    const int idx = light_pick<kImage>(P.lights, ul, &pmf);
                    if (idx >= 0) {
                        const DevLight &lt = P.lights.list[idx];
                        if (kImage && lt.type == 2) {
                            // ImageInfiniteLight::SampleLi with the compensated distribution
                            // (lights.h:588-613), shadow ray to 2 x sceneRadius (integrators.cpp:1311-1338)
                            float su, sv, lsPdf;
                            env::distrib_sample(lt.dist, uL0, uL1, &su, &sv, &lsPdf);
                            if (lsPdf != 0) {
                                V3 wl;
                                env::square_to_sphere(su, sv, &wl.x, &wl.y, &wl.z);
                                const V3 wi = xf_vec3(lt.rfl, wl);
                                lsPdf = lsPdf / (4 * kPi);
                                const Spec Ls = image_le(lt, su, sv, lam);
                                const float fval = hg_eval_c(dot(wo, wi), m.hg);
                                if (Ls.nonzero() && fval != 0) {
                                    const V3 pOut = po + wi * (2 * P.lights.scene_radius);
                                    const V3 d = pOut - po;
                                    light = idx;
                                    T_ray = sr_l = sr_u = sconst<S>(1.f);
                                    s_img[threadIdx.x] = make_float4(su, sv, pmf * lsPdf, fval);
                                    seqA = hash_3u32(f2u(po.x), f2u(po.y), f2u(po.z));
                                    seqB = hash_3u32(f2u(d.x), f2u(d.y), f2u(d.z));
                                    sd = d;
                                    segPending = true;
                                    mode = M_SHADOW;
                                    ev = EV_NONE;
                                    AVR_COUNT(nShadow, 4);
                                }
                            }
                        } else if (lt.type == 0) {
                            const V3 wi = {lt.w[0], lt.w[1], lt.w[2]};
                            const Spec Ls = sample_table(light_table(idx), lambda_index(lam)) * lt.scale;
                            const float fval = hg_eval_c(dot(wo, wi), m.hg);
                            if (Ls.nonzero() && fval != 0) {
                                s_ls[threadIdx.x] = to4(Ls);
                                s_fhat[threadIdx.x] = fval;
                                const V3 pOut = po + wi * (2 * P.lights.scene_radius);
                                const V3 d = pOut - po;
                                light = idx;
                                T_ray = sr_l = sr_u = sconst<S>(1.f);
                                // shadow-ray RNG (integrators.cpp:1338); u is its first draw
                                seqA = hash_3u32(f2u(po.x), f2u(po.y), f2u(po.z));
                                seqB = hash_3u32(f2u(d.x), f2u(d.y), f2u(d.z));
                                sd = d;
                                segPending = true;
                                mode = M_SHADOW;
                                ev = EV_NONE;
                                AVR_COUNT(nShadow, 4);
                            }
                        }
                    }
                }
            }
        }
        AVR_SEC(5)
        if (__ballot(ev == EV_SHADOW_DONE)) {
            [[maybe_unused]] const Params &P = fresh_params();
            [[maybe_unused]] const DevMedium &m = P.med;
            if (ev == EV_SHADOW_DONE) {
                // finish SampleLd (1379-1398); SampleT_maj returned 1 if the callback stopped
                const S Tm = shadowStopped ? sconst<S>(1.f) : T_maj;
                if constexpr (kGray) {
                    const float q = unit_quot(Tm);
                    T_ray = T_ray * q;
                    sr_l = sr_l * q;
                    sr_u = sr_u * q;
                } else {
                    T_ray = T_ray * (Tm / sv0(Tm));
                    sr_l = sr_l * (Tm / sv0(Tm));
                    sr_u = sr_u * (Tm / sv0(Tm));
                }
                Spec contrib = Spec::c(0.f);
                if (snz(T_ray)) {
                    const DevLight &lt = P.lights.list[light];
                    if (kImage && lt.type == 2) {
                        // non-delta light: r_l *= r_p * p_l, r_u *= r_p * scatterPDF (1391-1398)
                        const float4 im = s_img[threadIdx.x];
                        const S f_hat = sconst<S>(im.w);
                        const Spec Ls = image_le(lt, im.x, im.y, lam);
                        sr_l = sr_l * (r_u * im.z);
                        sr_u = sr_u * (r_u * im.w);
                        contrib = smul(Ls, beta * f_hat * T_ray) / savg(sr_l + sr_u);
                    } else {
                        // the delta light's spectrum and f_hat of the spawn (same wo, wi)
                        const float p_l = light_pmf<kImage>(P.lights, light) * 1.f;
                        const S f_hat = sconst<S>(s_fhat[threadIdx.x]);
                        const Spec Ls = spec4(s_ls[threadIdx.x]);
                        sr_l = sr_l * (r_u * p_l);
                        contrib = smul(Ls, beta * f_hat * T_ray) / savg(sr_l);
                    }
                }
                L = L + contrib;
                ev = EV_PHASE;
            }
        }
        AVR_SEC(6)
        if (__ballot(ev == EV_PHASE)) {
            [[maybe_unused]] const Params &P = fresh_params();
            [[maybe_unused]] const DevMedium &m = P.med;
            // ZSobol: the phase 2D draw and the next segment's three 1D draws of every lane in
            // EV_PHASE, evaluated cooperatively by the whole wave
            // (and, at offset 5, the next bounce's light-pick draw, parked in s_ul)
            [[maybe_unused]] const float *qr = nullptr;   // this lane's results in s_res (kCoopLds)
            if constexpr (kCoopLds) {
                // [u0, u1] phase 2D, [h0, h1, u] the next segment, [ul] the next light pick
                constexpr int off[5] = {0, 2, 3, 4, 5};
                constexpr bool two[5] = {true, false, false, false, false};
                constexpr int slot[5] = {0, 2, 3, 4, 5};
                float *sres = s_res + (threadIdx.x & ~63u) * 6;
                const int rk = coop_draws_lds<PathSampler<kSmp>::kW, 5, 6>(smp.z, P.zs, ev == EV_PHASE, off, two, slot, 5, sres,
                                                                          s_zst + (threadIdx.x & ~63u), s_dh,
                                                                          kZpt ? s_zpt : nullptr);
                qr = sres + rk * 6;
                if (ev == EV_PHASE) s_ul[threadIdx.x] = qr[5];
            }
            if (ev == EV_PHASE) {
                // phase-function sampling (integrators.cpp:1046-1061), then the next segment
                AVR_COUNT(nPhase, 2);
                float up0, up1;
                if constexpr (kCoopLds) {
                    up0 = qr[0];
                    up1 = qr[1];
                } else {
                    smp.get2d(P, &up0, &up1);
                }
                float phPdf;
                const V3 wi = hg_sample_c<kFast>(-pd, m.hg, up0, up1, &phPdf);
                if (phPdf == 0) {
                    ev = EV_END;
                } else {
                    beta = beta * unit_quot(phPdf);
                    r_l = r_u / phPdf;
                    pd = wi;
                    const float h0 = kCoopLds ? qr[2] : smp.get1d(P);
                    const float h1 = kCoopLds ? qr[3] : smp.get1d(P);
                    seqA = hash_u32(f2u(h0));
                    seqB = hash_u32(f2u(h1));
                    u = kCoopLds ? qr[4] : smp.get1d(P);
                    sd = pd;
                    segPending = true;
                    mode = M_MEDIUM;
                    ev = EV_NONE;
                }
            }
        }
        AVR_SEC(7)
        if (__ballot(ev == EV_ESCAPE)) {
            [[maybe_unused]] const Params &P = fresh_params();
            [[maybe_unused]] const DevMedium &m = P.med;
            if (ev == EV_ESCAPE) {
                // escaped (integrators.cpp:1078-1107)
                if constexpr (kGray) {
                    const float q = unit_quot(T_maj);
                    beta = beta * q;
                    r_u = r_u * q;
                    r_l = r_l * q;
                } else {
                    beta = beta * (T_maj / sv0(T_maj));
                    r_u = r_u * (T_maj / sv0(T_maj));
                    r_l = r_l * (T_maj / sv0(T_maj));
                }
                for (int k = 0; k < P.lights.n; ++k) {
                    const DevLight &lt = P.lights.list[k];
                    if (lt.type == 0 || (!kImage && lt.type == 2)) continue;
                    Spec Le;
                    float pdfLi = 0.f;
                    if (kImage && lt.type == 2) {
                        float eu = 0, evv = 0;
                        Le = image_le_dir(lt, pd, lam, &eu, &evv);
                        if (Le.nonzero() && depth != 0) pdfLi = image_pdf_li(lt, pd);
                    } else {
                        Le = sample_table(light_table(k), lambda_index(lam)) * lt.scale;
                    }
                    if (!Le.nonzero()) continue;
                    if (depth == 0) L = L + smul(Le, beta) / savg(r_u);
                    else {
                        // lightSampler.PMF * PDF_Li(prevIntrContext, ray.d, true): 0 for the uniform light
                        r_l = r_l * (light_pmf<kImage>(P.lights, k) * pdfLi);
                        L = L + smul(Le, beta) / savg(r_u + r_l);
                    }
                }
                ev = EV_END;
            }
        }
        if (__ballot(ev == EV_END)) {
            [[maybe_unused]] const Params &P = fresh_params();
            [[maybe_unused]] const DevMedium &m = P.med;
            if (ev == EV_END) {
                // the per-sample record: L (k_film takes the rest from the camera stage)
                P.ps.rec[g] = to4(L);
                mode = M_FETCH;
                ev = EV_NONE;
            }
        }

        AVR_SEC(1)
        // =================== refill idle lanes: one atomic per wave on a per-XCD head ======
        const uint64_t needMask = __ballot(mode == M_FETCH);
        const uint64_t busyMask = __ballot(mode == M_MEDIUM || mode == M_SHADOW);
        if (needMask && (busyMask == 0 || __popcll(needMask) >= P.refill_min)) {
            [[maybe_unused]] const Params &P = fresh_params();
            [[maybe_unused]] const DevMedium &m = P.med;
            const int cnt = __popcll(needMask);
            const int leader = __ffsll((long long)needMask) - 1;
            long long base = 0;
            int granted = 0, exhausted = 0;
            if (lane == leader) {
                exhausted = 1;
                for (int j = 0; j < 8; ++j) {
                    const int c = (xcc + j) & 7;
                    const long long lo = N * c / 8, hi = N * (c + 1) / 8;
                    if (lo >= hi) continue;
                    const int old = atomicAdd(P.heads + c, cnt);
                    if (lo + old < hi) {
                        base = lo + old;
                        granted = (int)((hi - base) < cnt ? (hi - base) : cnt);
                        exhausted = 0;
                        break;
                    }
                }
            }
            base = __shfl(base, leader);
            granted = __shfl(granted, leader);
            exhausted = __shfl(exhausted, leader);
            const uint64_t lt = lane == 0 ? 0ull : (needMask & ((~0ull) >> (64 - lane)));
            const int k = __popcll(lt);
            const bool fresh = mode == M_FETCH && k < granted;
            if (mode == M_FETCH) {
                if (fresh) {
                    AVR_COUNT(nPaths, 1);
                    // ---- a new path from the camera stage (k_paths_camera) ----
                    const int gn = (int)(base + k);
                    const float4 c0 = P.ps.cam0[gn], c1 = P.ps.cam1[gn], c2 = P.ps.cam2[gn];
                    const uint4 c3 = P.ps.cam3[gn];
                    // ZSobol: the first light pick drawn ahead; independent: the PCG32 state
                    [[maybe_unused]] float ul5 = 0.f;
                    [[maybe_unused]] uint4 c5{};
                    if constexpr (!kZSobol) c5 = P.ps.cam5[gn];
                    else ul5 = c1.w;
                    g = gn;
                    if constexpr (kZSobol) {
                        // the sample's ZSobol state past the camera draws and the first segment's three
                        // (hardware-sequence divisions: FastDiv splits here measured 1.2 % slower in
                        // k_paths, profiles/r05_ab_unit_quot_fastdiv.json; the camera stage keeps them)
                        const int slot = g % npix, sIdx = g / npix;
                        const int pix = P.pix_order ? P.pix_order[slot] : slot;
                        smp.start(P, pix % P.film.width, pix / P.film.width, P.sample_base + sIdx);
                        s_ul[threadIdx.x] = ul5;
                        smp.z.dimension = 9;
                    } else {
                        smp.rng.state = ((uint64_t)c5.y << 32) | c5.x;
                        smp.rng.inc = ((uint64_t)c5.w << 32) | c5.z;
                    }
                    po = {c0.x, c0.y, c0.z};
                    u = c0.w;
                    pd = {c1.x, c1.y, c1.z};
                    lam = spec4(c2);
                    seqA = ((uint64_t)c3.y << 32) | c3.x;
                    seqB = ((uint64_t)c3.w << 32) | c3.z;
                    L = Spec::c(0.f);
                    beta = r_u = r_l = sconst<S>(1.f);
                    depth = 0;
                    {
                        const LambdaIdx li = lambda_index(lam);
                        if constexpr (!kGray) {
                            sig_a = sfrom<S>(sample_table(tab_sa, li));
                            sig_s = sfrom<S>(sample_table(tab_ss, li));
                        }
                        if (kEmissive && (kMed == 0 || kMed == 1)) Le_l = sample_table(m.Le, li);
                    }
                    sd = pd;
                    segPending = true;
                    mode = M_MEDIUM;
                } else if (exhausted) {
                    mode = M_DONE;
                }
            }
        }
        AVR_SEC(2)
        // =================== segment starts, shared by the NEE shadow ray, the phase-sampled
        // continuation and the camera ray: RNG(seqA, seqB), then SampleT_maj's prologue
        // (medium-space ray, clip, DDA setup) once per batch for every lane that needs one
        if (__ballot(segPending)) {
            [[maybe_unused]] const Params &P = fresh_params();
            [[maybe_unused]] const DevMedium &m = P.med;
            if (segPending) {
                rng.set_sequence(seqA, seqB);
                if (mode == M_SHADOW) u = rng.uniform();
                float tMax = mode == M_SHADOW ? 1 - kShadowEpsilon : kInf;
                if (m.boundary) tMax = fminf_(tMax, interface_exit(m, po, sd));
                seg_start(m, po, sd, tMax);
                segPending = false;
            }
        }
        if (__ballot(mode != M_DONE) == 0) break;

        // =================== tracking: advance every busy lane collision by collision ======
        // until a batch of lanes needs service (events or refill) or none is busy.
        while (true) {
            AVR_SEC(3)
            const bool busy = (mode == M_MEDIUM || mode == M_SHADOW) && ev == EV_NONE;
            const uint64_t busyNow = __ballot(busy);
            const uint64_t service = __ballot(mode != M_DONE && !busy);
            if (busyNow == 0 || __popcll(service) >= P.refill_min) break;
            ++nIter;
            nActive += __popcll(busyNow);
            if (!busy) continue;
            // ---- advance to the next tentative collision (media.h:754-802) ----
            // Hot loop: on the S-cloud input a path crosses ~20 majorant cells per density
            // fetch. Bit-exact shortcuts: gray medium -> scalar state; a rejected candidate
            // (t >= segMax only consumes its RNG draw; its t is never used) is decided from
            // T_maj's FastExp factor outside a conservative error margin, exactly otherwise and
            // for every accepted collision; each lane crosses at most P.dda_budget cells per
            // iteration, bounding how long early lanes wait for the longest walk.
            float t = 0;
            const S sig_t = sig_a + sig_s;
            const float st0 = sv0(sig_t);
            // walk: 0 walking, 1 candidate pending (accepted or ambiguous), 2 segments exhausted.
            // Each step crosses at most one majorant cell and tests at most one candidate; the
            // loop has one wave-uniform exit so the body stays predicated (no per-exit masks).
            int walk = 0;
            for (int b = 0; b < P.dda_budget; ++b) {
                [[maybe_unused]] bool stepped = false;
                if (walk == 0 && needNext) {
                    float s0, s1;
                    if (!ddal_next(it, majp, maj_sy, maj_sz, &s0, &s1, &mv)) {
                        walk = 2;
                    } else {
                        stepped = true;
                        // zero-majorant cell: T_maj *= FastExp(-0 * dt); for a gray medium that
                        // factor is exactly 1, so the multiply is skipped
                        const S sigma_maj = sig_t * mv;
#ifdef AVR_PROBE_STATS
                        { const uint64_t z = __ballot(sv0(sigma_maj) == 0); AVR_PROBE(6, __popcll(z)) }
#endif
                        if (sv0(sigma_maj) == 0) {
                            if (!kGray) {
                                float dt = s1 - s0;
                                if (__builtin_isinf(dt)) dt = kFloatMax;
                                T_maj = T_maj * sexpm<kFast>(-(sigma_maj * dt));
                            }
                        } else {
                            tMin = s0;
                            segMax = s1;
                            needNext = false;
                        }
                    }
                }
                nStepsW += __popcll(__ballot(stepped));
                // unconditional (all busy lanes): in flight during the candidate test below
                // (the next cell's index is unclamped: LDS for the 16^3 majorants, a bounds-checked
                // buffer for NanoVDB's — +0.9 % grid, +2.2 % NanoVDB, profiles/r06_ab_walk.json)
                if constexpr (kVdb) {
                    if (useOcc) ddal_prefetch_occ_buf(it, majr, s_occ, maj_n);
                    else ddal_prefetch_buf(it, majr);
                } else {
                    ddal_prefetch(it, majp);
                }
                if (walk == 0 && !needNext) {
                    // Fast reject: the candidate t = tMin - log(1-u)/sigma_maj is decided against
                    // segMax from T_maj's own FastExp factor when 1-u lies outside an error margin
                    // (below); accepted and ambiguous candidates stay "pending" and are decided
                    // exactly, once per wave, after the walk.
                    const float sm0 = st0 * mv;
                    bool pending;
                    float dt = segMax - tMin;
                    // T_maj's factor should the candidate be rejected (media.h:790-801). Replay,
                    // gray medium: an infinite dt gives A = inf, i.e. a pending candidate, and the
                    // factor is used only for A < 40, where FastExp's range checks cannot fire —
                    // so neither the clamp nor the checks are evaluated (same bits; +1.6 % grid,
                    // +3.0 % NanoVDB, profiles/r06_ab_walk.json)
                    constexpr bool kLite = kGray && !kFast;
                    if (!kLite && __builtin_isinf(dt)) dt = kFloatMax;
                    S fac;
                    if constexpr (kLite) fac = fast_exp_m40(-((sig_t * mv) * dt));
                    else fac = sexpm<kFast>(-((sig_t * mv) * dt));
                    if constexpr (kFast) {
                        // fast mode: the hardware candidate is the candidate (decided once)
                        pending = tMin + m_exp_dist<true>(u, sm0) < segMax;
                    } else {
                        // t = tMin + (-log(1-u) / sm0) >= segMax  <=>  1-u <= exp(-sm0 (segMax - tMin))
                        // in real arithmetic; FastExp(-A) (relative error < 1.2e-4 for A < 40, the
                        // rounding of A = sm0 * dt and of pbrt's log / division / add all inside
                        // the 1e-3 + 5e-7 A margin) decides it for sure outside the margin: no
                        // transcendental of its own — the factor is T_maj's anyway
                        const float A = sm0 * dt;
                        pending = !(A < 40.f && (1 - u) <= sv0(fac) * (1 - 1e-3f - 5e-7f * A));
                    }
                    if (pending) {
                        walk = 1;
                    } else {
                        u = rng.uniform();
                        T_maj = T_maj * fac;
                        needNext = true;
                    }
                }
                const uint64_t walking = __ballot(walk == 0);
                AVR_PROBE(0, 1)
                AVR_PROBE(1, __popcll(walking))
                if (walking == 0) break;
            }
            AVR_SEC(4)
#ifdef AVR_PROBE_STATS
            { const uint64_t still = __ballot(walk == 0); AVR_PROBE(7, still != 0) }
#endif
            const bool segEnd = walk == 2, pend = walk == 1;
            if (segEnd) {
                if (mode == M_MEDIUM) ev = EV_ESCAPE;
                else { ev = EV_SHADOW_DONE; shadowStopped = false; }
                continue;
            }
            if (!pend) continue;   // walk budget used up: resume the DDA next iteration
            // exact candidate (media.h:770-777): t = tMin + SampleExponential(u, sigma_maj[0])
            t = tMin + m_exp_dist<kFast>(u, st0 * mv);
            u = rng.uniform();
            if (!(t < segMax)) {   // rejected after all: close the segment (media.h:790-801)
                float dt = segMax - tMin;
                if (__builtin_isinf(dt)) dt = kFloatMax;
                T_maj = T_maj * sexpm<kFast>(-((sig_t * mv) * dt));
                needNext = true;
                continue;
            }
            // ---- collision: density fetch for every lane that reached one ----
            const DevMedium &m = fresh_params().med;   // the medium's fields re-read here (s_load)
            const S sigma_maj = sig_t * mv;
            T_maj = T_maj * sexpm<kFast>(-(sigma_maj * (t - tMin)));
            const V3 pc = po + sd * t;
            // GridMedium::SamplePoint (media.h:287-319) / NanoVDBMedium::SamplePoint (624-637) /
            // RGBGridMedium / Homogeneous / Cloud
            V3 pm = xf_point_pair(m.medium_from_render, pc);
            S ms_a, ms_s;
            Spec rgbLe{};
            if constexpr (kRgb) {
                // RGBGridMedium::SamplePoint (media.h:377-403), as the wavefront kernels do it
                const MediumSample rs = sample_point(m, pc, Spec::c(1.f), Spec::c(0.f), Spec::c(0.f), lam, kEmissive);
                ms_a = sfrom<S>(rs.sigma_a);
                ms_s = sfrom<S>(rs.sigma_s);
                rgbLe = rs.Le;
            } else if constexpr (kAnalytic) {
                // HomogeneousMedium / CloudMedium::SamplePoint (media.h:230-238, 478-489)
                const MediumSample rs = sample_point(m, pc, to_spec(sig_a), to_spec(sig_s), Le_l, lam, kEmissive);
                ms_a = sfrom<S>(rs.sigma_a);
                ms_s = sfrom<S>(rs.sigma_s);
                rgbLe = rs.Le;
            } else {
                float dens;
                if constexpr (kVdb) {
                    dens = vdb::sample_world(m.vdb, pm.x, pm.y, pm.z);
                } else {
                    pm = m.unit_box ? V3{pm.x - m.bmin[0], pm.y - m.bmin[1], pm.z - m.bmin[2]} : box_offset(m.bmin, m.bmax, pm);
#ifdef AVR_PROBE_STATS
                    {
                        // the fat entry this lookup reads (fat_issue's index), per 32-B entry
                        const float psx = pm.x * m.nx - .5f, psy = pm.y * m.ny - .5f, psz = pm.z * m.nz - .5f;
                        const long long ent = ((long long)((int)__builtin_floorf(psz) + 1) * (m.ny + 1) +
                                               ((int)__builtin_floorf(psy) + 1)) * (m.nx + 1) +
                                              ((int)__builtin_floorf(psx) + 1);
                        AVR_PROBE(2, 1)
                        AVR_PROBE(3, __popcll(__ballot(1)))
                        AVR_PROBE(4, ProbeStats::distinct(ent >> 2))
                        AVR_PROBE(5, ProbeStats::distinct(ent >> 1))
                    }
#endif
                    dens = grid_density(m, pm);
                }
                ms_a = sig_a * dens;
                ms_s = sig_s * dens;
            }
            bool stop = false;
            if (mode == M_MEDIUM) {
                AVR_COUNT(nLookup, 0);
                // delta-tracking callback (integrators.cpp:990-1077)
                if (!snz(beta)) {
                    stop = true;
                    ev = EV_END;
                } else {
                    if (kEmissive && depth < P.max_depth) {
                        const Spec Le = (kRgb || kAnalytic) ? rgbLe : (kVdb ? vdb_emission(m, pm, lam) : grid_emission(m, pm, lam, Le_l));
                        if (Le.nonzero()) {
                            float pdf = sv0(sigma_maj) * sv0(T_maj);
                            S betap = beta * T_maj / pdf;
                            S r_e = r_u * sigma_maj * T_maj / pdf;
                            if (snz(r_e)) L = L + smul(Le, betap * ms_a) / savg(r_e);
                        }
                    }
                    const float pAbsorb = sv0(ms_a) / sv0(sigma_maj);
                    const float pScat = sv0(ms_s) / sv0(sigma_maj);
                    const float pNull = fmaxf_(0.f, 1 - pAbsorb - pScat);
                    const int e = sample_discrete3(pAbsorb, pScat, pNull, rng.uniform());
                    if (e == 0) {
                        stop = true;
                        ev = EV_END;
                    } else if (e == 1) {
                        stop = true;
                        ev = EV_END;
                        if (depth++ < P.max_depth) {
                            const float pdf = sv0(T_maj) * sv0(ms_s);
                            if constexpr (kGray) {   // T_maj * ms_s is pdf's product
                                const float q = unit_quot(pdf);
                                beta = beta * q;
                                r_u = r_u * q;
                            } else {
                                beta = beta * (T_maj * ms_s / pdf);
                                r_u = r_u * (T_maj * ms_s / pdf);
                            }
                            if (snz(beta) && snz(r_u)) {
                                po = pc;     // the scatter vertex: shadow-ray and next-segment origin
                                ev = EV_SCATTER;
                            }
                        }
                    } else {
                        const S sigma_n = sclamp0(sigma_maj - ms_a - ms_s);
                        const float pdf = sv0(T_maj) * sv0(sigma_n);
                        const S qn = kGray ? sconst<S>(unit_quot(pdf)) : T_maj * sigma_n / pdf;   // gray: pdf's product
                        beta = beta * qn;
                        if (pdf == 0) beta = sconst<S>(0.f);
                        r_u = r_u * qn;
                        r_l = r_l * (T_maj * sigma_maj / pdf);
                        if (!(snz(beta) && snz(r_u))) { stop = true; ev = EV_END; }
                    }
                }
            } else {
                AVR_COUNT(nShadowLookup, 3);
                // ratio-tracking callback with Russian roulette (integrators.cpp:1351-1378)
                const S sigma_n = sclamp0(sigma_maj - ms_a - ms_s);
                const float pdf = sv0(T_maj) * sv0(sigma_maj);
                T_ray = T_ray * (T_maj * sigma_n / pdf);
                if constexpr (kGray) sr_l = sr_l * unit_quot(pdf);   // T_maj * sigma_maj is pdf's product
                else sr_l = sr_l * (T_maj * sigma_maj / pdf);
                sr_u = sr_u * (T_maj * sigma_n / pdf);
                const S Tr = T_ray / savg(sr_l + sr_u);
                if (smaxc(Tr) < 0.05f) {
                    if (rng.uniform() < 0.75f) T_ray = sconst<S>(0.f);
                    else T_ray = T_ray / (1 - 0.75f);
                }
                if (!snz(T_ray)) { stop = true; ev = EV_SHADOW_DONE; shadowStopped = true; }
            }
            if (!stop) {
                T_maj = sconst<S>(1.f);
                tMin = t;
            }
        }
    }
    AVR_SEC_FLUSH
#ifdef AVR_PROBE_STATS
    probe.flush(P.stats);
#endif
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (lane < 5 && wcnt[lane]) atomicAdd(P.stats + lane, (unsigned long long)wcnt[lane]);
    if (lane == 0 && nStepsW) atomicAdd(P.stats + 5, nStepsW);
#undef AVR_COUNT
    if (lane == 0) {   // wave-uniform counters: one add per wave
        if (nIter) atomicAdd(P.stats + 8, nIter);
        if (nActive) atomicAdd(P.stats + 9, nActive);
    }
}

#ifndef AVR_KPATHS_TU
// ---------------------------------------------------------------------------
// Film — NaN/Inf guard (integrators.cpp:272-282), PixelSensor::ToSensorRGB (film.h:95-100),
// RGBFilm::AddSample (film.h:239-255): per pixel, the pass's samples in sampleIndex order.
// SpectralFilm: a pixel's bucket sums (up to kFilmLdsBuckets of them) are accumulated in this
// thread's LDS slice and written back once per pass — the same fp64 additions in the same
// order as the read-modify-writes on HBM, without their 2 x 4 dependent round trips per sample.
// One sample of the pass: L, the wavelengths, their pdfs and CameraSample::filterWeight —
// after k_paths: L from its record, the rest from its camera stage (k_paths_camera); after the
// wavefront kernels: their SoA (pdfs recomputed with the sampling function's pdf)
__device__ __forceinline__ void film_load_sample(const Params &P, size_t id, Spec *L, Spec *lam, Spec *pdf, float *w,
                                                 const double *canon_tabs) {
    *w = 1.f;
    if (P.rec_mode) {
        *L = spec4(P.ps.rec[id]);
        *lam = spec4(P.ps.cam2[id]);
        // the pdfs are evaluated from the wavelengths after the loads (film_pdfs)
        if (P.film.filter_type != 0) *w = P.ps.camw[id];
    } else {
        *L = spec4(P.ps.L[id]);
        *lam = spec4(P.ps.lambda[id]);
        *pdf = {film_lambda_pdf(P.film, lam->v0), film_lambda_pdf(P.film, lam->v1), film_lambda_pdf(P.film, lam->v2),
                film_lambda_pdf(P.film, lam->v3)};
        if (P.film.filter_type != 0) *w = P.ps.weight[id];
    }
}
// the camera stage's wavelength pdfs (film_lambda_pdf: the same canonical function of the same
// floats, so the same bits) when k_film evaluates them (k_paths' records)
// fast mode (its wavelengths come from the hardware log already): VisibleWavelengthsPDF
// (spectrum.h:255-259) with the hardware exp for cosh — about 1 ulp, statistical parity
__device__ __forceinline__ float film_lambda_pdf_fast(const DevFilm &f, float l) {
    if (f.nbuckets > 0) return 1 / (f.lmax - f.lmin);
    if (l < 360 || l > 830) return 0;
    const float x = 0.0072f * (l - 538);
    return 0.0039398042f / sqr(0.5f * (__expf(x) + __expf(-x)));
}
template <bool kFast = false>
__device__ __forceinline__ void film_pdfs(const Params &P, const Spec &lam, Spec *pdf, const double *canon_tabs) {
    if (!P.rec_mode) return;
    if constexpr (kFast)
        *pdf = {film_lambda_pdf_fast(P.film, lam.v0), film_lambda_pdf_fast(P.film, lam.v1),
                film_lambda_pdf_fast(P.film, lam.v2), film_lambda_pdf_fast(P.film, lam.v3)};
    else
        *pdf = {film_lambda_pdf(P.film, lam.v0, canon_tabs), film_lambda_pdf(P.film, lam.v1, canon_tabs),
                film_lambda_pdf(P.film, lam.v2, canon_tabs), film_lambda_pdf(P.film, lam.v3, canon_tabs)};
}
// The pass's wavelength pdfs into cam4 for the host accessor (avr_last_pass_samples): k_film's
// own evaluation (film_pdfs: the same overload over the same LDS-staged canonical tables), so
// the accessor returns exactly the pdfs the film divided by
__global__ void __launch_bounds__(256) k_lambda_pdfs(DevFilm film, const float4 *__restrict__ lam, float4 *__restrict__ pdf,
                                                     long long n, int fast) {
    __shared__ double s_canon[canon::kCanonTabDoubles];
    for (int i = threadIdx.x; i < canon::kCanonTabDoubles; i += blockDim.x)
        s_canon[i] = i < 128 ? canon::kLogInvC[i] : (i < 256 ? canon::kLogC[i - 128] : canon::kExp2J64[i - 256]);
    __syncthreads();
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        const float4 l = lam[i];
        pdf[i] = fast ? make_float4(film_lambda_pdf_fast(film, l.x), film_lambda_pdf_fast(film, l.y),
                                    film_lambda_pdf_fast(film, l.z), film_lambda_pdf_fast(film, l.w))
                      : make_float4(film_lambda_pdf(film, l.x, s_canon), film_lambda_pdf(film, l.y, s_canon),
                                    film_lambda_pdf(film, l.z, s_canon), film_lambda_pdf(film, l.w, s_canon));
    }
}
// The X, Y, Z matching tables interleaved per wavelength ({X, Y, Z, 0}, staged in LDS by
// k_film): one 16-B read per wavelength instead of four table gathers; same values, same sums
__device__ __forceinline__ float4 xyz_at(const float4 *t, int off) {
    return (off < 0 || off >= kNTable) ? make_float4(0.f, 0.f, 0.f, 0.f) : t[off];
}
// The NaN/Inf guard (integrators.cpp:272-282; a bad sample's L becomes 0, in place) and
// PixelSensor::ToSensorRGB with RGBFilm's maxComponentValue clamp (film.h:95-100, 239-250)
__device__ __forceinline__ void film_sensor_rgb(const Params &P, Spec &L, const Spec &lam, const Spec &pdf, float rgb[3],
                                                const float4 *xyz4) {
    const LambdaIdx li = lambda_index(lam);
    const float4 t0 = xyz_at(xyz4, li.o0), t1 = xyz_at(xyz4, li.o1), t2 = xyz_at(xyz4, li.o2), t3 = xyz_at(xyz4, li.o3);
    bool bad = __builtin_isnan(L.v0) || __builtin_isnan(L.v1) || __builtin_isnan(L.v2) || __builtin_isnan(L.v3);
    // y = avg(Y L / pdf) / CIE_Y_integral is finite whenever max|L| max|Y| < 1e37 min(pdf) (each
    // term below 1e37, the sum below 4e37 < FLT_MAX); only samples outside that bound (or with
    // an overflowing bound) evaluate it
    const float aL = fmaxf_(fmaxf_(__builtin_fabsf(L.v0), __builtin_fabsf(L.v1)),
                            fmaxf_(__builtin_fabsf(L.v2), __builtin_fabsf(L.v3)));
    const float aY = fmaxf_(fmaxf_(__builtin_fabsf(t0.y), __builtin_fabsf(t1.y)),
                            fmaxf_(__builtin_fabsf(t2.y), __builtin_fabsf(t3.y)));
    const float mp = fminf_(fminf_(pdf.v0, pdf.v1), fminf_(pdf.v2, pdf.v3));
    if (!bad && !(aL * aY < 1e37f * mp)) {
        const Spec Ys = {t0.y, t1.y, t2.y, t3.y};
        float y = safe_div(Ys * L, pdf).avg() / 106.856895f;
        bad = __builtin_isinf(y);
    }
    if (bad) L = Spec::c(0.f);
    const Spec Ld = safe_div(L, pdf);
    rgb[0] = (Spec{t0.x, t1.x, t2.x, t3.x} * Ld).avg() * P.film.imaging_ratio;
    rgb[1] = (Spec{t0.y, t1.y, t2.y, t3.y} * Ld).avg() * P.film.imaging_ratio;
    rgb[2] = (Spec{t0.z, t1.z, t2.z, t3.z} * Ld).avg() * P.film.imaging_ratio;
    float mx = fmaxf_(fmaxf_(rgb[0], rgb[1]), rgb[2]);
    if (mx > P.film.max_component)
        for (int c = 0; c < 3; ++c) rgb[c] *= P.film.max_component / mx;
}

constexpr int kFilmLdsBuckets = 16;
#ifndef AVR_FILM_BATCH
#define AVR_FILM_BATCH 4
#endif
constexpr int kFilmBatch = AVR_FILM_BATCH;
inline size_t film_lds_bytes(int nb) { return nb > 0 && nb <= kFilmLdsBuckets ? 2 * (size_t)nb * 256 * sizeof(double) : 0; }
// kBuckets: a SpectralFilm (P.film.nbuckets > 0); RGBFilm's instantiation has no bucket code
template <bool kBuckets, bool kFast = false>
#ifndef AVR_FILM_WAVES
#define AVR_FILM_WAVES 1   // minimum waves per SIMD asked of k_film (1: the compiler's choice)
#endif
__global__ void __launch_bounds__(256, AVR_FILM_WAVES) k_film(Params P) {
    extern __shared__ double s_bk[];   // [sum | weight][bucket][thread]: film_lds_bytes(nb)
    __shared__ float4 s_xyz[kNTable];
    for (int i = threadIdx.x; i < kNTable; i += blockDim.x)
        s_xyz[i] = make_float4(P.film.xyz[i], P.film.xyz[kNTable + i], P.film.xyz[2 * kNTable + i], 0.f);
    __shared__ double s_canon[canon::kCanonTabDoubles];   // the pdfs' cosh tables
    for (int i = threadIdx.x; i < canon::kCanonTabDoubles; i += blockDim.x)
        s_canon[i] = i < 128 ? canon::kLogInvC[i] : (i < 256 ? canon::kLogC[i - 128] : canon::kExp2J64[i - 256]);
    __syncthreads();
    const int npix = P.pass_pixels;
    const int nb = kBuckets ? P.film.nbuckets : 0;
    const bool ldsBuckets = nb > 0 && nb <= kFilmLdsBuckets;
    for (int pix = blockIdx.x * blockDim.x + threadIdx.x; pix < npix; pix += gridDim.x * blockDim.x) {
        double s0 = P.film.rgb_sum[3 * (size_t)pix], s1 = P.film.rgb_sum[3 * (size_t)pix + 1],
               s2 = P.film.rgb_sum[3 * (size_t)pix + 2], ws = P.film.w_sum[pix];
        double *gbs = P.film.bucket_sum + (size_t)pix * nb, *gbw = P.film.bucket_w + (size_t)pix * nb;
        double *bs = gbs, *bw = gbw;
        int bstride = 1;
        if (ldsBuckets) {
            bs = s_bk + threadIdx.x;
            bw = s_bk + nb * 256 + threadIdx.x;
            bstride = 256;
            for (int b = 0; b < nb; ++b) {
                bs[b * 256] = gbs[b];
                bw[b * 256] = gbw[b];
            }
        }
        const int slot = P.pix_slot ? P.pix_slot[pix] : pix;   // where k_paths traced this pixel
        // one sample into the sums, in sampleIndex order (the fp64 additions' order is the film's)
        auto add = [&](Spec L, const Spec &lam, const Spec &pdf, float w) {
            float rgb[3];
            film_sensor_rgb(P, L, lam, pdf, rgb, s_xyz);
            s0 += (double)(w * rgb[0]);
            s1 += (double)(w * rgb[1]);
            s2 += (double)(w * rgb[2]);
            ws += (double)w;
            if (kBuckets) {
                // SpectralFilm::AddSample (film.h:436-454): clamp by the max component, scale by
                // weight * CIE_Y_integral, one bucket per wavelength (LambdaToBucket, 500-504)
                const float lm = fmaxf_(fmaxf_(fmaxf_(L.v0, L.v1), L.v2), L.v3);
                if (lm > P.film.max_component) L = L * (P.film.max_component / lm);
                L = L * (w * 106.856895f);
                const float lv[4] = {lam.v0, lam.v1, lam.v2, lam.v3}, Lv[4] = {L.v0, L.v1, L.v2, L.v3};
                _Pragma("unroll") for (int i = 0; i < 4; ++i) {
                    int b = (int)((float)nb * (lv[i] - P.film.lmin) / (P.film.lmax - P.film.lmin));
                    b = b < 0 ? 0 : (b > nb - 1 ? nb - 1 : b);
                    bs[b * bstride] += (double)Lv[i];
                    bw[b * bstride] += (double)w;
                }
            }
        };
        // the pass's samples in groups of kFilmBatch: all of a group's loads are issued before
        // its (possibly storing) accumulation, so a wave keeps kFilmBatch x 52 B per lane in flight
        int s = 0;
        for (; s + kFilmBatch <= P.pass_samples; s += kFilmBatch) {
            Spec L[kFilmBatch], lam[kFilmBatch], pdf[kFilmBatch];
            float w[kFilmBatch];
            _Pragma("unroll") for (int k = 0; k < kFilmBatch; ++k)
                film_load_sample(P, (size_t)(s + k) * npix + slot, &L[k], &lam[k], &pdf[k], &w[k], s_canon);
            _Pragma("unroll") for (int k = 0; k < kFilmBatch; ++k) film_pdfs<kFast>(P, lam[k], &pdf[k], s_canon);
            _Pragma("unroll") for (int k = 0; k < kFilmBatch; ++k) add(L[k], lam[k], pdf[k], w[k]);
        }
        for (; s < P.pass_samples; ++s) {
            Spec L, lam, pdf;
            float w;
            film_load_sample(P, (size_t)s * npix + slot, &L, &lam, &pdf, &w, s_canon);
            film_pdfs<kFast>(P, lam, &pdf, s_canon);
            add(L, lam, pdf, w);
        }
        if (ldsBuckets)
            for (int b = 0; b < nb; ++b) {
                gbs[b] = bs[b * 256];
                gbw[b] = bw[b * 256];
            }
        P.film.rgb_sum[3 * (size_t)pix] = s0;
        P.film.rgb_sum[3 * (size_t)pix + 1] = s1;
        P.film.rgb_sum[3 * (size_t)pix + 2] = s2;
        P.film.w_sum[pix] = ws;
    }
}

// ---------------------------------------------------------------------------
// The density fetch alone: SampledGrid::Lookup (containers.h:804-835) over a batch of
// unit-box points (Bounds3::Offset applied), one trilinear lookup per point, through the
// same fat / linear layout code as the path kernels. Measurement kernel for the north star's
// density-fetch roofline (bench.py `density_fetch`: the recorded lookups of a pass in their
// trace order, sorted by voxel, shuffled).
__global__ void __launch_bounds__(256) k_density_fetch(DevMedium m, const float4 *__restrict__ pts, long long n,
                                                       float *__restrict__ out) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        const float4 p = pts[i];
        // clamped to the footprint's valid range: a stray point reads the zero border, never
        // past the grid (the layouts' own bounds checks assume finite coordinates)
        const V3 q{fminf_(fmaxf_(p.x, -1.f), 2.f), fminf_(fmaxf_(p.y, -1.f), 2.f), fminf_(fmaxf_(p.z, -1.f), 2.f)};
        out[i] = grid_density(m, q);
    }
}

// ---------------------------------------------------------------------------
// Integrator::Tr (cpu/integrators.cpp:324-374): ratio-tracking transmittance between
// points p0 -> p1 in the medium at four given wavelengths; one query per lane. RNG seeded
// with Hash(p0), Hash(p1); the ray is p0.SpawnRayTo(p1) (a medium interaction: no origin
// offset) clipped at 1 - ShadowEpsilon; result Tr / inv_w.Average().
__global__ void __launch_bounds__(256) k_transmittance(Params P, long long n, const float *__restrict__ p0,
                                                       const float *__restrict__ p1,
                                                       const float *__restrict__ lambda, float *__restrict__ out) {
    __shared__ float s_maj[4096];
    const float *maj = stage_majorant(P.med, s_maj);
    unsigned long long nLookup = 0, nSteps = 0, nIn = 0;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        ++nIn;
        const V3 a = {p0[3 * i], p0[3 * i + 1], p0[3 * i + 2]}, b = {p1[3 * i], p1[3 * i + 1], p1[3 * i + 2]};
        const Spec lamv = {lambda[4 * i], lambda[4 * i + 1], lambda[4 * i + 2], lambda[4 * i + 3]};
        Spec Tr = Spec::c(1.f), inv_w = Spec::c(1.f);
        Pcg32 rng;
        rng.set_sequence(hash_3u32(f2u(a.x), f2u(a.y), f2u(a.z)), hash_3u32(f2u(b.x), f2u(b.y), f2u(b.z)));
        Ray ray{a, b - a};
        if (dot(ray.d, ray.d) != 0) {
            const V3 pExit = ray.o + ray.d * (1 - kShadowEpsilon);
            ray.d = pExit - ray.o;
            const LambdaIdx li = lambda_index(lamv);
            const Spec sig_a = sample_table(P.med.sigma_a, li);
            const Spec sig_s = sample_table(P.med.sigma_s, li);
            const float u = rng.uniform();
            auto cb = [&](V3, const MediumSample &ms, const Spec &sigma_maj, const Spec &T_maj) -> bool {
                const Spec sigma_n = clamp_zero(sigma_maj - ms.sigma_a - ms.sigma_s);
                const float pr = T_maj.v0 * sigma_maj.v0;
                Tr = Tr * (T_maj * sigma_n / pr);
                inv_w = inv_w * (T_maj * sigma_maj / pr);
                return Tr.nonzero() && inv_w.nonzero();
            };
            const Spec T_maj = sample_t_maj(P.med, maj, ray, 1.f, u, rng, sig_a, sig_s, Spec::c(0.f), lamv, nLookup,
                                            nSteps, cb);
            Tr = Tr * (T_maj / T_maj.v0);
            inv_w = inv_w * (T_maj / T_maj.v0);
            Tr = Tr / inv_w.avg();
        }
        out[4 * i] = Tr.v0;
        out[4 * i + 1] = Tr.v1;
        out[4 * i + 2] = Tr.v2;
        out[4 * i + 3] = Tr.v3;
    }
    flush_stat(P.stats, 3, nLookup);
    flush_stat(P.stats, 4, nIn);
    flush_stat(P.stats, 6, nSteps);
}

// ---------------------------------------------------------------------------
// MajorantGrid build — GridMedium ctor (media.cpp:229, 241-246): each cell is
// SampledGrid::MaxValue over MajorantGrid::VoxelBounds (containers.h:838-857).
// One workgroup per majorant cell; wave max-reduction, then LDS.
__global__ void __launch_bounds__(256) k_majorant(const float *__restrict__ density, int nx, int ny, int nz, int rx,
                                                  int ry, int rz, float *out) {
    const int cell = blockIdx.x;
    const int x = cell % rx, y = (cell / rx) % ry, z = cell / (rx * ry);
    const float b0[3] = {float(x) / rx, float(y) / ry, float(z) / rz};
    const float b1[3] = {float(x + 1) / rx, float(y + 1) / ry, float(z + 1) / rz};
    const int n[3] = {nx, ny, nz};
    int lo[3], hi[3];
    _Pragma("unroll") for (int a = 0; a < 3; ++a) {
        float ps0 = b0[a] * n[a] - .5f, ps1 = b1[a] * n[a] - .5f;
        int l = (int)__builtin_floorf(ps0);
        lo[a] = l > 0 ? l : 0;
        int h = (int)__builtin_floorf(ps1) + 1;
        hi[a] = h < n[a] - 1 ? h : n[a] - 1;
    }
    float m = grid_at(density, nx, ny, nz, lo[0], lo[1], lo[2]);
    const int ex = hi[0] - lo[0] + 1, ey = hi[1] - lo[1] + 1, ez = hi[2] - lo[2] + 1;
    const long long total = (long long)ex * ey * ez;
    for (long long k = threadIdx.x; k < total; k += blockDim.x) {
        const int kx = (int)(k % ex), ky = (int)((k / ex) % ey), kz = (int)(k / ((long long)ex * ey));
        m = fmaxf_(m, grid_at(density, nx, ny, nz, lo[0] + kx, lo[1] + ky, lo[2] + kz));
    }
    for (int off = 32; off > 0; off >>= 1) m = fmaxf_(m, __shfl_xor(m, off));
    __shared__ float red[4];
    if (lane_id() == 0) red[threadIdx.x / 64] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        float r = red[0];
        for (int w = 1; w < (int)(blockDim.x / 64); ++w) r = fmaxf_(r, red[w]);
        out[cell] = r;
    }
}

// NanoVDBMedium's 64^3 majorant (media.cpp:556-613): each cell's world box is
// bounds.Lerp of its corners, mapped to index space by worldToIndexF, widened by one voxel
// of filter slop (int truncation of the f64 i -/+ 1), clamped to the active index bbox
// (inclusive); the cell holds the max of getValue over that box (0 when it is empty).
// One workgroup per cell.
__global__ void __launch_bounds__(256) k_majorant_vdb(vdb::Apron g, float3 bmin, float3 bmax, int4 ibmin, int4 ibmax,
                                                      int rx, int ry, int rz, float *out) {
    const int cell = blockIdx.x;
    const int x = cell % rx, y = (cell / rx) % ry, z = cell / (rx * ry);
    const float t0x = float(x) / rx, t0y = float(y) / ry, t0z = float(z) / rz;
    const float t1x = float(x + 1) / rx, t1y = float(y + 1) / ry, t1z = float(z + 1) / rz;
    const float ax = (1 - t0x) * bmin.x + t0x * bmax.x, ay = (1 - t0y) * bmin.y + t0y * bmax.y,
                az = (1 - t0z) * bmin.z + t0z * bmax.z;
    const float bx = (1 - t1x) * bmin.x + t1x * bmax.x, by = (1 - t1y) * bmin.y + t1y * bmax.y,
                bz = (1 - t1z) * bmin.z + t1z * bmax.z;
    float i0x, i0y, i0z, i1x, i1y, i1z;
    vdb::world_to_index(g, fminf_(ax, bx), fminf_(ay, by), fminf_(az, bz), &i0x, &i0y, &i0z);
    vdb::world_to_index(g, fmaxf_(ax, bx), fmaxf_(ay, by), fmaxf_(az, bz), &i1x, &i1y, &i1z);
    const int x0 = max((int)((double)i0x - 1.0), ibmin.x), x1 = min((int)((double)i1x + 1.0), ibmax.x);
    const int y0 = max((int)((double)i0y - 1.0), ibmin.y), y1 = min((int)((double)i1y + 1.0), ibmax.y);
    const int z0 = max((int)((double)i0z - 1.0), ibmin.z), z1 = min((int)((double)i1z + 1.0), ibmax.z);
    float m = 0.f;
    if (x0 <= x1 && y0 <= y1 && z0 <= z1) {
        const int ex = x1 - x0 + 1, ey = y1 - y0 + 1, ez = z1 - z0 + 1;
        const long long total = (long long)ex * ey * ez;
        for (long long k = threadIdx.x; k < total; k += blockDim.x) {
            const int kx = (int)(k % ex), ky = (int)((k / ex) % ey), kz = (int)(k / ((long long)ex * ey));
            const float v = vdb::get_value(g, x0 + kx, y0 + ky, z0 + kz);
            m = m < v ? v : m;   // std::max(maxValue, v)
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        const float o = __shfl_xor(m, off);
        m = m < o ? o : m;
    }
    __shared__ float red[4];
    if (lane_id() == 0) red[threadIdx.x / 64] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        float r = red[0];
        for (int w = 1; w < (int)(blockDim.x / 64); ++w) r = r < red[w] ? red[w] : r;
        out[cell] = r;
    }
}

// Apron blocks of a NanoVDB grid (avr_vdb.h "Apron layout"): block i holds getValue of the
// base layout over the 9^3 neighbourhood of extended block list[i]; one workgroup per block
__global__ void __launch_bounds__(256) k_vdb_apron(vdb::Grid base, const long long *__restrict__ list, long long n,
                                                   float *__restrict__ out) {
    const int ne_x = base.lnx + 1, ne_y = base.lny + 1;
    for (long long i = blockIdx.x; i < n; i += gridDim.x) {
        const long long e = list[i];
        const int ex = (int)(e % ne_x), ey = (int)((e / ne_x) % ne_y), ez = (int)(e / ((long long)ne_x * ne_y));
        for (int k = threadIdx.x; k < vdb::kApronVals; k += blockDim.x)
            out[i * vdb::kApronVals + k] = vdb::apron_value(base, ex, ey, ez, k);
    }
}

// The fat copy of a NanoVDB density grid's apron blocks (vdb::Apron::fat): entry (block i,
// base voxel k) = the eight stencil taps of apron_fat_entry as two float4
__global__ void __launch_bounds__(256) k_vdb_fat(const float *__restrict__ blocks, long long n, float4 *__restrict__ fat) {
    const long long total = n * 512;
    for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
        float t[8];
        vdb::apron_fat_entry(blocks, e >> 9, (int)(e & 511), t);
        fat[2 * e] = make_float4(t[0], t[1], t[2], t[3]);
        fat[2 * e + 1] = make_float4(t[4], t[5], t[6], t[7]);
    }
}

// Coarse occupancy level of a majorant grid (DevMedium::occ): one bit per pair of linear cells,
// set unless both cells' majorants are 0 (NaN counts as occupied).
__global__ void __launch_bounds__(256) k_majorant_occupancy(const float *__restrict__ maj, int n, unsigned *occ,
                                                            int nwords) {
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= nwords) return;
    unsigned bits = 0;
    for (int b = 0; b < 32; ++b) {
        const int i = 64 * w + 2 * b;
        const bool nz = (i < n && !(maj[i] == 0.f)) || (i + 1 < n && !(maj[i + 1] == 0.f));
        bits |= (unsigned)nz << b;
    }
    occ[w] = bits;
}

// RGBGridMedium's 16^3 majorant (media.cpp:364-377): per cell, sigmaScale * (max over the
// cell's voxel range of sigma_a's scale * rsp.MaxValue() (1 without a grid) + the same for
// sigma_s), the voxel range as SampledGrid::MaxValue (containers.h:838-857).
__global__ void __launch_bounds__(256) k_majorant_rgb(const float4 *__restrict__ ga, const float4 *__restrict__ gs,
                                                      int nx, int ny, int nz, int rx, int ry, int rz, float sigma_scale,
                                                      float *out) {
    const int cell = blockIdx.x;
    const int x = cell % rx, y = (cell / rx) % ry, z = cell / (rx * ry);
    const float b0[3] = {float(x) / rx, float(y) / ry, float(z) / rz};
    const float b1[3] = {float(x + 1) / rx, float(y + 1) / ry, float(z + 1) / rz};
    const int n[3] = {nx, ny, nz};
    int lo[3], hi[3];
    _Pragma("unroll") for (int a = 0; a < 3; ++a) {
        float ps0 = b0[a] * n[a] - .5f, ps1 = b1[a] * n[a] - .5f;
        int l = (int)__builtin_floorf(ps0);
        lo[a] = l > 0 ? l : 0;
        int h = (int)__builtin_floorf(ps1) + 1;
        hi[a] = h < n[a] - 1 ? h : n[a] - 1;
    }
    const int ex = hi[0] - lo[0] + 1, ey = hi[1] - lo[1] + 1, ez = hi[2] - lo[2] + 1;
    const long long total = (long long)ex * ey * ez;
    __shared__ float red[2][4];
    for (int gi = 0; gi < 2; ++gi) {
        const float4 *g = gi == 0 ? ga : gs;
        if (!g) continue;
        auto conv = [&](int vx, int vy, int vz) {
            const float4 c = g[(vz * ny + vy) * nx + vx];
            return c.w * rsp_max(c.x, c.y, c.z);
        };
        float m = conv(lo[0], lo[1], lo[2]);
        for (long long k = threadIdx.x; k < total; k += blockDim.x) {
            const int kx = (int)(k % ex), ky = (int)((k / ex) % ey), kz = (int)(k / ((long long)ex * ey));
            const float v = conv(lo[0] + kx, lo[1] + ky, lo[2] + kz);
            m = m < v ? v : m;
        }
        for (int off = 32; off > 0; off >>= 1) {
            const float o = __shfl_xor(m, off);
            m = m < o ? o : m;
        }
        if (lane_id() == 0) red[gi][threadIdx.x / 64] = m;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float r[2] = {1.f, 1.f};
        for (int gi = 0; gi < 2; ++gi) {
            if (!(gi == 0 ? ga : gs)) continue;
            r[gi] = red[gi][0];
            for (int w = 1; w < (int)(blockDim.x / 64); ++w) r[gi] = r[gi] < red[gi][w] ? red[gi][w] : r[gi];
        }
        out[cell] = sigma_scale * (r[0] + r[1]);
    }
}

// ZSobol pixel table: zsobol_upper for every pixel of the film and the first dmax
// dimensions, row Morton(pixel) (zp.upper must be null here: the digits are computed).
__global__ void __launch_bounds__(256) k_zsobol_table(smp::ZSobolParams zp, int width, int height, int dmax,
                                                      uint32_t *__restrict__ table) {
    const long long n = (long long)width * height * dmax;
    for (long long k = blockIdx.x * (long long)blockDim.x + threadIdx.x; k < n; k += (long long)gridDim.x * blockDim.x) {
        const int d = (int)(k % dmax);
        const long long pix = k / dmax;
        const uint32_t pm = (uint32_t)smp::encode_morton2((uint32_t)(pix % width), (uint32_t)(pix / width));
        table[(size_t)pm * dmax + d] = smp::zsobol_upper(pm, (uint32_t)d, zp);
    }
}

// ZSobol pass table: zsobol_pass_entry for every pixel of the film and the first pdims
// dimensions, for the pass whose sample indices agree with `base` above their low `plo` bits;
// row Morton(pixel). The pixel digits come from the pixel table (zp.upper) where it covers
// the dimension. zp.ptab must be null here. Built once per k_paths pass (a few hundred us);
// with `atab` (the same table built for plo + 2, plo + 2 <= log2spp) each entry is derived
// from its level-A entry by zsobol_pass_entry_from (one MixBits instead of ~5).
__global__ void __launch_bounds__(256) k_zsobol_pass_table(smp::ZSobolParams zp, int width, int height, int pdims,
                                                           int plo, long long base, uint64_t *__restrict__ table,
                                                           const uint64_t *__restrict__ atab, FastDiv div_pairs,
                                                           FastDiv div_width, uint64_t *__restrict__ ctab) {
    // one thread per PAIR of dimensions of a pixel's row (pdims is even, avr_set_sampler_pass_table):
    // 16-B loads and stores, and the pixel / Morton index arithmetic once per two entries;
    // 32-bit indices (the host checks width * height * pdims < 2^31) split by multiply-shift
    const uint32_t half = (uint32_t)pdims >> 1;
    const uint32_t n = (uint32_t)width * (uint32_t)height * half;
    const bool wide = smp::zsobol_wide(zp);
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
        const int pix = fdiv((int)k, div_pairs);
        const int d = 2 * (int)(k - (uint32_t)pix * half);
        const int py = fdiv(pix, div_width);
        const uint32_t pm = (uint32_t)smp::encode_morton2((uint32_t)(pix - py * width), (uint32_t)py);
        const uint64_t m = ((uint64_t)pm << zp.log2spp) | (uint64_t)base;
        const size_t row = (size_t)pm * pdims + d;
        ulonglong2 e;
        if (atab) {
            const ulonglong2 eA = *reinterpret_cast<const ulonglong2 *>(atab + row);
            e.x = wide ? smp::zsobol_pass_entry_from<uint64_t>(m, (uint32_t)d, zp, plo, eA.x)
                       : smp::zsobol_pass_entry_from<uint32_t>((uint32_t)m, (uint32_t)d, zp, plo, eA.x);
            e.y = wide ? smp::zsobol_pass_entry_from<uint64_t>(m, (uint32_t)d + 1, zp, plo, eA.y)
                       : smp::zsobol_pass_entry_from<uint32_t>((uint32_t)m, (uint32_t)d + 1, zp, plo, eA.y);
        } else {
            auto up_of = [&](int dd) -> uint32_t {
                return (zp.upper && dd < zp.dmax) ? zp.upper[(size_t)pm * zp.dmax + dd] : smp::zsobol_upper(pm, (uint32_t)dd, zp);
            };
            const uint32_t u0 = up_of(d), u1 = up_of(d + 1);
            e.x = wide ? smp::zsobol_pass_entry<uint64_t>(m, (uint32_t)d, zp, plo, u0)
                       : smp::zsobol_pass_entry<uint32_t>((uint32_t)m, (uint32_t)d, zp, plo, u0);
            e.y = wide ? smp::zsobol_pass_entry<uint64_t>(m, (uint32_t)d + 1, zp, plo, u1)
                       : smp::zsobol_pass_entry<uint32_t>((uint32_t)m, (uint32_t)d + 1, zp, plo, u1);
        }
        *reinterpret_cast<ulonglong2 *>(table + row) = e;
        // the camera stage's pairs (0, 1), (6, 7), (8, 9) also into its compact per-pixel copy
        if (ctab && (d == 0 || d == 6 || d == 8))
            *reinterpret_cast<ulonglong2 *>(ctab + 6 * (size_t)pix + (d == 0 ? 0 : d - 4)) = e;
    }
}

__global__ void __launch_bounds__(256) k_cloud(float *out, int n, long long first, long long count, float density,
                                               float wispiness, float frequency) {
    for (long long k = blockIdx.x * (long long)blockDim.x + threadIdx.x; k < count; k += (long long)gridDim.x * blockDim.x) {
        const long long idx = first + k;
        const int x = (int)(idx % n), y = (int)((idx / n) % n), z = (int)(idx / ((long long)n * n));
        out[k] = cloud_density(V3{(x + 0.5f) / n, (y + 0.5f) / n, (z + 0.5f) / n}, density, wispiness, frequency);
    }
}

// Synthetic RGB-coefficient explosion — BASELINE config C5's "emissive RGB-coefficient
// explosion volume" (asset absent) as an RGBGridMedium (media.h:355-427): per voxel
// {c0, c1, c2, scale} of RGBSigmoidPolynomial spectra (color.h:332-365) for sigma_a, sigma_s
// (RGBUnboundedSpectrum) and Le (RGBIlluminantSpectrum), voxel centres (i + 0.5) / n, in
// [first, first + count) of the x-fastest grid. A Perlin-perturbed ball: density
// d = clamp(1.2 (1 - r / 0.42) + 0.18 w1, 0, 1), heat t = clamp(1 - r / 0.3 + 0.25 w2, 0, 1);
// smoke sigma_a {0, 0, 0.3} x 2d (flat), sigma_s {0, 0.002, -1.1} x 6d (redder scattering),
// fire Le: a rising sigmoid with its edge at 650 - 180 t nm (hotter = whiter), scale 8 t^2.
__global__ void __launch_bounds__(256) k_rgb_explosion(float4 *sa, float4 *ss, float4 *le, int n, long long first,
                                                       long long count) {
    for (long long k = blockIdx.x * (long long)blockDim.x + threadIdx.x; k < count; k += (long long)gridDim.x * blockDim.x) {
        const long long idx = first + k;
        const int x = (int)(idx % n), y = (int)((idx / n) % n), z = (int)(idx / ((long long)n * n));
        const float px = (x + 0.5f) / n, py = (y + 0.5f) / n, pz = (z + 0.5f) / n;
        const float dx = px - 0.5f, dy = py - 0.5f, dz = pz - 0.5f;
        const float r = __builtin_sqrtf(dx * dx + dy * dy + dz * dz);
        const float w1 = perlin(8 * px, 8 * py, 8 * pz), w2 = perlin(6 * px + 3.1f, 6 * py + 1.7f, 6 * pz + 0.3f);
        const float d = clampf(1.2f * (1 - r / 0.42f) + 0.18f * w1, 0.f, 1.f);
        const float t = clampf(1 - r / 0.3f + 0.25f * w2, 0.f, 1.f);
        sa[k] = make_float4(0.f, 0.f, 0.3f, 2.f * d);
        ss[k] = make_float4(0.f, 0.002f, -1.1f, 6.f * d);
        const float edge = 650.f - 180.f * t;
        le[k] = make_float4(0.f, 0.03f, -0.03f * edge, 8.f * t * t);
    }
}

#endif  // AVR_KPATHS_TU
}  // namespace avr

#ifndef AVR_KPATHS_TU
#include "avr_image_kernels.h"   // the film image, image metrics and FLIP kernels
#endif

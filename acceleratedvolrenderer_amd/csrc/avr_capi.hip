// avr_capi.hip — host side of libavr_hip.so: the C-ABI (include/avr.h) and the
// wavefront scheduler that replaces pbrt's ImageTileIntegrator::Render /
// WavefrontPathIntegrator::Render loops (cpu/integrators.cpp:72-232,
// wavefront/integrator.cpp:290-493) for the volumetric path.
//
// Scheduling: the requested sample range is cut into passes of S sample indices
// over all P pixels (P*S <= max_paths, default 16M paths in flight for the wavefront
// kernels and 64M 32-B sample records for k_paths — HBM is 288 GB, pbrt's GPU path caps at 1M). Each pass: k_camera, then depth iterations of
// {k_medium, k_shadow} over compacted queues until no path survives, then k_film.
// Everything is enqueued on one HIP stream; the host reads back one int (the
// survivor count) per depth iteration to size the next launch and stop early.
#include "avr_kernels.hip"
#ifdef AVR_KP_SPLIT
// k_paths is instantiated in avr_kpaths.hip's translation units (one per medium kind and
// render mode, compiled in parallel by build.py); declared here, launched from avr_render
#include "avr_kpaths_list.h"
namespace avr {
#define AVR_KP_DECL(em, gr, zs, med, im, fa) extern template __global__ void k_paths<em, gr, zs, med, im, fa>(Params);
AVR_KP_ALL(AVR_KP_DECL)
#undef AVR_KP_DECL
}  // namespace avr
#endif
#include "avr_graph.hip"
#include "../../include/avr.h"

#include <rccl/rccl.h>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>
#include <algorithm>

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

#define HIP_TRY(expr)                                                                          \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess)                                                                  \
            return fail(AVR_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));       \
    } while (0)

#ifndef AVR_ZS_TWO_LEVEL
#define AVR_ZS_TWO_LEVEL 1   // build the ZSobol pass table from a level-A table shared by 4 passes
#endif

template <typename T>
hipError_t dalloc(T **p, size_t n) { return hipMalloc((void **)p, std::max<size_t>(n, 1) * sizeof(T)); }

}  // namespace

struct avr_context {
    int device = 0;
    // paths per pass: max_paths when the caller set one, else 16M for the wavefront kernels
    // (full SoA path state, ~250 B per path) and 64M for k_paths (a 32-B record per sample
    // only: 2 GiB of HBM; longer passes amortise the persistent kernel's drain tail)
    long long max_paths = 16ll << 20;
    bool max_paths_set = false;
    long long rec_cap = 0;   // k_paths records and camera stage allocated (samples)
    hipStream_t own_stream = nullptr, stream = nullptr;
    // medium
    avr::DevMedium med{};
    float *d_density_owned = nullptr;
    float *d_sigma_a = nullptr, *d_sigma_s = nullptr, *d_Le = nullptr, *d_lescale = nullptr, *d_majorant = nullptr;
    bool has_medium = false;
    // lights / camera / film
    avr::DevLights lights{};
    float *d_lightL = nullptr;
    avr::DevLight *d_lights = nullptr;
    avr::DevCamera cam{};
    bool has_camera = false;
    avr::DevFilm film{};
    float *d_xyz = nullptr;
    bool has_film = false;
    // path state
    long long cap = 0;
    avr::PathSoA ps{};
    avr::ShadowSoA sh{};
    int *d_queue[2] = {nullptr, nullptr};
    int *d_counts = nullptr;  // [0],[1] queue counts, [2] shadow count
    unsigned long long *d_stats = nullptr;
    int *h_count = nullptr;   // pinned
    avr_stats stats{};
    std::vector<hipEvent_t> evpool;   // timing events; the first ev_used are recorded, unresolved
    size_t ev_used = 0;
    struct Timed { int a, b; double avr_stats::*field; bool launch; };
    std::vector<Timed> timed;         // pending (event a -> event b) intervals to fold into stats
    int last_base = 0, last_S = 0;
    int kernel_mode = 0;      // 0: persistent k_paths (default), 1: wavefront k_medium/k_shadow
    bool last_persistent = false;   // which organisation the last avr_render ran
    bool last_fast = false;         // ... and whether k_paths ran in fast mode
    int *d_heads = nullptr;   // 8 per-XCD work counters of k_paths + the pass generation
    int pass_gen = 0;         // k_paths passes enqueued (the camera stage stamps it into d_heads[8])
    // k_paths' pixel order (avr_set_pixel_order): slot -> pixel and pixel -> slot, and the
    // host copy of the latter (to return the last pass in pixel order); empty = scanline
    int *d_pix_order = nullptr, *d_pix_slot = nullptr;
    std::vector<int> h_pix_slot;
    // bumped whenever the pixel order changes (avr_set_pixel_order, avr_film); the last
    // render's records are in the order of generation last_order_gen
    int order_gen = 0, last_order_gen = 0;
    // template arguments of the last k_paths instantiation launched ("k_paths<em, gray, smp,
    // med, image, fast>", avr_last_kernel), so a profiler pass can be matched to the timed run
    char last_kpaths[64] = "";
    // k_paths<emissive, gray, sampler, medium, image, fast> at slot
    // ((((fast*2 + image)*4 + medium(0 grid, 1 vdb, 2 rgb, 3 homogeneous/cloud))*3 + sampler(0
    // independent, 1 zsobol 32-bit, 2 zsobol 64-bit))*2 + emissive)*2 + gray
    static constexpr int kNumPaths = 192;
    int paths_grid[kNumPaths] = {};
    void (*kpaths[kNumPaths])(avr::Params) = {};
    int render_mode = 0;      // 0 replay (canonical math, per-sample parity), 1 fast (hardware math)
    int ray_binning = 0;      // wavefront organisation: counting-sort queues by (majorant cell, octant)
    int majorant_occupancy = 0;   // NanoVDB k_paths: coarse occupancy level of the majorant in LDS (opt-in)
    unsigned *d_occ = nullptr;
    float4 *d_planes = nullptr;   // convex interface half-spaces (avr_medium_boundary_convex)
    int *d_bin_keys = nullptr, *d_bin_out = nullptr, *d_bin_hist = nullptr;
    long long bin_cap = 0;
    // pixel sampler (avr_set_sampler) and filter (avr_set_filter)
    int sampler_kind = 0;     // 0 IndependentSampler, 1 ZSobolSampler
    int sampler_spp = 16;     // samplesPerPixel of the sampler (ZSobol's Morton layout)
    int filter_type = 0;      // 0 BoxFilter (radius from avr_film), 1 GaussianFilter
    float *d_filter = nullptr;
    float *d_temperature = nullptr;
    // NanoVDBMedium grids (0 density, 1 temperature): block slots, leaves, tile values
    int *d_vdb_slot[2] = {nullptr, nullptr};
    float *d_vdb_leaves[2] = {nullptr, nullptr}, *d_vdb_tiles[2] = {nullptr, nullptr};
    int vdb_ibbox[6] = {};    // density grid's active index bbox (majorant clamp)
    long long vdb_napron[2] = {0, 0};   // apron blocks of the density / temperature grid
    // RGBGridMedium grids (sigma_a, sigma_s, Le as float4 {c0, c1, c2, scale}) and illuminant
    float4 *d_rgb[3] = {nullptr, nullptr, nullptr};   // owned copies (avr_medium_rgbgrid only)
    float *d_illum = nullptr;
    // lights: host copy of the device list, ImageInfiniteLight buffers
    avr::DevLight h_lights[avr::kMaxLights] = {};
    // PowerLightSampler: each light's Phi-based weight (phi_ok once known: an image light's
    // needs its avr_light_image), and the sampler the render uses (0 BVH / uniform, 1 power)
    float h_phi[avr::kMaxLights] = {};
    bool phi_ok[avr::kMaxLights] = {};
    int light_sampler = 0;
    void *d_light_img[avr::kMaxLights] = {};
    int n_image_lights = 0, image_lights_ready = 0;
    // film image / --mse-reference-image state
    float *d_image = nullptr, *d_reference = nullptr;
    double *d_metric = nullptr;      // kMetricBlocks * kMetricSlots partials + kMetricSlots totals
    avr::Mat3 ref_out_from_sensor{};
    int ref_fp16 = 1;
    avr::smp::FilterTables ftab{};
    // ZSobol pixel table (zsobol_upper per Morton(pixel) x dimension < zs_dims), rebuilt
    // when the sampler's spp or the film resolution change; zs_dims 0 = no table
    uint32_t *d_zs_table = nullptr;
    int zs_dims = 256;
    int zs_key[3] = {-1, -1, -1};
    // ZSobol pass table (zsobol_pass_entry per Morton(pixel) x dimension < zs_pdims), rebuilt
    // for every k_paths pass: the digits its sample indices share; zs_pdims 0 = no table
    // Two buffers: a pass reads one while the next pass's table is built ahead into the other
    // (ptab_spec) on the low-priority side stream tstream
    uint64_t *d_zs_ptab[2] = {};
    size_t zs_ptab_cap[2] = {};   // entries allocated
    uint64_t *d_zs_ctab[2] = {};  // the camera stage's compact copy (6 entries per pixel)
    size_t zs_ctab_cap[2] = {};
    int zs_pdims = 96;
    int tab_buf = 1;              // the buffer the last pass read
    int ptab_spec = 1;            // avr_set_pass_table_ahead
    bool spec_valid = false;      // tstream holds (or is building) the table for spec_key
    long long spec_key[8] = {};
    int spec_buf = 0;
    hipStream_t tstream = nullptr;
    hipEvent_t ev_cam = nullptr, ev_tab = nullptr;
    long long prev_call_begin = -1;   // avr_render's previous spp_begin (the call stride)
    // Level-A pass table (the same table for plo + 2, shared by four consecutive passes);
    // zs_akey names the build it holds (rebuilt when any field changes), zs_two_level 0 = off
    uint64_t *d_zs_atab = nullptr;
    size_t zs_atab_cap = 0;
    long long zs_akey[6] = {-1, -1, -1, -1, -1, -1};
    int zs_two_level = AVR_ZS_TWO_LEVEL;
    int refill_min = 0;       // 0: the default (32 lanes; 20 for a non-emissive NanoVDB walk, 16 for RGB grids, 48 for a <= 2^3 GridMedium majorant)
    int dda_budget = 0;       // 0: by majorant resolution (12 cells up to 16^3, 32 for NanoVDB's 64^3)
    int grid_layout = 1;
    bool gray = false;        // sigma_a and sigma_s constant over 360..830 nm      // 1: build the fat (footprint) copy when memory allows, 0: linear only
    float4 *d_fat = nullptr;
    float *d_brick = nullptr;   // bricked GridMedium copy (grid_layout 2)
    uint64_t *d_advance = nullptr;  // per-pass PCG advance table {A, H}
    long long advance_cap = 0;
    // avr_film_reduce_rccl: this context's communicator and the clique (contexts in rank
    // order) it was created with by ncclCommInitAll; reused while the same clique reduces
    ncclComm_t comm = nullptr;
    std::vector<avr_context *> comm_group;
};

namespace {

// Destroy the communicators of c's RCCL clique (every member's: a clique with one member
// gone cannot run a collective) and forget the clique on each member.
void release_comms(avr_context *c) {
    if (!c || c->comm_group.empty()) return;
    const std::vector<avr_context *> group = c->comm_group;
    for (avr_context *m : group) {
        if (m->comm) {
            (void)hipSetDevice(m->device);
            (void)ncclCommDestroy(m->comm);
        }
        m->comm = nullptr;
        m->comm_group.clear();
    }
    (void)hipSetDevice(c->device);
}

void free_paths(avr_context *c) {
    float4 *f4[] = {c->ps.o, c->ps.d, c->ps.lambda, c->ps.pdf, c->ps.beta, c->ps.r_u, c->ps.r_l, c->ps.L,
                    c->sh.o, c->sh.d, c->sh.bf, c->sh.Ls, c->sh.rp};
    for (auto p : f4) if (p) (void)hipFree(p);
    if (c->ps.smp_state) (void)hipFree(c->ps.smp_state);
    if (c->ps.smp_inc) (void)hipFree(c->ps.smp_inc);
    if (c->ps.depth) (void)hipFree(c->ps.depth);
    if (c->ps.weight) (void)hipFree(c->ps.weight);
    if (c->sh.path) (void)hipFree(c->sh.path);
    if (c->sh.pdfs) (void)hipFree(c->sh.pdfs);
    for (auto &q : c->d_queue) if (q) (void)hipFree(q), q = nullptr;
    // the k_paths records and camera stage are managed by ensure_records
    float4 *rec = c->ps.rec, *cam0 = c->ps.cam0, *cam1 = c->ps.cam1, *cam2 = c->ps.cam2, *cam4 = c->ps.cam4;
    uint4 *cam3 = c->ps.cam3, *cam5 = c->ps.cam5;
    float *camw = c->ps.camw;
    c->ps = {};
    c->ps.rec = rec;
    c->ps.cam0 = cam0; c->ps.cam1 = cam1; c->ps.cam2 = cam2; c->ps.cam3 = cam3; c->ps.cam4 = cam4; c->ps.cam5 = cam5;
    c->ps.camw = camw;
    c->sh = {};
    c->cap = 0;
}

void free_pixel_order(avr_context *c) {
    if (c->d_pix_order) ++c->order_gen;   // back to scanline order
    if (c->d_pix_order) (void)hipFree(c->d_pix_order);
    if (c->d_pix_slot) (void)hipFree(c->d_pix_slot);
    c->d_pix_order = c->d_pix_slot = nullptr;
    c->h_pix_slot.clear();
}

void free_records(avr_context *c) {
    for (void *p : {(void *)c->ps.rec, (void *)c->ps.cam0, (void *)c->ps.cam1, (void *)c->ps.cam2, (void *)c->ps.cam3,
                    (void *)c->ps.cam4, (void *)c->ps.cam5, (void *)c->ps.camw})
        if (p) (void)hipFree(p);
    c->ps.rec = c->ps.cam0 = c->ps.cam1 = c->ps.cam2 = c->ps.cam4 = nullptr;
    c->ps.cam3 = c->ps.cam5 = nullptr;
    c->ps.camw = nullptr;
    c->rec_cap = 0;
}

// k_paths' per-sample records (L, 16 B) and its camera stage (k_paths_camera: 6 x 16 B + the
// 4-B filter weight), independent of the wavefront SoA
int ensure_records(avr_context *c, long long n) {
    if (n <= c->rec_cap) return AVR_OK;
    free_records(c);
    HIP_TRY(dalloc(&c->ps.rec, (size_t)n));
    HIP_TRY(dalloc(&c->ps.cam0, (size_t)n));
    HIP_TRY(dalloc(&c->ps.cam1, (size_t)n));
    HIP_TRY(dalloc(&c->ps.cam2, (size_t)n));
    HIP_TRY(dalloc(&c->ps.cam3, (size_t)n));
    HIP_TRY(dalloc(&c->ps.cam4, (size_t)n));
    HIP_TRY(dalloc(&c->ps.cam5, (size_t)n));
    HIP_TRY(dalloc(&c->ps.camw, (size_t)n));
    c->rec_cap = n;
    return AVR_OK;
}

int ensure_paths(avr_context *c, long long n) {
    if (n <= c->cap) return AVR_OK;
    free_paths(c);
    const size_t N = (size_t)n;
    HIP_TRY(dalloc(&c->ps.o, N)); HIP_TRY(dalloc(&c->ps.d, N)); HIP_TRY(dalloc(&c->ps.lambda, N));
    HIP_TRY(dalloc(&c->ps.pdf, N)); HIP_TRY(dalloc(&c->ps.beta, N)); HIP_TRY(dalloc(&c->ps.r_u, N));
    HIP_TRY(dalloc(&c->ps.r_l, N)); HIP_TRY(dalloc(&c->ps.L, N));
    HIP_TRY(dalloc(&c->ps.smp_state, N)); HIP_TRY(dalloc(&c->ps.smp_inc, N)); HIP_TRY(dalloc(&c->ps.depth, N));
    HIP_TRY(dalloc(&c->ps.weight, N));
    HIP_TRY(dalloc(&c->sh.path, N)); HIP_TRY(dalloc(&c->sh.o, N)); HIP_TRY(dalloc(&c->sh.d, N));
    HIP_TRY(dalloc(&c->sh.bf, N)); HIP_TRY(dalloc(&c->sh.Ls, N)); HIP_TRY(dalloc(&c->sh.rp, N));
    HIP_TRY(dalloc(&c->sh.pdfs, N));
    HIP_TRY(dalloc(&c->d_queue[0], N)); HIP_TRY(dalloc(&c->d_queue[1], N));
    c->cap = n;
    return AVR_OK;
}

void copy_xf(avr::Xf &x, const float m[16]) {
    for (int i = 0; i < 12; ++i) x.m[i] = m[i];
}

int upload_table(float **dst, const float *src, size_t n, hipStream_t s) {
    if (*dst) { (void)hipFree(*dst); *dst = nullptr; }
    if (!src) return AVR_OK;
    HIP_TRY(dalloc(dst, n));
    HIP_TRY(hipMemcpyAsync(*dst, src, n * sizeof(float), hipMemcpyHostToDevice, s));
    return AVR_OK;
}

int blocks_for(long long n, int per = 256, int cap = 256 * 16) {
    long long b = (n + per - 1) / per;
    if (b < 1) b = 1;
    return (int)std::min<long long>(b, cap);
}

bool affine(const float m[16]) { return m[12] == 0 && m[13] == 0 && m[14] == 0 && m[15] == 1; }

void free_rgb(avr_context *c) {
    for (auto &p : c->d_rgb) if (p) (void)hipFree(p), p = nullptr;
    if (c->d_illum) (void)hipFree(c->d_illum), c->d_illum = nullptr;
    c->med.rgb_a = c->med.rgb_s = c->med.rgb_le = nullptr;
    c->med.illuminant = nullptr;
}

void free_vdb(avr_context *c) {
    for (int k = 0; k < 2; ++k) {
        if (c->d_vdb_slot[k]) (void)hipFree(c->d_vdb_slot[k]);
        if (c->d_vdb_leaves[k]) (void)hipFree(c->d_vdb_leaves[k]);
        if (c->d_vdb_tiles[k]) (void)hipFree(c->d_vdb_tiles[k]);
        c->d_vdb_slot[k] = nullptr;
        c->d_vdb_leaves[k] = c->d_vdb_tiles[k] = nullptr;
    }
    c->med.vdb = {};
    c->med.vdb_temp = {};
}

// Map::set (NanoVDB): the float inverse matrix and translation are roundings of the f64 map
template <typename GridT>
bool vdb_map(const avr_vdb_grid *G, GridT &g) {
    for (int k = 0; k < 9; ++k) {
        if (!std::isfinite(G->world_to_index[k])) return false;
        g.inv[k] = (float)G->world_to_index[k];
    }
    for (int r = 0; r < 3; ++r) g.vec[r] = (float)G->index_to_world[4 * r + 3];
    return true;
}

// GridData::mWorldBBox: the map (Map::applyMap, f64) of the 8 corners of [min, max + 1]
void vdb_world_bbox(const avr_vdb_grid *G, double lo[3], double hi[3]) {
    for (int k = 0; k < 3; ++k) { lo[k] = INFINITY; hi[k] = -INFINITY; }
    const double *M = G->index_to_world;
    for (int corner = 0; corner < 8; ++corner) {
        const double x = (corner & 1) ? G->index_bbox[3] + 1.0 : G->index_bbox[0];
        const double y = (corner & 2) ? G->index_bbox[4] + 1.0 : G->index_bbox[1];
        const double z = (corner & 4) ? G->index_bbox[5] + 1.0 : G->index_bbox[2];
        for (int r = 0; r < 3; ++r) {
            const double w = M[4 * r] * x + M[4 * r + 1] * y + M[4 * r + 2] * z + M[4 * r + 3];
            lo[r] = std::min(lo[r], w);
            hi[r] = std::max(hi[r], w);
        }
    }
}

// Flatten one tree into the block-slot layout of avr_vdb.h, then into its apron layout on
// the device (what the kernels sample)
int upload_vdb(avr_context *c, const avr_vdb_grid *G, int k, avr::vdb::Apron &g) {
    if (G->n_leaves < 0 || G->n_tiles < 0 || (G->n_leaves && (!G->leaf_origin || !G->leaf_values)) ||
        (G->n_tiles && (!G->tile_origin || !G->tile_size || !G->tile_value)))
        return fail(AVR_ERR_ARG, "bad vdb grid arrays");
    for (int a = 0; a < 3; ++a)
        if (G->index_bbox[a] > G->index_bbox[3 + a]) return fail(AVR_ERR_ARG, "empty vdb index bbox");
    g = {};
    if (!vdb_map(G, g)) return fail(AVR_ERR_ARG, "non-finite vdb world-to-index map");
    g.background = G->background;
    long long lo[3] = {LLONG_MAX, LLONG_MAX, LLONG_MAX}, hi[3] = {LLONG_MIN, LLONG_MIN, LLONG_MIN};
    auto extend = [&](const int *o, long long size) {
        for (int a = 0; a < 3; ++a) { lo[a] = std::min<long long>(lo[a], o[a]); hi[a] = std::max<long long>(hi[a], o[a] + size); }
    };
    for (int l = 0; l < G->n_leaves; ++l) {
        const int *o = G->leaf_origin + 3 * l;
        if ((o[0] & 7) || (o[1] & 7) || (o[2] & 7)) return fail(AVR_ERR_ARG, "leaf origin not a multiple of 8");
        extend(o, 8);
    }
    for (int t = 0; t < G->n_tiles; ++t) {
        const int *o = G->tile_origin + 3 * t;
        const int sz = G->tile_size[t];
        if (sz < 8 || (sz & 7) || (o[0] & 7) || (o[1] & 7) || (o[2] & 7))
            return fail(AVR_ERR_ARG, "tile origin/size not multiples of 8");
        extend(o, sz);
    }
    long long nb[3] = {0, 0, 0};
    if (G->n_leaves + G->n_tiles > 0)
        for (int a = 0; a < 3; ++a) nb[a] = (hi[a] - lo[a]) / 8;
    const long long nslot = nb[0] * nb[1] * nb[2];
    if (nslot > (1ll << 31)) return fail(AVR_ERR_ARG, "vdb grid extent too large (> 2^31 blocks)");
    std::vector<int> slot((size_t)std::max<long long>(nslot, 1), avr::vdb::kBackgroundSlot);
    auto sidx = [&](long long bx, long long by, long long bz) { return (size_t)((bz * nb[1] + by) * nb[0] + bx); };
    for (int t = 0; t < G->n_tiles; ++t) {
        const int *o = G->tile_origin + 3 * t;
        const long long s = G->tile_size[t] / 8;
        const long long bx0 = (o[0] - lo[0]) / 8, by0 = (o[1] - lo[1]) / 8, bz0 = (o[2] - lo[2]) / 8;
        for (long long bz = bz0; bz < bz0 + s; ++bz)
            for (long long by = by0; by < by0 + s; ++by)
                for (long long bx = bx0; bx < bx0 + s; ++bx) slot[sidx(bx, by, bz)] = -(t + 1);
    }
    for (int l = 0; l < G->n_leaves; ++l) {
        const int *o = G->leaf_origin + 3 * l;
        int &s = slot[sidx((o[0] - lo[0]) / 8, (o[1] - lo[1]) / 8, (o[2] - lo[2]) / 8)];
        if (s >= 0) return fail(AVR_ERR_ARG, "duplicate leaf origin");
        s = l;
    }
    avr::vdb::Grid base{};
    base.background = g.background;
    for (int q = 0; q < 9; ++q) base.inv[q] = g.inv[q];
    for (int q = 0; q < 3; ++q) base.vec[q] = g.vec[q];
    base.ox = nslot ? (int)lo[0] : 0; base.oy = nslot ? (int)lo[1] : 0; base.oz = nslot ? (int)lo[2] : 0;
    base.lnx = (int)nb[0]; base.lny = (int)nb[1]; base.lnz = (int)nb[2];
    // the base layout (slots, leaves, tiles) lives on the device only while the apron blocks
    // are filled from it (avr_vdb.h "Apron layout"): a lookup then reads one slot and one block
    std::vector<int> aslot;
    std::vector<long long> list;
    avr::vdb::build_apron_slots(slot.data(), base.lnx, base.lny, base.lnz, G->tile_value, G->n_tiles, G->background,
                                aslot, list);
    std::vector<float> consts((size_t)G->n_tiles + 1);
    for (int t = 0; t < G->n_tiles; ++t) consts[t] = G->tile_value[t];
    consts[G->n_tiles] = G->background;
    struct Tmp {
        int *slot = nullptr;
        float *leaves = nullptr, *tiles = nullptr;
        long long *list = nullptr;
        ~Tmp() {
            if (slot) (void)hipFree(slot);
            if (leaves) (void)hipFree(leaves);
            if (tiles) (void)hipFree(tiles);
            if (list) (void)hipFree(list);
        }
    } tmp;
    HIP_TRY(dalloc(&tmp.slot, slot.size()));
    HIP_TRY(hipMemcpyAsync(tmp.slot, slot.data(), slot.size() * sizeof(int), hipMemcpyHostToDevice, c->stream));
    const size_t nleaf = (size_t)G->n_leaves * 512;
    HIP_TRY(dalloc(&tmp.leaves, std::max<size_t>(nleaf, 1)));
    if (nleaf)
        HIP_TRY(hipMemcpyAsync(tmp.leaves, G->leaf_values, nleaf * sizeof(float), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(dalloc(&tmp.tiles, std::max<size_t>((size_t)G->n_tiles, 1)));
    if (G->n_tiles)
        HIP_TRY(hipMemcpyAsync(tmp.tiles, G->tile_value, G->n_tiles * sizeof(float), hipMemcpyHostToDevice, c->stream));
    base.slot = tmp.slot;
    base.leaves = tmp.leaves;
    base.tiles = tmp.tiles;
    HIP_TRY(dalloc(&c->d_vdb_slot[k], aslot.size()));
    HIP_TRY(hipMemcpyAsync(c->d_vdb_slot[k], aslot.data(), aslot.size() * sizeof(int), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(dalloc(&c->d_vdb_tiles[k], consts.size()));
    HIP_TRY(hipMemcpyAsync(c->d_vdb_tiles[k], consts.data(), consts.size() * sizeof(float), hipMemcpyHostToDevice,
                           c->stream));
    HIP_TRY(dalloc(&c->d_vdb_leaves[k], std::max<size_t>(list.size(), 1) * avr::vdb::kApronVals));
    if (!list.empty()) {
        HIP_TRY(dalloc(&tmp.list, list.size()));
        HIP_TRY(hipMemcpyAsync(tmp.list, list.data(), list.size() * sizeof(long long), hipMemcpyHostToDevice, c->stream));
        const long long nl = (long long)list.size();
        const int nblk = (int)std::min<long long>(nl, 1 << 20);
        hipLaunchKernelGGL(avr::k_vdb_apron, dim3(nblk), dim3(256), 0, c->stream, base, tmp.list, nl,
                           c->d_vdb_leaves[k]);
        HIP_TRY(hipGetLastError());
    }
    // the host vectors and the base layout die here: finish the copies and the fill first
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->vdb_napron[k] = (long long)list.size();
    g.slot = c->d_vdb_slot[k];
    g.blocks = c->d_vdb_leaves[k];
    g.consts = c->d_vdb_tiles[k];
    g.ox = base.ox; g.oy = base.oy; g.oz = base.oz;
    g.lnx = base.lnx; g.lny = base.lny; g.lnz = base.lnz;
    return AVR_OK;
}

// (Re)build the current medium's majorant grid at resolution mres on the device:
// GridMedium MaxValue per cell (media.cpp:229-246), RGBGridMedium's sigma scale x (max
// sigma_a + max sigma_s) (media.cpp:339-378), NanoVDBMedium's slop-widened cell maxima
// (media.cpp:585-613); Homogeneous / Cloud: one segment with majorant 1.
int build_majorant(avr_context *c, const int mres[3]) {
    avr::DevMedium &m = c->med;
    const int type = m.type;
    if (c->d_majorant) (void)hipFree(c->d_majorant);
    c->d_majorant = nullptr;
    const int nm = mres[0] * mres[1] * mres[2];
    if (c->d_occ) (void)hipFree(c->d_occ);
    c->d_occ = nullptr;
    m.occ = nullptr;
    // nm cells + one trailing 0: the read target of empty cells under the occupancy level
    HIP_TRY(dalloc(&c->d_majorant, (size_t)nm + 1));
    HIP_TRY(hipMemsetAsync(c->d_majorant + nm, 0, sizeof(float), c->stream));
    for (int i = 0; i < 3; ++i) {
        m.mres[i] = mres[i];
        m.fres[i] = (float)mres[i];
        m.fresm1[i] = (float)(mres[i] - 1);
    }
    if (type == 0) {
        hipLaunchKernelGGL(avr::k_majorant, dim3(nm), dim3(256), 0, c->stream, m.density, m.nx, m.ny, m.nz, mres[0],
                           mres[1], mres[2], c->d_majorant);
        HIP_TRY(hipGetLastError());
    } else if (type == 4) {
        hipLaunchKernelGGL(avr::k_majorant_rgb, dim3(nm), dim3(256), 0, c->stream, m.rgb_a, m.rgb_s, m.nx, m.ny, m.nz,
                           mres[0], mres[1], mres[2], m.rgb_sigma_scale, c->d_majorant);
        HIP_TRY(hipGetLastError());
    } else if (type == 3) {
        const int *b = c->vdb_ibbox;
        hipLaunchKernelGGL(avr::k_majorant_vdb, dim3(nm), dim3(256), 0, c->stream, m.vdb,
                           make_float3(m.bmin[0], m.bmin[1], m.bmin[2]), make_float3(m.bmax[0], m.bmax[1], m.bmax[2]),
                           make_int4(b[0], b[1], b[2], 0), make_int4(b[3], b[4], b[5], 0), mres[0], mres[1], mres[2],
                           c->d_majorant);
        HIP_TRY(hipGetLastError());
        const int nw = (nm + 63) / 64;
        if (c->majorant_occupancy && nw <= avr::kOccWords) {
            HIP_TRY(hipMalloc(&c->d_occ, (size_t)nw * sizeof(unsigned)));
            hipLaunchKernelGGL(avr::k_majorant_occupancy, dim3((nw + 255) / 256), dim3(256), 0, c->stream,
                               c->d_majorant, nm, c->d_occ, nw);
            HIP_TRY(hipGetLastError());
            m.occ = c->d_occ;
        }
    } else {   // single segment, sigma_maj = sigma_t * 1 (density <= 1 for the cloud)
        const float one = 1.f;
        HIP_TRY(hipMemcpyAsync(c->d_majorant, &one, sizeof(float), hipMemcpyHostToDevice, c->stream));
    }
    m.majorant = c->d_majorant;
    return AVR_OK;
}

int medium_common(avr_context *c, const float *d_density, int nx, int ny, int nz, const float bounds[6],
                  const float rfm[16], const float mfr[16], const float *sigma_a, const float *sigma_s, float g,
                  const float *Le, const float *Lescale, int lnx, int lny, int lnz, const int mres[3],
                  int type = 0, const float cloud[3] = nullptr) {
    if (!affine(rfm) || !affine(mfr)) return fail(AVR_ERR_ARG, "medium transforms must be affine");
    if (!sigma_a || !sigma_s) return fail(AVR_ERR_ARG, "sigma_a/sigma_s tables required");
    if (mres[0] < 1 || mres[1] < 1 || mres[2] < 1) return fail(AVR_ERR_ARG, "bad majorant resolution");
    if (Lescale && (lnx < 1 || lny < 1 || lnz < 1)) return fail(AVR_ERR_ARG, "bad Lescale grid");
    int rc;
    if ((rc = upload_table(&c->d_sigma_a, sigma_a, avr::kNTable, c->stream))) return rc;
    if ((rc = upload_table(&c->d_sigma_s, sigma_s, avr::kNTable, c->stream))) return rc;
    // Le and LeScale are always resident: a temperature grid attached later makes the medium
    // emissive without an Le spectrum (zeros), and LeScale defaults to pbrt's 1^3 {LeNorm}
    // grid with LeNorm = 1 (media.cpp:288-296)
    static const float zeros[avr::kNTable] = {};
    static const float one = 1.f;
    if ((rc = upload_table(&c->d_Le, Le ? Le : zeros, avr::kNTable, c->stream))) return rc;
    if (!Lescale) { Lescale = &one; lnx = lny = lnz = 1; }
    if ((rc = upload_table(&c->d_lescale, Lescale, (size_t)lnx * lny * lnz, c->stream))) return rc;
    avr::DevMedium &m = c->med;
    if (type != 3) free_vdb(c);
    if (type != 4) free_rgb(c);
    if (c->d_temperature) { (void)hipFree(c->d_temperature); c->d_temperature = nullptr; }
    m.temperature = nullptr;
    m.temp_scale = 1.f;
    m.temp_offset = 0.f;
    m.type = type;
    m.boundary = 0;   // the bounds box until avr_medium_boundary_sphere
    m.trace = nullptr;
    m.trace_count = nullptr;
    m.trace_cap = 0;
    m.cloud_density = cloud ? cloud[0] : 0.f;
    m.cloud_wispiness = cloud ? cloud[1] : 0.f;
    m.cloud_frequency = cloud ? cloud[2] : 0.f;
    m.density = d_density;
    m.nx = nx; m.ny = ny; m.nz = nz;
    for (int i = 0; i < 3; ++i) { m.bmin[i] = bounds[i]; m.bmax[i] = bounds[3 + i]; m.mres[i] = mres[i]; }
    m.unit_box = (m.bmax[0] - m.bmin[0] == 1.f && m.bmax[1] - m.bmin[1] == 1.f && m.bmax[2] - m.bmin[2] == 1.f) ? 1 : 0;
    copy_xf(m.render_from_medium, rfm);
    copy_xf(m.medium_from_render, mfr);
    m.sigma_a = c->d_sigma_a;
    m.sigma_s = c->d_sigma_s;
    m.g = g;
    m.hg = avr::hg_consts(g);
    m.fn[0] = (float)nx;
    m.fn[1] = (float)ny;
    m.fn[2] = (float)nz;
    c->gray = true;
    for (int i = 1; i < avr::kNTable; ++i) c->gray &= sigma_a[i] == sigma_a[0] && sigma_s[i] == sigma_s[0];
    c->med.gray_sigma_a = sigma_a[0];
    c->med.gray_sigma_s = sigma_s[0];
    // isEmissive = Le_spec.MaxValue() > 0 (media.cpp:238)
    bool emissive = false;
    if (Le) for (int i = 0; i < avr::kNTable; ++i) emissive |= Le[i] > 0;
    m.emissive = emissive ? 1 : 0;
    m.Le = c->d_Le;
    m.lescale = c->d_lescale;
    m.lnx = lnx; m.lny = lny; m.lnz = lnz;
    if ((rc = build_majorant(c, mres))) return rc;
    if (c->d_fat) { (void)hipFree(c->d_fat); c->d_fat = nullptr; }
    if (c->d_brick) { (void)hipFree(c->d_brick); c->d_brick = nullptr; }
    m.fat = nullptr;
    m.brick = nullptr;
    m.nb[0] = m.nb[1] = m.nb[2] = 0;
    if (c->grid_layout == 2 && type == 0) {
        // bricked copy: 8^3 base voxels + apron per brick (k_brickify), 1.42x the grid
        const int nb[3] = {(nx + 8) / 8, (ny + 8) / 8, (nz + 8) / 8};
        const long long nbricks = (long long)nb[0] * nb[1] * nb[2];
        const size_t bytes = (size_t)nbricks * avr::kBrickFloats * sizeof(float);
        size_t freeB = 0, totalB = 0;
        HIP_TRY(hipMemGetInfo(&freeB, &totalB));
        if (bytes + (8ull << 30) < freeB && hipMalloc((void **)&c->d_brick, bytes) == hipSuccess) {
            hipLaunchKernelGGL(avr::k_brickify, dim3(blocks_for(nbricks * avr::kBrickFloats, 256, 256 * 64)), dim3(256), 0,
                               c->stream, d_density, nx, ny, nz, nb[0], nb[1], nbricks, c->d_brick);
            HIP_TRY(hipGetLastError());
            m.brick = c->d_brick;
            for (int a = 0; a < 3; ++a) m.nb[a] = nb[a];
        } else {
            (void)hipGetLastError();
            c->d_brick = nullptr;
        }
    }
    if (c->grid_layout == 1 && type == 0) {
        const size_t nfat = (size_t)(nx + 1) * (ny + 1) * (nz + 1);
        size_t freeB = 0, totalB = 0;
        HIP_TRY(hipMemGetInfo(&freeB, &totalB));
        // keep >= 8 GiB for path state / film / other ranks' traffic
        if (nfat * 32 + (8ull << 30) < freeB && hipMalloc((void **)&c->d_fat, nfat * 32) == hipSuccess) {
            hipLaunchKernelGGL(avr::k_fatten, dim3(blocks_for((long long)nfat, 256, 256 * 64)), dim3(256), 0,
                               c->stream, d_density, nx, ny, nz, c->d_fat);
            HIP_TRY(hipGetLastError());
            m.fat = c->d_fat;
        } else {
            (void)hipGetLastError();
            c->d_fat = nullptr;
        }
    }
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->has_medium = true;
    return AVR_OK;
}

}  // namespace

extern "C" {

const char *avr_last_error(void) { return g_err.c_str(); }


// Setup calls replace or free device buffers that queued work on the context's stream may
// still read, and readbacks through hipMemcpy (the null stream) do not order against a
// non-blocking stream: both first drain the context's stream.
#define AVR_QUIESCE(c)                                                                              \
    do {                                                                                            \
        if ((c) && (c)->stream) {                                                                   \
            hipError_t qe_ = hipStreamSynchronize((c)->stream);                                     \
            if (qe_ == hipSuccess && (c)->tstream) qe_ = hipStreamSynchronize((c)->tstream);        \
            if (qe_ != hipSuccess) return fail(AVR_ERR_HIP, std::string("stream: ") + hipGetErrorString(qe_)); \
        }                                                                                           \
    } while (0)

int avr_context_create(int device, long long max_paths, avr_context **out) {
    if (!out) return fail(AVR_ERR_ARG, "null out");
    // path ids (s * pixels + pixel) are 32-bit in the kernels: passes hold < 2^31 paths
    if (max_paths > INT_MAX) return fail(AVR_ERR_ARG, "max_paths above 2^31 - 1 (32-bit path ids)");
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(AVR_ERR_ARG, "device index out of range");
    HIP_TRY(hipSetDevice(device));
    auto *c = new avr_context();
    c->device = device;
    if (max_paths > 0) c->max_paths = max_paths, c->max_paths_set = true;
    // the path stream at the greatest priority, the side stream (ptab_spec's tables built
    // ahead) at the least, so the dispatcher serves the side stream's blocks only from CUs the
    // path kernels leave free
    int prLeast = 0, prGreatest = 0;
    hipError_t e = hipDeviceGetStreamPriorityRange(&prLeast, &prGreatest);
    if (e == hipSuccess) e = hipStreamCreateWithPriority(&c->own_stream, hipStreamNonBlocking, prGreatest);
    if (e == hipSuccess) e = hipStreamCreateWithPriority(&c->tstream, hipStreamNonBlocking, prLeast);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_cam, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_tab, hipEventDisableTiming);
    if (e != hipSuccess) { (void)avr_context_destroy(c); return fail(AVR_ERR_HIP, hipGetErrorString(e)); }
    c->stream = c->own_stream;
    if (dalloc(&c->d_counts, 4) != hipSuccess || dalloc(&c->d_stats, avr::kNumStats + 8) != hipSuccess ||
        hipHostMalloc((void **)&c->h_count, sizeof(int) * 4) != hipSuccess) {
        delete c;
        return fail(AVR_ERR_HIP, "context allocation failed");
    }
    if (dalloc(&c->d_heads, 9) != hipSuccess || hipMemset(c->d_heads, 0xff, 9 * sizeof(int)) != hipSuccess ||
        hipMemset(c->d_stats, 0, sizeof(unsigned long long) * (avr::kNumStats + 8)) != hipSuccess) {
        delete c;
        return fail(AVR_ERR_HIP, "context allocation failed");
    }
    {
        // persistent grid per k_paths variant: every admitted block resident. No block ever
        // waits on another (work is pulled from counters), so the API's answer is safe as is.
        // The variants differ in VGPRs (gray: 3 waves/SIMD, 4-wavelength: 2), so each gets
        // its own grid.
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, device) != hipSuccess) {
            delete c;
            return fail(AVR_ERR_HIP, "device query failed");
        }
        // slot 32*image + 8*medium(0 grid, 1 vdb, 2 rgb, 3 homogeneous/cloud) + 4*zsobol + 2*emissive + gray; RGB grids
        // are never gray (their gray slots hold the 4-wavelength kernel)
#define AVR_KP(em, gr, zs, med, im, fa) avr::k_paths<em, (med == 4 ? false : gr), zs, med, im, fa>
#define AVR_KP4(zs, med, im, fa)                                                                                      \
    AVR_KP(false, false, zs, med, im, fa), AVR_KP(false, true, zs, med, im, fa), AVR_KP(true, false, zs, med, im, fa), \
        AVR_KP(true, true, zs, med, im, fa)
#define AVR_KP12(med, im, fa) AVR_KP4(0, med, im, fa), AVR_KP4(2, med, im, fa), AVR_KP4(3, med, im, fa)
#define AVR_KP48(im, fa) AVR_KP12(0, im, fa), AVR_KP12(3, im, fa), AVR_KP12(4, im, fa), AVR_KP12(1, im, fa)
        void (*kerns[avr_context::kNumPaths])(avr::Params) = {AVR_KP48(false, false), AVR_KP48(true, false),
                                                              AVR_KP48(false, true), AVR_KP48(true, true)};
#undef AVR_KP48
#undef AVR_KP12
#undef AVR_KP4
#undef AVR_KP
        for (int k = 0; k < avr_context::kNumPaths; ++k) {
            int blocksPerCU = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocksPerCU, kerns[k], 256, 0) != hipSuccess) {
                delete c;
                return fail(AVR_ERR_HIP, "occupancy query failed");
            }
            c->paths_grid[k] = prop.multiProcessorCount * std::max(1, blocksPerCU);
            c->kpaths[k] = kerns[k];
        }
    }
    *out = c;
    return AVR_OK;
}

int avr_set_grid_layout(avr_context *c, int layout) {
    AVR_QUIESCE(c);
    if (!c || layout < 0 || layout > 2) return fail(AVR_ERR_ARG, "grid layout must be 0 (linear), 1 (fat) or 2 (bricked)");
    c->grid_layout = layout;
    return AVR_OK;
}

int avr_grid_layout_active(avr_context *c) { return !c ? 0 : (c->d_fat ? 1 : (c->med.brick ? 2 : 0)); }

int avr_set_dda_budget(avr_context *c, int cells) {
    if (!c || cells < 0) return fail(AVR_ERR_ARG, "DDA budget must be >= 1 cell (0: default)");
    c->dda_budget = cells;
    return AVR_OK;
}

int avr_set_refill_min(avr_context *c, int lanes) {
    if (!c || lanes < 0 || lanes > 64) return fail(AVR_ERR_ARG, "refill threshold must be 0..64 lanes (0 = default)");
    c->refill_min = lanes;
    return AVR_OK;
}

int avr_set_render_mode(avr_context *c, int mode) {
    AVR_QUIESCE(c);
    if (!c || (mode != 0 && mode != 1)) return fail(AVR_ERR_ARG, "render mode must be 0 (replay) or 1 (fast)");
    c->render_mode = mode;
    return AVR_OK;
}

int avr_set_ray_binning(avr_context *c, int on) {
    AVR_QUIESCE(c);
    if (!c || (on != 0 && on != 1)) return fail(AVR_ERR_ARG, "ray binning must be 0 or 1");
    c->ray_binning = on;
    return AVR_OK;
}

int avr_set_pass_table_ahead(avr_context *c, int on) {
    AVR_QUIESCE(c);
    if (!c || (on != 0 && on != 1)) return fail(AVR_ERR_ARG, "pass table ahead must be 0 or 1");
    c->ptab_spec = on;
    c->spec_valid = false;   // (the side stream is idle after the quiesce)
    return AVR_OK;
}

int avr_set_majorant_occupancy(avr_context *c, int on) {
    AVR_QUIESCE(c);
    if (!c || (on != 0 && on != 1)) return fail(AVR_ERR_ARG, "majorant occupancy must be 0 or 1");
    HIP_TRY(hipSetDevice(c->device));
    c->majorant_occupancy = on;
    if (c->has_medium) {   // rebuild the current majorant (same values) with / without the level
        const int r[3] = {c->med.mres[0], c->med.mres[1], c->med.mres[2]};
        return build_majorant(c, r);
    }
    return AVR_OK;
}

int avr_set_kernel_mode(avr_context *c, int mode) {
    if (!c || (mode != 0 && mode != 1)) return fail(AVR_ERR_ARG, "kernel mode must be 0 (persistent) or 1 (wavefront)");
    c->kernel_mode = mode;
    return AVR_OK;
}

int avr_context_destroy(avr_context *c) {
    if (!c) return AVR_OK;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    if (c->tstream) (void)hipStreamSynchronize(c->tstream);
    release_comms(c);
    free_paths(c);
    free_records(c);
    float *fs[] = {c->d_density_owned, c->d_sigma_a, c->d_sigma_s, c->d_Le, c->d_lescale, c->d_majorant,
                   c->d_lightL, c->d_xyz};
    if (c->d_lights) (void)hipFree(c->d_lights);
    for (auto p : fs) if (p) (void)hipFree(p);
    if (c->film.rgb_sum) (void)hipFree(c->film.rgb_sum);
    if (c->film.w_sum) (void)hipFree(c->film.w_sum);
    if (c->film.bucket_sum) (void)hipFree(c->film.bucket_sum);
    if (c->d_counts) (void)hipFree(c->d_counts);
    if (c->d_heads) (void)hipFree(c->d_heads);
    for (int *b : {c->d_bin_keys, c->d_bin_out, c->d_bin_hist}) if (b) (void)hipFree(b);
    if (c->d_planes) (void)hipFree(c->d_planes);
    if (c->d_occ) (void)hipFree(c->d_occ);
    if (c->d_advance) (void)hipFree(c->d_advance);
    if (c->d_filter) (void)hipFree(c->d_filter);
    if (c->d_temperature) (void)hipFree(c->d_temperature);
    free_vdb(c);
    free_rgb(c);
    for (auto &b : c->d_light_img) if (b) (void)hipFree(b), b = nullptr;
    if (c->d_zs_table) (void)hipFree(c->d_zs_table);
    for (int b = 0; b < 2; ++b) {
        if (c->d_zs_ptab[b]) (void)hipFree(c->d_zs_ptab[b]);
        if (c->d_zs_ctab[b]) (void)hipFree(c->d_zs_ctab[b]);
    }
    if (c->d_zs_atab) (void)hipFree(c->d_zs_atab);
    if (c->d_image) (void)hipFree(c->d_image);
    if (c->d_reference) (void)hipFree(c->d_reference);
    if (c->d_metric) (void)hipFree(c->d_metric);
    if (c->d_fat) (void)hipFree(c->d_fat);
    if (c->d_brick) (void)hipFree(c->d_brick);
    free_pixel_order(c);
    if (c->d_stats) (void)hipFree(c->d_stats);
    if (c->h_count) (void)hipHostFree(c->h_count);
    for (auto e : c->evpool) (void)hipEventDestroy(e);
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    if (c->tstream) (void)hipStreamDestroy(c->tstream);
    if (c->ev_cam) (void)hipEventDestroy(c->ev_cam);
    if (c->ev_tab) (void)hipEventDestroy(c->ev_tab);
    delete c;
    return AVR_OK;
}

int avr_set_stream(avr_context *c, void *s) {
    if (!c) return fail(AVR_ERR_ARG, "null context");
    c->stream = s ? (hipStream_t)s : c->own_stream;
    return AVR_OK;
}

int avr_medium_grid(avr_context *c, const float *density, int nx, int ny, int nz, const float bounds[6],
                    const float rfm[16], const float mfr[16], const float *sigma_a, const float *sigma_s, float g,
                    const float *Le, const float *Lescale, int lnx, int lny, int lnz, const int mres[3]) {
    AVR_QUIESCE(c);
    if (!c || !density || nx < 1 || ny < 1 || nz < 1) return fail(AVR_ERR_ARG, "bad grid");
    HIP_TRY(hipSetDevice(c->device));
    if (c->d_density_owned) { (void)hipFree(c->d_density_owned); c->d_density_owned = nullptr; }
    const size_t n = (size_t)nx * ny * nz;
    if (n > (size_t)INT32_MAX) return fail(AVR_ERR_ARG, "grid too large for int32 indexing (containers.h:834)");
    HIP_TRY(dalloc(&c->d_density_owned, n));
    HIP_TRY(hipMemcpyAsync(c->d_density_owned, density, n * sizeof(float), hipMemcpyHostToDevice, c->stream));
    return medium_common(c, c->d_density_owned, nx, ny, nz, bounds, rfm, mfr, sigma_a, sigma_s, g, Le, Lescale, lnx,
                         lny, lnz, mres);
}

int avr_medium_grid_device(avr_context *c, const float *d_density, int nx, int ny, int nz, const float bounds[6],
                           const float rfm[16], const float mfr[16], const float *sigma_a, const float *sigma_s,
                           float g, const float *Le, const float *Lescale, int lnx, int lny, int lnz,
                           const int mres[3]) {
    AVR_QUIESCE(c);
    if (!c || !d_density || nx < 1 || ny < 1 || nz < 1) return fail(AVR_ERR_ARG, "bad grid");
    if ((size_t)nx * ny * nz > (size_t)INT32_MAX) return fail(AVR_ERR_ARG, "grid too large for int32 indexing");
    HIP_TRY(hipSetDevice(c->device));
    if (c->d_density_owned) { (void)hipFree(c->d_density_owned); c->d_density_owned = nullptr; }
    return medium_common(c, d_density, nx, ny, nz, bounds, rfm, mfr, sigma_a, sigma_s, g, Le, Lescale, lnx, lny, lnz,
                         mres);
}

int avr_medium_temperature(avr_context *c, const float *temperature, float temperature_scale,
                           float temperature_offset) {
    AVR_QUIESCE(c);
    if (!c || !temperature) return fail(AVR_ERR_ARG, "null temperature grid");
    if (!c->has_medium || c->med.type != 0) return fail(AVR_ERR_STATE, "temperature needs a grid medium first");
    if (!c->med.Le || !c->med.lescale) return fail(AVR_ERR_STATE, "medium emission tables missing");
    if (c->med.Le && c->med.emissive && !c->med.temperature)
        return fail(AVR_ERR_ARG, "both \"Le\" and \"temperature\" given (media.cpp:283-284)");
    HIP_TRY(hipSetDevice(c->device));
    const size_t n = (size_t)c->med.nx * c->med.ny * c->med.nz;
    if (c->d_temperature) (void)hipFree(c->d_temperature);
    c->d_temperature = nullptr;
    HIP_TRY(dalloc(&c->d_temperature, n));
    HIP_TRY(hipMemcpy(c->d_temperature, temperature, n * sizeof(float), hipMemcpyHostToDevice));
    c->med.temperature = c->d_temperature;
    c->med.temp_scale = temperature_scale;
    c->med.temp_offset = temperature_offset;
    c->med.emissive = 1;   // isEmissive = temperatureGrid ? true : ... (media.cpp:238)
    return AVR_OK;
}

int avr_medium_homogeneous(avr_context *c, const float bounds[6], const float rfm[16], const float mfr[16],
                           const float *sigma_a, const float *sigma_s, float g, const float *Le) {
    AVR_QUIESCE(c);
    if (!c || !bounds || !rfm || !mfr) return fail(AVR_ERR_ARG, "null medium argument");
    HIP_TRY(hipSetDevice(c->device));
    static const float one = 1.f;
    const int mres[3] = {1, 1, 1};
    return medium_common(c, nullptr, 1, 1, 1, bounds, rfm, mfr, sigma_a, sigma_s, g, Le, Le ? &one : nullptr, 1, 1, 1,
                         mres, 1, nullptr);
}

int avr_medium_cloud(avr_context *c, const float bounds[6], const float rfm[16], const float mfr[16],
                     const float *sigma_a, const float *sigma_s, float g, float density, float wispiness,
                     float frequency) {
    AVR_QUIESCE(c);
    if (!c || !bounds || !rfm || !mfr) return fail(AVR_ERR_ARG, "null medium argument");
    HIP_TRY(hipSetDevice(c->device));
    const int mres[3] = {1, 1, 1};
    const float cloud[3] = {density, wispiness, frequency};
    return medium_common(c, nullptr, 1, 1, 1, bounds, rfm, mfr, sigma_a, sigma_s, g, nullptr, nullptr, 1, 1, 1, mres,
                         2, cloud);
}

int avr_medium_nanovdb(avr_context *c, const avr_vdb_grid *density, const avr_vdb_grid *temperature, const float rfm[16],
                       const float mfr[16], const float *sigma_a, const float *sigma_s, float g, float Lescale,
                       float temperature_offset, float temperature_scale) {
    AVR_QUIESCE(c);
    if (!c || !density || !rfm || !mfr) return fail(AVR_ERR_ARG, "null medium argument");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(c->stream));
    free_vdb(c);
    int rc;
    avr::vdb::Apron gd{}, gt{};
    if ((rc = upload_vdb(c, density, 0, gd))) return rc;
    if (temperature && (rc = upload_vdb(c, temperature, 1, gt))) return rc;
    // bounds: density world bbox, union the temperature grid's (media.cpp:531-549)
    double lo[3], hi[3];
    vdb_world_bbox(density, lo, hi);
    float bounds[6];
    for (int a = 0; a < 3; ++a) { bounds[a] = (float)lo[a]; bounds[3 + a] = (float)hi[a]; }
    if (temperature) {
        vdb_world_bbox(temperature, lo, hi);
        for (int a = 0; a < 3; ++a) {
            bounds[a] = std::min(bounds[a], (float)lo[a]);
            bounds[3 + a] = std::max(bounds[3 + a], (float)hi[a]);
        }
    }
    for (int a = 0; a < 6; ++a) c->vdb_ibbox[a] = density->index_bbox[a];
    c->med.vdb = gd;
    c->med.vdb_temp = gt;
    const int mres[3] = {64, 64, 64};   // majorantGrid(Bounds3f(), {64, 64, 64}) (media.cpp:520)
    if ((rc = medium_common(c, nullptr, 1, 1, 1, bounds, rfm, mfr, sigma_a, sigma_s, g, nullptr, nullptr, 1, 1, 1, mres,
                            3, nullptr)))
        return rc;
    // the density grid's fat copy (avr_set_grid_layout 1, as for GridMedium): 32 B per base voxel
    // of every apron block, when it fits in free HBM with 8 GiB to spare
    if (c->grid_layout == 1 && c->vdb_napron[0] > 0) {
        const size_t nfat = (size_t)c->vdb_napron[0] * 512;
        size_t freeB = 0, totalB = 0;
        HIP_TRY(hipMemGetInfo(&freeB, &totalB));
        if (nfat * 32 + (8ull << 30) < freeB && hipMalloc((void **)&c->d_fat, nfat * 32) == hipSuccess) {
            hipLaunchKernelGGL(avr::k_vdb_fat, dim3(blocks_for((long long)nfat, 256, 256 * 64)), dim3(256), 0, c->stream,
                               c->med.vdb.blocks, c->vdb_napron[0], c->d_fat);
            HIP_TRY(hipGetLastError());
            HIP_TRY(hipStreamSynchronize(c->stream));
            c->med.vdb.fat = reinterpret_cast<const float *>(c->d_fat);
        } else {
            (void)hipGetLastError();
            c->d_fat = nullptr;
        }
    }
    c->med.vdb_lescale = Lescale;
    c->med.temp_offset = temperature_offset;
    c->med.temp_scale = temperature_scale;
    c->med.emissive = temperature ? 1 : 0;
    return AVR_OK;
}

static int medium_rgbgrid(avr_context *c, int nx, int ny, int nz, const float bounds[6], const float rfm[16],
                          const float mfr[16], const float *sigma_a, const float *sigma_s, float sigma_scale, float g,
                          const float *Le, const float *illuminant, float Le_scale, bool on_device) {
    AVR_QUIESCE(c);
    if (!c || !bounds || !rfm || !mfr) return fail(AVR_ERR_ARG, "null medium argument");
    if (nx < 1 || ny < 1 || nz < 1) return fail(AVR_ERR_ARG, "bad grid");
    if (!sigma_a && !sigma_s)
        return fail(AVR_ERR_ARG, "RGB grid requires \"sigma_a\" and/or \"sigma_s\" (media.cpp:404-406)");
    if (Le && !sigma_a) return fail(AVR_ERR_ARG, "RGB grid requires \"sigma_a\" if \"Le\" given (media.cpp:418-419)");
    if (Le && !illuminant) return fail(AVR_ERR_ARG, "Le needs the colour space's illuminant table");
    const size_t n = (size_t)nx * ny * nz;
    if (n > (size_t)INT32_MAX) return fail(AVR_ERR_ARG, "grid too large for int32 indexing");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(c->stream));
    free_rgb(c);
    const float *src[3] = {sigma_a, sigma_s, Le};
    const float4 *grid[3] = {nullptr, nullptr, nullptr};
    for (int k = 0; k < 3; ++k) {
        if (!src[k]) continue;
        if (on_device) {   // the caller's device arrays, adopted (not copied)
            grid[k] = reinterpret_cast<const float4 *>(src[k]);
            continue;
        }
        HIP_TRY(dalloc(&c->d_rgb[k], n));
        HIP_TRY(hipMemcpyAsync(c->d_rgb[k], src[k], n * sizeof(float4), hipMemcpyHostToDevice, c->stream));
        grid[k] = c->d_rgb[k];
    }
    int rc;
    if (Le && (rc = upload_table(&c->d_illum, illuminant, avr::kNTable, c->stream))) return rc;
    c->med.rgb_a = grid[0];
    c->med.rgb_s = grid[1];
    c->med.rgb_le = grid[2];
    c->med.illuminant = c->d_illum;
    c->med.rgb_sigma_scale = sigma_scale;
    c->med.rgb_le_scale = Le_scale;
    // SampleRay's sigma_t = 1 (media.h:417): tables {1} + {0} make the segments' sigma_maj the
    // majorant value itself; SamplePoint reads the RGB grids instead of the tables
    static float ones[avr::kNTable], zeros[avr::kNTable];
    for (int i = 0; i < avr::kNTable; ++i) ones[i] = 1.f;
    const int mres[3] = {16, 16, 16};   // majorantGrid(bounds, {16, 16, 16}) (media.cpp:352)
    if ((rc = medium_common(c, nullptr, nx, ny, nz, bounds, rfm, mfr, ones, zeros, g, nullptr, nullptr, 1, 1, 1, mres,
                            4, nullptr)))
        return rc;
    c->med.emissive = (Le && Le_scale > 0) ? 1 : 0;   // IsEmissive (media.h:374)
    return AVR_OK;
}

int avr_medium_rgbgrid(avr_context *c, int nx, int ny, int nz, const float bounds[6], const float rfm[16],
                       const float mfr[16], const float *sigma_a, const float *sigma_s, float sigma_scale, float g,
                       const float *Le, const float *illuminant, float Le_scale) {
    return medium_rgbgrid(c, nx, ny, nz, bounds, rfm, mfr, sigma_a, sigma_s, sigma_scale, g, Le, illuminant, Le_scale,
                          false);
}

int avr_medium_rgbgrid_device(avr_context *c, int nx, int ny, int nz, const float bounds[6], const float rfm[16],
                              const float mfr[16], const float *d_sigma_a, const float *d_sigma_s, float sigma_scale,
                              float g, const float *d_Le, const float *illuminant, float Le_scale) {
    return medium_rgbgrid(c, nx, ny, nz, bounds, rfm, mfr, d_sigma_a, d_sigma_s, sigma_scale, g, d_Le, illuminant,
                          Le_scale, true);
}

int avr_generate_rgb_explosion(avr_context *c, float *d_sigma_a, float *d_sigma_s, float *d_Le, int n, long long first,
                               long long count) {
    if (!c || !d_sigma_a || !d_sigma_s || !d_Le || n < 1 || count < 0 || first < 0 ||
        first + count > (long long)n * n * n)
        return fail(AVR_ERR_ARG, "bad rgb explosion args");
    HIP_TRY(hipSetDevice(c->device));
    hipLaunchKernelGGL(avr::k_rgb_explosion, dim3(blocks_for(count, 256, 256 * 32)), dim3(256), 0, c->stream,
                       reinterpret_cast<float4 *>(d_sigma_a), reinterpret_cast<float4 *>(d_sigma_s),
                       reinterpret_cast<float4 *>(d_Le), n, first, count);
    HIP_TRY(hipGetLastError());
    return AVR_OK;
}

int avr_medium_bounds(avr_context *c, float bounds[6]) {
    AVR_QUIESCE(c);
    if (!c || !c->has_medium || !bounds) return fail(AVR_ERR_STATE, "no medium");
    for (int a = 0; a < 3; ++a) { bounds[a] = c->med.bmin[a]; bounds[3 + a] = c->med.bmax[a]; }
    return AVR_OK;
}

int avr_generate_cloud(avr_context *c, float *d_out, int n, long long first, long long count, float density,
                       float wispiness, float frequency) {
    if (!c || !d_out || n < 1 || count < 0) return fail(AVR_ERR_ARG, "bad cloud args");
    HIP_TRY(hipSetDevice(c->device));
    hipLaunchKernelGGL(avr::k_cloud, dim3(blocks_for(count, 256, 256 * 32)), dim3(256), 0, c->stream, d_out, n, first,
                       count, density, wispiness, frequency);
    HIP_TRY(hipGetLastError());
    return AVR_OK;
}

int avr_read_majorant(avr_context *c, float *out) {
    AVR_QUIESCE(c);
    if (!c || !c->has_medium || !out) return fail(AVR_ERR_STATE, "no medium");
    const int nm = c->med.mres[0] * c->med.mres[1] * c->med.mres[2];
    HIP_TRY(hipMemcpyAsync(out, c->d_majorant, nm * sizeof(float), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return AVR_OK;
}

int avr_medium_boundary_sphere(avr_context *c, const float center[3], float radius) {
    AVR_QUIESCE(c);
    if (!c || !c->has_medium) return fail(AVR_ERR_STATE, "no medium");
    if (radius > 0 && !center) return fail(AVR_ERR_ARG, "null sphere centre");
    if (!(radius <= 0 || std::isfinite(radius))) return fail(AVR_ERR_ARG, "sphere radius must be finite");
    c->med.boundary = radius > 0 ? 1 : 0;
    for (int i = 0; i < 3; ++i) c->med.sph[i] = radius > 0 ? center[i] : 0.f;
    c->med.sph[3] = radius > 0 ? radius : 0.f;
    return AVR_OK;
}

int avr_medium_boundary_convex(avr_context *c, const float *planes, int n_planes) {
    AVR_QUIESCE(c);
    if (!c || !c->has_medium) return fail(AVR_ERR_STATE, "no medium");
    if (n_planes < 0 || n_planes > 256 || (n_planes > 0 && !planes))
        return fail(AVR_ERR_ARG, "convex interface: 0..256 planes {nx, ny, nz, h}");
    for (int i = 0; i < 4 * n_planes; ++i)
        if (!std::isfinite(planes[i])) return fail(AVR_ERR_ARG, "convex interface planes must be finite");
    HIP_TRY(hipSetDevice(c->device));
    if (c->d_planes) { (void)hipFree(c->d_planes); c->d_planes = nullptr; }
    c->med.planes = nullptr;
    c->med.n_planes = 0;
    if (n_planes == 0) {
        if (c->med.boundary == 2) c->med.boundary = 0;
        return AVR_OK;
    }
    HIP_TRY(dalloc(&c->d_planes, (size_t)n_planes));
    HIP_TRY(hipMemcpyAsync(c->d_planes, planes, 4 * sizeof(float) * n_planes, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->med.planes = c->d_planes;
    c->med.n_planes = n_planes;
    c->med.boundary = 2;
    return AVR_OK;
}

int avr_record_lookups(avr_context *c, void *d_points, long long cap, void *d_count) {
    AVR_QUIESCE(c);
    if (!c || !c->has_medium) return fail(AVR_ERR_STATE, "no medium");
    if (d_points && (cap < 0 || !d_count)) return fail(AVR_ERR_ARG, "lookup trace needs a capacity and a counter");
    c->med.trace = (float4 *)d_points;
    c->med.trace_count = d_points ? (unsigned long long *)d_count : nullptr;
    c->med.trace_cap = d_points ? cap : 0;
    return AVR_OK;
}

int avr_density_fetch(avr_context *c, const void *d_points, long long n, float *d_out, float *ms) {
    AVR_QUIESCE(c);
    if (!c || !c->has_medium || c->med.type != 0) return fail(AVR_ERR_STATE, "density fetch needs a GridMedium");
    if (n < 0 || (n > 0 && (!d_points || !d_out))) return fail(AVR_ERR_ARG, "bad density fetch batch");
    HIP_TRY(hipSetDevice(c->device));
    hipEvent_t e0 = nullptr, e1 = nullptr;
    HIP_TRY(hipEventCreate(&e0));
    HIP_TRY(hipEventCreate(&e1));
    const int blocks = (int)std::min<long long>((n + 255) / 256, 256LL * 64);
    HIP_TRY(hipEventRecord(e0, c->stream));
    if (n > 0)
        hipLaunchKernelGGL(avr::k_density_fetch, dim3(blocks), dim3(256), 0, c->stream, c->med,
                           (const float4 *)d_points, n, d_out);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(e1, c->stream));
    HIP_TRY(hipEventSynchronize(e1));
    float t = 0.f;
    HIP_TRY(hipEventElapsedTime(&t, e0, e1));
    if (ms) *ms = t;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return AVR_OK;
}

int avr_set_majorant_res(avr_context *c, const int res[3]) {
    AVR_QUIESCE(c);
    if (!c || !c->has_medium || !res) return fail(AVR_ERR_STATE, "no medium");
    if (c->med.type == 1 || c->med.type == 2)
        return fail(AVR_ERR_ARG, "homogeneous / cloud media have a single majorant segment");
    if (res[0] < 1 || res[1] < 1 || res[2] < 1 || res[0] > 255 || res[1] > 255 || res[2] > 255)
        return fail(AVR_ERR_ARG, "majorant resolution must be 1..255 per axis");
    HIP_TRY(hipSetDevice(c->device));
    int rc = build_majorant(c, res);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(c->stream));
    return AVR_OK;
}

// The probe loop of the device-side tuners (avr_tune_majorant, avr_tune_walk): render
// [spp_begin, spp_end) after setup(k) for each k < n, twice (k ascending, then descending) —
// plus one untimed render after setup(0) first (the first render after a scene change builds
// one-off tables) — timed with HIP events on the context stream; each candidate's time is the
// faster of its two probes; *bestk = the fastest, ms[k] the times when non-null. The
// film sums are saved before and restored after (also when a probe fails; the first error is
// kept); restore() then re-applies the chosen (or, after a failure, the original) setting.
// prefer >= 0: that candidate (the default schedule) is kept unless the fastest probe beats it
// by more than kProbeNoise — the probes' run-to-run spread — so the choice is reproducible. Its
// time is the fastest probe of every candidate marked in `same` (those that run the very same
// schedule, e.g. refill 0 and refill 32 when 32 is the default), not one noisy probe.
constexpr float kProbeNoise = 0.02f;
extern "C++" {
template <typename Setup, typename Restore>
static int probe_loop(avr_context *c, int n, Setup setup, Restore restore, int spp_begin, int spp_end, int seed,
                      int max_depth, int *bestk, float *ms, int prefer = -1, const std::vector<char> *same = nullptr) {
    HIP_TRY(hipSetDevice(c->device));
    const size_t np = (size_t)c->film.width * c->film.height;
    const size_t nd = (4 + 2 * (size_t)std::max(0, c->film.nbuckets)) * np;
    double *saved = nullptr;
    HIP_TRY(dalloc(&saved, nd));
    int rc = avr_film_export_device(c, saved);
    const bool haveSaved = rc == AVR_OK;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (!rc && (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess)) rc = fail(AVR_ERR_HIP, "event");
    float best = -1.f, tPrefer = -1.f;
    *bestk = 0;
    // the probes render one range over and over: no pass table built ahead on the side stream
    // (a probe would wait for the previous one's), restored afterwards
    const int spec0 = c->ptab_spec;
    c->ptab_spec = 0;
    c->spec_valid = false;
    // two rounds over the candidates, the second in reverse order, each candidate's time the
    // faster of its two probes (one probe each left 1^3 and 2^3 of fast mode to noise)
    std::vector<float> tmin(n, -1.f);
    for (int it = -1; it < 2 * n && !rc; ++it) {
        const int k = it < 0 ? -1 : (it < n ? it : 2 * n - 1 - it);
        if ((rc = setup(k < 0 ? 0 : k))) break;
        if (hipEventRecord(e0, c->stream) != hipSuccess) { rc = fail(AVR_ERR_HIP, "event record"); break; }
        if ((rc = avr_render(c, spp_begin, spp_end, seed, max_depth))) break;
        if (hipEventRecord(e1, c->stream) != hipSuccess || hipEventSynchronize(e1) != hipSuccess) {
            rc = fail(AVR_ERR_HIP, "event sync");
            break;
        }
        float t = 0.f;
        (void)hipEventElapsedTime(&t, e0, e1);
        if (k >= 0 && (tmin[k] < 0 || t < tmin[k])) tmin[k] = t;
    }
    c->ptab_spec = spec0;
    for (int k = 0; k < n && !rc; ++k) {
        const float t = tmin[k];
        if (ms) ms[k] = t;
        if ((k == prefer || (same && (*same)[k])) && (tPrefer < 0 || t < tPrefer)) tPrefer = t;
        if (best < 0 || t < best) { best = t; *bestk = k; }
    }
    if (!rc && prefer >= 0 && tPrefer >= 0 && tPrefer <= best * (1 + kProbeNoise)) *bestk = prefer;
    const std::string err = g_err;
    const int rcProbe = rc;
    int rcRestore = restore(rc != 0, *bestk);
    if (haveSaved) {
        const double *d = saved;
        hipError_t e = hipMemcpyAsync(c->film.rgb_sum, d, 3 * np * sizeof(double), hipMemcpyDeviceToDevice, c->stream);
        if (e == hipSuccess)
            e = hipMemcpyAsync(c->film.w_sum, d + 3 * np, np * sizeof(double), hipMemcpyDeviceToDevice, c->stream);
        if (e == hipSuccess && c->film.nbuckets > 0)
            e = hipMemcpyAsync(c->film.bucket_sum, d + 4 * np, 2 * np * c->film.nbuckets * sizeof(double),
                               hipMemcpyDeviceToDevice, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        if (e != hipSuccess && !rcRestore) rcRestore = fail(AVR_ERR_HIP, std::string("film restore: ") + hipGetErrorString(e));
    }
    if (rcProbe) {
        rc = rcProbe;
        g_err = err;
    } else {
        rc = rcRestore;
    }
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    (void)hipFree(saved);
    if (!rc) rc = avr_reset_stats(c);
    return rc;
}
}  // extern "C++"

int avr_tune_majorant(avr_context *c, const int *candidates, int n, int spp_begin, int spp_end, int seed,
                      int max_depth, int chosen[3], float *ms) {
    AVR_QUIESCE(c);
    if (!c || !candidates || n < 1 || !chosen) return fail(AVR_ERR_ARG, "null argument");
    if (!c->has_medium || !c->has_film || !c->has_camera) return fail(AVR_ERR_STATE, "scene incomplete");
    if (c->med.type == 1 || c->med.type == 2)
        return fail(AVR_ERR_ARG, "homogeneous / cloud media have a single majorant segment");
    if (spp_end <= spp_begin) return fail(AVR_ERR_ARG, "empty probe sample range");
    for (int k = 0; k < 3 * n; ++k)
        if (candidates[k] < 1 || candidates[k] > 255) return fail(AVR_ERR_ARG, "majorant resolution must be 1..255");
    const int mres0[3] = {c->med.mres[0], c->med.mres[1], c->med.mres[2]};
    int bestk = 0;
    const int rc = probe_loop(
        c, n, [&](int k) { return build_majorant(c, candidates + 3 * k); },
        [&](bool failed, int b) { return build_majorant(c, failed ? mres0 : candidates + 3 * b); }, spp_begin, spp_end,
        seed, max_depth, &bestk, ms);
    if (!rc)
        for (int i = 0; i < 3; ++i) chosen[i] = candidates[3 * bestk + i];
    return rc;
}

// k_paths' effective walk schedule for requested (refill lanes, DDA cells), 0 = the defaults —
// measured optima: refill at 32 idle lanes and 10 DDA cells per iteration for 16^3
// majorants, 32 cells for finer ones; a non-emissive NanoVDB medium (pbrt's 64^3 majorant: ~4x the
// DDA steps of the grid) refills at 20 lanes with 28 cells (S-cloud-1024: 1239 -> 1352
// Msamples/s at 12 / 28 in round 3, 1435 -> 1464 at 16 / 28 in round 5, 1619 -> 1638 at 20 / 28
// in round 6, profiles/r06_walk_sweep.json); an RGBGridMedium (8 sigmoid taps x 4 wavelengths per
// lookup, 2 waves / SIMD) at 16 lanes with 32 cells (C5's RGB explosion: 1770 -> 2094 Msamples/s)
static void walk_schedule(const avr_context *c, int refill, int dda, int *r_eff, int *d_eff) {
    const int mres = std::max(c->med.mres[0], std::max(c->med.mres[1], c->med.mres[2]));
    const bool vdbWalk = c->med.type == 3 && !c->med.emissive && mres > 16;
    const bool rgbWalk = c->med.type == 4;
    // a GridMedium majorant of at most 2 cells per axis (fast mode's tuned 1^3): walks of one
    // or two cells, so the event handlers dominate and larger batches win
    const bool coarse = c->med.type == 0 && mres <= 2;
    // measured optima (profiles/r06_walk_sweep.json for the round-6 kernels: NanoVDB 20 / 28,
    // coarse 48)
    *r_eff = refill > 0 ? refill : (vdbWalk ? 20 : (rgbWalk ? 16 : (coarse ? 48 : 32)));
    *d_eff = dda > 0 ? dda : (vdbWalk ? 28 : (rgbWalk || mres > 16 ? 32 : 10));
}

int avr_tune_walk(avr_context *c, const int *refill, int nr, const int *dda, int nd, int spp_begin, int spp_end,
                  int seed, int max_depth, int chosen[2], float *ms) {
    AVR_QUIESCE(c);
    if (!c || !refill || !dda || nr < 1 || nd < 1 || !chosen) return fail(AVR_ERR_ARG, "null argument");
    if (!c->has_medium || !c->has_film || !c->has_camera) return fail(AVR_ERR_STATE, "scene incomplete");
    if (spp_end <= spp_begin) return fail(AVR_ERR_ARG, "empty probe sample range");
    for (int k = 0; k < nr; ++k)
        if (refill[k] < 0 || refill[k] > 64) return fail(AVR_ERR_ARG, "refill candidates must be 0..64 lanes");
    for (int k = 0; k < nd; ++k)
        if (dda[k] < 0) return fail(AVR_ERR_ARG, "DDA budget candidates must be >= 0 cells");
    const int r0 = c->refill_min, d0 = c->dda_budget;
    // the default schedule (0, 0) when listed, else the current one, wins ties within the noise
    int prefer = -1;
    for (int k = 0; k < nr * nd && prefer < 0; ++k)
        if (refill[k / nd] == 0 && dda[k % nd] == 0) prefer = k;
    for (int k = 0; k < nr * nd && prefer < 0; ++k)
        if (refill[k / nd] == r0 && dda[k % nd] == d0) prefer = k;
    // every candidate that resolves to the preferred schedule counts as the same probe
    std::vector<char> same((size_t)nr * nd, 0);
    if (prefer >= 0) {
        int rp, dp;
        walk_schedule(c, refill[prefer / nd], dda[prefer % nd], &rp, &dp);
        for (int k = 0; k < nr * nd; ++k) {
            int rk, dk;
            walk_schedule(c, refill[k / nd], dda[k % nd], &rk, &dk);
            same[(size_t)k] = rk == rp && dk == dp;
        }
    }
    int bestk = 0;
    const int rc = probe_loop(
        c, nr * nd,
        [&](int k) {
            c->refill_min = refill[k / nd];
            c->dda_budget = dda[k % nd];
            return AVR_OK;
        },
        [&](bool failed, int b) {
            c->refill_min = failed ? r0 : refill[b / nd];
            c->dda_budget = failed ? d0 : dda[b % nd];
            return AVR_OK;
        },
        spp_begin, spp_end, seed, max_depth, &bestk, ms, prefer, &same);
    if (!rc) {
        chosen[0] = refill[bestk / nd];
        chosen[1] = dda[bestk % nd];
    }
    return rc;
}

static void pc1d_build(const float *f, int n, float mn, float mx, float *cdf, float *funcInt);

// ---------------------------------------------------------------------------
// PowerLightSampler (lightsamplers.cpp:76-96): weight = Average(SafeDiv(Phi(lambda),
// lambda.PDF())) at lambda = SampledWavelengths::SampleVisible(0.5) (canonical wavelength
// math, as the device's), then an AliasTable over the weights (util/sampling.cpp:563-618).
static avr::Spec visible_half_lambda(avr::Spec *pdf) {
    const avr::Spec l = avr::sample_visible_lambda(0.5f);
    *pdf = {avr::visible_wavelength_pdf(l.v0), avr::visible_wavelength_pdf(l.v1), avr::visible_wavelength_pdf(l.v2),
            avr::visible_wavelength_pdf(l.v3)};
    return l;
}
static float phi_weight(const avr::Spec &phi, const avr::Spec &pdf) {
    // SafeDiv then SampledSpectrum::Average (spectrum.h:175-181): sum in order, / 4
    const float a = pdf.v0 != 0 ? phi.v0 / pdf.v0 : 0.f, b = pdf.v1 != 0 ? phi.v1 / pdf.v1 : 0.f;
    const float c2 = pdf.v2 != 0 ? phi.v2 / pdf.v2 : 0.f, d = pdf.v3 != 0 ? phi.v3 / pdf.v3 : 0.f;
    return (((a + b) + c2) + d) / 4;
}
// DistantLight::Phi (lights.cpp:216-218): scale * Lemit(lambda) * Pi * Sqr(sceneRadius);
// UniformInfiniteLight::Phi (lights.cpp:974-976): 4 * Pi * Pi * Sqr(sceneRadius) * scale * Lemit(lambda)
static float phi_table_light(int type, const float *L, float scale, float r) {
    avr::Spec pdf;
    const avr::Spec l = visible_half_lambda(&pdf);
    const avr::Spec Le = avr::sample_table(L, avr::lambda_index(l));
    avr::Spec phi;
    if (type == 0) {
        phi = Le * scale * avr::kPi * (r * r);
    } else {
        const float k = 4 * avr::kPi * avr::kPi * (r * r) * scale;
        phi = avr::Spec{k * Le.v0, k * Le.v1, k * Le.v2, k * Le.v3};
    }
    return phi_weight(phi, pdf);
}
// RGBSigmoidPolynomial (util/color.h:332-365), the host twin of the device's rsp_eval
static float rsp_host(float c0, float c1, float c2, float lambda) {
    const float x = std::fma(lambda, std::fma(lambda, c0, c1), c2);
    if (std::isinf(x)) return x > 0 ? 1.f : 0.f;
    return .5f + x / (2 * std::sqrt(1 + x * x));
}
// ImageInfiniteLight::Phi (lights.cpp:1042-1060): the image's RGBIlluminantSpectrum summed over
// the pixels (rows y, then x) at lambda, times 4 Pi^2 R^2 scale / (width * height)
static float phi_image_light(const float *coeffs, int res, const float *illum, float scale, float r) {
    avr::Spec pdf;
    const avr::Spec l = visible_half_lambda(&pdf);
    const avr::Spec il = avr::sample_table(illum, avr::lambda_index(l));
    avr::Spec sum = avr::Spec::c(0.f);
    for (size_t p = 0; p < (size_t)res * res; ++p) {
        const float *c = coeffs + 4 * p;
        const avr::Spec s{c[3] * rsp_host(c[0], c[1], c[2], l.v0), c[3] * rsp_host(c[0], c[1], c[2], l.v1),
                          c[3] * rsp_host(c[0], c[1], c[2], l.v2), c[3] * rsp_host(c[0], c[1], c[2], l.v3)};
        sum = sum + s * il;
    }
    const float k = 4 * avr::kPi * avr::kPi * (r * r) * scale;
    const float wh = (float)(res * res);
    const avr::Spec phi{k * sum.v0 / wh, k * sum.v1 / wh, k * sum.v2 / wh, k * sum.v3 / wh};
    return phi_weight(phi, pdf);
}
// AliasTable construction (util/sampling.cpp:563-618): p = w / sum (double accumulation),
// then the under / over work lists popped from the back
static void build_alias(const float *w, int n, float *q, float *p, int *alias) {
    double acc = 0.;
    for (int i = 0; i < n; ++i) acc += w[i];
    const float sum = (float)acc;
    for (int i = 0; i < n; ++i) p[i] = w[i] / sum;
    struct Outcome { float pHat; int index; };
    std::vector<Outcome> under, over;
    for (int i = 0; i < n; ++i) {
        const float pHat = p[i] * (float)n;
        (pHat < 1 ? under : over).push_back({pHat, i});
    }
    while (!under.empty() && !over.empty()) {
        const Outcome un = under.back(), ov = over.back();
        under.pop_back();
        over.pop_back();
        q[un.index] = un.pHat;
        alias[un.index] = ov.index;
        const float pExcess = un.pHat + ov.pHat - 1;
        (pExcess < 1 ? under : over).push_back({pExcess, ov.index});
    }
    for (const Outcome &o : over) q[o.index] = 1, alias[o.index] = -1;
    for (const Outcome &u : under) q[u.index] = 1, alias[u.index] = -1;
}
// (Re)build the device light list's sampler fields after any light or sampler change
static int update_light_sampler(avr_context *c) {
    const int n = c->lights.n;
    bool ready = c->light_sampler == 1 && n > 0;
    for (int i = 0; i < n && ready; ++i) ready = c->phi_ok[i];
    c->lights.power = ready ? 1 : 0;
    if (n == 0) return AVR_OK;
    float q[avr::kMaxLights], pm[avr::kMaxLights];
    int al[avr::kMaxLights];
    if (ready) {
        float w[avr::kMaxLights];
        float tot = 0.f;
        for (int i = 0; i < n; ++i) tot += (w[i] = c->h_phi[i]);   // std::accumulate(..., 0.f)
        if (tot == 0.f) std::fill(w, w + n, 1.f);
        build_alias(w, n, q, pm, al);
    } else {
        // BVH / uniform (the kernels' pick ignores the bins then): q = 1, p = pInf / n
        for (int i = 0; i < n; ++i) q[i] = 1.f, pm[i] = float(n) / float(n + 0) / n, al[i] = -1;
    }
    for (int i = 0; i < n; ++i) {
        c->h_lights[i].aq = q[i];
        c->h_lights[i].ap = pm[i];
        c->h_lights[i].alias = al[i];
    }
    if (c->d_lights) {
        HIP_TRY(hipMemcpyAsync(c->d_lights, c->h_lights, sizeof(c->h_lights), hipMemcpyHostToDevice, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
    }
    return AVR_OK;
}

int avr_lights(avr_context *c, int n, const int *types, const float *w3, const float *L, const float *scale,
               float scene_radius) {
    AVR_QUIESCE(c);
    if (!c || n < 0 || n > avr::kMaxLights) return fail(AVR_ERR_ARG, "0..8 lights supported");
    if (n > 0 && (!types || !w3 || !L || !scale)) return fail(AVR_ERR_ARG, "null light arrays");
    HIP_TRY(hipSetDevice(c->device));
    int rc = upload_table(&c->d_lightL, n ? L : nullptr, (size_t)n * avr::kNTable, c->stream);
    if (rc) return rc;
    avr::DevLight h[avr::kMaxLights] = {};
    for (int i = 0; i < n; ++i) {
        if (types[i] < 0 || types[i] > 2)
            return fail(AVR_ERR_ARG, "light type must be 0 (distant), 1 (uniform infinite) or 2 (image infinite)");
        h[i].type = types[i];
        for (int k = 0; k < 3; ++k) h[i].w[k] = w3[3 * i + k];
        h[i].L = c->d_lightL + (size_t)i * avr::kNTable;
        h[i].scale = scale[i];
    }
    if (!c->d_lights) HIP_TRY(dalloc(&c->d_lights, avr::kMaxLights));
    HIP_TRY(hipMemcpyAsync(c->d_lights, h, sizeof(h), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    for (auto &b : c->d_light_img) if (b) (void)hipFree(b), b = nullptr;
    for (int i = 0; i < avr::kMaxLights; ++i) c->h_lights[i] = h[i];
    c->lights = {};
    c->lights.n = n;
    c->lights.list = c->d_lights;
    c->lights.scene_radius = scene_radius;
    c->n_image_lights = 0;
    for (int i = 0; i < n; ++i) c->n_image_lights += types[i] == 2 ? 1 : 0;
    c->image_lights_ready = 0;
    for (int i = 0; i < avr::kMaxLights; ++i) {
        c->phi_ok[i] = i < n && types[i] != 2;
        c->h_phi[i] = c->phi_ok[i] ? phi_table_light(types[i], L + (size_t)i * avr::kNTable, scale[i], scene_radius) : 0.f;
    }
    return update_light_sampler(c);
}

int avr_light_sampler(avr_context *c, int kind) {
    AVR_QUIESCE(c);
    if (!c || (kind != 0 && kind != 1)) return fail(AVR_ERR_ARG, "light sampler must be 0 (bvh / uniform) or 1 (power)");
    HIP_TRY(hipSetDevice(c->device));
    c->light_sampler = kind;
    return update_light_sampler(c);
}

// ImageInfiniteLight: pixel spectra, the compensated PiecewiseConstant2D (lights.cpp:1026-1038)
int avr_light_image(avr_context *c, int index, int res, const float *pixel_coeffs, const float *distribution,
                    const float *illuminant, const float render_from_light[16], const float light_from_render[16]) {
    AVR_QUIESCE(c);
    if (!c || index < 0 || index >= c->lights.n || c->h_lights[index].type != 2)
        return fail(AVR_ERR_ARG, "avr_light_image: index must name a type-2 light of the last avr_lights call");
    if (res < 1 || !pixel_coeffs || !distribution || !illuminant || !render_from_light || !light_from_render)
        return fail(AVR_ERR_ARG, "avr_light_image: bad image arguments");
    HIP_TRY(hipSetDevice(c->device));
    const size_t np = (size_t)res * res;
    // compensated distribution: d - average (f64 accumulate, lights.cpp:1031), clamped at 0;
    // all zero -> ones
    double sum = 0.;
    for (size_t i = 0; i < np; ++i) sum += distribution[i];
    const float average = (float)(sum / np);
    std::vector<float> d(np);
    bool allZero = true;
    for (size_t i = 0; i < np; ++i) {
        d[i] = std::max<float>(distribution[i] - average, 0);
        allZero &= d[i] == 0;
    }
    if (allZero) std::fill(d.begin(), d.end(), 1.f);
    const int nx = res, ny = res;
    const size_t ntab = (size_t)avr::smp::filter_table_floats(nx, ny);
    const size_t bytes = np * sizeof(float4) + ntab * sizeof(float) + avr::kNTable * sizeof(float);
    std::vector<unsigned char> blob(bytes);
    std::memcpy(blob.data(), pixel_coeffs, np * sizeof(float4));
    float *t = (float *)(blob.data() + np * sizeof(float4));
    float *f = t, *ccdf = f + nx * ny, *cint = ccdf + ny * (nx + 1), *mcdf = cint + ny, *mint = mcdf + ny + 1;
    for (size_t i = 0; i < np; ++i) f[i] = std::abs(d[i]);
    for (int y = 0; y < ny; ++y) pc1d_build(f + (size_t)y * nx, nx, 0.f, 1.f, ccdf + (size_t)y * (nx + 1), cint + y);
    pc1d_build(cint, ny, 0.f, 1.f, mcdf, mint);
    std::memcpy(t + ntab, illuminant, avr::kNTable * sizeof(float));
    if (c->d_light_img[index]) (void)hipFree(c->d_light_img[index]);
    c->d_light_img[index] = nullptr;
    HIP_TRY(hipMalloc((void **)&c->d_light_img[index], bytes));
    HIP_TRY(hipMemcpy(c->d_light_img[index], blob.data(), bytes, hipMemcpyHostToDevice));
    unsigned char *base = (unsigned char *)c->d_light_img[index];
    avr::DevLight &L = c->h_lights[index];
    L.img = (const float4 *)base;
    L.res = res;
    const float *dt = (const float *)(base + np * sizeof(float4));
    L.dist.nx = nx;
    L.dist.ny = ny;
    L.dist.f = dt;
    L.dist.ccdf = dt + nx * ny;
    L.dist.cint = L.dist.ccdf + ny * (nx + 1);
    L.dist.mcdf = L.dist.cint + ny;
    L.dist.mint = *mint;
    L.illum = dt + ntab;
    for (int r = 0; r < 3; ++r)
        for (int k = 0; k < 3; ++k) {
            L.rfl[3 * r + k] = render_from_light[4 * r + k];
            L.lfr[3 * r + k] = light_from_render[4 * r + k];
        }
    HIP_TRY(hipMemcpyAsync(c->d_lights, c->h_lights, sizeof(c->h_lights), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    ++c->image_lights_ready;
    c->h_phi[index] = phi_image_light(pixel_coeffs, res, illuminant, L.scale, c->lights.scene_radius);
    c->phi_ok[index] = true;
    return update_light_sampler(c);
}

int avr_camera(avr_context *c, int type, const float cfr[16], const float rfc[16]) {
    if (!c || (type != 0 && type != 1) || !cfr || !rfc) return fail(AVR_ERR_ARG, "bad camera");
    if (!affine(rfc)) return fail(AVR_ERR_ARG, "render_from_camera must be affine");
    c->cam.type = type;
    for (int i = 0; i < 16; ++i) c->cam.raster[i] = cfr[i];
    copy_xf(c->cam.render_from_camera, rfc);
    c->has_camera = true;
    return AVR_OK;
}

int avr_film(avr_context *c, int width, int height, const float fr[2], const float *sensor, float imaging_ratio,
             float max_component_value) {
    AVR_QUIESCE(c);
    if (!c || width < 1 || height < 1 || !fr || !sensor) return fail(AVR_ERR_ARG, "bad film");
    HIP_TRY(hipSetDevice(c->device));
    int rc = upload_table(&c->d_xyz, sensor, 3 * (size_t)avr::kNTable, c->stream);
    if (rc) return rc;
    if (c->film.rgb_sum) (void)hipFree(c->film.rgb_sum);
    if (c->film.w_sum) (void)hipFree(c->film.w_sum);
    if (c->film.bucket_sum) (void)hipFree(c->film.bucket_sum);
    free_pixel_order(c);   // an order is for one film resolution
    c->film = {};
    c->film.width = width;
    c->film.height = height;
    c->film.filter_rx = fr[0];
    c->film.filter_ry = fr[1];
    c->film.xyz = c->d_xyz;
    c->film.imaging_ratio = imaging_ratio;
    c->film.max_component = max_component_value;
    const size_t np = (size_t)width * height;
    HIP_TRY(dalloc(&c->film.rgb_sum, 3 * np));
    HIP_TRY(dalloc(&c->film.w_sum, np));
    c->has_film = true;
    return avr_film_clear(c);
}

// FilterSampler tables of GaussianFilter(radius, sigma) — filters.h:80-118,
// filters.cpp:133-147, PiecewiseConstant1D/2D sampling.h:603-770 — built on the host in
// pbrt's float operation order (this file is compiled with -ffp-contract=off).
static float gaussian_1d(float x, float mu, float sigma) {   // util/math.h:477-480
    return 1 / std::sqrt(2 * avr::kPi * sigma * sigma) * avr::fast_exp(-avr::sqr(x - mu) / (2 * sigma * sigma));
}
static void pc1d_build(const float *f, int n, float mn, float mx, float *cdf, float *funcInt) {
    cdf[0] = 0;
    for (int i = 1; i < n + 1; ++i) cdf[i] = cdf[i - 1] + std::abs(f[i - 1]) * (mx - mn) / n;
    *funcInt = cdf[n];
    if (*funcInt == 0)
        for (int i = 1; i < n + 1; ++i) cdf[i] = float(i) / float(n);
    else
        for (int i = 1; i < n + 1; ++i) cdf[i] /= *funcInt;
}

int avr_set_filter(avr_context *c, int type, const float radius[2], float sigma) {
    AVR_QUIESCE(c);
    if (!c || (type != 0 && type != 1) || !radius || !(radius[0] > 0) || !(radius[1] > 0))
        return fail(AVR_ERR_ARG, "filter: type 0 (box) or 1 (gaussian) with a positive radius");
    HIP_TRY(hipSetDevice(c->device));
    if (type == 0) {
        c->filter_type = 0;
        c->film.filter_rx = radius[0];
        c->film.filter_ry = radius[1];
        return AVR_OK;
    }
    const int nx = int(32 * radius[0]), ny = int(32 * radius[1]);
    if (nx < 1 || ny < 1 || nx > 128 || ny > 128) return fail(AVR_ERR_ARG, "gaussian filter radius out of range");
    const float expX = gaussian_1d(radius[0], 0, sigma), expY = gaussian_1d(radius[1], 0, sigma);
    std::vector<float> t((size_t)avr::smp::filter_table_floats(nx, ny));
    float *f = t.data(), *ccdf = f + nx * ny, *cint = ccdf + ny * (nx + 1), *mcdf = cint + ny, *mint = mcdf + ny + 1;
    for (int y = 0; y < ny; ++y)
        for (int x = 0; x < nx; ++x) {
            // Bounds2f::Lerp of ((x + 0.5) / nx, (y + 0.5) / ny) over [-r, r]
            const float tx = (x + 0.5f) / nx, ty = (y + 0.5f) / ny;
            const float px = (1 - tx) * -radius[0] + tx * radius[0], py = (1 - ty) * -radius[1] + ty * radius[1];
            f[(size_t)y * nx + x] = std::max<float>(0, gaussian_1d(px, 0, sigma) - expX) *
                                    std::max<float>(0, gaussian_1d(py, 0, sigma) - expY);
        }
    for (int y = 0; y < ny; ++y) pc1d_build(f + (size_t)y * nx, nx, -radius[0], radius[0], ccdf + (size_t)y * (nx + 1), cint + y);
    pc1d_build(cint, ny, -radius[1], radius[1], mcdf, mint);
    // the search guides (camera stage): one row per conditional CDF, then the marginal's
    t.resize((size_t)avr::smp::filter_blob_floats(nx, ny), 0.f);
    f = t.data();
    ccdf = f + nx * ny;
    cint = ccdf + ny * (nx + 1);
    mcdf = cint + ny;
    const float mint_v = t[(size_t)avr::smp::filter_table_floats(nx, ny) - 1];
    uint8_t *guide = (uint8_t *)(t.data() + avr::smp::filter_table_floats(nx, ny));
    for (int y = 0; y < ny; ++y)
        avr::smp::filter_guide_build(ccdf + (size_t)y * (nx + 1), nx, guide + (size_t)y * (avr::smp::kFilterGuideK + 1));
    avr::smp::filter_guide_build(mcdf, ny, guide + (size_t)ny * (avr::smp::kFilterGuideK + 1));
    // the cell weights (after the guides)
    float *wt = t.data() + avr::smp::filter_table_floats(nx, ny) + avr::smp::filter_guide_floats(ny);
    for (int y = 0; y < ny; ++y)
        for (int x = 0; x < nx; ++x) wt[(size_t)y * nx + x] = avr::smp::filter_cell_weight(f, cint, mint_v, nx, y, x);
    if (c->d_filter) (void)hipFree(c->d_filter);
    c->d_filter = nullptr;
    HIP_TRY(dalloc(&c->d_filter, t.size()));
    HIP_TRY(hipMemcpy(c->d_filter, t.data(), t.size() * sizeof(float), hipMemcpyHostToDevice));
    c->ftab.nx = nx;
    c->ftab.ny = ny;
    c->ftab.rx = radius[0];
    c->ftab.ry = radius[1];
    c->ftab.f = c->d_filter;
    c->ftab.ccdf = c->d_filter + nx * ny;
    c->ftab.cint = c->ftab.ccdf + ny * (nx + 1);
    c->ftab.mcdf = c->ftab.cint + ny;
    c->ftab.mint = mint_v;
    c->ftab.guide = (const uint8_t *)(c->d_filter + avr::smp::filter_table_floats(nx, ny));
    c->ftab.wt = c->d_filter + avr::smp::filter_table_floats(nx, ny) + avr::smp::filter_guide_floats(ny);
    c->filter_type = 1;
    return AVR_OK;
}

int avr_set_pixel_order(avr_context *c, const int *order, long long n) {
    AVR_QUIESCE(c);
    if (!c || !c->has_film) return fail(AVR_ERR_STATE, "pixel order needs a film");
    HIP_TRY(hipSetDevice(c->device));
    free_pixel_order(c);
    if (!order) return AVR_OK;   // scanline
    const long long np = (long long)c->film.width * c->film.height;
    if (n != np) return fail(AVR_ERR_ARG, "pixel order must list every pixel of the film once");
    std::vector<int> slot((size_t)np, -1);
    for (long long j = 0; j < np; ++j) {
        const int p = order[j];
        if (p < 0 || p >= np || slot[(size_t)p] >= 0) return fail(AVR_ERR_ARG, "pixel order is not a permutation");
        slot[(size_t)p] = (int)j;
    }
    HIP_TRY(dalloc(&c->d_pix_order, (size_t)np));
    HIP_TRY(dalloc(&c->d_pix_slot, (size_t)np));
    HIP_TRY(hipMemcpy(c->d_pix_order, order, np * sizeof(int), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->d_pix_slot, slot.data(), np * sizeof(int), hipMemcpyHostToDevice));
    c->h_pix_slot.swap(slot);
    ++c->order_gen;
    return AVR_OK;
}

int avr_set_sampler_table(avr_context *c, int dims) {
    AVR_QUIESCE(c);
    if (!c || dims < 0 || dims > 4096) return fail(AVR_ERR_ARG, "sampler table dimensions must be 0..4096");
    c->zs_dims = dims;
    c->zs_key[0] = -1;   // rebuild (or drop) at the next render
    return AVR_OK;
}

int avr_set_sampler_pass_table(avr_context *c, int dims) {
    AVR_QUIESCE(c);
    if (!c || dims < 0 || dims > 4096) return fail(AVR_ERR_ARG, "sampler pass table dimensions must be 0..4096");
    // rows of an even number of 8-B entries: the camera stage loads a draw pair's entries as one
    // 16-B ulonglong2 at ptab + row * dims, aligned only for even dims (the extra dimension is
    // never read — same results)
    c->zs_pdims = (dims + 1) & ~1;
    return AVR_OK;
}

int avr_set_sampler(avr_context *c, int kind, int samples_per_pixel) {
    if (!c || (kind != 0 && kind != 1) || samples_per_pixel < 1)
        return fail(AVR_ERR_ARG, "sampler: kind 0 (independent) or 1 (zsobol), samples_per_pixel >= 1");
    c->sampler_kind = kind;
    c->sampler_spp = samples_per_pixel;
    return AVR_OK;
}

int avr_film_clear(avr_context *c) {
    if (!c || !c->has_film) return fail(AVR_ERR_STATE, "no film");
    const size_t np = (size_t)c->film.width * c->film.height;
    HIP_TRY(hipMemsetAsync(c->film.rgb_sum, 0, 3 * np * sizeof(double), c->stream));
    HIP_TRY(hipMemsetAsync(c->film.w_sum, 0, np * sizeof(double), c->stream));
    if (c->film.nbuckets > 0)
        HIP_TRY(hipMemsetAsync(c->film.bucket_sum, 0, 2 * np * c->film.nbuckets * sizeof(double), c->stream));
    return AVR_OK;
}

// SpectralFilm (film.h:401-530, Create film.cpp:1037-1066): buckets over [lambda_min,
// lambda_max]; n_buckets = 0 returns to RGBFilm. Both sums live in one allocation.
int avr_film_spectral(avr_context *c, int n_buckets, float lambda_min, float lambda_max) {
    if (!c || !c->has_film) return fail(AVR_ERR_STATE, "no film");
    if (n_buckets < 0) return fail(AVR_ERR_ARG, "n_buckets must be >= 0");
    if (n_buckets > 0 && !(360.f <= lambda_min && lambda_min < lambda_max && lambda_max <= 830.f))
        return fail(AVR_ERR_ARG, "SpectralFilm wavelength range must lie within 360..830 nm");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (c->film.bucket_sum) (void)hipFree(c->film.bucket_sum);
    c->film.bucket_sum = c->film.bucket_w = nullptr;
    c->film.nbuckets = n_buckets;
    c->film.lmin = lambda_min;
    c->film.lmax = lambda_max;
    if (n_buckets > 0) {
        const size_t nb = (size_t)c->film.width * c->film.height * n_buckets;
        HIP_TRY(dalloc(&c->film.bucket_sum, 2 * nb));
        c->film.bucket_w = c->film.bucket_sum + nb;
    }
    return avr_film_clear(c);
}

// Stats are resolved lazily so that a render stays asynchronous: every timed interval
// records two pool events and is folded (one stream sync) when stats are read.
static int fold_stats(avr_context *c) {
    if (c->timed.empty()) return AVR_OK;
    HIP_TRY(hipStreamSynchronize(c->stream));
    for (const auto &t : c->timed) {
        float ms = 0;
        HIP_TRY(hipEventElapsedTime(&ms, c->evpool[t.a], c->evpool[t.b]));
        c->stats.*(t.field) += ms;
        if (t.launch) c->stats.medium_launches++;
    }
    c->timed.clear();
    c->ev_used = 0;
    unsigned long long h[avr::kNumStats];
    HIP_TRY(hipStreamSynchronize(c->stream));
    HIP_TRY(hipMemcpy(h, c->d_stats, sizeof(h), hipMemcpyDeviceToHost));
    c->stats.medium_lookups = h[0];
    c->stats.medium_items_in = h[1];
    c->stats.medium_items_out = h[2];
    c->stats.shadow_lookups = h[3];
    c->stats.shadow_items = h[4];
    c->stats.medium_dda_steps = h[5];
    c->stats.shadow_dda_steps = h[6];
    c->stats.loop_iterations = h[8];
    c->stats.active_lane_iterations = h[9];
    if (h[7]) {
        HIP_TRY(hipMemset(c->d_stats + 7, 0, sizeof(unsigned long long)));
        return fail(AVR_ERR_STATE, "k_paths launched without its pass's camera stage (work heads not reset): pass not rendered");
    }
    return AVR_OK;
}

// The ZSobol pass table of sample indices [base, base + S): its entries hold the digits above
// the lowest plo bits, where the pass's indices differ
static int pass_plo(long long base, int S) {
    int plo = 0;
    while ((base >> plo) != ((base + S - 1) >> plo)) ++plo;
    return plo;
}
constexpr int kPtabKey = 8;
// what a built table depends on (a table built ahead is used only when the pass's key equals it)
static void ptab_key(const avr_context *c, const avr::smp::ZSobolParams &zs, long long base, int plo, long long *key) {
    const long long k[kPtabKey] = {base, plo, (long long)zs.log2spp, (long long)zs.seed,
                                   (long long)c->film.width * 65536 + c->film.height, c->zs_pdims,
                                   (long long)(uintptr_t)zs.upper, zs.dmax};
    for (int i = 0; i < kPtabKey; ++i) key[i] = k[i];
}
// Build the pass table (and the camera stage's compact copy) of [base, base + S) into buffer buf
// on stream s, with its level-A table when the two-level build applies. No room for a buffer:
// d_zs_ptab[buf] stays null (the pixel table / every digit per call serve the pass).
static int ptab_build(avr_context *c, hipStream_t s, const avr::smp::ZSobolParams &zs, long long base, int plo, int buf,
                      bool two_level) {
    const long long P = (long long)c->film.width * c->film.height;
    const size_t prow = (size_t)avr::smp::encode_morton2((uint32_t)c->film.width - 1, (uint32_t)c->film.height - 1) + 1;
    const size_t need_e = prow * (size_t)c->zs_pdims;
    // the same headroom policy as the fat / bricked density copies: allocate only with >= 8 GiB
    // of HBM to spare
    auto fits = [](size_t bytes) {
        size_t freeB = 0, totalB = 0;
        return hipMemGetInfo(&freeB, &totalB) == hipSuccess && bytes + (8ull << 30) < freeB;
    };
    if (need_e > c->zs_ptab_cap[buf]) {
        if (c->d_zs_ptab[buf]) (void)hipFree(c->d_zs_ptab[buf]);
        c->d_zs_ptab[buf] = nullptr;
        c->zs_ptab_cap[buf] = 0;
        if (!fits(need_e * sizeof(uint64_t)) ||
            hipMalloc((void **)&c->d_zs_ptab[buf], need_e * sizeof(uint64_t)) != hipSuccess) {
            (void)hipGetLastError();
            c->d_zs_ptab[buf] = nullptr;
            return AVR_OK;
        }
        c->zs_ptab_cap[buf] = need_e;
    }
    // two-level build: the plo + 2 table is shared by the four passes whose indices agree above
    // plo + 2 bits; each pass then derives its own from it (not when the caller's passes stride
    // past each other's group: a sample shard's rank would rebuild it for every pass)
    const uint64_t *atab = nullptr;
    if (two_level && c->zs_two_level && plo + 2 <= zs.log2spp) {
        if (need_e > c->zs_atab_cap) {
            if (c->d_zs_atab) (void)hipFree(c->d_zs_atab);
            c->d_zs_atab = nullptr;
            c->zs_atab_cap = 0;
            for (long long &k : c->zs_akey) k = -1;
            if (!fits(need_e * sizeof(uint64_t)) ||
                hipMalloc((void **)&c->d_zs_atab, need_e * sizeof(uint64_t)) != hipSuccess) {
                (void)hipGetLastError();
                c->d_zs_atab = nullptr;   // no room: one-level build
            } else {
                c->zs_atab_cap = need_e;
            }
        }
        if (c->d_zs_atab) {
            const long long key[6] = {base >> (plo + 2), plo, (long long)zs.log2spp, zs.seed,
                                      (long long)c->film.width * 65536 + c->film.height, c->zs_pdims};
            bool same = true;
            for (int k = 0; k < 6; ++k) same = same && key[k] == c->zs_akey[k];
            if (!same) {
                hipLaunchKernelGGL(avr::k_zsobol_pass_table,
                                   dim3(blocks_for(P * (c->zs_pdims / 2), 256, 256 * 64)), dim3(256), 0, s, zs,
                                   c->film.width, c->film.height, c->zs_pdims, plo + 2, (base >> (plo + 2)) << (plo + 2),
                                   c->d_zs_atab, (const uint64_t *)nullptr, avr::fastdiv_make((uint32_t)(c->zs_pdims / 2)),
                                   avr::fastdiv_make((uint32_t)c->film.width), (uint64_t *)nullptr);
                HIP_TRY(hipGetLastError());
                for (int k = 0; k < 6; ++k) c->zs_akey[k] = key[k];
            }
            atab = c->d_zs_atab;
        }
    }
    // the camera stage's six entries per pixel (dimensions 0, 1, 6..9) also as a compact
    // scanline-ordered copy (48 B per pixel), when the table holds them
    const size_t need_c = c->zs_pdims >= 10 ? 6 * (size_t)P : 0;
    if (need_c > c->zs_ctab_cap[buf]) {
        if (c->d_zs_ctab[buf]) (void)hipFree(c->d_zs_ctab[buf]);
        c->d_zs_ctab[buf] = nullptr;
        c->zs_ctab_cap[buf] = 0;
        if (hipMalloc((void **)&c->d_zs_ctab[buf], need_c * sizeof(uint64_t)) != hipSuccess) {
            (void)hipGetLastError();
            c->d_zs_ctab[buf] = nullptr;   // no room: the camera reads the rows
        } else {
            c->zs_ctab_cap[buf] = need_c;
        }
    }
    uint64_t *ctab = need_c ? c->d_zs_ctab[buf] : nullptr;
    hipLaunchKernelGGL(avr::k_zsobol_pass_table, dim3(blocks_for(P * (c->zs_pdims / 2), 256, 256 * 64)), dim3(256), 0, s,
                       zs, c->film.width, c->film.height, c->zs_pdims, plo, base, c->d_zs_ptab[buf], atab,
                       avr::fastdiv_make((uint32_t)(c->zs_pdims / 2)), avr::fastdiv_make((uint32_t)c->film.width), ctab);
    HIP_TRY(hipGetLastError());
    return AVR_OK;
}

// next free pool event (folds first when the pool is full)
static int next_event(avr_context *c, int *idx) {
    if (c->ev_used >= 512) {
        int rc = fold_stats(c);
        if (rc) return rc;
    }
    if (c->ev_used == c->evpool.size()) {
        hipEvent_t e;
        HIP_TRY(hipEventCreate(&e));
        c->evpool.push_back(e);
    }
    *idx = (int)c->ev_used++;
    HIP_TRY(hipEventRecord(c->evpool[*idx], c->stream));
    return AVR_OK;
}
#define EV_MARK(var)                      \
    int var;                              \
    do {                                  \
        int rc_ = next_event(c, &var);    \
        if (rc_) return rc_;              \
    } while (0)

int avr_render(avr_context *c, int spp_begin, int spp_end, int seed, int max_depth) {
    if (!c) return fail(AVR_ERR_ARG, "null context");
    if (!c->has_medium || !c->has_camera || !c->has_film) return fail(AVR_ERR_STATE, "medium, camera and film required");
    if (spp_begin < 0 || spp_end < spp_begin || max_depth < 0) return fail(AVR_ERR_ARG, "bad sample range");
    if (c->image_lights_ready < c->n_image_lights) return fail(AVR_ERR_STATE, "image light without avr_light_image");
    if (c->light_sampler == 1 && c->lights.n > 0 && !c->lights.power)
        return fail(AVR_ERR_STATE, "power light sampler: light weights incomplete");
    avr::smp::ZSobolParams zs{};
    if (c->sampler_kind == 1) {
        // ZSobolSampler indexes (Morton(pixel) << log2(spp)) | sampleIndex: indices must stay
        // below the sampler's samplesPerPixel and the Sobol' index below 2^32
        if (spp_end > c->sampler_spp) return fail(AVR_ERR_ARG, "zsobol: sample index beyond samplesPerPixel");
        zs = avr::smp::zsobol_params(c->sampler_spp, c->film.width, c->film.height, seed);
        // SobolSample takes indices below 2^SobolMatrixSize = 2^52 (lowdiscrepancy.h:170)
        if (2 * zs.nBase4Digits - (zs.log2spp & 1) > 52)
            return fail(AVR_ERR_ARG, "zsobol: resolution x spp beyond the 2^52 Sobol' index range");
        // Morton(pixel) and the pixel-only digits (zsobol_upper, the pixel table) are 32-bit
        const int res = (int)avr::smp::round_up_pow2((uint32_t)std::max(c->film.width, c->film.height));
        if (2 * avr::smp::ilog2((uint32_t)res) > 32)
            return fail(AVR_ERR_ARG, "zsobol: film resolution beyond 65536 (Morton(pixel) exceeds 32 bits)");
    }
    HIP_TRY(hipSetDevice(c->device));
    if (c->sampler_kind == 1) {
        // The digits of GetSampleIndex above log2(spp) depend on (pixel, dimension) only:
        // tabulate them once per film/sampler (k_zsobol_table), so each sampler call computes
        // the log2(spp)/2 sample digits plus one load instead of all nBase4Digits
        const int key[3] = {c->sampler_spp, c->film.width, c->film.height};
        if (c->zs_key[0] != key[0] || c->zs_key[1] != key[1] || c->zs_key[2] != key[2]) {
            // a table built ahead reads the pixel table: let it finish, and drop it
            if (c->tstream) HIP_TRY(hipStreamSynchronize(c->tstream));
            c->spec_valid = false;
            if (c->d_zs_table) (void)hipFree(c->d_zs_table);
            c->d_zs_table = nullptr;
            for (int k = 0; k < 3; ++k) c->zs_key[k] = key[k];
            if (c->zs_dims > 0) {
                const size_t rows =
                    (size_t)avr::smp::encode_morton2((uint32_t)c->film.width - 1, (uint32_t)c->film.height - 1) + 1;
                if (hipMalloc((void **)&c->d_zs_table, rows * c->zs_dims * sizeof(uint32_t)) != hipSuccess) {
                    (void)hipGetLastError();
                    c->d_zs_table = nullptr;   // no room: every call computes all digits
                } else {
                    EV_MARK(t0);
                    hipLaunchKernelGGL(avr::k_zsobol_table, dim3(blocks_for((long long)c->film.width * c->film.height *
                                                                            c->zs_dims, 256, 256 * 64)),
                                       dim3(256), 0, c->stream, zs, c->film.width, c->film.height, c->zs_dims,
                                       c->d_zs_table);
                    HIP_TRY(hipGetLastError());
                    EV_MARK(t1);
                    c->timed.push_back({t0, t1, &avr_stats::ms_setup, false});
                }
            }
        }
        zs.upper = c->d_zs_table;
        zs.dmax = c->d_zs_table ? c->zs_dims : 0;
    }
    const long long P = (long long)c->film.width * c->film.height;
    if (P > (1ll << 30)) return fail(AVR_ERR_ARG, "film too large");
    // k_paths runs every medium type with every light type: GridMedium, RGBGridMedium and
    // the single-segment Homogeneous/CloudMedium keep the majorant in LDS (at most 4096
    // cells = pbrt's 16^3; larger grids take the wavefront kernels), NanoVDBMedium reads
    // its 64^3 majorant through L2
    const int mcells = c->med.mres[0] * c->med.mres[1] * c->med.mres[2];
    const bool persistent = c->kernel_mode == 0 &&
                            (((c->med.type != 3) && mcells <= 4096) || c->med.type == 3) &&
                            c->med.mres[0] <= 255 && c->med.mres[1] <= 255 && c->med.mres[2] <= 255;
    const long long maxp = c->max_paths_set ? c->max_paths : (persistent ? (64ll << 20) : c->max_paths);
    const long long Smax = std::max<long long>(1, maxp / P);
    const long long need = P * std::min<long long>(Smax, std::max(1, spp_end - spp_begin));
    int rc = persistent ? ensure_records(c, need) : ensure_paths(c, need);
    if (rc) return rc;
    EV_MARK(evStart);
    // the stride between consecutive calls' first sample indices (S for pbrt's pass loop and the
    // one-GPU bench, N x S for a rank of an N-GPU sample shard): where the pass after this call's
    // last one is expected to start, for the pass table built ahead
    const long long call_stride = (c->prev_call_begin >= 0 && spp_begin > c->prev_call_begin) ? spp_begin - c->prev_call_begin : 0;
    c->prev_call_begin = spp_begin;
    for (long long base = spp_begin; base < spp_end; base += Smax) {
        const int S = (int)std::min<long long>(Smax, spp_end - base);
        bool spec_next = false;   // build the next pass's ZSobol table ahead (ptab_spec)
        avr::smp::ZSobolParams spec_zs{};
        avr::Params p{};
        p.med = c->med;
        p.lights = c->lights;
        p.cam = c->cam;
        p.film = c->film;
        p.film.filter_type = c->filter_type;
        p.film.gauss = c->ftab;
        p.sampler_kind = c->sampler_kind;
        p.zs = zs;
        p.ps = c->ps;
        p.sh = c->sh;
        p.max_depth = max_depth;
        p.seed = seed;
        p.pass_pixels = (int)P;
        p.div_pixels = avr::fastdiv_make((uint32_t)P);
        p.div_width = avr::fastdiv_make((uint32_t)c->film.width);
        p.pass_samples = S;
        p.sample_base = (int)base;
        p.stats = c->d_stats;
        const long long n0 = P * S;
        c->last_persistent = persistent;
        c->last_fast = persistent && c->render_mode == 1;
        if (persistent) {
            // PCG32 Advance(s*65536) as an affine map state' = A*state + inc*H (rng.h:132-146:
            // every step is linear in inc, so H = accPlus computed with inc = 1).
            if (S > c->advance_cap) {
                if (c->d_advance) (void)hipFree(c->d_advance);
                HIP_TRY(dalloc(&c->d_advance, 2 * (size_t)S));
                c->advance_cap = S;
            }
            if (c->sampler_kind == 0) {   // read by the IndependentSampler's camera stage only
                hipLaunchKernelGGL(avr::k_advance, dim3((S + 255) / 256), dim3(256), 0, c->stream, c->d_advance,
                                   (long long)base, S);
                HIP_TRY(hipGetLastError());
            }
            p.advance = c->d_advance;
            walk_schedule(c, c->refill_min, c->dda_budget, &p.refill_min, &p.dda_budget);   // defaults: measured optima
            // zeroed by the camera stage (k_paths_camera), which must run first on this stream: it
            // stamps pass_gen into heads[8], and a k_paths launched without it renders nothing and
            // makes the stats readback fail (stats[7])
            p.heads = c->d_heads;
            p.pass_gen = ++c->pass_gen & 0x7fffffff;
            // the camera stage: one lane per sample (k_paths_camera)
            {
                const int sv = c->sampler_kind == 0 ? 0 : (avr::smp::zsobol_wide(p.zs) ? 2 : 1);
                p.pix_order = c->d_pix_order;
                // ZSobol quads: 4-aligned sample ranges, at most 8 lower base-4 digits
                p.cam_quad = (base % 4 == 0 && S % 4 == 0 && p.zs.log2spp <= 16) ? 1 : 0;
                using KC = void (*)(avr::Params);
                static const KC kcam[2][3] = {
                    {avr::k_paths_camera<0, false>, avr::k_paths_camera<2, false>, avr::k_paths_camera<3, false>},
                    {avr::k_paths_camera<0, true>, avr::k_paths_camera<2, true>, avr::k_paths_camera<3, true>}};
                EV_MARK(ec);
                // rows = Morton(w-1, h-1) + 1 (up to ~4x the pixels of a non-square film): the
                // table kernel indexes entries with 32 bits
                const long long prow = (long long)avr::smp::encode_morton2((uint32_t)c->film.width - 1,
                                                                           (uint32_t)c->film.height - 1) + 1;
                if (c->sampler_kind == 1 && c->zs_pdims > 0 &&
                    (long long)c->film.width * c->film.height * c->zs_pdims < (1ll << 31) &&
                    prow * c->zs_pdims < (1ll << 31)) {
                    // ZSobol pass table: the digits of GetSampleIndex that the pass's sample
                    // indices [base, base + S) share (those above their lowest differing bits),
                    // for the first zs_pdims dimensions; the camera stage and k_paths then
                    // evaluate only the digits below (two MixBits at 64 indices per pass)
                    const int plo = pass_plo(base, S);
                    long long key[kPtabKey];
                    ptab_key(c, zs, base, plo, key);
                    int buf = -1;
                    if (c->spec_valid) {
                        // the table the previous pass built ahead on the side stream (ptab_build's
                        // caller below): this stream waits for it, whether it is used or not, so
                        // no build of this pass overlaps it
                        HIP_TRY(hipStreamWaitEvent(c->stream, c->ev_tab, 0));
                        bool same = true;
                        for (int k = 0; k < kPtabKey; ++k) same = same && key[k] == c->spec_key[k];
                        if (same) buf = c->spec_buf;
                        c->spec_valid = false;
                    }
                    if (buf < 0) {
                        buf = 1 - c->tab_buf;
                        int rc2 = ptab_build(c, c->stream, zs, base, plo, buf, call_stride == 0 || call_stride == S);
                        if (rc2) return rc2;
                        if (!c->d_zs_ptab[buf]) buf = -1;
                    }
                    if (buf >= 0) {
                        c->tab_buf = buf;
                        p.zs.ptab = c->d_zs_ptab[buf];
                        p.zs.ctab = c->zs_pdims >= 10 ? c->d_zs_ctab[buf] : nullptr;
                        p.zs.pdims = c->zs_pdims;
                        p.zs.plo = plo;
                        spec_next = c->ptab_spec != 0;
                        spec_zs = zs;
                    }
                }
                // 16384 blocks (64 per CU, ~14 samples per thread at the bench's pass): the measured optimum
                // between one round of resident blocks and one sample per thread
                // (profiles/r06_ab_camera_grid.json)
                const int cgrid = blocks_for(n0, 256, 256 * 64);
                hipLaunchKernelGGL(kcam[c->render_mode ? 1 : 0][sv], dim3(cgrid), dim3(256), 0, c->stream, p);
                HIP_TRY(hipGetLastError());
                EV_MARK(ec1);
                c->timed.push_back({ec, ec1, &avr_stats::ms_camera, false});
                if (spec_next) HIP_TRY(hipEventRecord(c->ev_cam, c->stream));
            }
            EV_MARK(e0);
            // gray medium: sigma_a and sigma_s tables constant over all 471 wavelengths
            const int mk = c->med.type == 3 ? 1 : (c->med.type == 4 ? 2 : (c->med.type == 1 || c->med.type == 2 ? 3 : 0));
            const int sv = c->sampler_kind == 0 ? 0 : (avr::smp::zsobol_wide(p.zs) ? 2 : 1);
            // the kImage instantiation also carries the power light sampler's pick (light_pick)
            const bool general_lights = c->n_image_lights > 0 || c->lights.power;
            const int kv = ((((c->render_mode * 2 + (general_lights ? 1 : 0)) * 4 + mk) * 3 + sv) * 2 +
                            (c->med.emissive ? 1 : 0)) * 2 + (c->gray && c->med.type != 4 ? 1 : 0);
            hipLaunchKernelGGL(c->kpaths[kv], dim3(c->paths_grid[kv]), dim3(256), 0, c->stream, p);
            HIP_TRY(hipGetLastError());
            {
                const int kmed = c->med.type == 3 ? 3 : (c->med.type == 4 ? 4 : (c->med.type == 1 || c->med.type == 2 ? 1 : 0));
                std::snprintf(c->last_kpaths, sizeof(c->last_kpaths), "k_paths<%s, %s, %d, %d, %s, %s>",
                              c->med.emissive ? "true" : "false", (c->gray && c->med.type != 4) ? "true" : "false",
                              sv == 0 ? 0 : (sv == 1 ? 2 : 3), kmed, general_lights ? "true" : "false",
                              c->render_mode ? "true" : "false");
            }
            EV_MARK(e1);
            p.rec_mode = 1;   // k_film reads the records k_paths wrote (in slot order)
            p.pix_slot = c->d_pix_slot;
            p.fast = c->render_mode;
            // fast mode: the wavelength pdfs with the hardware exp (its wavelengths are the hardware log's)
            using KF = void (*)(avr::Params);
            static const KF kfilm[2][2] = {{avr::k_film<false, false>, avr::k_film<true, false>},
                                           {avr::k_film<false, true>, avr::k_film<true, true>}};
            hipLaunchKernelGGL(kfilm[c->render_mode ? 1 : 0][c->film.nbuckets > 0 ? 1 : 0], dim3(blocks_for(P)), dim3(256), avr::film_lds_bytes(c->film.nbuckets),
                               c->stream, p);
            HIP_TRY(hipGetLastError());
            EV_MARK(e2);
            c->timed.push_back({e0, e1, &avr_stats::ms_medium, true});
            c->timed.push_back({e1, e2, &avr_stats::ms_film, false});
            if (spec_next) {
                // the NEXT pass's table (sample indices [base + S, base + 2S): the next loop
                // iteration's, or the next avr_render call's when the caller walks the indices in
                // order) built ahead into the other buffer on the low-priority side stream: it
                // waits for this pass's camera stage (the last reader of that buffer, k_paths of
                // the previous pass, is then done too) and is dispatched as k_paths' blocks retire
                // in its drain, instead of in front of the next camera stage. A pass whose key
                // differs builds its own table (and this one is discarded).
                const bool in_call = base + Smax < spp_end || call_stride == 0;
                const long long nb = in_call ? base + S : spp_begin + call_stride;
                const int nplo = pass_plo(nb, S);
                HIP_TRY(hipStreamWaitEvent(c->tstream, c->ev_cam, 0));
                const int tb = 1 - c->tab_buf;
                // (not timed: events around it would measure its wait for the drain too)
                { int rc2 = ptab_build(c, c->tstream, spec_zs, nb, nplo, tb, in_call || call_stride == S); if (rc2) return rc2; }
                HIP_TRY(hipEventRecord(c->ev_tab, c->tstream));
                if (c->d_zs_ptab[tb]) {
                    ptab_key(c, spec_zs, nb, nplo, c->spec_key);
                    c->spec_buf = tb;
                    c->spec_valid = true;
                }
            }
            c->last_base = (int)base;
            c->last_S = S;
            c->last_order_gen = c->order_gen;
            continue;
        }
        EV_MARK(c0);
        if (c->sampler_kind) hipLaunchKernelGGL(avr::k_camera<true>, dim3(blocks_for(n0)), dim3(256), 0, c->stream, p);
        else hipLaunchKernelGGL(avr::k_camera<false>, dim3(blocks_for(n0)), dim3(256), 0, c->stream, p);
        HIP_TRY(hipGetLastError());
        EV_MARK(c1);
        c->timed.push_back({c0, c1, &avr_stats::ms_camera, false});
        c->h_count[0] = (int)n0;
        HIP_TRY(hipMemcpyAsync(c->d_counts, c->h_count, sizeof(int), hipMemcpyHostToDevice, c->stream));
        int cur = 0;
        long long count = n0;
        bool first = true;
        while (count > 0) {
            const int nxt = cur ^ 1;
            HIP_TRY(hipMemsetAsync(c->d_counts + nxt, 0, sizeof(int), c->stream));
            HIP_TRY(hipMemsetAsync(c->d_counts + 2, 0, sizeof(int), c->stream));
            p.queue_in = first ? nullptr : c->d_queue[cur];
            p.count_in = c->d_counts + cur;
            const int nbins = 8 * c->med.mres[0] * c->med.mres[1] * c->med.mres[2];
            const bool bin = c->ray_binning && nbins <= 8 * 4096;
            if (bin && c->bin_cap < n0) {
                for (int **b : {&c->d_bin_keys, &c->d_bin_out}) {
                    if (*b) (void)hipFree(*b);
                    HIP_TRY(dalloc(b, (size_t)n0));
                }
                if (!c->d_bin_hist) HIP_TRY(dalloc(&c->d_bin_hist, (size_t)8 * 4096));
                c->bin_cap = n0;
            }
            auto bin_queue = [&](const int *queue, const int *count_p, const float4 *o, const float4 *d) -> int {
                HIP_TRY(hipMemsetAsync(c->d_bin_hist, 0, nbins * sizeof(int), c->stream));
                const int nbk = blocks_for(count);
                hipLaunchKernelGGL(avr::k_bin_count, dim3(nbk), dim3(256), 0, c->stream, c->med, queue, count_p, o, d,
                                   c->d_bin_keys, c->d_bin_hist);
                hipLaunchKernelGGL(avr::k_bin_scan, dim3(1), dim3(1024), 0, c->stream, c->d_bin_hist, nbins);
                hipLaunchKernelGGL(avr::k_bin_scatter, dim3(nbk), dim3(256), 0, c->stream, queue, count_p,
                                   c->d_bin_keys, c->d_bin_hist, c->d_bin_out);
                HIP_TRY(hipGetLastError());
                return AVR_OK;
            };
            // camera rays keep their pixel order (already coherent); later depths are binned
            if (bin && !first) {
                EV_MARK(s0);
                int rc = bin_queue(c->d_queue[cur], c->d_counts + cur, c->ps.o, c->ps.d);
                if (rc) return rc;
                EV_MARK(s1);
                c->timed.push_back({s0, s1, &avr_stats::ms_binning, false});
                HIP_TRY(hipMemcpyAsync(c->d_queue[cur], c->d_bin_out, (size_t)count * sizeof(int),
                                       hipMemcpyDeviceToDevice, c->stream));
            }
            p.queue_out = c->d_queue[nxt];
            p.count_out = c->d_counts + nxt;
            p.shadow_count = c->d_counts + 2;
            const int nb = blocks_for(count);
            EV_MARK(m0);
            if (c->sampler_kind) hipLaunchKernelGGL(avr::k_medium<true>, dim3(nb), dim3(256), 0, c->stream, p);
            else hipLaunchKernelGGL(avr::k_medium<false>, dim3(nb), dim3(256), 0, c->stream, p);
            HIP_TRY(hipGetLastError());
            EV_MARK(m1);
            p.sh_perm = nullptr;
            if (bin) {
                // the shadow rays k_medium just pushed, binned the same way (read through sh_perm)
                EV_MARK(s2);
                int rc = bin_queue(nullptr, c->d_counts + 2, c->sh.o, c->sh.d);
                if (rc) return rc;
                EV_MARK(s3);
                c->timed.push_back({s2, s3, &avr_stats::ms_binning, false});
                p.sh_perm = c->d_bin_out;
            }
            EV_MARK(m15);
            hipLaunchKernelGGL(avr::k_shadow, dim3(nb), dim3(256), 0, c->stream, p);
            HIP_TRY(hipGetLastError());
            EV_MARK(m2);
            c->timed.push_back({m0, m1, &avr_stats::ms_medium, true});
            c->timed.push_back({m15, m2, &avr_stats::ms_shadow, false});
            // the queue length decides the next launch: the wavefront organisation syncs here
            HIP_TRY(hipMemcpyAsync(c->h_count, c->d_counts + nxt, sizeof(int), hipMemcpyDeviceToHost, c->stream));
            HIP_TRY(hipStreamSynchronize(c->stream));
            count = c->h_count[0];
            cur = nxt;
            first = false;
        }
        EV_MARK(f0);
        hipLaunchKernelGGL((c->film.nbuckets > 0 ? avr::k_film<true> : avr::k_film<false>), dim3(blocks_for(P)), dim3(256), avr::film_lds_bytes(c->film.nbuckets), c->stream, p);
        HIP_TRY(hipGetLastError());
        EV_MARK(f1);
        c->timed.push_back({f0, f1, &avr_stats::ms_film, false});
        c->last_base = (int)base;
        c->last_S = S;
    }
    EV_MARK(evEnd);
    c->timed.push_back({evStart, evEnd, &avr_stats::ms_total, false});
    return AVR_OK;
}

int avr_transmittance_device(avr_context *c, long long n, const float *p0, const float *p1, const float *lambda,
                             float *tr) {
    if (!c || n < 0 || (n > 0 && (!p0 || !p1 || !lambda || !tr))) return fail(AVR_ERR_ARG, "bad transmittance query");
    if (!c->has_medium) return fail(AVR_ERR_STATE, "medium required");
    if (n == 0) return AVR_OK;
    HIP_TRY(hipSetDevice(c->device));
    avr::Params p{};
    p.med = c->med;
    p.stats = c->d_stats;
    const int blocks = (int)std::min<long long>((n + 255) / 256, 8192);
    EV_MARK(t0);
    hipLaunchKernelGGL(avr::k_transmittance, dim3(blocks), dim3(256), 0, c->stream, p, n, p0, p1, lambda, tr);
    HIP_TRY(hipGetLastError());
    EV_MARK(t1);
    c->timed.push_back({t0, t1, &avr_stats::ms_shadow, false});
    return AVR_OK;
}

int avr_transmittance(avr_context *c, long long n, const float *p0, const float *p1, const float *lambda, float *tr) {
    if (!c || n < 0 || (n > 0 && (!p0 || !p1 || !lambda || !tr))) return fail(AVR_ERR_ARG, "bad transmittance query");
    if (n == 0) return AVR_OK;
    HIP_TRY(hipSetDevice(c->device));
    float *d = nullptr;
    HIP_TRY(dalloc(&d, (size_t)n * 14));
    float *dp0 = d, *dp1 = d + 3 * n, *dl = d + 6 * n, *dtr = d + 10 * n;
    HIP_TRY(hipMemcpyAsync(dp0, p0, 3 * n * sizeof(float), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(dp1, p1, 3 * n * sizeof(float), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(dl, lambda, 4 * n * sizeof(float), hipMemcpyHostToDevice, c->stream));
    int rc = avr_transmittance_device(c, n, dp0, dp1, dl, dtr);
    if (rc == AVR_OK) {
        hipError_t e = hipMemcpyAsync(tr, dtr, 4 * n * sizeof(float), hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        if (e != hipSuccess) rc = fail(AVR_ERR_HIP, hipGetErrorString(e));
    }
    (void)hipStreamSynchronize(c->stream);
    (void)hipFree(d);
    return rc;
}

int avr_sync(avr_context *c) {
    if (!c) return fail(AVR_ERR_ARG, "null context");
    HIP_TRY(hipStreamSynchronize(c->stream));
    return AVR_OK;
}

int avr_get_stats(avr_context *c, avr_stats *out) {
    if (!c || !out) return fail(AVR_ERR_ARG, "null arg");
    HIP_TRY(hipSetDevice(c->device));
    int rc = fold_stats(c);
    if (rc) return rc;
    *out = c->stats;
    return AVR_OK;
}

int avr_reset_stats(avr_context *c) {
    if (!c) return fail(AVR_ERR_ARG, "null context");
    HIP_TRY(hipSetDevice(c->device));
    int rc = fold_stats(c);
    if (rc) return rc;
    c->stats = {};
    HIP_TRY(hipMemsetAsync(c->d_stats, 0, sizeof(unsigned long long) * avr::kNumStats, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return AVR_OK;
}

static constexpr int kMetricBlocks = 1024;

static int film_image(avr_context *c, const avr::Mat3 &M, int fp16, float *d_out) {
    const long long np = (long long)c->film.width * c->film.height;
    hipLaunchKernelGGL(avr::k_film_image, dim3(blocks_for(np, 256, 4096)), dim3(256), 0, c->stream, c->film, M,
                       fp16, d_out);
    HIP_TRY(hipGetLastError());
    return AVR_OK;
}

int avr_film_image_device(avr_context *c, const float out_from_sensor[9], int fp16, float *d_out) {
    if (!c || !c->has_film || !out_from_sensor || !d_out) return fail(AVR_ERR_STATE, "no film or null argument");
    HIP_TRY(hipSetDevice(c->device));
    avr::Mat3 M;
    for (int i = 0; i < 9; ++i) M.m[i] = out_from_sensor[i];
    return film_image(c, M, fp16 ? 1 : 0, d_out);
}

int avr_film_set_reference(avr_context *c, const float *reference_rgb, const float out_from_sensor[9], int fp16) {
    if (!c || !c->has_film || !reference_rgb || !out_from_sensor) return fail(AVR_ERR_STATE, "no film or null argument");
    HIP_TRY(hipSetDevice(c->device));
    const size_t np = (size_t)c->film.width * c->film.height;
    if (c->d_reference) (void)hipFree(c->d_reference);
    if (c->d_image) (void)hipFree(c->d_image);
    c->d_reference = nullptr;
    c->d_image = nullptr;
    HIP_TRY(dalloc(&c->d_reference, 3 * np));
    HIP_TRY(dalloc(&c->d_image, 3 * np));
    if (!c->d_metric) HIP_TRY(dalloc(&c->d_metric, (size_t)(kMetricBlocks + 1) * avr::kMetricSlots));
    HIP_TRY(hipMemcpyAsync(c->d_reference, reference_rgb, 3 * np * sizeof(float), hipMemcpyHostToDevice, c->stream));
    for (int i = 0; i < 9; ++i) c->ref_out_from_sensor.m[i] = out_from_sensor[i];
    c->ref_fp16 = fp16 ? 1 : 0;
    HIP_TRY(hipStreamSynchronize(c->stream));
    return AVR_OK;
}

int avr_film_metric(avr_context *c, int metric, float *out) {
    if (!c || !c->has_film || !out) return fail(AVR_ERR_STATE, "no film");
    if (!c->d_reference) return fail(AVR_ERR_STATE, "no reference image (avr_film_set_reference)");
    if (metric < 0 || metric > 3) return fail(AVR_ERR_ARG, "metric must be 0 MSE, 1 MAE, 2 MRSE, 3 ME");
    HIP_TRY(hipSetDevice(c->device));
    int rc;
    if ((rc = film_image(c, c->ref_out_from_sensor, c->ref_fp16, c->d_image))) return rc;
    const int np = c->film.width * c->film.height;
    double *tot = c->d_metric + (size_t)kMetricBlocks * avr::kMetricSlots;
    hipLaunchKernelGGL(avr::k_metric, dim3(kMetricBlocks), dim3(256), 0, c->stream, c->d_image, c->d_reference, np,
                       metric, c->d_metric);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(avr::k_metric_final, dim3(1), dim3(64), 0, c->stream, c->d_metric, kMetricBlocks, tot);
    HIP_TRY(hipGetLastError());
    double h[avr::kMetricSlots];
    HIP_TRY(hipMemcpyAsync(h, tot, sizeof(h), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    // / (Float(xres) * Float(yres)); ME rounds its sums to float first (image.cpp:573-577)
    const float npix = (float)c->film.width * (float)c->film.height;
    const int n = metric == 3 ? 9 : 3;
    for (int k = 0; k < n; ++k) out[k] = metric == 3 ? (float)h[k] / npix : (float)(h[k] / npix);
    return AVR_OK;
}

// FLIP for `imgtool diff --metric FLIP` (src/ext/flip/flip.cpp:1085-1112, ComputeFLIPError)
int avr_flip(avr_context *c, const float *test, const float *ref, int width, int height, float ppd, float *error) {
    if (!c || !test || !ref || !error || width < 1 || height < 1) return fail(AVR_ERR_ARG, "avr_flip: bad arguments");
    HIP_TRY(hipSetDevice(c->device));
    if (!(ppd > 0)) ppd = avr::flip::ppd_default();
    std::vector<float> sf, ef, pf;
    const int rs = avr::flip::spatial_filter(ppd, sf);
    const int rd = avr::flip::detection_filter(ppd, false, ef);
    (void)avr::flip::detection_filter(ppd, true, pf);
    const float cmax = avr::flip::max_distance();
    const size_t n = (size_t)width * height;
    float *d_in = nullptr, *d_f = nullptr, *d_out = nullptr;
    avr::flip::F4 *d_yc = nullptr;
    auto cleanup = [&]() {
        if (d_in) (void)hipFree(d_in);
        if (d_f) (void)hipFree(d_f);
        if (d_out) (void)hipFree(d_out);
        if (d_yc) (void)hipFree(d_yc);
    };
    const size_t nf = sf.size() + ef.size() + pf.size();
    if (dalloc(&d_in, 6 * n) != hipSuccess || dalloc(&d_f, nf) != hipSuccess || dalloc(&d_out, n) != hipSuccess ||
        dalloc(&d_yc, 2 * n) != hipSuccess) {
        cleanup();
        return fail(AVR_ERR_HIP, "avr_flip: allocation failed");
    }
    std::vector<float> filt(nf);
    std::copy(sf.begin(), sf.end(), filt.begin());
    std::copy(ef.begin(), ef.end(), filt.begin() + sf.size());
    std::copy(pf.begin(), pf.end(), filt.begin() + sf.size() + ef.size());
    hipError_t e = hipMemcpyAsync(d_in, test, 3 * n * sizeof(float), hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(d_in + 3 * n, ref, 3 * n * sizeof(float), hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(d_f, filt.data(), nf * sizeof(float), hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(avr::k_flip_prep, dim3(blocks_for((long long)n)), dim3(256), 0, c->stream, d_in, d_in + 3 * n,
                           (int)n, d_yc, d_yc + n);
        hipLaunchKernelGGL(avr::k_flip_error, dim3(blocks_for((long long)n)), dim3(256), 0, c->stream, d_yc, d_yc + n,
                           width, height, d_f, rs, d_f + sf.size(), d_f + sf.size() + ef.size(), rd, cmax, d_out);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(error, d_out, n * sizeof(float), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    cleanup();
    if (e != hipSuccess) return fail(AVR_ERR_HIP, std::string("avr_flip: ") + hipGetErrorString(e));
    return AVR_OK;
}

int avr_film_read(avr_context *c, double *rgb, double *w) {
    if (!c || !c->has_film || !rgb || !w) return fail(AVR_ERR_STATE, "no film");
    const size_t np = (size_t)c->film.width * c->film.height;
    HIP_TRY(hipMemcpyAsync(rgb, c->film.rgb_sum, 3 * np * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipMemcpyAsync(w, c->film.w_sum, np * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return AVR_OK;
}

int avr_film_read_spectral(avr_context *c, double *bucket_sums, double *weight_sums) {
    if (!c || !c->has_film || c->film.nbuckets <= 0) return fail(AVR_ERR_STATE, "no spectral film");
    if (!bucket_sums || !weight_sums) return fail(AVR_ERR_ARG, "null buffer");
    const size_t nb = (size_t)c->film.width * c->film.height * c->film.nbuckets;
    HIP_TRY(hipMemcpyAsync(bucket_sums, c->film.bucket_sum, nb * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipMemcpyAsync(weight_sums, c->film.bucket_w, nb * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return AVR_OK;
}

int avr_film_spectral_device_ptrs(avr_context *c, void **bucket_sums, void **weight_sums) {
    if (!c || !c->has_film || c->film.nbuckets <= 0 || !bucket_sums || !weight_sums)
        return fail(AVR_ERR_STATE, "no spectral film");
    *bucket_sums = c->film.bucket_sum;
    *weight_sums = c->film.bucket_w;
    return AVR_OK;
}

int avr_film_device_ptrs(avr_context *c, void **rgb, void **w) {
    if (!c || !c->has_film || !rgb || !w) return fail(AVR_ERR_STATE, "no film");
    *rgb = c->film.rgb_sum;
    *w = c->film.w_sum;
    return AVR_OK;
}

int avr_last_pass_samples(avr_context *c, float *L, float *lambda, float *pdf, long long n_max, int *first,
                          int *ns) {
    AVR_QUIESCE(c);
    if (!c || !c->has_film || !L || !lambda || !pdf || !first || !ns) return fail(AVR_ERR_ARG, "null arg");
    const long long n = (long long)c->film.width * c->film.height * c->last_S;
    if (n_max < n) return fail(AVR_ERR_ARG, "buffer too small for the last pass");
    if (n > 0 && c->last_persistent && c->last_order_gen != c->order_gen)
        return fail(AVR_ERR_STATE, "the pixel order changed since the last render (its records are in the old order)");
    if (n > 0 && c->last_persistent) {
        // k_paths' records (L), its camera stage's wavelengths and their pdfs as k_film evaluates them
        HIP_TRY(hipMemcpy(L, c->ps.rec, n * sizeof(float4), hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(lambda, c->ps.cam2, n * sizeof(float4), hipMemcpyDeviceToHost));
        {
            avr::DevFilm f = c->film;
            hipLaunchKernelGGL(avr::k_lambda_pdfs, dim3(blocks_for(n)), dim3(256), 0, c->stream, f, c->ps.cam2, c->ps.cam4, n,
                               c->last_fast ? 1 : 0);
            HIP_TRY(hipGetLastError());
            HIP_TRY(hipStreamSynchronize(c->stream));
        }
        HIP_TRY(hipMemcpy(pdf, c->ps.cam4, n * sizeof(float4), hipMemcpyDeviceToHost));
        if (!c->h_pix_slot.empty()) {   // slot order -> pixel order
            const long long np = (long long)c->film.width * c->film.height;
            std::vector<float> tmp(4 * (size_t)np);
            for (float *a : {L, lambda, pdf})
                for (long long sb = 0; sb < n; sb += np) {
                    std::memcpy(tmp.data(), a + 4 * sb, 4 * np * sizeof(float));
                    for (long long p = 0; p < np; ++p)
                        std::memcpy(a + 4 * (sb + p), tmp.data() + 4 * (size_t)c->h_pix_slot[(size_t)p], 4 * sizeof(float));
                }
        }
    } else if (n > 0) {
        HIP_TRY(hipMemcpy(L, c->ps.L, n * sizeof(float4), hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(lambda, c->ps.lambda, n * sizeof(float4), hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(pdf, c->ps.pdf, n * sizeof(float4), hipMemcpyDeviceToHost));
    }
    *first = c->last_base;
    *ns = c->last_S;
    return AVR_OK;
}

int avr_last_kernel(avr_context *c, char *buf, int cap) {
    if (!c || !buf || cap <= 0) return fail(AVR_ERR_ARG, "null arg");
    std::snprintf(buf, (size_t)cap, "%s", c->last_kpaths);
    return AVR_OK;
}

int avr_last_pass_weights(avr_context *c, float *w, long long n_max) {
    AVR_QUIESCE(c);
    if (!c || !c->has_film || !w) return fail(AVR_ERR_ARG, "null arg");
    const long long n = (long long)c->film.width * c->film.height * c->last_S;
    if (n_max < n) return fail(AVR_ERR_ARG, "buffer too small for the last pass");
    if (n > 0 && c->last_persistent && c->filter_type != 0 && c->last_order_gen != c->order_gen)
        return fail(AVR_ERR_STATE, "the pixel order changed since the last render (its records are in the old order)");
    if (c->filter_type == 0) {
        for (long long i = 0; i < n; ++i) w[i] = 1.f;   // BoxFilter::Sample weight
    } else if (n > 0 && c->last_persistent) {
        std::vector<float> camw((size_t)n);
        HIP_TRY(hipMemcpy(camw.data(), c->ps.camw, n * sizeof(float), hipMemcpyDeviceToHost));
        const long long np = (long long)c->film.width * c->film.height;
        for (long long i = 0; i < n; ++i)
            w[i] = camw[c->h_pix_slot.empty() ? i : (i / np) * np + c->h_pix_slot[(size_t)(i % np)]];
    } else if (n > 0) {
        HIP_TRY(hipMemcpy(w, c->ps.weight, n * sizeof(float), hipMemcpyDeviceToHost));
    }
    return AVR_OK;
}

int avr_film_export_device(avr_context *c, void *dst) {
    if (!c || !c->has_film || !dst) return fail(AVR_ERR_STATE, "no film");
    const size_t np = (size_t)c->film.width * c->film.height;
    double *d = (double *)dst;
    HIP_TRY(hipMemcpyAsync(d, c->film.rgb_sum, 3 * np * sizeof(double), hipMemcpyDeviceToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(d + 3 * np, c->film.w_sum, np * sizeof(double), hipMemcpyDeviceToDevice, c->stream));
    if (c->film.nbuckets > 0)   // SpectralFilm: bucket sums then weights follow
        HIP_TRY(hipMemcpyAsync(d + 4 * np, c->film.bucket_sum, 2 * np * c->film.nbuckets * sizeof(double),
                               hipMemcpyDeviceToDevice, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return AVR_OK;
}

// RGBFilm sums of several contexts (one per GPU, one process: pbrt's in-process multi-GPU
// render) SUM-reduced into the root context's film with RCCL over xGMI: rgb, weights and,
// for a SpectralFilm, the bucket sums — in place on the root.
int avr_film_reduce_rccl(avr_context **ctxs, int n, int root) {
    if (!ctxs || n < 1 || root < 0 || root >= n) return fail(AVR_ERR_ARG, "film reduce: bad context list");
    for (int i = 0; i < n; ++i) {
        if (!ctxs[i] || !ctxs[i]->has_film) return fail(AVR_ERR_STATE, "film reduce: context without a film");
        const avr::DevFilm &a = ctxs[i]->film, &b = ctxs[root]->film;
        if (a.width != b.width || a.height != b.height || a.nbuckets != b.nbuckets)
            return fail(AVR_ERR_ARG, "film reduce: films differ in resolution or buckets");
        for (int j = 0; j < i; ++j)
            if (ctxs[j]->device == ctxs[i]->device) return fail(AVR_ERR_ARG, "film reduce: one context per GPU");
    }
    std::vector<int> devs(n);
    for (int i = 0; i < n; ++i) {
        devs[i] = ctxs[i]->device;
        HIP_TRY(hipSetDevice(devs[i]));
        HIP_TRY(hipStreamSynchronize(ctxs[i]->stream));
    }
    // communicators are created once per clique (ncclCommInitAll costs a bootstrap) and
    // cached on the contexts; a different context list releases the old cliques first
    const std::vector<avr_context *> clique(ctxs, ctxs + n);
    bool cached = true;
    for (int i = 0; i < n && cached; ++i) cached = ctxs[i]->comm && ctxs[i]->comm_group == clique;
    if (!cached) {
        for (int i = 0; i < n; ++i) release_comms(ctxs[i]);
        std::vector<ncclComm_t> fresh(n);
        if (ncclCommInitAll(fresh.data(), n, devs.data()) != ncclSuccess)
            return fail(AVR_ERR_HIP, "ncclCommInitAll failed");
        for (int i = 0; i < n; ++i) {
            ctxs[i]->comm = fresh[i];
            ctxs[i]->comm_group = clique;
        }
    }
    std::vector<ncclComm_t> comms(n);
    for (int i = 0; i < n; ++i) comms[i] = ctxs[i]->comm;
    const size_t np = (size_t)ctxs[root]->film.width * ctxs[root]->film.height;
    const size_t nb = (size_t)ctxs[root]->film.nbuckets;
    ncclResult_t r = ncclGroupStart();
    for (int i = 0; r == ncclSuccess && i < n; ++i) {
        avr::DevFilm &f = ctxs[i]->film;
        r = ncclReduce(f.rgb_sum, f.rgb_sum, 3 * np, ncclDouble, ncclSum, root, comms[i], ctxs[i]->stream);
        if (r == ncclSuccess) r = ncclReduce(f.w_sum, f.w_sum, np, ncclDouble, ncclSum, root, comms[i], ctxs[i]->stream);
        if (r == ncclSuccess && nb > 0)
            r = ncclReduce(f.bucket_sum, f.bucket_sum, 2 * np * nb, ncclDouble, ncclSum, root, comms[i], ctxs[i]->stream);
    }
    const ncclResult_t re = ncclGroupEnd();
    if (r == ncclSuccess) r = re;
    hipError_t e = hipSuccess;
    for (int i = 0; i < n; ++i) {
        (void)hipSetDevice(devs[i]);
        const hipError_t ei = hipStreamSynchronize(ctxs[i]->stream);
        if (e == hipSuccess) e = ei;
    }
    if (r != ncclSuccess) return fail(AVR_ERR_HIP, std::string("film reduce: ") + ncclGetErrorString(r));
    if (e != hipSuccess) return fail(AVR_ERR_HIP, std::string("film reduce: ") + hipGetErrorString(e));
    return AVR_OK;
}

}  // extern "C"

#include "avr_graph_capi.hip"

#if defined(AVR_PROFILE_SECTIONS) || defined(AVR_PROBE_STATS)
// Variant builds only (not part of include/avr.h): read and clear the k_paths section cycles
// (or, with AVR_PROBE_STATS, the walk / gather probe counters)
// of this context (stats[kNumStats .. kNumStats + 4], written by every k_paths unit).
extern "C" int avr_debug_sections(avr_context *c, unsigned long long *out) {
    if (!c || !out) return fail(AVR_ERR_ARG, "null argument");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(c->stream));
    HIP_TRY(hipMemcpy(out, c->d_stats + avr::kNumStats, 8 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemset(c->d_stats + avr::kNumStats, 0, 8 * sizeof(unsigned long long)));
    return AVR_OK;
}
#endif

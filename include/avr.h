/* avr.h — C-ABI of the MI355X-native volumetric path integrator (libavr_hip.so).
 *
 * Drop-in boundary for pbrt-v4's volumetric path in tsvdh/AcceleratedVolRenderer
 * (paths relative to /root/reference/src/pbrt). Plain C types only: opaque
 * handles, host pointers + sizes, int status codes (0 = ok), a thread-local
 * error string. No exceptions cross the ABI; buffers passed in are copied
 * during the call. One context per GPU; calls on one context are serialised
 * by the caller (pbrt drives Render() from one thread: cpu/render.cpp:159).
 *
 * Replaces:
 *   VolPathIntegrator::Render/Li/SampleLd   cpu/integrators.cpp:72-298, 962-1399
 *   SampleT_maj + DDAMajorantIterator        media.h:136-214, 730-806
 *   GridMedium SamplePoint/SampleRay/ctor    media.h:265-352, media.cpp:212-330
 *   WorkQueue push / ForAllQueued            wavefront/workqueue.h:41-172
 *   RGBFilm::AddSample / GetPixelRGB         film.h:232-316
 */
#ifndef AVR_H
#define AVR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AVR_OK 0
#define AVR_ERR_ARG 1
#define AVR_ERR_HIP 2
#define AVR_ERR_STATE 3

#define AVR_TABLE_SIZE 471 /* DenselySampledSpectrum over 360..830 nm (spectrum.h:374-420) */

typedef struct avr_context avr_context;

/* Work counters and kernel times accumulated over every avr_render call since the context
 * was created or avr_reset_stats (pbrt's ReportKernelStats analogue,
 * wavefront/wavefront.cpp:47-56). Resolved when read: rendering never waits for them. */
typedef struct avr_stats {
    unsigned long long medium_lookups;  /* SamplePoint density fetches in k_medium   */
    unsigned long long medium_items_in; /* work items consumed by k_medium           */
    unsigned long long medium_items_out;/* survivors + shadow rays pushed by k_medium;
                                           k_paths: phase-function samples (real scatters
                                           that continue the path)                  */
    unsigned long long shadow_lookups;  /* density fetches in k_shadow               */
    unsigned long long shadow_items;    /* shadow rays traced                        */
    unsigned long long medium_dda_steps;
    unsigned long long shadow_dda_steps;
    unsigned long long medium_launches;
    unsigned long long loop_iterations;        /* k_paths: wave tracking iterations       */
    unsigned long long active_lane_iterations; /* k_paths: sum of busy lanes per iteration */
    double ms_camera, ms_medium, ms_shadow, ms_film; /* summed hipEvent times      */
    double ms_total;                                  /* first launch .. film done  */
    double ms_setup;   /* one-off device tables built by avr_render (ZSobol pixel table) */
    double ms_binning; /* wavefront ray binning (avr_set_ray_binning): key, scan, scatter passes */
} avr_stats;

/* Last error message of the calling thread ("" if none). */
const char *avr_last_error(void);

/* Context on HIP device `device` (one process per GPU; no implicit peer access).
 * `max_paths` bounds the paths in flight per pass (0 = default: 64M for the persistent
 * kernel, whose per-sample HBM state is 116 B — the 16-B radiance record plus the camera
 * stage's 6 x 16 B + 4 B, about 7.4 GB at 64M — 16M for the wavefront
 * kernels; at most 2^31 - 1: path ids are 32-bit, AVR_ERR_ARG above). */
int avr_context_create(int device, long long max_paths, avr_context **out);
/* Also releases the RCCL communicators the context shares with the other contexts of its
 * last avr_film_reduce_rccl list (see there: not concurrently with work on those contexts). */
int avr_context_destroy(avr_context *ctx);
/* Kernel organisation: 0 = persistent-wave megakernel k_paths (default: path state in
 * VGPRs, ballot-based lane refill), 1 = wavefront kernels k_camera/k_medium/k_shadow with
 * compacted SoA queues between events (pbrt wavefront decomposition). Same estimator. */
int avr_set_kernel_mode(avr_context *ctx, int mode);
/* Lookup trace (measurement): while d_points is non-null, the wavefront kernels append the
 * unit-box point of every GridMedium density fetch (float4 {x, y, z, 0}, fetch order) to
 * d_points (device, capacity cap) and count them in *d_count (device u64, zeroed by the
 * caller; counts past cap are not stored). NULL stops tracing. */
int avr_record_lookups(avr_context *ctx, void *d_points, long long cap, void *d_count);
/* The density fetch alone (SampledGrid::Lookup, containers.h:804-835, through the same fat /
 * linear layout code as the path kernels) over n unit-box points (device float4), results
 * to d_out (device, n floats); synchronous; *ms = the kernel's HIP-event time. */
int avr_density_fetch(avr_context *ctx, const void *d_points, long long n, float *d_out, float *ms);
/* Render mode for later renders (SURVEY.md §7 "replay / fast"): 0 = replay (default) — the
 * device evaluates log/atanh/cosh/sin/cos by the canonical f64 sequences and FastExp by pbrt's
 * CPU polynomial (util/math.h:450-471), so every sample replays the CPU VolPathIntegrator's bit
 * for bit; 1 = fast — the hardware v_log/v_exp/v_sin/v_cos (about 1 ulp) and a single
 * free-flight decision per candidate: the same estimator with different last bits, so parity
 * is statistical (film error within the Monte Carlo noise). Applies to the persistent kernel
 * (kernel mode 0); the wavefront kernels always replay. */
int avr_set_render_mode(avr_context *ctx, int mode);
/* Wavefront organisation (kernel mode 1) only: 1 = counting-sort the medium queue (depths
 * after the camera rays) and the shadow queue by (majorant cell of the ray origin, direction
 * octant) before each k_medium / k_shadow launch, so a wave's lanes gather from nearby voxels
 * (north star "density fetches coalesced along sorted ray packets"). Results unchanged. */
int avr_set_ray_binning(avr_context *ctx, int on);
/* NanoVDBMedium in the persistent kernel: 1 = stage a coarse occupancy level of the majorant
 * grid (one bit per cell pair, up to 64^3 cells) in LDS, so majorant-0 cells skip the L2 read
 * of the majorant; 0 (default) = read every cell's majorant (measured 2 % faster: occupied
 * cells then wait for the LDS bit before their L2 read). Rebuilds the current majorant.
 * Results unchanged (no reference counterpart: a DDAMajorantIterator, media.h:141-214, memory
 * schedule only). */
int avr_set_majorant_occupancy(avr_context *ctx, int on);
/* ZSobolSampler passes of the persistent kernel: 1 (default) = after launching a pass, build the
 * NEXT pass's ZSobol pass table (sample indices [base + S, base + 2S)) into a second buffer on a
 * low-priority side stream, where the dispatcher serves it as the pass's k_paths blocks retire;
 * the next pass (in the same avr_render call, or the next call when the caller's calls advance
 * by a fixed stride: pbrt's pass loop, a rank of a sample shard) then skips its own build. A
 * pass whose indices differ builds its table as before. 0 = build every table in front of its camera stage.
 * Results unchanged (a schedule of ZSobolSampler::GetSampleIndex's digits, samplers.h:225-330). */
int avr_set_pass_table_ahead(avr_context *ctx, int on);
/* k_paths: refill a wave's idle lanes with new samples once at least `lanes` (1..64)
 * are idle (or none is busy); larger values batch the per-event handlers across lanes.
 * 0 = default (the measured optima in both render modes: 32; 20 for a non-emissive
 * NanoVDB medium at pbrt's 64^3 majorant, whose longer DDA walks favour smaller batches;
 * 16 for an RGBGridMedium; 48 for a GridMedium majorant of at most 2 cells per axis, e.g.
 * fast mode's tuned 1^3, whose one-cell walks leave the handlers dominant). */
int avr_set_refill_min(avr_context *ctx, int lanes);
/* k_paths: majorant-grid cells a lane may cross per tracking iteration before yielding to
 * the wave (0 = default: 10 for majorant grids up to 16^3, 32 for finer ones and for
 * RGBGridMedium, 28 for a non-emissive NanoVDB medium at 64^3 — measured optima); bounds the
 * divergence of the DDA walk. No effect on results. */
int avr_set_dda_budget(avr_context *ctx, int cells);
/* Density layout for the NEXT avr_medium_grid* / avr_medium_nanovdb call: 1 (default) also
 * builds a "fat" footprint copy — GridMedium: entry (ix,iy,iz) holds the 8 trilinear taps as
 * 32 contiguous bytes, (n+1)^3 x 32 B; NanoVDBMedium: the same 32 B per base voxel of every
 * 9^3 apron block of the density grid (512 x 32 B per block) — built on device if it fits in
 * free HBM with 8 GiB to spare, so a density fetch is one 32-B access in one cache line; 0
 * keeps only pbrt's linear layout (containers.h:834) / the apron blocks; 2 (GridMedium) builds a
 * bricked copy instead — 8^3 base voxels per brick with a +1 apron (9^3 floats, padded to 736),
 * bricks x-fastest, so a footprint's 8 taps lie in one brick (4 x 8 B within 368 B), 1.42x the
 * grid. Results are bit-identical in every layout. */
int avr_set_grid_layout(avr_context *ctx, int layout);
/* The current medium's density copy: 1 fat, 2 bricked, 0 none (pbrt's linear layout only). */
int avr_grid_layout_active(avr_context *ctx);
/* The persistent kernel's pixel order (SURVEY §7 step 6 / north star "density-grid fetches
 * coalesced along sorted ray packets"): `order` lists every pixel of the current film once
 * (row-major ids); within each sample index of a pass the camera stage and k_paths hand
 * pixels to lanes in that order, so consecutive lanes start coherent camera rays (e.g.
 * sorted by the majorant cell where the ray enters the medium). NULL restores scanline
 * order; a new film resets it. Results are identical in any order (per-pixel sums still
 * add the pixel's samples in sampleIndex order). */
int avr_set_pixel_order(avr_context *ctx, const int *order, long long n);
/* Run all work of this context on `hip_stream` (a hipStream_t; NULL = the context's own stream). */
int avr_set_stream(avr_context *ctx, void *hip_stream);

/* GridMedium (media.h:271-275, media.cpp:249-330). density is nx*ny*nz floats,
 * x fastest ((z*ny + y)*nx + x, util/containers.h:830-835). sigma_a/sigma_s/Le are
 * DenselySampled tables already scaled (sigmaScale / LeNorm folded in, as the ctor's
 * Scale() calls do). Le may be NULL (non-emissive). Lescale is the LeScale grid
 * (lnx*lny*lnz, LeNorm folded in) and may be NULL when Le is NULL.
 * Transforms are row-major 4x4 (renderFromMedium and its inverse).
 * The majorant grid (majorant_res, pbrt uses 16^3, media.cpp:229) is built on device. */
int avr_medium_grid(avr_context *ctx, const float *density, int nx, int ny, int nz, const float bounds[6],
                    const float render_from_medium[16], const float medium_from_render[16],
                    const float *sigma_a, const float *sigma_s, float g, const float *Le, const float *Lescale,
                    int lnx, int lny, int lnz, const int majorant_res[3]);
/* Same, but the density already lives in device memory of this context's GPU
 * (e.g. a 4 GiB grid generated on device). The caller keeps ownership and must keep
 * it alive while the context renders. */
int avr_medium_grid_device(avr_context *ctx, const float *d_density, int nx, int ny, int nz, const float bounds[6],
                           const float render_from_medium[16], const float medium_from_render[16],
                           const float *sigma_a, const float *sigma_s, float g, const float *Le,
                           const float *Lescale, int lnx, int lny, int lnz, const int majorant_res[3]);
/* Attach a temperature grid (nx*ny*nz f32, same layout as the density) to the current
 * GridMedium: emission Le = LeScale(p) * BlackbodySpectrum(T)(lambda) with
 * T = (temperature(p) - offset) * scale where T > 100 K (media.h:299-316, media.cpp:
 * 256-329: "temperature", "temperaturescale", "temperatureoffset"). The medium must have
 * been created without an Le spectrum (pbrt rejects both). */
int avr_medium_temperature(avr_context *ctx, const float *temperature, float temperature_scale,
                           float temperature_offset);
/* HomogeneousMedium (media.h:217-262, Create media.cpp:165-210) filling the interface box
 * `bounds` (medium space): constant sigma_a/sigma_s tables (sigmaScale folded in), g, and
 * optionally Le (471, LeScale folded in; null = not emissive). Its majorant segment is the
 * box crossing with sigma_maj = sigma_t (HomogeneousMajorantIterator). */
int avr_medium_homogeneous(avr_context *ctx, const float bounds[6], const float render_from_medium[16],
                           const float medium_from_render[16], const float *sigma_a, const float *sigma_s, float g,
                           const float *Le);
/* CloudMedium (media.h:430-528, Create media.cpp:455-485): procedural density (Perlin noise;
 * parameters density, wispiness, frequency) inside `bounds`, one majorant segment per ray
 * with sigma_maj = sigma_t. */
int avr_medium_cloud(avr_context *ctx, const float bounds[6], const float render_from_medium[16],
                     const float medium_from_render[16], const float *sigma_a, const float *sigma_s, float g,
                     float density, float wispiness, float frequency);
/* One NanoVDB FloatGrid as NanoVDBMedium reads it (media.h:624-672; NanoVDB is the
 * un-vendored openvdb@414bed84 feature/nanovdb submodule): the 8^3 leaf nodes (origin =
 * index coordinate of the leaf's voxel (0,0,0), multiples of 8; 512 values each, x-major
 * ((x&7)*8 + (y&7))*8 + (z&7) as LeafNode stores them), the constant tiles of the upper tree
 * levels (origin and edge length in voxels, multiples of 8), the background value returned
 * everywhere else, the active-voxel index bbox (inclusive, GridData::mIndexBBox) and the map:
 * index->world as a row-major 3x4 (Map::mMatD with mVecD as the last column) and the inverse
 * 3x3 (Map::mInvMatD); the float copies worldToIndexF uses are their roundings, as Map::set
 * makes them. World bbox = the map of the corners of [min, max + 1], each row evaluated
 * ((m0*x + m1*y) + m2*z) + t in f64. */
typedef struct avr_vdb_grid {
    int n_leaves;
    const int *leaf_origin;      /* 3 per leaf */
    const float *leaf_values;    /* 512 per leaf */
    int n_tiles;
    const int *tile_origin;      /* 3 per tile (may be NULL when n_tiles == 0) */
    const int *tile_size;        /* 1 per tile */
    const float *tile_value;     /* 1 per tile */
    float background;
    int index_bbox[6];           /* min xyz, max xyz */
    double index_to_world[12];
    double world_to_index[9];
} avr_vdb_grid;
/* NanoVDBMedium (media.h:602-685, ctor media.cpp:511-616, Create media.cpp:618-665):
 * density grid, optional temperature grid (NULL = not emissive), sigma tables with
 * sigmaScale folded in, g, LeScale, temperatureoffset, temperaturescale. Bounds are the
 * density grid's world bbox (union the temperature grid's); the 64^3 majorant is built on
 * the device with pbrt's one-voxel filter slop. Replaces NanoVDBMedium::Create's
 * readGrid + ctor: the caller hands over the tree it read. */
int avr_medium_nanovdb(avr_context *ctx, const avr_vdb_grid *density, const avr_vdb_grid *temperature,
                       const float render_from_medium[16], const float medium_from_render[16],
                       const float *sigma_a, const float *sigma_s, float g, float Lescale,
                       float temperature_offset, float temperature_scale);
/* RGBGridMedium (media.h:355-427, ctor media.cpp:339-378, Create media.cpp:380-453): an
 * nx*ny*nz grid (x fastest) on the box `bounds` whose voxels hold RGBUnboundedSpectrum
 * sigma_a / sigma_s and RGBIlluminantSpectrum Le as 4 floats {c0, c1, c2, scale} — the
 * RGBSigmoidPolynomial coefficients RGBColorSpace::ToRGBCoeffs gave the caller and the
 * spectrum's scale (spectrum.cpp:236-247). sigma_a or sigma_s may be NULL (treated as 1);
 * Le (NULL = none) needs sigma_a and the colour space's illuminant table (471, e.g. D65
 * for sRGB). sigma_scale is "scale", Le_scale "Lescale". The 16^3 majorant
 * sigma_scale * (max sigma_a + max sigma_s) is built on the device. */
int avr_medium_rgbgrid(avr_context *ctx, int nx, int ny, int nz, const float bounds[6],
                       const float render_from_medium[16], const float medium_from_render[16],
                       const float *sigma_a, const float *sigma_s, float sigma_scale, float g, const float *Le,
                       const float *illuminant, float Le_scale);
/* Same, but sigma_a / sigma_s / Le are float4 arrays already in device memory of this context's
 * GPU (e.g. a 1024^3 grid generated on device, 16 GiB per field); the caller keeps ownership
 * and keeps them alive while the context renders. */
int avr_medium_rgbgrid_device(avr_context *ctx, int nx, int ny, int nz, const float bounds[6],
                              const float render_from_medium[16], const float medium_from_render[16],
                              const float *d_sigma_a, const float *d_sigma_s, float sigma_scale, float g,
                              const float *d_Le, const float *illuminant, float Le_scale);
/* Medium interface of the current medium (pbrt: a shape with no material
 * whose MediumInterface has this medium inside and none outside, interaction.cpp:91-97
 * SkipIntersection, shapes.h:152-200 Sphere). radius > 0: a sphere of that radius at `center`
 * (render space) bounds the medium — camera rays start their first segment where they enter
 * it, every segment and shadow ray ends at its exit, rays that miss it see no medium (the
 * medium's SampleT_maj still clips to its bounds box, media.h:325-328); radius <= 0 returns
 * to the default model (the bounds box is the interface). Reset by every avr_medium_* call.
 * Both kernel organisations. */
int avr_medium_boundary_sphere(avr_context *ctx, const float center[3], float radius);
/* A convex polyhedral medium interface (e.g. a convex triangle mesh — a box mesh, a prism —
 * given by its face planes): n_planes half-spaces {nx, ny, nz, h} in render space, the
 * medium inside every n.p <= h (outward normals, 1..256 planes; 0 returns to the box). Same
 * semantics as the sphere; crossings by the parametric slab clip (vecmath.h:1547-1571
 * generalised), not pbrt's watertight triangle test, so paths match pbrt statistically. */
int avr_medium_boundary_convex(avr_context *ctx, const float *planes, int n_planes);
/* The medium bounds the last avr_medium_* call set (medium space, min xyz then max xyz). */
int avr_medium_bounds(avr_context *ctx, float bounds[6]);
/* Fill d_out[first .. first+count) of an n^3 grid with CloudMedium::Density
 * (media.h:496-520) at voxel centres (i+0.5)/n — the synthetic S-cloud input. */
int avr_generate_cloud(avr_context *ctx, float *d_out, int n, long long first, long long count, float density,
                       float wispiness, float frequency);
/* Fill voxels [first, first + count) of three n^3 float4 device arrays with the synthetic
 * RGB-coefficient explosion (BASELINE config C5's stand-in as an RGBGridMedium): {c0, c1, c2,
 * scale} of sigma_a, sigma_s and Le at voxel centres (i + 0.5) / n; each pointer is the
 * array's element `first`. */
int avr_generate_rgb_explosion(avr_context *ctx, float *d_sigma_a, float *d_sigma_s, float *d_Le, int n,
                               long long first, long long count);
/* Copy the device majorant grid to host (mres product floats). */
int avr_read_majorant(avr_context *ctx, float *out);
/* Rebuild the current medium's majorant grid at res[3] cells (1..255 per axis) from the
 * medium's own data (GridMedium / RGBGridMedium / NanoVDBMedium; the single-segment media
 * refuse). pbrt fixes 16^3 for grids (media.cpp:229) and 64^3 for NanoVDB (media.cpp:521):
 * replay parity with pbrt assumes those; any conservative majorant gives the same estimator
 * in expectation (SURVEY §7 "fast": tuned majorant, statistical parity). The persistent
 * kernel keeps grids of up to 4096 cells in LDS; finer grid majorants run the wavefront kernels. */
int avr_set_majorant_res(avr_context *ctx, const int res[3]);
/* The "tuned majorant": render the probe sample range [spp_begin, spp_end) twice per
 * candidate resolution (n triples in `candidates`; candidates ascending, then descending),
 * timed with HIP events on the context stream, keep the fastest (chosen[3]; each candidate's
 * faster probe in ms[n] when non-null). The film sums are restored and the work counters
 * reset afterwards; no pass table is built ahead during the probes. */
int avr_tune_majorant(avr_context *ctx, const int *candidates, int n, int spp_begin, int spp_end, int seed,
                      int max_depth, int chosen[3], float *ms);
/* k_paths' lane schedule chosen on the device for the current scene (replaces fixed
 * per-medium defaults): render the probe sample range twice per (refill lanes, DDA cells)
 * candidate pair (the faster probe counts), refill[i] x dda[j] (0 = the library default for either), timed with HIP
 * events on the context stream, and keep the fastest (chosen[2] = {refill, dda}; the nr*nd
 * probe times in ms[i * nd + j] when non-null) — except that the default pair (0, 0), when
 * listed (else the current schedule, when listed), is kept unless the fastest probe beats
 * every probe of that same effective schedule (e.g. refill 0 and refill 32 where 32 is the
 * default) by more than 2 % (the probes' run-to-run spread), so repeated runs choose the same
 * schedule. Film sums restored and work counters reset
 * afterwards, as avr_tune_majorant. The schedule never changes results, only how a wave
 * batches its lanes' events and walks. */
int avr_tune_walk(avr_context *ctx, const int *refill, int nr, const int *dda, int nd, int spp_begin, int spp_end,
                  int seed, int max_depth, int chosen[2], float *ms);

/* Lights (lights.h:244-305 DistantLight, lights.cpp:950-972 UniformInfiniteLight).
 * type 0 = distant: w = render-space unit vector towards the light
 *          (Normalize(renderFromLight(0,0,1)), lights.h:287); type 1 = uniform infinite;
 * type 2 = image infinite (then avr_light_image).
 * L = n tables of 471 floats; scale = final light scale (1/SpectrumToPhotometric folded in).
 * scene_radius = Bounds3::BoundingSphere radius of the scene bounds (lights.h:280). */
int avr_lights(avr_context *ctx, int n, const int *types, const float *w3, const float *L, const float *scale,
               float scene_radius);
/* ImageInfiniteLight (lights.h:552-640, ctor lights.cpp:1007-1040, Create lights.cpp:1527-1660)
 * for light `index` of the last avr_lights call, which lists it with type 2 (its L table is
 * ignored; `scale` is the final scale: "scale" / SpectrumToPhotometric(illuminant), times the
 * "illuminance" factor when given). A res x res equal-area octahedral map: per pixel the
 * RGBIlluminantSpectrum {c0, c1, c2, scale} of ClampZero(rgb) in the image's colour space,
 * `distribution` = Image::GetSamplingDistribution() (res*res, row y), the colour space's
 * illuminant (471) and renderFromLight / its inverse (row-major 4x4, the 3x3 part is used).
 * The library builds the compensated PiecewiseConstant2D that SampleLi / PDF_Li use with
 * allowIncompletePDF (VolPath always passes true). Scenes with image lights render with
 * the wavefront kernels. */
int avr_light_image(avr_context *ctx, int index, int res, const float *pixel_coeffs, const float *distribution,
                    const float *illuminant, const float render_from_light[16], const float light_from_render[16]);

/* VolPath's light sampler (VolPathIntegrator::Create "lightsampler", integrators.cpp:1402-1420;
 * LightSampler::Create, lightsamplers.cpp:22-37): 0 = "bvh" (default) or "uniform" — identical
 * for infinite lights (lightsamplers.h:266-277, 35-50); 1 = "power": PowerLightSampler
 * (lightsamplers.h:63-99, lightsamplers.cpp:76-96), lights picked by an AliasTable over
 * Average(Phi(lambda) / pdf) at SampleVisible(0.5) (DistantLight / UniformInfiniteLight /
 * ImageInfiniteLight::Phi, lights.cpp:216, 974, 1042). Kept across avr_lights calls; a power
 * render needs every image light's avr_light_image first. */
int avr_light_sampler(avr_context *ctx, int kind);

/* Camera: type 0 orthographic, 1 perspective (cameras.cpp:284-306, 404-427).
 * camera_from_raster: full 4x4 (projective for perspective); render_from_camera: affine 4x4. */
int avr_camera(avr_context *ctx, int type, const float camera_from_raster[16], const float render_from_camera[16]);

/* RGBFilm with a box filter and a PixelSensor (film.h:95-100, 232-316): sensor_rgb is the
 * 3 x 471 r̄ḡb̄ (cie1931: X, Y, Z) tables, imaging_ratio = exposureTime*ISO/100.
 * Allocates and zeroes the fp64 film sums (3 + 1 doubles per pixel). */
int avr_film(avr_context *ctx, int width, int height, const float filter_radius[2], const float *sensor_rgb,
             float imaging_ratio, float max_component_value);
int avr_film_clear(avr_context *ctx);
/* Pixel filter for later renders (GetCameraSample, samplers.h:797-815): type 0 BoxFilter
 * (filters.h:48-77, radius), 1 GaussianFilter(radius, sigma) (filters.h:80-118; sampled with
 * FilterSampler's tabulated distribution, filters.cpp:133-147, weight f/pdf; radius <= 4).
 * pbrt's default filter is gaussian radius 1.5, sigma 0.5 (scene.cpp:94, filters.cpp). */
int avr_set_filter(avr_context *ctx, int type, const float radius[2], float sigma);
/* Pixel sampler for later renders: 0 IndependentSampler (samplers.h:442-476, default here),
 * 1 ZSobolSampler with FastOwen randomisation (samplers.h:225-330; pbrt's default,
 * scene.cpp:93). samples_per_pixel is the sampler's pixelsamples: ZSobol lays out
 * (Morton(pixel) << log2(spp)) | sampleIndex, so avr_render must stay below it. */
int avr_set_sampler(avr_context *ctx, int kind, int samples_per_pixel);
/* ZSobolSampler: GetSampleIndex's digits above log2(spp) depend on (pixel, dimension) only;
 * the first render after a sampler/film change tabulates them for the first `dims`
 * dimensions (4 B per pixel-Morton row and dimension; default 256, 0 = compute every digit
 * per call). Results are identical either way. */
int avr_set_sampler_table(avr_context *ctx, int dims);
/* ZSobolSampler in the persistent kernel: a pass renders sample indices [b, b + S) that agree
 * above their lowest L differing bits, so every digit of GetSampleIndex above them — and the
 * permutation of the one just below, whose hash reads only those bits — is shared by the
 * pass's samples of one pixel. Each pass tabulates them for the first `dims` dimensions
 * (8 B per pixel-Morton row and dimension; default 96, 0 = off) and a sampler call then
 * evaluates only the digits below (2 base-4 digits for 64-index passes instead of
 * log2(spp)/2). Results are identical either way. Odd `dims` are rounded up to even (rows
 * of 16-B aligned entry pairs). Memory: two tables of rows x dims x 8 B (the pass's and the
 * level-A table it is derived from), rows = Morton(width - 1, height - 1) + 1 — 1.64 M rows at
 * 720p, 1.26 GB per table at 96 dimensions, up to ~4x the pixel count for non-square films —
 * allocated lazily by the first render, only with >= 8 GiB of HBM to spare (else the pixel
 * table serves every draw), next to max_paths' records; with dims >= 10 also a 48-B per-pixel
 * copy of the camera stage's six entries (44 MB at 720p). */
int avr_set_sampler_pass_table(avr_context *ctx, int dims);

/* Render sample indices [spp_begin, spp_end) of every pixel (the avr_set_sampler sampler,
 * seed), VolPathIntegrator maxdepth. Asynchronous on the context stream. */
int avr_render(avr_context *ctx, int spp_begin, int spp_end, int seed, int max_depth);
/* Integrator::Tr (cpu/integrators.cpp:324-374): ratio-tracking transmittance from p0[i] to
 * p1[i] (render space, xyz) at the four wavelengths lambda[4i..4i+3] (nm), n queries; writes
 * tr[4i..4i+3] = Tr / inv_w.Average(). RNG per query seeded with Hash(p0), Hash(p1), as pbrt.
 * avr_transmittance: host arrays, synchronous. _device: device arrays, async on the stream. */
int avr_transmittance(avr_context *ctx, long long n, const float *p0, const float *p1, const float *lambda,
                      float *tr);
int avr_transmittance_device(avr_context *ctx, long long n, const float *p0, const float *p1, const float *lambda,
                             float *tr);
int avr_sync(avr_context *ctx);
int avr_get_stats(avr_context *ctx, avr_stats *out);   /* waits for queued work */
int avr_reset_stats(avr_context *ctx);

/* Film readback: rgb_sum[W*H*3] and w_sum[W*H] (fp64 RGBFilm::Pixel sums). */
int avr_film_read(avr_context *ctx, double *rgb_sum, double *w_sum);
/* SpectralFilm (film.h:401-530; SpectralFilm::Create film.cpp:1037-1066 "nbuckets",
 * "lambdamin", "lambdamax"): after avr_film, n_buckets > 0 switches the film to uniform
 * wavelength sampling (SampledWavelengths::SampleUniform) over [lambda_min, lambda_max]
 * (within 360..830 nm here) and per-pixel bucket sums next to the RGB sums
 * (SpectralFilm::AddSample, film.h:413-455); 0 returns to RGBFilm. Readback: the fp64
 * Pixel::bucketSums / weightSums, [pixel * n_buckets + bucket]. */
int avr_film_spectral(avr_context *ctx, int n_buckets, float lambda_min, float lambda_max);
int avr_film_read_spectral(avr_context *ctx, double *bucket_sums, double *weight_sums);
int avr_film_spectral_device_ptrs(avr_context *ctx, void **d_bucket_sums, void **d_weight_sums);
/* In-process multi-GPU render (one context per GPU, e.g. avr_render(ctx_k, k*spp/N,
 * (k+1)*spp/N, ...)): SUM-reduce the n contexts' film sums (rgb, weights, SpectralFilm
 * buckets) into ctxs[root]'s film over RCCL (xGMI); the other films are left as they are.
 * Films must match in resolution and buckets; one context per device. The communicators
 * are created on the first reduce of a context list (ncclCommInitAll) and cached on the
 * contexts for later reduces of the same list; avr_context_destroy releases them.
 * Threading: the cached communicators tie the listed contexts together. Destroying one of
 * them, or reducing over a different list that contains one of them, destroys the whole
 * group's communicators; neither may run while another thread renders, reduces or reads on
 * any context of that group (calls on one context are serialized by the caller anyway). */
int avr_film_reduce_rccl(avr_context **ctxs, int n, int root);
/* Device pointers of the film sums (for an RCCL reduce across GPUs). */
int avr_film_device_ptrs(avr_context *ctx, void **d_rgb_sum, void **d_w_sum);
/* Device-to-device copy of the film sums into caller memory on the same GPU, laid out
 * [rgb_sum (W*H*3) | w_sum (W*H)] as doubles — the buffer handed to the RCCL reduce; a
 * SpectralFilm appends [bucket_sums (W*H*nb) | weight_sums (W*H*nb)]. */
int avr_film_export_device(avr_context *ctx, void *d_dst);

/* RGBFilm::GetImage on the device (film.cpp:533-565): per pixel GetPixelRGB (film.h:258-274)
 * with the caller's outputRGBFromSensorRGB (row-major 3x3), optionally as the fp16 image
 * ("savefp16": clamp to 65504, round to half). d_out: W*H*3 floats on this GPU. */
int avr_film_image_device(avr_context *ctx, const float output_from_sensor[9], int fp16, float *d_out);
/* --mse-reference-image (integrators.cpp:119-148, 209-219): keep a W*H*3 reference image
 * (host, row-major RGB) on the device; avr_film_metric then compares the film's GetImage
 * with it: metric 0 MSE, 1 MAE, 2 MRSE -> 3 per-channel values; 3 ME -> 9 values
 * (absolute, positive, negative per channel) with Image::MSE/MAE/MRSE/ME's definitions
 * (util/image.cpp:543-678), f64 sums by a fixed-order device reduction. */
int avr_film_set_reference(avr_context *ctx, const float *reference_rgb, const float output_from_sensor[9],
                           int fp16);
int avr_film_metric(avr_context *ctx, int metric, float *out);

/* FLIP error map (src/ext/flip/flip.cpp ComputeFLIPError, used by `imgtool diff --metric
 * FLIP`): test and reference are width*height RGB (interleaved, row-major) sRGB-encoded
 * values as the caller passes them (imgtool clamps to [0,1] first); ppd <= 0 takes the
 * reference's default 0.7 m / 0.7 m / 3840 px monitor. error: width*height floats. */
int avr_flip(avr_context *ctx, const float *test_rgb, const float *reference_rgb, int width, int height, float ppd,
             float *error);

/* ---- Lighting graph (src/graph/, the fork's own SampleT_maj callers) ----
 * The medium is the context's (avr_medium_*); geometry model: the medium's bounds box is
 * the boundary primitive. Sampling follows the reference's graph tools
 * (cmd/graph_maker.cpp:97-104): the scene sampler at its film resolution with
 * Options->pixelSamples, sampling index i -> pixel (i % resolution_x, i / resolution_x)
 * (graph/util.h:816-817). */
typedef struct avr_graph_sampling {
    int sampler;             /* 0 IndependentSampler, 1 ZSobolSampler                     */
    int seed;                /* sampler seed (Options->seed)                              */
    int samples_per_pixel;   /* Options->pixelSamples (RoundUpPow2(lightIterations))      */
    int film_width, film_height; /* the sampler's full resolution (ZSobol Morton layout)  */
    int resolution_x;        /* Options->graph.samplingResolution.x                       */
} avr_graph_sampling;

/* FreeGraphBuilder::TracePath (free/free_graph_builder.cpp:19-141), the medium walk: for
 * each of n_rays rays (origin o, direction d, first segment end t_first = the medium exit
 * after SkipIntersection, BuildGraph :166-196) `iterations` walks, walk w = ray*iterations+i
 * started with StartPixelSample(pixel(index0[ray] + i), sample_index). Writes up to
 * max_depth scatter points per walk to points[(w*max_depth + k)*3 ..] and the count to
 * counts[w] (count == max_depth: the reference's forcedEnd). Host arrays, synchronous. */
int avr_graph_walks(avr_context *ctx, const avr_graph_sampling *smp, long long n_rays, const float *o, const float *d,
                    const float *t_first, const long long *index0, int iterations, int sample_index, int max_depth,
                    float *points, int *counts);

/* avr_graph_walks with skip_dims sampler dimensions drawn after StartPixelSample before the
 * walk (the reinforcement walks continue the stream their ray's phase sample started). */
int avr_graph_walks_from(avr_context *ctx, const avr_graph_sampling *smp, long long n_rays, const float *o,
                         const float *d, const float *t_first, const long long *index0, int iterations,
                         int sample_index, int skip_dims, int max_depth, float *points, int *counts);

/* FreeGraphBuilder::ReinforceSparseVertices' rays (free_graph_builder.cpp:434-475): for each of
 * n vertices (ids, points n*3), GetSphereVolumePointsRandom(vertex_radius, point, n_rays) with
 * the sampler at StartPixelSample({0, 0}, cycle), then per sphere point p the medium's HG
 * Sample_p((1,0,0), Get2D()) at StartPixelSample(pixel(id * n_rays + p), cycle) and the medium
 * box crossing: o/d (n*n_rays*3), t_first (medium exit after SkipIntersection), valid
 * (RayEntersVolume). The walk from each valid ray: avr_graph_walks_from(.., index0 =
 * id * n_rays + p, iterations 1, sample_index cycle, skip_dims 2, max_depth - 1). */
int avr_graph_reinforce_rays(avr_context *ctx, const avr_graph_sampling *smp, int n, const int *vertex_ids,
                             const float *points, float vertex_radius, int n_rays, int cycle, float *o, float *d,
                             float *t_first, int *valid);

/* LightingCalculator::GetLightVector (lighting_calculator.cpp:84-155) with
 * ComputeRaysToSphere (graph/util.h:814-840) and SampleTransmittance (util.h:344-366):
 * light[v] = Inv4Pi * average over the disk points of vertex v (GetDiskPoints(vertex -
 * in_dir * max_dist_to_center * 2, sphere_radius, points_on_radius, in_dir)) whose ray along
 * in_dir crosses the medium box and the vertex's sphere inside the medium, of the average of
 * `iterations` ratio-tracking transmittances to a uniform point of the sphere chord.
 * vertices: n_vertices*3 (ids 0..n-1 in order). Host arrays, synchronous. */
int avr_graph_light(avr_context *ctx, const avr_graph_sampling *smp, int n_vertices, const float *vertices,
                    const float in_dir[3], float sphere_radius, int points_on_radius, int iterations,
                    float max_dist_to_center, float *light);

/* LightingCalculator::ComputeFinalLight (lighting_calculator.cpp:23-59): total = light +
 * sum of T^k light for k = 1..bounces, T in CSR (row_ptr[n+1], col ascending per row, val),
 * stopping before the first bounce whose vector holds a NaN/Inf; *iterations = bounces
 * completed. _device: device arrays, async on the context's stream (iterations read back
 * synchronously when non-null). */
int avr_graph_propagate(avr_context *ctx, int n, const int *row_ptr, const int *col, const float *val,
                        const float *light, int bounces, float *total, int *iterations);
int avr_graph_propagate_device(avr_context *ctx, int n, long long nnz, const int *row_ptr, const int *col,
                               const float *val, const float *light, int bounces, float *total, int *iterations);

/* FreeGraph assembly on the host (free_graph_builder.cpp:100-131, graph.cpp:134-229):
 * walks merged in walk order into vertices of radius `vertex_radius` — a scatter point joins
 * the nearest vertex strictly within the radius (nanoflann's RadiusResultSet bound; the
 * reference takes the first one its kd-tree reports), else the path's previous vertex when
 * within the radius, else becomes a new vertex; consecutive path vertices add edge samples;
 * each traced segment after a scatter counts a sample of the path's last vertex
 * (HandlePotentialPathEnd). avr_graph_transport: GetTransportMatrix (:61-82) as CSR rows
 * (row = vertex, col ascending, val = edge samples / vertex samples); row_ptr n+1, col/val
 * n_edges entries. */
typedef struct avr_graph avr_graph;
int avr_graph_create(float vertex_radius, avr_graph **out);
int avr_graph_destroy(avr_graph *g);
int avr_graph_add_walks(avr_graph *g, long long n_walks, int max_depth, const float *points, const int *counts);
/* Walks that start at an existing vertex (TracePath's startingVertex; -1 = none), traced with
 * max_depth - 1 scatters when a start vertex is given (max_depth counts path vertices). */
int avr_graph_add_walks_from(avr_graph *g, long long n_walks, int max_depth, const float *points, const int *counts,
                             const int *start_vertex);
/* Vertex::outEdges.size() per vertex; CountInRadius (squared distance < radius^2, self included) */
int avr_graph_out_degrees(avr_graph *g, int *out);
int avr_graph_count_in_radius(avr_graph *g, int n, const int *vertex_ids, float radius, int *counts);
int avr_graph_size(avr_graph *g, long long *n_vertices, long long *n_edges);
int avr_graph_vertices(avr_graph *g, float *xyz, int *samples);
int avr_graph_edges(avr_graph *g, int *from, int *to, int *samples);
int avr_graph_transport(avr_graph *g, int *row_ptr, int *col, float *val);
/* UseAndRemovePathInfo's in-node path length average (free_graph_builder.cpp:241-273) */
int avr_graph_in_node_path_length(avr_graph *g, float *average, long long *count);

/* Per-sample radiance of the LAST wavefront pass of the last avr_render (replay checks;
 * pbrt's --debugstart analogue, integrators.cpp:74-102). Element id = s*W*H + pixel,
 * s = sampleIndex - first sample of that pass. Writes n_max*4 floats into each of
 * L, lambda, pdf and returns the pass's first sample index and sample count. */
int avr_last_pass_samples(avr_context *ctx, float *L, float *lambda, float *pdf, long long n_max,
                          int *first_sample, int *n_samples);
/* Filter weights (CameraSample::filterWeight) of the last pass's samples, same indexing.
 * Both readbacks fail with AVR_ERR_STATE once the pixel order (avr_set_pixel_order, or a new
 * avr_film that drops it) changed after that render: its records are in the old slot order. */
int avr_last_pass_weights(avr_context *ctx, float *weight, long long n_max);
/* Template arguments of the last k_paths instantiation avr_render launched, as
 * "k_paths<emissive, gray, sampler, medium, image, fast>" (sampler 0 independent, 2 / 3 ZSobol
 * with 32- / 64-bit indices; "" before the first persistent render): lets a profiler pass
 * (rocprofv3 kernel names) be matched to the configuration that was timed. NUL-terminated,
 * truncated to cap bytes. */
int avr_last_kernel(avr_context *ctx, char *buf, int cap);

#ifdef __cplusplus
}
#endif
#endif /* AVR_H */

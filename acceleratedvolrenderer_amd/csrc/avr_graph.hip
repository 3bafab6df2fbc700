// avr_graph.hip — device kernels of the lighting-graph precompute (src/graph/ of the
// reference: the fork's own SampleT_maj callers), included by
// avr_capi.hip after avr_kernels.hip.
//
//  k_graph_walks   FreeGraphBuilder::TracePath (free/free_graph_builder.cpp:19-141), the
//                  medium part: one lane per light path, delta tracking segment by segment,
//                  scatter points written out; the order-dependent vertex merging stays on the
//                  host (avr_graph_add_walks), because a walk never depends on the graph.
//  k_graph_disk    LightingCalculator::GetLightVector (lighting_calculator.cpp:84-155): one
//                  lane per vertex enumerates its disk points (graph/util.h:179-204) and the
//                  ray/box/sphere crossings (util.h:419-503).
//  k_graph_tr      ComputeRaysToSphere (util.h:814-840) + SampleTransmittance (util.h:344-366):
//                  one lane per (vertex, disk point, iteration) ratio-tracking estimate.
//  k_graph_average the two Averager::GetAverage levels (util.h:545-565) and Inv4Pi.
//  k_graph_spmv    ComputeFinalLight's transport product (lighting_calculator.cpp:23-59):
//                  CSR row per lane, terms summed in ascending column order (Eigen's
//                  column-major sparse x sparse-vector order), NaN/Inf flag per bounce; the
//                  previous bounce's vector is added to the total in the same pass.
//
// Geometry model (shared with the oracle): the medium's boundary primitive is
// its bounds box (medium-space slab test, ray mapped without error offsets); spheres solve
// Sphere::BasicIntersect's interval quadric once for both roots.
namespace avr {
namespace graph {

// ray / sphere crossings and the hit kinds: avr_boundary.h (shared with the path kernels)
using namespace ::avr::shape;

// GetHits(primitive) in the model (util.h:419-458): slab test in medium space
__device__ __forceinline__ Hits box_hits(const DevMedium &m, V3 o, V3 d) {
    const V3 om = xf_point_lr(m.medium_from_render, o), dm = xf_vector(m.medium_from_render, d);
    float t0, t1;
    if (!intersect_box(m.bmin, m.bmax, om, dm, kInf, &t0, &t1)) return {kOutsideZeroHits, 0.f, 0.f};
    if (t0 > 0) return {kOutsideTwoHits, t0, t1};
    return {kInsideOneHit, t1, 0.f};
}


__device__ __forceinline__ void coordinate_system(V3 v1, V3 *v2, V3 *v3) {   // vecmath.h:1007-1013
    const float sign = __builtin_copysignf(1.f, v1.z);
    const float a = -1 / (sign + v1.z);
    const float b = v1.x * v1.y * a;
    *v2 = {1 + sign * sqr(v1.x) * a, sign * b, -sign * v1.x};
    *v3 = {b, sign + sqr(v1.y) * a, -v1.y};
}

// Sampling index -> pixel (util.h:816-817)
__device__ __forceinline__ void index_pixel(unsigned long long index, int resX, int *px, int *py) {
    *py = (int)(index / (unsigned long long)resX);
    *px = (int)(index - (unsigned long long)*py * (unsigned long long)resX);
}

// One disk point's ray after the crossings (k_graph_disk -> k_graph_tr)
struct DiskRec {
    float4 o_start;      // ray origin at the medium entry (SkipIntersection), startScatterT
    float dist;          // distInSphere (endScatterT - startScatterT)
    int valid;           // crossed both the box and the sphere inside the medium
};

}  // namespace graph

// skipDims: sampler dimensions already drawn after StartPixelSample before TracePath (the
// reinforcement rays' phase sample, free_graph_builder.cpp:448-451)
template <bool kZSobol>
__global__ void __launch_bounds__(256) k_graph_walks(Params P, long long nPaths, int iterations, const float *__restrict__ o,
                                                     const float *__restrict__ d, const float *__restrict__ tFirst,
                                                     const long long *__restrict__ index0, int sampleIndex, int skipDims,
                                                     int resX, int maxDepth, float *__restrict__ points,
                                                     int *__restrict__ counts) {
    __shared__ float s_maj[4096];
    const float *maj = stage_majorant(P.med, s_maj);
    const Lambda lw = sample_visible(0.f);   // mediumData.defaultLambda = film.SampleWavelengths(0)
    const Spec lam = lw.l;
    const LambdaIdx li = lambda_index(lam);
    const Spec sig_a = sample_table(P.med.sigma_a, li), sig_s = sample_table(P.med.sigma_s, li);
    unsigned long long nLookup = 0, nSteps = 0, nIn = 0;
    for (long long path = blockIdx.x * (long long)blockDim.x + threadIdx.x; path < nPaths;
         path += (long long)gridDim.x * blockDim.x) {
        ++nIn;
        const long long r = path / iterations, i = path - r * iterations;
        int px, py;
        graph::index_pixel((unsigned long long)(index0[r] + i), resX, &px, &py);
        PathSampler<kZSobol> smp;
        smp.start(P, px, py, sampleIndex);
        for (int k = 0; k < skipDims; ++k) (void)smp.get1d(P);
        V3 ro = {o[3 * r], o[3 * r + 1], o[3 * r + 2]}, rd = {d[3 * r], d[3 * r + 1], d[3 * r + 2]};
        bool usedTHit = false;
        int k = 0;
        while (k < maxDepth) {
            const float h0 = smp.get1d(P);
            const float h1 = smp.get1d(P);
            Pcg32 rng;
            rng.set_sequence(hash_u32(f2u(h0)), hash_u32(f2u(h1)));
            float tMax;
            if (!usedTHit) {
                tMax = tFirst[r];
                usedTHit = true;
            } else {
                const graph::Hits h = graph::box_hits(P.med, ro, rd);
                if (h.type == graph::kOutsideZeroHits) break;
                tMax = h.t0;
            }
            bool scattered = false;
            V3 pS = {0.f, 0.f, 0.f};
            const float u = smp.get1d(P);
            auto cb = [&](V3 p, const MediumSample &ms, const Spec &sigma_maj, const Spec &) -> bool {
                const float pAbsorb = ms.sigma_a.v0 / sigma_maj.v0;
                const float pScat = ms.sigma_s.v0 / sigma_maj.v0;
                const float pNull = fmaxf_(0.f, 1 - pAbsorb - pScat);
                const int mode = sample_discrete3(pAbsorb, pScat, pNull, rng.uniform());
                if (mode == 0) return false;
                if (mode == 1) {
                    scattered = true;
                    pS = p;
                    return false;
                }
                return true;
            };
            sample_t_maj(P.med, maj, Ray{ro, rd}, tMax, u, rng, sig_a, sig_s, Spec::c(0.f), lam, nLookup, nSteps, cb);
            if (!scattered) break;
            float *dst = points + 3 * (path * maxDepth + k);
            dst[0] = pS.x;
            dst[1] = pS.y;
            dst[2] = pS.z;
            ++k;
            if (k == maxDepth) break;
            float u0, u1, pdf;
            smp.get2d(P, &u0, &u1);
            const V3 wi = hg_sample(-rd, P.med.g, u0, u1, &pdf);
            ro = pS;
            rd = wi;
        }
        counts[path] = k;
    }
    flush_stat(P.stats, 3, nLookup);
    flush_stat(P.stats, 4, nIn);
    flush_stat(P.stats, 6, nSteps);
}

// FreeGraphBuilder::ReinforceSparseVertices' rays (free_graph_builder.cpp:434-475), one lane
// per listed vertex: StartPixelSample({0, 0}, cycle) on a copy of the sampler, then
// GetSphereVolumePointsRandom (util.h:238-252: rejection sampling in the cube; the three
// Get1D of one Point3f are GCC-evaluated right to left, so the first draw is z; the
// arithmetic is (double(u) - 0.5) * 2 * radius), then per point StartPixelSample(pixel(id *
// nRays + point), cycle), the medium's HG Sample_p((1, 0, 0), Get2D()), GetHits(box) and
// SkipIntersection. valid = RayEntersVolume (OutsideTwoHits or InsideOneHit).
template <bool kZSobol>
__global__ void __launch_bounds__(256) k_graph_reinforce_rays(Params P, int n, const int *__restrict__ ids,
                                                              const float *__restrict__ pts, float radius, int nRays,
                                                              int cycle, int resX, float *__restrict__ o,
                                                              float *__restrict__ d, float *__restrict__ tFirst,
                                                              int *__restrict__ valid) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n) return;
    const V3 c = {pts[3 * v], pts[3 * v + 1], pts[3 * v + 2]};
    PathSampler<kZSobol> cube;
    cube.start(P, 0, 0, cycle);
    const double r = (double)radius;
    for (int k = 0; k < nRays;) {
        const float pz = (float)(((double)cube.get1d(P) - 0.5) * 2 * r);
        const float py = (float)(((double)cube.get1d(P) - 0.5) * 2 * r);
        const float px = (float)(((double)cube.get1d(P) - 0.5) * 2 * r);
        const V3 q = {px, py, pz};
        if (!(length(q) < radius)) continue;
        const long long ray = (long long)v * nRays + k;
        const V3 sp = q + c;
        int pxl, pyl;
        graph::index_pixel((unsigned long long)ids[v] * (unsigned long long)nRays + (unsigned long long)k, resX, &pxl,
                           &pyl);
        PathSampler<kZSobol> smp;
        smp.start(P, pxl, pyl, cycle);
        float u0, u1, pdf;
        smp.get2d(P, &u0, &u1);
        const V3 dir = hg_sample(V3{1.f, 0.f, 0.f}, P.med.g, u0, u1, &pdf);
        const graph::Hits h = graph::box_hits(P.med, sp, dir);
        V3 og = sp;
        float t = 0.f;
        int ok = 0;
        if (h.type == graph::kOutsideTwoHits) {
            og = sp + dir * h.t0;
            t = h.t1 - h.t0;
            ok = 1;
        } else if (h.type == graph::kInsideOneHit) {
            t = h.t0;
            ok = 1;
        }
        o[3 * ray] = og.x; o[3 * ray + 1] = og.y; o[3 * ray + 2] = og.z;
        d[3 * ray] = dir.x; d[3 * ray + 1] = dir.y; d[3 * ray + 2] = dir.z;
        tFirst[ray] = t;
        valid[ray] = ok;
        ++k;
    }
}

// Per vertex: disk points around vertex - inDir * maxDistToCenter * 2 (GetDiskPoints, util.h:179-204,
// grid order x then y), the medium-box and sphere crossings of the ray along inDir from each,
// GetStartEndT (util.h:484-503), SkipIntersection to the medium entry and SkipForward.
__global__ void __launch_bounds__(256) k_graph_disk(DevMedium m, int nv, const float *__restrict__ verts, V3 dir,
                                                    float radius, int n, float maxDist, int maxPts,
                                                    graph::DiskRec *__restrict__ rec, int *__restrict__ npts) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= nv) return;
    const V3 c = {verts[3 * v], verts[3 * v + 1], verts[3 * v + 2]};
    const V3 origin = c - (dir * maxDist) * 2.f;
    V3 xv, yv;
    graph::coordinate_system(dir, &xv, &yv);
    const float step = radius / (float)(n + 1);
    xv = xv * step;
    yv = yv * step;
    int k = 0;
    for (int x = -n; x <= n; ++x)
        for (int y = -n; y <= n; ++y) {
            V3 p = (n == 0) ? origin : (origin + (float)x * xv) + (float)y * yv;
            if (n != 0 && length(p - origin) > radius) continue;
            graph::DiskRec r;
            r.valid = 0;
            r.dist = 0.f;
            r.o_start = make_float4(0.f, 0.f, 0.f, 0.f);
            const graph::Hits mh = graph::box_hits(m, p, dir), sh = graph::sphere_hits(c, radius, p, dir);
            if (mh.type == graph::kOutsideTwoHits && sh.type == graph::kOutsideTwoHits) {
                const float startT = mh.t0, endT = graph::smin(mh.t1, sh.t1), startScatterT = graph::smax(mh.t0, sh.t0);
                const float endScatterT = endT;
                if (!(endT < startScatterT || endScatterT < startT)) {
                    const V3 os = p + dir * startT;
                    r.o_start = make_float4(os.x, os.y, os.z, startScatterT - startT);
                    r.dist = (endScatterT - startT) - (startScatterT - startT);
                    r.valid = 1;
                }
            }
            if (k < maxPts) rec[(long long)v * maxPts + k] = r;
            ++k;
        }
    npts[v] = k;
}

// One ratio-tracking estimate per lane: (vertex v0 + j / (maxPts * iterations), point, iteration).
template <bool kZSobol>
__global__ void __launch_bounds__(256) k_graph_tr(Params P, int v0, int nvChunk, int maxPts, int iterations, V3 dir,
                                                  int resX, const graph::DiskRec *__restrict__ rec,
                                                  const int *__restrict__ npts, float *__restrict__ tr) {
    __shared__ float s_maj[4096];
    const float *maj = stage_majorant(P.med, s_maj);
    const Lambda lw = sample_visible(0.f);
    const Spec lam = lw.l;
    const LambdaIdx li = lambda_index(lam);
    const Spec sig_a = sample_table(P.med.sigma_a, li), sig_s = sample_table(P.med.sigma_s, li);
    unsigned long long nLookup = 0, nSteps = 0, nIn = 0;
    const long long total = (long long)nvChunk * maxPts * iterations;
    for (long long j = blockIdx.x * (long long)blockDim.x + threadIdx.x; j < total;
         j += (long long)gridDim.x * blockDim.x) {
        const int i = (int)(j % iterations);
        const long long vk = j / iterations;
        const int k = (int)(vk % maxPts);
        const int v = v0 + (int)(vk / maxPts);
        const int np = npts[v];
        if (k >= np) continue;
        const graph::DiskRec r = rec[(long long)v * maxPts + k];
        if (!r.valid) continue;
        ++nIn;
        int px, py;
        graph::index_pixel((unsigned long long)v * (unsigned long long)np + (unsigned long long)k, resX, &px, &py);
        PathSampler<kZSobol> smp;
        smp.start(P, px, py, i);
        const float curDist = r.dist * smp.get1d(P);
        const float curT = r.o_start.w + curDist;
        // RNG rng(Hash(Get1D()), Hash(Get1D())) (util.h:346): GCC evaluates the two arguments
        // right to left, so the first draw is the offset and the second the sequence index
        const float uOff = smp.get1d(P);
        const float uSeq = smp.get1d(P);
        Pcg32 rng;
        rng.set_sequence(hash_u32(f2u(uSeq)), hash_u32(f2u(uOff)));
        float Tr = 1.f;
        const float u = smp.get1d(P);
        auto cb = [&](V3, const MediumSample &ms, const Spec &sigma_maj, const Spec &) -> bool {
            const float sigma_n = fmaxf_(0.f, (sigma_maj.v0 - ms.sigma_a.v0) - ms.sigma_s.v0);
            Tr *= sigma_n / sigma_maj.v0;
            return Tr != 0;
        };
        sample_t_maj(P.med, maj, Ray{{r.o_start.x, r.o_start.y, r.o_start.z}, dir}, curT, u, rng, sig_a, sig_s,
                     Spec::c(0.f), lam, nLookup, nSteps, cb);
        tr[j] = Tr;
    }
    flush_stat(P.stats, 3, nLookup);
    flush_stat(P.stats, 4, nIn);
    flush_stat(P.stats, 6, nSteps);
}

// Averager::GetAverage (util.h:545-565, unit weights) over the iterations of each valid disk
// point, then over the points; light = average * Inv4Pi (lighting_calculator.cpp:151-152).
__global__ void __launch_bounds__(256) k_graph_average(int v0, int nvChunk, int maxPts, int iterations,
                                                       const graph::DiskRec *__restrict__ rec,
                                                       const int *__restrict__ npts, const float *__restrict__ tr,
                                                       float *__restrict__ light) {
    const int vc = blockIdx.x * blockDim.x + threadIdx.x;
    if (vc >= nvChunk) return;
    const int v = v0 + vc;
    const int np = npts[v] < maxPts ? npts[v] : maxPts;
    float avg = 0.f, w = 0.f;
    for (int k = 0; k < np; ++k) {
        if (!rec[(long long)v * maxPts + k].valid) continue;
        const float *t = tr + ((long long)vc * maxPts + k) * iterations;
        float a = 0.f, wi = 0.f;
        for (int i = 0; i < iterations; ++i) {
            a += t[i] * 1.f;
            wi += 1.f;
        }
        a = wi == 0 ? 0.f : a / wi;
        avg += a * 1.f;
        w += 1.f;
    }
    light[v] = (w == 0 ? 0.f : avg / w) * kInv4Pi;
}

// One bounce of ComputeFinalLight: next = T * cur by CSR rows (terms in ascending column order,
// the first product starting the sum), flag[it] |= NaN/Inf in next; and, unless an earlier
// bounce was flagged, total += cur for it >= 1 (the previous bounce's product).
__global__ void __launch_bounds__(256) k_graph_spmv(int n, const int *__restrict__ rowptr, const int *__restrict__ col,
                                                    const float *__restrict__ val, const float *__restrict__ cur,
                                                    float *__restrict__ next, float *__restrict__ total,
                                                    int *__restrict__ flags, int it) {
    bool stopped = false;
    if (it >= 1)
        for (int j = 0; j < it; ++j) stopped |= flags[j] != 0;
    bool bad = false;
    for (int row = blockIdx.x * blockDim.x + threadIdx.x; row < n; row += gridDim.x * blockDim.x) {
        const int e0 = rowptr[row], e1 = rowptr[row + 1];
        float acc = 0.f;
        if (e0 < e1) {
            acc = val[e0] * cur[col[e0]];
            for (int e = e0 + 1; e < e1; ++e) acc = acc + val[e] * cur[col[e]];
        }
        next[row] = acc;
        bad |= __builtin_isnan(acc) || __builtin_isinf(acc);
        if (it >= 1 && !stopped) total[row] += cur[row];
    }
    if (__ballot(bad) != 0 && __lane_id() == 0) atomicOr(flags + it, 1);
}

// The last bounce's product added unless a flag stopped the iteration (also the first-order
// copy total = light happens on the host side of the stream, hipMemcpyAsync).
__global__ void __launch_bounds__(256) k_graph_accumulate(int n, const float *__restrict__ cur, float *__restrict__ total,
                                                          const int *__restrict__ flags, int it) {
    for (int j = 0; j < it; ++j)
        if (flags[j]) return;
    for (int row = blockIdx.x * blockDim.x + threadIdx.x; row < n; row += gridDim.x * blockDim.x) total[row] += cur[row];
}

}  // namespace avr

// avr_graph_capi.hip — C-ABI of the lighting-graph precompute (include/avr.h, "Lighting
// graph"), included at the end of avr_capi.hip (shares avr_context, fail(), HIP_TRY).
#include "avr_graph_host.h"

namespace {

// Params for the graph kernels: the context's medium plus the graph's sampler
int graph_params(avr_context *c, const avr_graph_sampling *s, unsigned long long maxIndex, int maxSampleIndex,
                 avr::Params *p) {
    if (!s) return fail(AVR_ERR_ARG, "null sampling");
    if (s->sampler != 0 && s->sampler != 1) return fail(AVR_ERR_ARG, "sampler must be 0 (independent) or 1 (zsobol)");
    if (s->resolution_x <= 0) return fail(AVR_ERR_ARG, "resolution_x must be positive");
    *p = avr::Params{};
    p->med = c->med;
    p->stats = c->d_stats;
    p->seed = s->seed;
    p->sampler_kind = s->sampler;
    if (s->sampler == 1) {
        if (s->samples_per_pixel <= 0 || s->film_width <= 0 || s->film_height <= 0)
            return fail(AVR_ERR_ARG, "zsobol: samples_per_pixel and film resolution required");
        avr::smp::ZSobolParams zs = avr::smp::zsobol_params(s->samples_per_pixel, s->film_width, s->film_height, s->seed);
        if (zs.nBase4Digits > 16) return fail(AVR_ERR_ARG, "zsobol: film resolution x spp beyond 2^32 sample indices");
        // (Morton(pixel) << log2(spp)) | sampleIndex must fit 32 bits (the device's ZSobol index)
        const unsigned long long yMax = maxIndex / (unsigned long long)s->resolution_x;
        const unsigned long long xMax = std::min<unsigned long long>(maxIndex, (unsigned long long)s->resolution_x - 1);
        int bits = 0;
        while ((1ull << bits) <= std::max(xMax, yMax)) ++bits;
        int sbits = 0;
        while ((1ll << sbits) <= (long long)maxSampleIndex) ++sbits;
        if (2 * bits + std::max(zs.log2spp, sbits) > 32)
            return fail(AVR_ERR_ARG, "zsobol: graph sampling indices beyond the 2^32 Sobol' index range");
        p->zs = zs;
    }
    return AVR_OK;
}

}  // namespace

extern "C" {

int avr_graph_walks(avr_context *c, const avr_graph_sampling *s, long long n_rays, const float *o, const float *d,
                    const float *t_first, const long long *index0, int iterations, int sample_index, int max_depth,
                    float *points, int *counts) {
    return avr_graph_walks_from(c, s, n_rays, o, d, t_first, index0, iterations, sample_index, 0, max_depth, points,
                                counts);
}

int avr_graph_walks_from(avr_context *c, const avr_graph_sampling *s, long long n_rays, const float *o, const float *d,
                         const float *t_first, const long long *index0, int iterations, int sample_index,
                         int skip_dims, int max_depth, float *points, int *counts) {
    if (!c || n_rays < 0 || iterations < 0 || max_depth < 0 || skip_dims < 0)
        return fail(AVR_ERR_ARG, "bad walk arguments");
    if (!c->has_medium) return fail(AVR_ERR_STATE, "medium required");
    const long long nPaths = n_rays * (long long)iterations;
    if (nPaths == 0) return AVR_OK;
    if (!o || !d || !t_first || !index0 || !counts || (max_depth > 0 && !points)) return fail(AVR_ERR_ARG, "null buffer");
    long long maxIdx = 0;
    for (long long r = 0; r < n_rays; ++r) {
        if (index0[r] < 0) return fail(AVR_ERR_ARG, "negative sampling index");
        maxIdx = std::max(maxIdx, index0[r] + iterations - 1);
    }
    avr::Params p;
    int rc = graph_params(c, s, (unsigned long long)maxIdx, sample_index, &p);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(c->device));
    const int md = std::max(max_depth, 1);
    char *buf = nullptr;
    const size_t szRay = (size_t)n_rays * 3 * sizeof(float), szT = (size_t)n_rays * sizeof(float);
    const size_t szI = (size_t)n_rays * sizeof(long long), szP = (size_t)nPaths * md * 3 * sizeof(float);
    const size_t szC = (size_t)nPaths * sizeof(int);
    HIP_TRY(dalloc(&buf, 2 * szRay + szT + szI + szP + szC + 64));
    float *dO = (float *)buf, *dD = (float *)(buf + szRay), *dT = (float *)(buf + 2 * szRay);
    long long *dI = (long long *)(buf + ((2 * szRay + szT + 7) & ~(size_t)7));
    float *dP = (float *)((char *)dI + szI);
    int *dC = (int *)((char *)dP + szP);
    hipError_t e = hipMemcpyAsync(dO, o, szRay, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(dD, d, szRay, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(dT, t_first, szT, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(dI, index0, szI, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) {
        const int blocks = blocks_for(nPaths, 256, 256 * 64);
        if (p.sampler_kind == 1)
            hipLaunchKernelGGL(avr::k_graph_walks<true>, dim3(blocks), dim3(256), 0, c->stream, p, nPaths, iterations,
                               dO, dD, dT, dI, sample_index, skip_dims, s->resolution_x, max_depth, dP, dC);
        else
            hipLaunchKernelGGL(avr::k_graph_walks<false>, dim3(blocks), dim3(256), 0, c->stream, p, nPaths, iterations,
                               dO, dD, dT, dI, sample_index, skip_dims, s->resolution_x, max_depth, dP, dC);
        e = hipGetLastError();
    }
    if (e == hipSuccess && max_depth > 0) e = hipMemcpyAsync(points, dP, szP, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(counts, dC, szC, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    (void)hipStreamSynchronize(c->stream);
    (void)hipFree(buf);
    if (e != hipSuccess) return fail(AVR_ERR_HIP, std::string("graph walks: ") + hipGetErrorString(e));
    return AVR_OK;
}

int avr_graph_reinforce_rays(avr_context *c, const avr_graph_sampling *s, int n, const int *vertex_ids,
                             const float *points, float vertex_radius, int n_rays, int cycle, float *o, float *d,
                             float *t_first, int *valid) {
    if (!c || n < 0 || n_rays < 0 || cycle < 0 || !(vertex_radius > 0)) return fail(AVR_ERR_ARG, "bad reinforce arguments");
    if (!c->has_medium) return fail(AVR_ERR_STATE, "medium required");
    const long long nr = (long long)n * n_rays;
    if (nr == 0) return AVR_OK;
    if (!vertex_ids || !points || !o || !d || !t_first || !valid) return fail(AVR_ERR_ARG, "null buffer");
    long long maxId = 0;
    for (int i = 0; i < n; ++i) {
        if (vertex_ids[i] < 0) return fail(AVR_ERR_ARG, "negative vertex id");
        maxId = std::max<long long>(maxId, vertex_ids[i]);
    }
    avr::Params p;
    int rc = graph_params(c, s, (unsigned long long)(maxId + 1) * (unsigned long long)n_rays, cycle, &p);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(c->device));
    char *buf = nullptr;
    const size_t szI = (size_t)n * 4, szP = (size_t)n * 12, szR = (size_t)nr * 12, szT = (size_t)nr * 4;
    HIP_TRY(dalloc(&buf, szI + szP + 2 * szR + 2 * szT));
    int *dId = (int *)buf;
    float *dPt = (float *)(buf + szI), *dO = (float *)(buf + szI + szP), *dD = (float *)(buf + szI + szP + szR);
    float *dT = (float *)(buf + szI + szP + 2 * szR);
    int *dV = (int *)(buf + szI + szP + 2 * szR + szT);
    hipError_t e = hipMemcpyAsync(dId, vertex_ids, szI, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(dPt, points, szP, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) {
        if (p.sampler_kind == 1)
            hipLaunchKernelGGL(avr::k_graph_reinforce_rays<true>, dim3((n + 255) / 256), dim3(256), 0, c->stream, p, n,
                               dId, dPt, vertex_radius, n_rays, cycle, s->resolution_x, dO, dD, dT, dV);
        else
            hipLaunchKernelGGL(avr::k_graph_reinforce_rays<false>, dim3((n + 255) / 256), dim3(256), 0, c->stream, p, n,
                               dId, dPt, vertex_radius, n_rays, cycle, s->resolution_x, dO, dD, dT, dV);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(o, dO, szR, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(d, dD, szR, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(t_first, dT, szT, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(valid, dV, szT, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    (void)hipStreamSynchronize(c->stream);
    (void)hipFree(buf);
    if (e != hipSuccess) return fail(AVR_ERR_HIP, std::string("graph reinforce rays: ") + hipGetErrorString(e));
    return AVR_OK;
}

int avr_graph_light(avr_context *c, const avr_graph_sampling *s, int n_vertices, const float *vertices,
                    const float in_dir[3], float sphere_radius, int points_on_radius, int iterations,
                    float max_dist_to_center, float *light) {
    if (!c || n_vertices < 0 || points_on_radius < 0 || iterations < 0) return fail(AVR_ERR_ARG, "bad light arguments");
    if (!c->has_medium) return fail(AVR_ERR_STATE, "medium required");
    if (n_vertices == 0) return AVR_OK;
    if (!vertices || !in_dir || !light) return fail(AVR_ERR_ARG, "null buffer");
    if (iterations < 1) return fail(AVR_ERR_ARG, "Must have at least one light ray iteration");   // :10-11
    const int maxPts = (2 * points_on_radius + 1) * (2 * points_on_radius + 1);
    avr::Params p;
    int rc = graph_params(c, s, (unsigned long long)n_vertices * (unsigned long long)maxPts, iterations - 1, &p);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(c->device));
    // tr scratch: at most 2^28 estimates per chunk of vertices (1 GiB)
    const long long perV = (long long)maxPts * iterations;
    const int chunk = (int)std::max<long long>(1, std::min<long long>(n_vertices, (1ll << 28) / perV));
    float *dV = nullptr, *dL = nullptr, *dTr = nullptr;
    avr::graph::DiskRec *dRec = nullptr;
    int *dN = nullptr;
    hipError_t e = dalloc(&dV, (size_t)n_vertices * 3);
    if (e == hipSuccess) e = dalloc(&dL, (size_t)n_vertices);
    if (e == hipSuccess) e = dalloc(&dRec, (size_t)n_vertices * maxPts);
    if (e == hipSuccess) e = dalloc(&dN, (size_t)n_vertices);
    if (e == hipSuccess) e = dalloc(&dTr, (size_t)chunk * perV);
    if (e == hipSuccess) e = hipMemcpyAsync(dV, vertices, (size_t)n_vertices * 3 * sizeof(float), hipMemcpyHostToDevice, c->stream);
    const avr::V3 dir = {in_dir[0], in_dir[1], in_dir[2]};
    if (e == hipSuccess) {
        hipLaunchKernelGGL(avr::k_graph_disk, dim3((n_vertices + 255) / 256), dim3(256), 0, c->stream, c->med, n_vertices,
                           dV, dir, sphere_radius, points_on_radius, max_dist_to_center, maxPts, dRec, dN);
        e = hipGetLastError();
    }
    for (int v0 = 0; e == hipSuccess && v0 < n_vertices; v0 += chunk) {
        const int nv = std::min(chunk, n_vertices - v0);
        const long long n = (long long)nv * perV;
        const int blocks = blocks_for(n, 256, 256 * 64);
        if (p.sampler_kind == 1)
            hipLaunchKernelGGL(avr::k_graph_tr<true>, dim3(blocks), dim3(256), 0, c->stream, p, v0, nv, maxPts, iterations,
                               dir, s->resolution_x, dRec, dN, dTr);
        else
            hipLaunchKernelGGL(avr::k_graph_tr<false>, dim3(blocks), dim3(256), 0, c->stream, p, v0, nv, maxPts, iterations,
                               dir, s->resolution_x, dRec, dN, dTr);
        e = hipGetLastError();
        if (e != hipSuccess) break;
        hipLaunchKernelGGL(avr::k_graph_average, dim3((nv + 255) / 256), dim3(256), 0, c->stream, v0, nv, maxPts,
                           iterations, dRec, dN, dTr, dL);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(light, dL, (size_t)n_vertices * sizeof(float), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    (void)hipStreamSynchronize(c->stream);
    (void)hipFree(dV); (void)hipFree(dL); (void)hipFree(dRec); (void)hipFree(dN); (void)hipFree(dTr);
    if (e != hipSuccess) return fail(AVR_ERR_HIP, std::string("graph light: ") + hipGetErrorString(e));
    return AVR_OK;
}

int avr_graph_propagate_device(avr_context *c, int n, long long nnz, const int *row_ptr, const int *col,
                               const float *val, const float *light, int bounces, float *total, int *iterations) {
    if (!c || n < 0 || nnz < 0 || bounces < 0) return fail(AVR_ERR_ARG, "bad propagate arguments");
    if (n == 0) { if (iterations) *iterations = bounces; return AVR_OK; }
    if (!row_ptr || !light || !total || (nnz > 0 && (!col || !val))) return fail(AVR_ERR_ARG, "null buffer");
    HIP_TRY(hipSetDevice(c->device));
    float *buf = nullptr;
    int *flags = nullptr;
    HIP_TRY(dalloc(&buf, (size_t)2 * n));
    hipError_t e = dalloc(&flags, (size_t)std::max(bounces, 1));
    float *cur = buf, *next = buf + n;
    if (e == hipSuccess) e = hipMemsetAsync(flags, 0, sizeof(int) * std::max(bounces, 1), c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(total, light, (size_t)n * sizeof(float), hipMemcpyDeviceToDevice, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(cur, light, (size_t)n * sizeof(float), hipMemcpyDeviceToDevice, c->stream);
    const int blocks = blocks_for(n, 256, 256 * 64);
    for (int it = 0; e == hipSuccess && it < bounces; ++it) {
        hipLaunchKernelGGL(avr::k_graph_spmv, dim3(blocks), dim3(256), 0, c->stream, n, row_ptr, col, val, cur, next,
                           total, flags, it);
        e = hipGetLastError();
        std::swap(cur, next);
    }
    if (e == hipSuccess && bounces > 0) {
        hipLaunchKernelGGL(avr::k_graph_accumulate, dim3(blocks), dim3(256), 0, c->stream, n, cur, total, flags, bounces);
        e = hipGetLastError();
    }
    if (e == hipSuccess && iterations) {
        std::vector<int> h(std::max(bounces, 1));
        e = hipMemcpyAsync(h.data(), flags, sizeof(int) * h.size(), hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        int done = bounces;
        for (int j = 0; j < bounces; ++j)
            if (h[j]) { done = j; break; }
        *iterations = done;
    }
    // the scratch is freed after the stream drains (hipFree synchronises the device)
    (void)hipStreamSynchronize(c->stream);
    (void)hipFree(buf);
    (void)hipFree(flags);
    if (e != hipSuccess) return fail(AVR_ERR_HIP, std::string("graph propagate: ") + hipGetErrorString(e));
    return AVR_OK;
}

int avr_graph_propagate(avr_context *c, int n, const int *row_ptr, const int *col, const float *val,
                        const float *light, int bounces, float *total, int *iterations) {
    if (!c || n < 0 || bounces < 0) return fail(AVR_ERR_ARG, "bad propagate arguments");
    if (n == 0) { if (iterations) *iterations = bounces; return AVR_OK; }
    if (!row_ptr || !light || !total) return fail(AVR_ERR_ARG, "null buffer");
    const long long nnz = row_ptr[n];
    if (nnz < 0 || row_ptr[0] != 0) return fail(AVR_ERR_ARG, "bad row_ptr");
    for (int i = 0; i < n; ++i) {
        if (row_ptr[i + 1] < row_ptr[i]) return fail(AVR_ERR_ARG, "row_ptr not monotone");
        for (int k = row_ptr[i]; k < row_ptr[i + 1]; ++k) {
            if (col[k] < 0 || col[k] >= n) return fail(AVR_ERR_ARG, "column out of range");
            if (k > row_ptr[i] && col[k] <= col[k - 1]) return fail(AVR_ERR_ARG, "columns must ascend within a row");
        }
    }
    HIP_TRY(hipSetDevice(c->device));
    char *buf = nullptr;
    const size_t szR = (size_t)(n + 1) * 4, szE = (size_t)nnz * 4, szN = (size_t)n * 4;
    HIP_TRY(dalloc(&buf, szR + 2 * szE + 2 * szN));
    int *dR = (int *)buf, *dC = (int *)(buf + szR);
    float *dVal = (float *)(buf + szR + szE), *dL = (float *)(buf + szR + 2 * szE), *dT = (float *)(buf + szR + 2 * szE + szN);
    hipError_t e = hipMemcpyAsync(dR, row_ptr, szR, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess && nnz) e = hipMemcpyAsync(dC, col, szE, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess && nnz) e = hipMemcpyAsync(dVal, val, szE, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(dL, light, szN, hipMemcpyHostToDevice, c->stream);
    int rc = AVR_OK;
    if (e == hipSuccess) rc = avr_graph_propagate_device(c, n, nnz, dR, dC, dVal, dL, bounces, dT, iterations);
    if (e == hipSuccess && rc == AVR_OK) e = hipMemcpyAsync(total, dT, szN, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess && rc == AVR_OK) e = hipStreamSynchronize(c->stream);
    (void)hipStreamSynchronize(c->stream);
    (void)hipFree(buf);
    if (rc) return rc;
    if (e != hipSuccess) return fail(AVR_ERR_HIP, std::string("graph propagate: ") + hipGetErrorString(e));
    return AVR_OK;
}

struct avr_graph {
    avr::graph::Builder b;
    explicit avr_graph(float r) : b(r) {}
};

int avr_graph_create(float vertex_radius, avr_graph **out) {
    if (!out || !(vertex_radius > 0)) return fail(AVR_ERR_ARG, "vertex radius must be positive");
    *out = new avr_graph(vertex_radius);
    return AVR_OK;
}
int avr_graph_destroy(avr_graph *g) {
    delete g;
    return AVR_OK;
}
int avr_graph_add_walks(avr_graph *g, long long n_walks, int max_depth, const float *points, const int *counts) {
    if (!g || n_walks < 0 || max_depth < 0) return fail(AVR_ERR_ARG, "bad walks");
    if (n_walks > 0 && (!counts || (max_depth > 0 && !points))) return fail(AVR_ERR_ARG, "null buffer");
    for (long long w = 0; w < n_walks; ++w) {
        const int k = counts[w];
        if (k < 0 || k > max_depth) return fail(AVR_ERR_ARG, "walk count out of range");
        g->b.AddWalk(points + (size_t)w * max_depth * 3, k, k == max_depth);
    }
    return AVR_OK;
}
int avr_graph_add_walks_from(avr_graph *g, long long n_walks, int max_depth, const float *points, const int *counts,
                             const int *start_vertex) {
    if (!g || n_walks < 0 || max_depth < 0) return fail(AVR_ERR_ARG, "bad walks");
    if (n_walks > 0 && (!counts || !start_vertex || (max_depth > 0 && !points))) return fail(AVR_ERR_ARG, "null buffer");
    for (long long w = 0; w < n_walks; ++w) {
        const int k = counts[w], sv = start_vertex[w];
        if (k < 0 || k > max_depth) return fail(AVR_ERR_ARG, "walk count out of range");
        if (sv < -1 || sv >= (long long)g->b.NumVertices()) return fail(AVR_ERR_ARG, "start vertex out of range");
        // with a starting vertex the path holds one vertex before the first scatter, so the
        // walk was traced with max_depth - 1 scatters
        const int cap = sv >= 0 ? max_depth - 1 : max_depth;
        if (k > cap) return fail(AVR_ERR_ARG, "walk count out of range");
        g->b.AddWalk(points + (size_t)w * max_depth * 3, k, k == cap, sv);
    }
    return AVR_OK;
}
int avr_graph_out_degrees(avr_graph *g, int *out) {
    if (!g || !out) return fail(AVR_ERR_ARG, "null buffer");
    g->b.OutDegrees(out);
    return AVR_OK;
}
int avr_graph_count_in_radius(avr_graph *g, int n, const int *vertex_ids, float radius, int *counts) {
    if (!g || n < 0 || !(radius > 0)) return fail(AVR_ERR_ARG, "bad radius query");
    if (n > 0 && (!vertex_ids || !counts)) return fail(AVR_ERR_ARG, "null buffer");
    for (int i = 0; i < n; ++i) {
        if (vertex_ids[i] < 0 || vertex_ids[i] >= (long long)g->b.NumVertices()) return fail(AVR_ERR_ARG, "vertex id");
        counts[i] = g->b.CountInRadius(vertex_ids[i], radius);
    }
    return AVR_OK;
}
int avr_graph_size(avr_graph *g, long long *n_vertices, long long *n_edges) {
    if (!g) return fail(AVR_ERR_ARG, "null graph");
    if (n_vertices) *n_vertices = (long long)g->b.NumVertices();
    if (n_edges) *n_edges = (long long)g->b.NumEdges();
    return AVR_OK;
}
int avr_graph_vertices(avr_graph *g, float *xyz, int *samples) {
    if (!g) return fail(AVR_ERR_ARG, "null graph");
    if (xyz) std::copy(g->b.Vertices().begin(), g->b.Vertices().end(), xyz);
    if (samples) std::copy(g->b.VertexSamples().begin(), g->b.VertexSamples().end(), samples);
    return AVR_OK;
}
int avr_graph_edges(avr_graph *g, int *from, int *to, int *samples) {
    if (!g) return fail(AVR_ERR_ARG, "null graph");
    if (from) std::copy(g->b.EdgeFrom().begin(), g->b.EdgeFrom().end(), from);
    if (to) std::copy(g->b.EdgeTo().begin(), g->b.EdgeTo().end(), to);
    if (samples) std::copy(g->b.EdgeSamples().begin(), g->b.EdgeSamples().end(), samples);
    return AVR_OK;
}
int avr_graph_transport(avr_graph *g, int *row_ptr, int *col, float *val) {
    if (!g || !row_ptr || (g->b.NumEdges() > 0 && (!col || !val))) return fail(AVR_ERR_ARG, "null buffer");
    g->b.Transport(row_ptr, col, val);
    return AVR_OK;
}
int avr_graph_in_node_path_length(avr_graph *g, float *average, long long *count) {
    if (!g) return fail(AVR_ERR_ARG, "null graph");
    // Averager::GetAverage over the added values (util.h:545-565); a double sum here
    if (average) *average = g->b.PathLengthCount() ? (float)(g->b.PathLengthSum() / g->b.PathLengthCount()) : 0.f;
    if (count) *count = g->b.PathLengthCount();
    return AVR_OK;
}

}  // extern "C"

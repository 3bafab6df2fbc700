// graph_ref.cpp — ORACLE TEST INFRASTRUCTURE (never shipped, never on the product path).
//
// Our own harness, compiled by oracle/ref/Makefile against the UNMODIFIED reference
// sources under /root/reference/src. It prints golden vectors for the lighting-graph
// row that pin oracle/volpath_oracle.cpp's graph section:
//  * GetHits(sphere) (src/graph/util.h:419-463): pbrt's own Sphere::Intersect
//    (shapes.h:141-150, BasicIntersect 152-236) on a SphereContainer-style sphere
//    (util.h:285-300: Translate(center)), SkipIntersection = SurfaceInteraction::SpawnRay
//    (interaction.cpp:91-97), the second Intersect, and the from-far disambiguation;
//  * LightingCalculator's transport iteration (lighting_calculator.cpp:23-59) with the
//    reference's vendored Eigen (src/graph/deps/Eigen, header-only): SparseMatrix<float>
//    from triplets (GetTransportMatrix, :61-82), curLight = T * curLight, the NaN/Inf stop,
//    totalLight += curLight.
// graph/util.h itself is not included: it pulls media.h, which needs the absent NanoVDB
// submodule; the few lines of GetHits are restated here over the reference's primitives.
#include <pbrt/shapes.h>
#include <pbrt/interaction.h>
#include <pbrt/util/rng.h>

#include "graph/deps/Eigen/SparseCore"

#include <cstdio>
#include <cstring>
#include <vector>

using namespace pbrt;

static uint32_t bits(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }

// GetHits(const Sphere&, ray) — graph/util.h:419-463 (distBack = maxDistToCenter * 2)
static int SphereGetHits(const Sphere &sphere, Ray ray, float distBack, float *t0, float *t1) {
    Ray rayOutside = ray;
    rayOutside.o -= ray.d * distBack;
    pstd::optional<ShapeIntersection> first = sphere.Intersect(ray, Infinity);
    if (!first) return 2;   // OutsideZeroHits
    *t0 = first->tHit;
    Ray skipped = first->intr.SpawnRay(ray.d);   // SkipIntersection (interaction.cpp:91-97)
    pstd::optional<ShapeIntersection> second = sphere.Intersect(skipped, Infinity);
    if (second) { *t1 = *t0 + second->tHit; return 0; }   // OutsideTwoHits
    pstd::optional<ShapeIntersection> far = sphere.Intersect(rayOutside, Infinity);
    if (!far) return 2;
    float adjusted = far->tHit - distBack;
    float diff = std::abs(first->tHit - adjusted);
    if (diff < std::pow(10, -3)) return 2;   // OutsideOneHit -> reported as zero hits
    *t1 = 0;
    return 3;                                // InsideOneHit
}

int main() {
    RNG rng(7, 11);
    auto U = [&]() { return rng.Uniform<float>(); };
    printf("{\n\"sphere_hits\": [\n");
    const int nSph = 400;
    for (int i = 0; i < nSph; ++i) {
        Point3f c(U() * 2 - 1, U() * 2 - 1, U() * 2 - 1);
        float r = 0.002f + 0.3f * U();
        Transform rfo = Translate(Vector3f(c)), ofr = Inverse(rfo);
        Sphere sphere(&rfo, &ofr, false, r, -r, r, 360);
        // rays: from far outside towards a point near the sphere (hits, misses, grazes),
        // and every 5th ray from inside the sphere
        Vector3f d = Normalize(Vector3f(U() * 2 - 1, U() * 2 - 1, U() * 2 - 1));
        Point3f target = c + Vector3f(U() * 2 - 1, U() * 2 - 1, U() * 2 - 1) * (r * 1.2f);
        Point3f o = (i % 5 == 4) ? c + Vector3f(U() - .5f, U() - .5f, U() - .5f) * r : target - d * (2 + 3 * U());
        float t0 = 0, t1 = 0;
        int type = SphereGetHits(sphere, Ray(o, d), 4.f, &t0, &t1);
        printf("  [%u,%u,%u, %u, %u,%u,%u, %u,%u,%u, %d, %u, %u]%s\n", bits(c.x), bits(c.y), bits(c.z), bits(r),
               bits(o.x), bits(o.y), bits(o.z), bits(d.x), bits(d.y), bits(d.z), type, bits(t0), bits(t1),
               i + 1 < nSph ? "," : "");
    }
    printf("],\n\"transport\": [\n");
    // graphs: n vertices, each with 0..6 out-edges; T(v, w) = edgeSamples / samples with
    // samples >= sum of edge samples (each traced segment from v contributes at most one edge)
    const int nCases = 6;
    for (int cs = 0; cs < nCases; ++cs) {
        int n = 5 + cs * 37;
        int bounces = (cs == nCases - 1) ? 200 : 3 + cs * 4;
        std::vector<Eigen::Triplet<float>> trip;
        std::vector<int> rows, cols;
        std::vector<float> vals;
        for (int v = 0; v < n; ++v) {
            int deg = (int)(U() * 7) + (cs == nCases - 1 && v == 0 ? 1 : 0);
            int samples = 0;
            std::vector<int> es;
            std::vector<int> targets;
            for (int e = 0; e < deg; ++e) {
                int w = (int)(U() * n);
                if (cs == nCases - 1 && v == 0 && e == 0) w = 0;   // self-loop carrying the huge entry
                if (std::find(targets.begin(), targets.end(), w) != targets.end()) continue;
                targets.push_back(w);
                int s = 1 + (int)(U() * 9);
                es.push_back(s);
                samples += s;
            }
            samples += (int)(U() * 5);
            for (size_t e = 0; e < targets.size(); ++e) {
                float val = static_cast<float>(es[e]) / static_cast<float>(samples);
                if (cs == nCases - 1 && v == 0 && e == 0) val = val * 3e38f;   // drives the NaN/Inf stop
                trip.emplace_back(v, targets[e], val);
                rows.push_back(v); cols.push_back(targets[e]); vals.push_back(val);
            }
        }
        Eigen::SparseMatrix<float> T(n, n);
        T.setFromTriplets(trip.begin(), trip.end());
        Eigen::SparseVector<float> light(n);
        std::vector<float> l0(n);
        for (int v = 0; v < n; ++v) { l0[v] = U() * Inv4Pi; light.coeffRef(v) = l0[v]; }
        // ComputeFinalLight (lighting_calculator.cpp:23-59)
        Eigen::SparseVector<float> total(light);
        int it = 0;
        Eigen::SparseVector<float> cur = total;
        for (; it < bounces; ++it) {
            cur = T * cur;
            bool invalid = false;
            for (int i = 0; i < n; ++i)
                if (IsNaN(cur.coeff(i)) || IsInf(cur.coeff(i))) { invalid = true; break; }
            if (invalid) break;
            total += cur;
        }
        printf("  {\"n\": %d, \"bounces\": %d, \"iterations\": %d, \"rows\": [", n, bounces, it);
        for (size_t k = 0; k < rows.size(); ++k) printf("%d%s", rows[k], k + 1 < rows.size() ? "," : "");
        printf("], \"cols\": [");
        for (size_t k = 0; k < cols.size(); ++k) printf("%d%s", cols[k], k + 1 < cols.size() ? "," : "");
        printf("], \"vals\": [");
        for (size_t k = 0; k < vals.size(); ++k) printf("%u%s", bits(vals[k]), k + 1 < vals.size() ? "," : "");
        printf("], \"light\": [");
        for (int v = 0; v < n; ++v) printf("%u%s", bits(l0[v]), v + 1 < n ? "," : "");
        printf("], \"total\": [");
        for (int v = 0; v < n; ++v) printf("%u%s", bits(total.coeff(v)), v + 1 < n ? "," : "");
        printf("]}%s\n", cs + 1 < nCases ? "," : "");
    }
    printf("]\n}\n");
    return 0;
}

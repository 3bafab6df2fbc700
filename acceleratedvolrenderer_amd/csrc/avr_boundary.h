// avr_boundary.h — medium boundary shapes shared by the path kernels (interface spheres,
// f3 of SURVEY §8f) and the lighting-graph kernels (graph/util.h:280-300, 419-503).
// A sphere's crossings solve Sphere::BasicIntersect's interval quadric (shapes.h:152-191)
// exactly as the reference's CPU build evaluates it (t0 pinned bit for bit against pbrt's
// own Sphere in oracle/_ref/graph_ref); the oracle restates the same code.
#pragma once

namespace avr {
namespace shape {

enum : int { kOutsideTwoHits = 0, kOutsideOneHit = 1, kOutsideZeroHits = 2, kInsideOneHit = 3 };

struct Hits {
    int type;
    float t0, t1;
};

// Interval arithmetic of util/math.h:818-1071 on the CPU branch (round-to-nearest op, then one
// NextFloatUp/Down), which is what the reference's CPU build runs.
struct Iv {
    float lo, hi;
};
// std::min / std::max exactly (first argument kept on ties, as the oracle's std:: calls)
__device__ __forceinline__ float smin(float a, float b) { return b < a ? b : a; }
__device__ __forceinline__ float smax(float a, float b) { return a < b ? b : a; }
__device__ __forceinline__ Iv iv(float a, float b) { return {smin(a, b), smax(a, b)}; }
__device__ __forceinline__ Iv iv_err(float v, float e) {   // Interval::FromValueAndError
    if (e == 0) return {v, v};
    return {next_down(v - e), next_up(v + e)};
}
__device__ __forceinline__ Iv iadd(Iv a, Iv b) { return iv(next_down(a.lo + b.lo), next_up(a.hi + b.hi)); }
__device__ __forceinline__ Iv isub(Iv a, Iv b) { return iv(next_down(a.lo - b.hi), next_up(a.hi - b.lo)); }
__device__ __forceinline__ float min4(float a, float b, float c, float d) { return smin(smin(smin(a, b), c), d); }
__device__ __forceinline__ float max4(float a, float b, float c, float d) { return smax(smax(smax(a, b), c), d); }
__device__ __forceinline__ Iv imul(Iv a, Iv b) {
    const float p0 = a.lo * b.lo, p1 = a.hi * b.lo, p2 = a.lo * b.hi, p3 = a.hi * b.hi;
    return iv(min4(next_down(p0), next_down(p1), next_down(p2), next_down(p3)),
              max4(next_up(p0), next_up(p1), next_up(p2), next_up(p3)));
}
__device__ __forceinline__ bool in_range0(Iv i) { return 0 >= i.lo && 0 <= i.hi; }
__device__ __forceinline__ Iv idiv(Iv a, Iv b) {
    if (in_range0(b)) return {-kInf, kInf};
    const float q0 = a.lo / b.lo, q1 = a.hi / b.lo, q2 = a.lo / b.hi, q3 = a.hi / b.hi;
    return iv(min4(next_down(q0), next_down(q1), next_down(q2), next_down(q3)),
              max4(next_up(q0), next_up(q1), next_up(q2), next_up(q3)));
}
__device__ __forceinline__ Iv iscale(float f, Iv i) {
    if (f > 0) return iv(next_down(f * i.lo), next_up(f * i.hi));
    return iv(next_down(f * i.hi), next_up(f * i.lo));
}
__device__ __forceinline__ Iv isqr(Iv i) {
    float alo = fabsf(i.lo), ahi = fabsf(i.hi);
    if (alo > ahi) { const float t = alo; alo = ahi; ahi = t; }
    if (in_range0(i)) return iv(0.f, next_up(ahi * ahi));
    return iv(next_down(alo * alo), next_up(ahi * ahi));
}
__device__ __forceinline__ Iv isqrt(Iv i) {
    return iv(smax(0.f, next_down(__builtin_sqrtf(i.lo))), next_up(__builtin_sqrtf(i.hi)));
}
__device__ __forceinline__ float mid(Iv i) { return (i.lo + i.hi) / 2; }

// Sphere of radius r at c (SphereContainer: Translate(c), util.h:285-300): the ray as exact
// Point3fi / Vector3fi through objectFromRender = Translate(-c) (transform.h:136-180,
// 276-310), then Sphere::BasicIntersect's quadric (shapes.h:152-191), tMax = Infinity.
__device__ __forceinline__ Hits sphere_hits(V3 c, float r, V3 o, V3 d) {
    const float ov[3] = {o.x, o.y, o.z}, dv[3] = {d.x, d.y, d.z}, cv[3] = {-c.x, -c.y, -c.z};
    Iv oi[3], di[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float m0 = k == 0 ? 1.f : 0.f, m1 = k == 1 ? 1.f : 0.f, m2 = k == 2 ? 1.f : 0.f;
        const float xp = (m0 * ov[0] + m1 * ov[1]) + (m2 * ov[2] + cv[k]);
        const float e = gamma_n(3) * (((fabsf(m0 * ov[0]) + fabsf(m1 * ov[1])) + fabsf(m2 * ov[2])) + fabsf(cv[k]));
        oi[k] = iv_err(xp, e);
        const float vp = (m0 * dv[0] + m1 * dv[1]) + m2 * dv[2];
        const float ve = gamma_n(3) * ((fabsf(m0 * dv[0]) + fabsf(m1 * dv[1])) + fabsf(m2 * dv[2]));
        di[k] = iv_err(vp, ve);
    }
    const Iv a = iadd(iadd(isqr(di[0]), isqr(di[1])), isqr(di[2]));
    const Iv b = iscale(2.f, iadd(iadd(imul(di[0], oi[0]), imul(di[1], oi[1])), imul(di[2], oi[2])));
    const Iv R = {r, r};
    const Iv cc = isub(iadd(iadd(isqr(oi[0]), isqr(oi[1])), isqr(oi[2])), isqr(R));
    const Iv bq = idiv(b, iscale(2.f, a));
    Iv v[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) v[k] = isub(oi[k], imul(bq, di[k]));   // Tuple3: (s * t) = t * s = {s * x, ..}
    const Iv len = isqrt(iadd(iadd(isqr(v[0]), isqr(v[1])), isqr(v[2])));
    const Iv discrim = imul(imul(iscale(4.f, a), iadd(R, len)), isub(R, len));
    if (discrim.lo < 0) return {kOutsideZeroHits, 0.f, 0.f};
    const Iv root = isqrt(discrim);
    const Iv q = mid(b) < 0 ? iscale(-.5f, isub(b, root)) : iscale(-.5f, iadd(b, root));
    Iv t0 = idiv(q, a), t1 = idiv(cc, q);
    if (t0.lo > t1.lo) { const Iv t = t0; t0 = t1; t1 = t; }
    if (t0.hi > kInf || t1.lo <= 0) return {kOutsideZeroHits, 0.f, 0.f};
    if (t0.lo <= 0) return {kInsideOneHit, mid(t1), 0.f};
    return {kOutsideTwoHits, mid(t0), mid(t1)};
}

// Convex polyhedron as the intersection of half-spaces n.p <= h (outward normals; e.g. the
// face planes of a convex triangle mesh): the ray's parametric slab clip, the generalisation
// of Bounds3::IntersectP (vecmath.h:1547-1571) to arbitrary planes. Same hit kinds as above:
// InsideOneHit {exit} for an origin inside, OutsideTwoHits {entry, exit}, else no hit.
// Float operation order fixed (dot products left to right, -ffp-contract=off): the oracle's
// restatement is bit-identical.
__host__ __device__ __forceinline__ Hits convex_hits(const float4 *planes, int n, V3 o, V3 d) {
    float t0 = -kInf, t1 = kInf;
    for (int i = 0; i < n; ++i) {
        const float4 pl = planes[i];
        const float denom = (pl.x * d.x + pl.y * d.y) + pl.z * d.z;
        const float num = pl.w - ((pl.x * o.x + pl.y * o.y) + pl.z * o.z);
        if (denom == 0.f) {
            if (num < 0.f) return {kOutsideZeroHits, 0.f, 0.f};   // parallel and outside this plane
        } else {
            const float t = num / denom;
            if (denom > 0.f) t1 = t < t1 ? t : t1;   // leaving through this plane
            else t0 = t > t0 ? t : t0;                // entering through this plane
        }
    }
    if (!(t0 <= t1) || t1 <= 0.f) return {kOutsideZeroHits, 0.f, 0.f};
    if (t0 <= 0.f) return {kInsideOneHit, t1, 0.f};
    return {kOutsideTwoHits, t0, t1};
}

}  // namespace shape
}  // namespace avr

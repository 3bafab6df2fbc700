// avr_graph_host.h — host-side FreeGraph assembly (the order-dependent part of
// FreeGraphBuilder, free/free_graph_builder.cpp:19-141 and 241-273, over Graph's
// AddVertex / AddEdge / AddVertexToPath, graph.cpp:79-229). The walks themselves come from
// the GPU (k_graph_walks); merging them into vertices depends on every earlier walk, so it
// runs here in walk order, as the reference's single-threaded BuildGraph loop does.
//
// Radius search: a uniform hash grid with cells of the vertex radius (the 27 cells around a
// point hold every vertex within the radius). GetClosestInRadius takes result[0] of
// nanoflann's RadiusResultSet — distances strictly below the squared radius, in kd-tree
// traversal order; this builder takes the nearest such vertex (ties: lowest id), which is the
// same vertex whenever at most one vertex is within the radius.
#pragma once

#include <cmath>
#include <cstdint>
#include <unordered_map>
#include <vector>

namespace avr {
namespace graph {

class Builder {
  public:
    explicit Builder(float radius) : r_(radius), r2_(radius * radius) {}   // Sqr(nodeRadius), :14

    // One walk: k scatter points; forced = the walk stopped at maxDepth (PathData::forcedEnd);
    // start >= 0: TracePath's startingVertex (free_graph_builder.cpp:24-25), the path's
    // first vertex before any scatter (the reinforcement walks)
    void AddWalk(const float *pts, int k, bool forced, int start = -1) {
        path_.clear();
        if (start >= 0) path_.push_back(start);
        for (int j = 0; j < k; ++j) {
            const float p[3] = {pts[3 * j], pts[3 * j + 1], pts[3 * j + 2]};
            // HandlePotentialPathEnd after the segment that produced this scatter
            if (!path_.empty()) ++vsamples_[path_.back()];
            int v = Closest(p);
            if (v < 0 && !path_.empty() && DistSq(&vxyz_[3 * (size_t)path_.back()], p) <= r2_) v = path_.back();
            if (v < 0) v = NewVertex(p);
            path_.push_back(v);
            if (path_.size() >= 2) AddEdge(path_[path_.size() - 2], v);
        }
        // the segment after the last scatter (escape / absorption / no boundary hit) — none
        // when the walk was cut at maxDepth
        if (!forced && !path_.empty()) ++vsamples_[path_.back()];
        PathInfo(forced);
    }

    // Vertex::outEdges.size(): distinct targets per vertex
    void OutDegrees(int *out) const {
        for (size_t v = 0; v < NumVertices(); ++v) out[v] = 0;
        for (int f : efrom_) ++out[f];
    }
    // CountInRadius (free_graph_builder.cpp:229-236): vertices with squared distance strictly
    // below Sqr(radius) (nanoflann RadiusResultSet), the vertex itself included
    int CountInRadius(int v, float radius) const {
        const float r2 = radius * radius;
        const float *p = &vxyz_[3 * (size_t)v];
        const int reach = (int)std::ceil(radius / r_);
        const int64_t cx = Cell(p[0]), cy = Cell(p[1]), cz = Cell(p[2]);
        int n = 0;
        if ((int64_t)reach * 2 + 1 > 64) {   // wide query: scan every vertex
            for (size_t u = 0; u < NumVertices(); ++u) n += DistSq(&vxyz_[3 * u], p) < r2;
            return n;
        }
        for (int64_t z = cz - reach; z <= cz + reach; ++z)
            for (int64_t y = cy - reach; y <= cy + reach; ++y)
                for (int64_t x = cx - reach; x <= cx + reach; ++x) {
                    auto it = grid_.find(Key(x, y, z));
                    if (it == grid_.end()) continue;
                    for (int u : it->second) n += DistSq(&vxyz_[3 * (size_t)u], p) < r2;
                }
        return n;
    }

    size_t NumVertices() const { return vsamples_.size(); }
    size_t NumEdges() const { return efrom_.size(); }
    const std::vector<float> &Vertices() const { return vxyz_; }
    const std::vector<int> &VertexSamples() const { return vsamples_; }
    const std::vector<int> &EdgeFrom() const { return efrom_; }
    const std::vector<int> &EdgeTo() const { return eto_; }
    const std::vector<int> &EdgeSamples() const { return esamples_; }
    double PathLengthSum() const { return plSum_; }
    long long PathLengthCount() const { return plCount_; }

    // GetTransportMatrix (lighting_calculator.cpp:61-82) as CSR: row = vertex, col ascending
    void Transport(int *rowptr, int *col, float *val) const {
        const size_t n = NumVertices();
        std::vector<std::vector<std::pair<int, int>>> rows(n);
        for (size_t e = 0; e < efrom_.size(); ++e) rows[efrom_[e]].push_back({eto_[e], esamples_[e]});
        size_t off = 0;
        for (size_t v = 0; v < n; ++v) {
            rowptr[v] = (int)off;
            std::sort(rows[v].begin(), rows[v].end());
            for (auto &ce : rows[v]) {
                col[off] = ce.first;
                val[off] = static_cast<float>(ce.second) / static_cast<float>(vsamples_[v]);
                ++off;
            }
        }
        rowptr[n] = (int)off;
    }

  private:
    static float DistSq(const float *a, const float *b) {   // nanoflann L2_Simple / DistanceSquared
        const float dx = a[0] - b[0], dy = a[1] - b[1], dz = a[2] - b[2];
        return dx * dx + dy * dy + dz * dz;
    }
    int64_t Cell(float x) const { return (int64_t)std::floor(x / r_); }
    static uint64_t Key(int64_t x, int64_t y, int64_t z) {
        return ((uint64_t)(x & 0x1fffff) << 42) | ((uint64_t)(y & 0x1fffff) << 21) | (uint64_t)(z & 0x1fffff);
    }
    int Closest(const float *p) const {
        const int64_t cx = Cell(p[0]), cy = Cell(p[1]), cz = Cell(p[2]);
        int best = -1;
        float bestD = 0;
        for (int64_t z = cz - 1; z <= cz + 1; ++z)
            for (int64_t y = cy - 1; y <= cy + 1; ++y)
                for (int64_t x = cx - 1; x <= cx + 1; ++x) {
                    auto it = grid_.find(Key(x, y, z));
                    if (it == grid_.end()) continue;
                    for (int v : it->second) {
                        const float d = DistSq(&vxyz_[3 * (size_t)v], p);
                        if (!(d < r2_)) continue;
                        if (best < 0 || d < bestD || (d == bestD && v < best)) { best = v; bestD = d; }
                    }
                }
        return best;
    }
    int NewVertex(const float *p) {
        const int id = (int)vsamples_.size();
        vxyz_.insert(vxyz_.end(), p, p + 3);
        vsamples_.push_back(0);
        grid_[Key(Cell(p[0]), Cell(p[1]), Cell(p[2]))].push_back(id);
        return id;
    }
    void AddEdge(int from, int to) {   // Graph::AddEdge with EdgeData{1}: merge adds samples
        const uint64_t key = ((uint64_t)(uint32_t)from << 32) | (uint32_t)to;
        auto it = edges_.find(key);
        if (it != edges_.end()) {
            ++esamples_[it->second];
            return;
        }
        edges_[key] = (int)efrom_.size();
        efrom_.push_back(from);
        eto_.push_back(to);
        esamples_.push_back(1);
    }
    // UseAndRemovePathInfo (free_graph_builder.cpp:241-273): runs of one vertex in a path
    void PathInfo(bool forced) {
        const size_t n = path_.size();
        if (n == 0) return;
        if (n == 1) {
            if (!forced) Add(1);
            return;
        }
        float run = 1;
        for (size_t i = 0; i + 1 < n; ++i) {
            if (path_[i] == path_[i + 1]) ++run;
            else { Add(run); run = 1; }
        }
        if (!forced) Add(run);
    }
    void Add(float v) { plSum_ += v; ++plCount_; }

    float r_, r2_;
    std::vector<float> vxyz_;
    std::vector<int> vsamples_;
    std::vector<int> efrom_, eto_, esamples_;
    std::unordered_map<uint64_t, int> edges_;
    std::unordered_map<uint64_t, std::vector<int>> grid_;
    std::vector<int> path_;
    double plSum_ = 0;
    long long plCount_ = 0;
};

}  // namespace graph
}  // namespace avr

// Host replay of the reference's radius-search ORDER for the few queries whose
// order the GPU's (distance, index) sort cannot decide.
//
// cpp_neighbors (c2p-net/ngenet/cpp_wrappers/cpp_neighbors/neighbors/neighbors.cpp
// :211-332) answers each query with nanoflann 1.3.0 (the header vendored at
// cpp_wrappers/cpp_utils/nanoflann/nanoflann.hpp): a KD-tree with leaf size 10
// over the query's support batch, RadiusResultSet appending (index, d) pairs in
// leaf-visit order, then std::sort by d alone (IndexDist_Sorter, :208-214), which
// is not stable.  Equal distances therefore come out in an order that depends on
// the tree and on introsort, and the float box-distance pruning could in principle
// drop a point within a few ulps of the radius.  The GPU path flags exactly those
// rows (a tie in the row, or a distance within 2^-17 relative of r^2) and this
// file recomputes them: it builds the same tree (same split rule, same in-place
// partition, same float arithmetic) and runs the same search, then sorts with
// std::sort and the same comparator -- libstdc++'s introsort is deterministic
// given its input sequence, so the output equals the reference's.
//
// The tree build and search below follow nanoflann 1.3.0's divideTree /
// middleSplit_ / planeSplit and searchLevel closely (their order of operations
// is what fixes the output order), so nanoflann's licence applies to those
// parts.  Its notice, as the vendored header carries it:
//
//   Software License Agreement (BSD License)
//
//   Copyright 2008-2009  Marius Muja (mariusm@cs.ubc.ca). All rights reserved.
//   Copyright 2008-2009  David G. Lowe (lowe@cs.ubc.ca). All rights reserved.
//   Copyright 2011-2016  Jose Luis Blanco (joseluisblancoc@gmail.com).
//     All rights reserved.
//
//   THE BSD LICENSE
//
//   Redistribution and use in source and binary forms, with or without
//   modification, are permitted provided that the following conditions
//   are met:
//
//   1. Redistributions of source code must retain the above copyright
//      notice, this list of conditions and the following disclaimer.
//   2. Redistributions in binary form must reproduce the above copyright
//      notice, this list of conditions and the following disclaimer in the
//      documentation and/or other materials provided with the distribution.
//
//   THIS SOFTWARE IS PROVIDED BY THE AUTHOR ``AS IS'' AND ANY EXPRESS OR
//   IMPLIED WARRANTIES, INCLUDING, BUT NOT LIMITED TO, THE IMPLIED WARRANTIES
//   OF MERCHANTABILITY AND FITNESS FOR A PARTICULAR PURPOSE ARE DISCLAIMED.
//   IN NO EVENT SHALL THE AUTHOR BE LIABLE FOR ANY DIRECT, INDIRECT,
//   INCIDENTAL, SPECIAL, EXEMPLARY, OR CONSEQUENTIAL DAMAGES (INCLUDING, BUT
//   NOT LIMITED TO, PROCUREMENT OF SUBSTITUTE GOODS OR SERVICES; LOSS OF USE,
//   DATA, OR PROFITS; OR BUSINESS INTERRUPTION) HOWEVER CAUSED AND ON ANY
//   THEORY OF LIABILITY, WHETHER IN CONTRACT, STRICT LIABILITY, OR TORT
//   (INCLUDING NEGLIGENCE OR OTHERWISE) ARISING IN ANY WAY OUT OF THE USE OF
//   THIS SOFTWARE, EVEN IF ADVISED OF THE POSSIBILITY OF SUCH DAMAGE.
#include <cstddef>
#include <algorithm>
#include <utility>
#include <vector>

namespace pcr {

namespace {

struct KdNode {
    int child1 = -1, child2 = -1;  // -1: leaf
    size_t left = 0, right = 0;    // leaf range in vind
    int divfeat = 0;
    float divlow = 0.f, divhigh = 0.f;
};

struct Box {
    float lo[3], hi[3];
};

class KdTree {
  public:
    KdTree(const float *pts, size_t n) : p_(pts), n_(n) {
        vind_.resize(n);
        for (size_t i = 0; i < n; ++i) vind_[i] = i;
        if (n == 0) return;
        // bounding box: first point, then strict < / > updates
        for (int d = 0; d < 3; ++d) root_.lo[d] = root_.hi[d] = at(0, d);
        for (size_t k = 1; k < n; ++k)
            for (int d = 0; d < 3; ++d) {
                const float v = at(k, d);
                if (v < root_.lo[d]) root_.lo[d] = v;
                if (v > root_.hi[d]) root_.hi[d] = v;
            }
        Box b = root_;
        nodes_.reserve(2 * (n / 5 + 1));
        root_node_ = divide(0, n, b);
    }

    // nanoflann radiusSearch(query, r2, out, sorted=true): (local index, d) pairs
    void radius(const float *q, float r2, std::vector<std::pair<size_t, float>> &out) const {
        out.clear();
        if (n_ == 0) return;
        float dists[3] = {0.f, 0.f, 0.f};
        float distsq = 0.f;
        for (int d = 0; d < 3; ++d) {
            if (q[d] < root_.lo[d]) {
                dists[d] = (q[d] - root_.lo[d]) * (q[d] - root_.lo[d]);
                distsq += dists[d];
            }
            if (q[d] > root_.hi[d]) {
                dists[d] = (q[d] - root_.hi[d]) * (q[d] - root_.hi[d]);
                distsq += dists[d];
            }
        }
        search(root_node_, q, r2, distsq, dists, out);
        std::sort(out.begin(), out.end(),
                  [](const std::pair<size_t, float> &a, const std::pair<size_t, float> &b) {
                      return a.second < b.second;
                  });
    }

  private:
    float at(size_t i, int d) const { return p_[3 * i + d]; }

    void minmax(const size_t *ind, size_t count, int d, float &mn, float &mx) const {
        mn = mx = at(ind[0], d);
        for (size_t i = 1; i < count; ++i) {
            const float v = at(ind[i], d);
            if (v < mn) mn = v;
            if (v > mx) mx = v;
        }
    }

    // partition ind[0..count) around cutval on axis d: < first, then ==, then >
    void plane_split(size_t *ind, size_t count, int d, float cutval, size_t &lim1,
                     size_t &lim2) const {
        size_t l = 0, r = count - 1;
        for (;;) {
            while (l <= r && at(ind[l], d) < cutval) ++l;
            while (r && l <= r && at(ind[r], d) >= cutval) --r;
            if (l > r || !r) break;
            std::swap(ind[l], ind[r]);
            ++l;
            --r;
        }
        lim1 = l;
        r = count - 1;
        for (;;) {
            while (l <= r && at(ind[l], d) <= cutval) ++l;
            while (r && l <= r && at(ind[r], d) > cutval) --r;
            if (l > r || !r) break;
            std::swap(ind[l], ind[r]);
            ++l;
            --r;
        }
        lim2 = l;
    }

    // split axis: the widest bbox axes (within a 1e-5 relative band), largest
    // actual spread first; cut at the bbox middle clamped to the points' range
    void middle_split(size_t *ind, size_t count, size_t &index, int &cutfeat, float &cutval,
                      const Box &b) const {
        const float eps = 0.00001f;
        float max_span = b.hi[0] - b.lo[0];
        for (int d = 1; d < 3; ++d) {
            const float s = b.hi[d] - b.lo[d];
            if (s > max_span) max_span = s;
        }
        float max_spread = -1.f;
        cutfeat = 0;
        for (int d = 0; d < 3; ++d) {
            const float s = b.hi[d] - b.lo[d];
            if (s > (1 - eps) * max_span) {
                float mn, mx;
                minmax(ind, count, d, mn, mx);
                const float spread = mx - mn;
                if (spread > max_spread) {
                    cutfeat = d;
                    max_spread = spread;
                }
            }
        }
        const float split_val = (b.lo[cutfeat] + b.hi[cutfeat]) / 2;
        float mn, mx;
        minmax(ind, count, cutfeat, mn, mx);
        cutval = split_val < mn ? mn : (split_val > mx ? mx : split_val);
        size_t lim1, lim2;
        plane_split(ind, count, cutfeat, cutval, lim1, lim2);
        if (lim1 > count / 2)
            index = lim1;
        else if (lim2 < count / 2)
            index = lim2;
        else
            index = count / 2;
    }

    int divide(size_t left, size_t right, Box &b) {
        const int id = (int)nodes_.size();
        nodes_.emplace_back();
        if (right - left <= kLeaf) {
            nodes_[id].left = left;
            nodes_[id].right = right;
            for (int d = 0; d < 3; ++d) b.lo[d] = b.hi[d] = at(vind_[left], d);
            for (size_t k = left + 1; k < right; ++k)
                for (int d = 0; d < 3; ++d) {
                    const float v = at(vind_[k], d);
                    if (b.lo[d] > v) b.lo[d] = v;
                    if (b.hi[d] < v) b.hi[d] = v;
                }
            return id;
        }
        size_t idx;
        int cutfeat;
        float cutval;
        middle_split(vind_.data() + left, right - left, idx, cutfeat, cutval, b);
        Box lb = b, rb = b;
        lb.hi[cutfeat] = cutval;
        const int c1 = divide(left, left + idx, lb);
        rb.lo[cutfeat] = cutval;
        const int c2 = divide(left + idx, right, rb);
        KdNode &nd = nodes_[id];
        nd.child1 = c1;
        nd.child2 = c2;
        nd.divfeat = cutfeat;
        nd.divlow = lb.hi[cutfeat];
        nd.divhigh = rb.lo[cutfeat];
        for (int d = 0; d < 3; ++d) {
            b.lo[d] = std::min(lb.lo[d], rb.lo[d]);
            b.hi[d] = std::max(lb.hi[d], rb.hi[d]);
        }
        return id;
    }

    void search(int id, const float *q, float r2, float mindistsq, float *dists,
                std::vector<std::pair<size_t, float>> &out) const {
        const KdNode &nd = nodes_[id];
        if (nd.child1 < 0 && nd.child2 < 0) {
            for (size_t i = nd.left; i < nd.right; ++i) {
                const size_t j = vind_[i];
                float d = 0.f;
                for (int k = 0; k < 3; ++k) {
                    const float diff = q[k] - at(j, k);
                    d += diff * diff;
                }
                if (d < r2) out.emplace_back(j, d);
            }
            return;
        }
        const int f = nd.divfeat;
        const float val = q[f];
        const float diff1 = val - nd.divlow, diff2 = val - nd.divhigh;
        int best, other;
        float cut;
        if ((diff1 + diff2) < 0) {
            best = nd.child1;
            other = nd.child2;
            cut = (val - nd.divhigh) * (val - nd.divhigh);
        } else {
            best = nd.child2;
            other = nd.child1;
            cut = (val - nd.divlow) * (val - nd.divlow);
        }
        search(best, q, r2, mindistsq, dists, out);
        const float dst = dists[f];
        mindistsq = mindistsq + cut - dst;
        dists[f] = cut;
        if (mindistsq * 1.0f <= r2) search(other, q, r2, mindistsq, dists, out);
        dists[f] = dst;
    }

    static constexpr size_t kLeaf = 10;
    const float *p_;
    size_t n_;
    std::vector<size_t> vind_;
    std::vector<KdNode> nodes_;
    Box root_{};
    int root_node_ = -1;
};

}  // namespace

// rows: query indices (ascending) to recompute; qbatch[k] = batch of rows[k].
// q (nq,3) / s (ns,3) host copies; soff the support batch offsets.  Writes
// res[k] = the reference's neighbour list of rows[k] as global support indices.
void kd_replay_rows(const float *q, const float *s, const int *soff, const std::vector<int> &rows,
                    const std::vector<int> &qbatch, float r2,
                    std::vector<std::vector<int>> &res) {
    res.assign(rows.size(), {});
    std::vector<std::pair<size_t, float>> hits;
    size_t k = 0;
    while (k < rows.size()) {
        const int b = qbatch[k];
        const KdTree tree(s + 3 * (size_t)soff[b], (size_t)(soff[b + 1] - soff[b]));
        for (; k < rows.size() && qbatch[k] == b; ++k) {
            tree.radius(q + 3 * (size_t)rows[k], r2, hits);
            res[k].reserve(hits.size());
            for (const auto &h : hits) res[k].push_back((int)h.first + soff[b]);
        }
    }
}

}  // namespace pcr

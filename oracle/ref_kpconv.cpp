// TEST INFRASTRUCTURE ONLY.  C-ABI driver around the REFERENCE's own KPConv
// helpers (c2p-net/ngenet/cpp_wrappers): cpp_subsampling/grid_subsampling/
// grid_subsampling.cpp (batch_grid_subsampling) and cpp_neighbors/neighbors/
// neighbors.cpp (batch_nanoflann_neighbors, vendored nanoflann), compiled in place
// with the reference's flags (setup.py: -std=c++11 -D_GLIBCXX_USE_CXX11_ABI=0)
// by oracle/build_ref.sh into oracle/_ref/libref_kpconv.so.
//
// This file replaces only the CPython marshalling of the reference's wrapper.cpp
// files (cpp_subsampling/wrapper.cpp:232-263, cpp_neighbors/wrapper.cpp:183-224),
// which no longer compile against the numpy 2 headers in this image: arrays in
// -> std::vector<PointXYZ> -> the reference function -> arrays out.
#include <cstdlib>
#include <cstring>
#include <vector>

#include "cloud/cloud.h"
#include "grid_subsampling/grid_subsampling.h"
#include "neighbors/neighbors.h"

extern "C" {

// subsample_batch(points, batches, features=..., sampleDl, max_p): results are
// malloc'ed; free with ref_free.  Returns the number of output points.
int ref_subsample_batch(const float *pts, int n, const int *batches, int nb, const float *feats,
                        int fdim, float dl, int max_p, float **out_pts, int **out_batches,
                        float **out_feats) {
    std::vector<PointXYZ> op((const PointXYZ *)pts, (const PointXYZ *)pts + n);
    std::vector<int> ob(batches, batches + nb);
    std::vector<float> of;
    if (feats && fdim > 0) of.assign(feats, feats + (size_t)n * fdim);
    std::vector<int> oc, sc, sb;
    std::vector<PointXYZ> sp;
    std::vector<float> sf;
    batch_grid_subsampling(op, sp, of, sf, oc, sc, ob, sb, dl, max_p);
    const int m = (int)sp.size();
    *out_pts = (float *)malloc(sizeof(float) * 3 * (m > 0 ? m : 1));
    memcpy(*out_pts, sp.data(), sizeof(float) * 3 * m);
    *out_batches = (int *)malloc(sizeof(int) * (nb > 0 ? nb : 1));
    memcpy(*out_batches, sb.data(), sizeof(int) * sb.size());
    if (out_feats) {
        *out_feats = (float *)malloc(sizeof(float) * (sf.size() > 0 ? sf.size() : 1));
        memcpy(*out_feats, sf.data(), sizeof(float) * sf.size());
    }
    return m;
}

// batch_query(queries, supports, q_batches, s_batches, radius): (nq, max_count)
// int32, padded with supports.size().  Returns max_count.
int ref_batch_neighbors(const float *q, int nq, const float *s, int ns, const int *qb,
                        const int *sb, int nb, float radius, int **out) {
    std::vector<PointXYZ> queries((const PointXYZ *)q, (const PointXYZ *)q + nq);
    std::vector<PointXYZ> supports((const PointXYZ *)s, (const PointXYZ *)s + ns);
    std::vector<int> q_batches(qb, qb + nb), s_batches(sb, sb + nb), idx;
    batch_nanoflann_neighbors(queries, supports, q_batches, s_batches, idx, radius);
    const int mc = nq > 0 ? (int)(idx.size() / (size_t)nq) : 0;
    *out = (int *)malloc(sizeof(int) * (idx.size() > 0 ? idx.size() : 1));
    memcpy(*out, idx.data(), sizeof(int) * idx.size());
    return mc;
}

void ref_free(void *p) { free(p); }
}

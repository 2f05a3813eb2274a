/*
 * TEST INFRASTRUCTURE ONLY (never linked by the product): a restatement of
 * Open3D 0.13 PointCloud::VoxelDownSample (geometry/PointCloud.cpp), the call
 * at dip/demo.py:73-74.  Open3D is absent from this image, so this
 * follows its published algorithm; parity vs Open3D itself is unpinned beyond
 * it, and the tests also check it against an independent numpy grouping.
 *
 *   voxel_min_bound = GetMinBound() - voxel_size3 * 0.5
 *   ref_coord = (p - voxel_min_bound) / voxel_size
 *   voxel_index = (int(floor(x)), int(floor(y)), int(floor(z)))
 *   voxelindex_to_accpoint[voxel_index].AddPoint(cloud, i)   (point_ += p,
 *       normal_ += n unless a component is NaN, color_ += c, ++count)
 *   for (auto accpoint : voxelindex_to_accpoint): emit point_ / double(count)
 *       (normals and colors likewise)
 *
 * The map is std::unordered_map<Eigen::Vector3i, AccumulatedPoint,
 * utility::hash_eigen<Eigen::Vector3i>>; the key and hash are restated below
 * (hash_eigen = boost-style hash_combine over the coefficients).
 */
#include <climits>
#include <cmath>
#include <cstdint>
#include <functional>
#include <unordered_map>

namespace {

struct Key {
    int v[3];
    bool operator==(const Key &o) const { return v[0] == o.v[0] && v[1] == o.v[1] && v[2] == o.v[2]; }
};

struct HashEigen {
    std::size_t operator()(const Key &m) const {
        std::size_t seed = 0;
        for (int i = 0; i < 3; i++)
            seed ^= std::hash<int>()(m.v[i]) + 0x9e3779b9 + (seed << 6) + (seed >> 2);
        return seed;
    }
};

struct AccumulatedPoint {
    double point[3] = {0.0, 0.0, 0.0}, normal[3] = {0.0, 0.0, 0.0}, color[3] = {0.0, 0.0, 0.0};
    int num = 0;
};

}  // namespace

/* returns the number of output points (rows of out_*), or -1 on the reference's
   errors (voxel_size <= 0, voxel_size too small); normals / colors may be NULL */
extern "C" int oracle_voxel_down_sample(const double *pts, int n, double voxel_size,
                                        const double *normals, const double *colors,
                                        double *out_p, double *out_n, double *out_c)
{
    if (voxel_size <= 0.0) return -1;
    if (n <= 0) return 0;
    double mn[3], mx[3];
    for (int c = 0; c < 3; c++) { mn[c] = pts[c]; mx[c] = pts[c]; }
    for (int i = 1; i < n; i++)
        for (int c = 0; c < 3; c++) {
            mn[c] = std::min(mn[c], pts[3 * i + c]);
            mx[c] = std::max(mx[c], pts[3 * i + c]);
        }
    const double half = voxel_size * 0.5;
    double vmin[3], ext = 0.0;
    for (int c = 0; c < 3; c++) {
        vmin[c] = mn[c] - half;
        ext = std::max(ext, (mx[c] + half) - vmin[c]);
    }
    if (voxel_size * (double)INT_MAX < ext) return -1;
    std::unordered_map<Key, AccumulatedPoint, HashEigen> acc;
    for (int i = 0; i < n; i++) {
        Key k;
        for (int c = 0; c < 3; c++) k.v[c] = (int)std::floor((pts[3 * i + c] - vmin[c]) / voxel_size);
        AccumulatedPoint &a = acc[k];
        for (int c = 0; c < 3; c++) a.point[c] += pts[3 * i + c];
        if (normals) {
            const double *nv = normals + 3 * i;
            if (!std::isnan(nv[0]) && !std::isnan(nv[1]) && !std::isnan(nv[2]))
                for (int c = 0; c < 3; c++) a.normal[c] += nv[c];
        }
        if (colors)
            for (int c = 0; c < 3; c++) a.color[c] += colors[3 * i + c];
        a.num++;
    }
    int k = 0;
    for (const auto &kv : acc) {
        const AccumulatedPoint &a = kv.second;
        for (int c = 0; c < 3; c++) {
            out_p[3 * k + c] = a.point[c] / (double)a.num;
            if (normals && out_n) out_n[3 * k + c] = a.normal[c] / (double)a.num;
            if (colors && out_c) out_c[3 * k + c] = a.color[c] / (double)a.num;
        }
        k++;
    }
    return k;
}

/* the iteration order of the same map type for keys inserted in the given order
   (order[k] = insertion index of the k-th visited key): the check for the
   product's array simulation of it (csrc/voxel.hip voxel3i_map_order) */
extern "C" void oracle_voxel3i_map_order(const int *xyz, int n, int *order)
{
    std::unordered_map<Key, int, HashEigen> m;
    for (int r = 0; r < n; r++) m.emplace(Key{{xyz[3 * r], xyz[3 * r + 1], xyz[3 * r + 2]}}, r);
    int k = 0;
    for (const auto &kv : m) order[k++] = kv.second;
}

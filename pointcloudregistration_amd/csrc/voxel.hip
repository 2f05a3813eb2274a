// f2: Open3D PointCloud::VoxelDownSample for a batch of clouds
// (dip/demo.py:73-74 `pcd.voxel_down_sample(voxel_size)`, the C3 input stage).
//
// Semantics (Open3D 0.13 geometry/PointCloud.cpp, restated in
// oracle/voxel_oracle.cpp):
//   voxel_min_bound = min_bound - voxel/2 (per axis), every point p goes to the
//   voxel int(floor((p - voxel_min_bound) / voxel)) (Eigen::Vector3i key of an
//   unordered_map with utility::hash_eigen); each voxel accumulates its points
//   in input order (point_ += p; normals without NaN components; colors) and
//   emits point_ / double(count) -- normals and colors divided the same way --
//   in the map's iteration order.  f64 throughout (Open3D stores double).
//
// MI355X design: bounding boxes, voxel keys, a stable radix sort by (cloud,
// voxel), the run heads, the per-voxel sums (sequential in input order: the
// same roundings) and the output rows run on the GPU.  The map's iteration
// order is a property of libstdc++'s hashtable (bucket growth and node
// splicing), so the host replays it: the distinct voxels of a cloud, in
// first-occurrence order, are inserted into a std::unordered_map with the same
// key type and hash -- the reference's insertion sequence, hence its order --
// and the GPU writes each voxel's row to its slot.
#include "pcr_internal.h"

#include <cstring>

#include <rocprim/rocprim.hpp>

#include <climits>
#include <cmath>
#include <unordered_map>
#include <thread>
#include <vector>

namespace pcr {
namespace {

typedef unsigned long long u64;

struct VArgs {
    const double *pts, *nrm, *col;
    int n, nb;
    const int *off;      // [nb+1]
    double voxel;
    double *bbox;        // [nb][6] min xyz, max xyz
    int *bad;            // non-finite coordinate seen
    const double *vmb;   // [nb][3] voxel_min_bound
    int sx, sy, sz, sb;  // key bit shifts (x | y | z | cloud)
    u64 *key;
    int *iota;
};

__device__ __forceinline__ int cloud_of(const int *off, int nb, int i) {
    int lo = 0, hi = nb - 1;  // largest b with off[b] <= i
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (off[mid] <= i) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// one block per cloud: min / max corners (PointCloud::GetMinBound / GetMaxBound)
__global__ __launch_bounds__(256) void vd_bbox(VArgs a) {
    const int b = blockIdx.x, t = threadIdx.x;
    const int i0 = a.off[b], i1 = a.off[b + 1];
    double lo[3] = {__builtin_inf(), __builtin_inf(), __builtin_inf()};
    double hi[3] = {-__builtin_inf(), -__builtin_inf(), -__builtin_inf()};
    int bad = 0;
    for (int i = i0 + t; i < i1; i += 256)
        for (int c = 0; c < 3; ++c) {
            const double v = a.pts[3 * (size_t)i + c];
            bad |= !__builtin_isfinite(v);
            lo[c] = fmin(lo[c], v);
            hi[c] = fmax(hi[c], v);
        }
    __shared__ double sl[3][4], sh[3][4];
    __shared__ int sb[4];
    for (int c = 0; c < 3; ++c)
        for (int o = 32; o; o >>= 1) {
            lo[c] = fmin(lo[c], __shfl_xor(lo[c], o, 64));
            hi[c] = fmax(hi[c], __shfl_xor(hi[c], o, 64));
        }
    for (int o = 32; o; o >>= 1) bad |= __shfl_xor(bad, o, 64);
    if ((t & 63) == 0) {
        for (int c = 0; c < 3; ++c) { sl[c][t >> 6] = lo[c]; sh[c][t >> 6] = hi[c]; }
        sb[t >> 6] = bad;
    }
    __syncthreads();
    if (t != 0) return;
    if (sb[0] | sb[1] | sb[2] | sb[3]) atomicOr(a.bad, 1);
    for (int c = 0; c < 3; ++c) {
        double l = sl[c][0], h = sh[c][0];
        for (int w = 1; w < 4; ++w) { l = fmin(l, sl[c][w]); h = fmax(h, sh[c][w]); }
        a.bbox[6 * b + c] = l;
        a.bbox[6 * b + 3 + c] = h;
    }
}

__device__ __forceinline__ int voxel_index(double p, double vmb, double voxel) {
    return (int)__builtin_floor((p - vmb) / voxel);
}

__global__ void vd_key(VArgs a) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const int b = cloud_of(a.off, a.nb, i);
    const double *p = a.pts + 3 * (size_t)i;
    const double *m = a.vmb + 3 * b;
    const u64 ix = (u64)voxel_index(p[0], m[0], a.voxel), iy = (u64)voxel_index(p[1], m[1], a.voxel),
              iz = (u64)voxel_index(p[2], m[2], a.voxel);
    a.key[i] = ((u64)b << a.sb) | (ix << a.sx) | (iy << a.sy) | (iz << a.sz);
    a.iota[i] = i;
}

__global__ void vd_heads(const u64 *key, int n, unsigned char *head) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) head[i] = (i == 0) || key[i] != key[i - 1];
}

// mark[first input index of voxel r] = r (the sort is stable: a run's first
// entry is its lowest input index)
__global__ void vd_mark(const int *start, const int *v, int V, int *mark) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r < V) mark[v[start[r]]] = r;
}

struct NonNeg {
    __device__ bool operator()(int x) const { return x >= 0; }
};

__global__ void vd_okey(const int *list, const int *start, const u64 *skey, int V, u64 *okey) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r < V) okey[r] = skey[start[list[r]]];
}

// output row pos <- voxel list[outr[pos]]: sums in input order from zero
// (AccumulatedPoint::AddPoint), then / double(count)
__global__ void vd_emit(VArgs a, const int *outr, int total, const int *list, const int *start,
                        const int *v, double *op, double *on, double *oc) {
    const int pos = blockIdx.x * blockDim.x + threadIdx.x;
    if (pos >= total) return;
    const int vox = list[outr[pos]];
    const int s0 = start[vox], s1 = start[vox + 1];
    const double cnt = (double)(s1 - s0);
    double s[3] = {0.0, 0.0, 0.0};
    for (int q = s0; q < s1; ++q)
        for (int c = 0; c < 3; ++c) s[c] = s[c] + a.pts[3 * (size_t)v[q] + c];
    for (int c = 0; c < 3; ++c) op[3 * (size_t)pos + c] = s[c] / cnt;
    if (a.nrm && on) {
        double t[3] = {0.0, 0.0, 0.0};
        for (int q = s0; q < s1; ++q) {
            const double *nv = a.nrm + 3 * (size_t)v[q];
            if (!__builtin_isnan(nv[0]) && !__builtin_isnan(nv[1]) && !__builtin_isnan(nv[2]))
                for (int c = 0; c < 3; ++c) t[c] = t[c] + nv[c];
        }
        for (int c = 0; c < 3; ++c) on[3 * (size_t)pos + c] = t[c] / cnt;
    }
    if (a.col && oc) {
        double t[3] = {0.0, 0.0, 0.0};
        for (int q = s0; q < s1; ++q)
            for (int c = 0; c < 3; ++c) t[c] = t[c] + a.col[3 * (size_t)v[q] + c];
        for (int c = 0; c < 3; ++c) oc[3 * (size_t)pos + c] = t[c] / cnt;
    }
}

inline unsigned nbits(u64 x) { return x ? 64u - (unsigned)__builtin_clzll(x) : 0u; }
inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

struct Carve {
    size_t used = 0;
    template <class T> size_t take(size_t count) {
        const size_t at = used;
        used = align256(used + sizeof(T) * (count > 0 ? count : 1));
        return at;
    }
};

// Eigen::Vector3i key with Open3D's utility::hash_eigen (boost hash_combine
// over the coefficients; std::hash<int> is the identity in libstdc++)
struct V3i {
    int x, y, z;
    bool operator==(const V3i &o) const { return x == o.x && y == o.y && z == o.z; }
};
struct HashEigenV3i {
    size_t operator()(const V3i &k) const {
        size_t seed = 0;
        const int e[3] = {k.x, k.y, k.z};
        for (int i = 0; i < 3; ++i)
            seed ^= std::hash<int>()(e[i]) + 0x9e3779b9 + (seed << 6) + (seed >> 2);
        return seed;
    }
};

}  // namespace

// host replay of the reference's unordered_map<Vector3i, AccumulatedPoint,
// hash_eigen> iteration order for the voxels of ONE cloud given in
// first-occurrence order; order[k] = index (into keys) of the k-th emitted voxel.
//
// libstdc++'s unique-key _Hashtable keeps all nodes in one singly linked list
// and, per bucket, a pointer to the node BEFORE the bucket's first node; its
// iteration order is that list.  It is simulated here with index arrays (no node
// allocation): the same hash codes (hash_eigen), the same bucket counts (the
// library's own _Prime_rehash_policy, asked exactly when the container asks it:
// before every insertion of a new key), the same insertion rule (a new node goes
// first in its bucket; into an empty bucket it goes first in the whole list and
// the bucket of the former first node is re-pointed at it) and the same rehash
// relinking (old list order, each node to the front of its new bucket, or of the
// list when that bucket is empty).  oracle_voxel3i_map_order builds the real
// container for the parity test.
void voxel3i_map_order(const int32_t *xyz, int n, int32_t *order) {
    if (n <= 0) return;
    constexpr int kNil = -2, kBefore = -1;  // bucket slot: empty / the list head
    std::vector<size_t> code((size_t)n);
    for (int r = 0; r < n; ++r) code[r] = HashEigenV3i()(V3i{xyz[3 * r], xyz[3 * r + 1], xyz[3 * r + 2]});
    std::vector<int> nxt((size_t)n, kNil), bkt(1, kNil), nb;
    int head = kNil;
    size_t nbkt = 1;
    std::__detail::_Prime_rehash_policy pol;  // max_load_factor 1
    auto link_after = [&](int before, int node) {  // node after `before` (head if kBefore)
        int &slot = before == kBefore ? head : nxt[before];
        nxt[node] = slot;
        slot = node;
    };
    for (int r = 0; r < n; ++r) {
        const std::pair<bool, size_t> rh = pol._M_need_rehash(nbkt, (size_t)r, 1);
        if (rh.first) {
            const size_t nn = rh.second;
            nb.assign(nn, kNil);
            int p = head;
            head = kNil;
            size_t bbegin = 0;
            while (p != kNil) {
                const int next = nxt[p];
                const size_t b = code[p] % nn;
                if (nb[b] == kNil) {
                    nxt[p] = head;
                    head = p;
                    nb[b] = kBefore;
                    if (nxt[p] != kNil) nb[bbegin] = p;
                    bbegin = b;
                } else {
                    link_after(nb[b], p);
                }
                p = next;
            }
            bkt.swap(nb);
            nbkt = nn;
        }
        const size_t b = code[r] % nbkt;
        if (bkt[b] != kNil) {
            link_after(bkt[b], r);
        } else {
            nxt[r] = head;
            head = r;
            if (nxt[r] != kNil) bkt[code[nxt[r]] % nbkt] = r;
            bkt[b] = kBefore;
        }
    }
    int k = 0;
    for (int p = head; p != kNil; p = nxt[p]) order[k++] = p;
}

}  // namespace pcr

extern "C" int pcr_voxel3i_map_order(const int32_t *xyz, int32_t n, int32_t *order) {
    pcr::clear_error();
    PCR_REQUIRE(n >= 0 && (n == 0 || (xyz && order)), PCR_ERR_ARG, "voxel3i_map_order: bad arguments");
    pcr::voxel3i_map_order(xyz, n, order);
    return PCR_OK;
}

extern "C" int pcr_voxel_down_sample(const double *points, int32_t n, const int32_t *cloud_len,
                                     int32_t nb, double voxel_size, const double *normals,
                                     const double *colors, double *out_points, double *out_normals,
                                     double *out_colors, int32_t *out_cloud_len, int32_t *out_total,
                                     pcr_stream_t stream) {
    using namespace pcr;
    clear_error();
    PCR_REQUIRE(n >= 0 && nb >= 1 && cloud_len && out_cloud_len && out_total, PCR_ERR_ARG,
                "voxel_down_sample: bad arguments");
    PCR_REQUIRE(n == 0 || (points && out_points), PCR_ERR_ARG, "voxel_down_sample: null points");
    // PointCloud::VoxelDownSample: "[VoxelDownSample] voxel_size <= 0."
    PCR_REQUIRE(voxel_size > 0.0, PCR_ERR_ARG, "[VoxelDownSample] voxel_size <= 0.");
    std::vector<int> off(nb + 1, 0);
    for (int b = 0; b < nb; ++b) {
        PCR_REQUIRE(cloud_len[b] >= 0, PCR_ERR_ARG, "voxel_down_sample: negative cloud length");
        off[b + 1] = off[b] + cloud_len[b];
    }
    PCR_REQUIRE(off[nb] <= n, PCR_ERR_ARG, "voxel_down_sample: clouds sum to %d > %d points", off[nb], n);
    const int N = off[nb];
    *out_total = 0;
    for (int b = 0; b < nb; ++b) out_cloud_len[b] = 0;
    if (N == 0) return PCR_OK;
    hipStream_t st = as_stream(stream);
    Carve c;
    const size_t o_off = c.take<int>(nb + 1), o_bb = c.take<double>(6 * (size_t)nb),
                 o_vmb = c.take<double>(3 * (size_t)nb), o_bad = c.take<int>(2),
                 o_key = c.take<u64>(N), o_skey = c.take<u64>(N), o_iota = c.take<int>(N),
                 o_v = c.take<int>(N), o_head = c.take<unsigned char>(N), o_start = c.take<int>(N + 1),
                 o_mark = c.take<int>(N), o_list = c.take<int>(N), o_okey = c.take<u64>(N),
                 o_outr = c.take<int>(N), o_cnt = c.take<int>(2);
    char *ws = (char *)workspace(27, c.used);
    PCR_REQUIRE(ws, PCR_ERR_NOMEM, "voxel_down_sample: %s", pcr_last_error());
    VArgs a;
    a.pts = points; a.nrm = normals; a.col = colors; a.n = N; a.nb = nb;
    a.off = (int *)(ws + o_off); a.voxel = voxel_size;
    a.bbox = (double *)(ws + o_bb); a.vmb = (const double *)(ws + o_vmb); a.bad = (int *)(ws + o_bad);
    a.key = (u64 *)(ws + o_key); a.iota = (int *)(ws + o_iota);
    u64 *skey = (u64 *)(ws + o_skey);
    int *v = (int *)(ws + o_v);
    unsigned char *head = (unsigned char *)(ws + o_head);
    int *start = (int *)(ws + o_start), *mark = (int *)(ws + o_mark), *list = (int *)(ws + o_list);
    u64 *okey = (u64 *)(ws + o_okey);
    int *outr = (int *)(ws + o_outr), *dcnt = (int *)(ws + o_cnt);

    PCR_HIP_CHECK(hipMemcpyAsync((void *)a.off, off.data(), sizeof(int) * (nb + 1), hipMemcpyHostToDevice, st));
    PCR_HIP_CHECK(hipMemsetAsync(a.bad, 0, sizeof(int), st));
    hipLaunchKernelGGL(vd_bbox, dim3(nb), dim3(256), 0, st, a);
    PCR_LAUNCH_CHECK();
    std::vector<double> bb(6 * (size_t)nb);
    int hbad = 0;
    PCR_HIP_CHECK(hipMemcpyAsync(bb.data(), a.bbox, sizeof(double) * bb.size(), hipMemcpyDeviceToHost, st));
    PCR_HIP_CHECK(hipMemcpyAsync(&hbad, a.bad, sizeof(int), hipMemcpyDeviceToHost, st));
    PCR_HIP_CHECK(hipStreamSynchronize(st));
    PCR_REQUIRE(!hbad, PCR_ERR_ARG,
                "voxel_down_sample: non-finite point coordinates (the reference's voxel index is undefined there)");
    // voxel_min_bound = min - voxel/2 (Eigen: voxel_size3 * 0.5), the too-small
    // check of the reference, and the widest voxel index per axis (monotone:
    // the last point's floor((max - vmb) / voxel))
    std::vector<double> vmb(3 * (size_t)nb);
    u64 mx[3] = {0, 0, 0};
    const double half = voxel_size * 0.5;
    for (int b = 0; b < nb; ++b) {
        if (off[b + 1] == off[b]) { vmb[3 * b] = vmb[3 * b + 1] = vmb[3 * b + 2] = 0.0; continue; }
        double ext = 0.0;
        for (int q = 0; q < 3; ++q) {
            const double lo = bb[6 * b + q] - half, hi = bb[6 * b + 3 + q] + half;
            vmb[3 * b + q] = lo;
            ext = std::max(ext, hi - lo);
        }
        PCR_REQUIRE(!(voxel_size * (double)INT_MAX < ext), PCR_ERR_ARG,
                    "[VoxelDownSample] voxel_size is too small.");
        for (int q = 0; q < 3; ++q) {
            const double r = std::floor((bb[6 * b + 3 + q] - vmb[3 * b + q]) / voxel_size);
            mx[q] = std::max(mx[q], (u64)r);
        }
    }
    const unsigned bz = std::max(1u, nbits(mx[2])), by = std::max(1u, nbits(mx[1])),
                   bx = std::max(1u, nbits(mx[0])), bbat = nbits((u64)(nb - 1));
    PCR_REQUIRE(bx + by + bz + bbat <= 64, PCR_ERR_ARG,
                "voxel_down_sample: %u-bit voxel keys (the grid is too fine for one 64-bit sort key)",
                bx + by + bz + bbat);
    a.sz = 0; a.sy = (int)bz; a.sx = (int)(bz + by); a.sb = (int)(bz + by + bx);
    PCR_HIP_CHECK(hipMemcpyAsync((void *)a.vmb, vmb.data(), sizeof(double) * vmb.size(), hipMemcpyHostToDevice, st));
    const dim3 gN((N + 255) / 256), blk(256);
    hipLaunchKernelGGL(vd_key, gN, blk, 0, st, a);
    PCR_LAUNCH_CHECK();
    // stable radix sort by (cloud, voxel): input order kept inside a voxel
    const unsigned kb = bx + by + bz + bbat;
    size_t tb = 0, t1 = 0;
    PCR_HIP_CHECK(rocprim::radix_sort_pairs(nullptr, t1, a.key, skey, a.iota, v, N, 0, kb, st));
    tb = t1;
    PCR_HIP_CHECK(rocprim::select(nullptr, t1, rocprim::counting_iterator<int>(0), head, start, dcnt, (size_t)N, st));
    tb = std::max(tb, t1);
    PCR_HIP_CHECK(rocprim::select(nullptr, t1, mark, list, dcnt + 1, (size_t)N, NonNeg(), st));
    tb = std::max(tb, t1);
    void *tmp = workspace(28, tb);
    PCR_REQUIRE(tmp, PCR_ERR_NOMEM, "voxel_down_sample: %s", pcr_last_error());
    t1 = tb;
    PCR_HIP_CHECK(rocprim::radix_sort_pairs(tmp, t1, a.key, skey, a.iota, v, N, 0, kb, st));
    hipLaunchKernelGGL(vd_heads, gN, blk, 0, st, skey, N, head);
    PCR_LAUNCH_CHECK();
    t1 = tb;
    PCR_HIP_CHECK(rocprim::select(tmp, t1, rocprim::counting_iterator<int>(0), head, start, dcnt, (size_t)N, st));
    int V = 0;
    PCR_HIP_CHECK(hipMemcpyAsync(&V, dcnt, sizeof(int), hipMemcpyDeviceToHost, st));
    PCR_HIP_CHECK(hipStreamSynchronize(st));
    PCR_HIP_CHECK(hipMemcpyAsync(start + V, &N, sizeof(int), hipMemcpyHostToDevice, st));
    PCR_HIP_CHECK(hipMemsetAsync(mark, 0xFF, sizeof(int) * N, st));
    const dim3 gV((V + 255) / 256);
    hipLaunchKernelGGL(vd_mark, gV, blk, 0, st, start, v, V, mark);
    PCR_LAUNCH_CHECK();
    t1 = tb;
    PCR_HIP_CHECK(rocprim::select(tmp, t1, mark, list, dcnt + 1, (size_t)N, NonNeg(), st));
    hipLaunchKernelGGL(vd_okey, gV, blk, 0, st, list, start, skey, V, okey);
    PCR_LAUNCH_CHECK();
    std::vector<u64> hk(V);
    PCR_HIP_CHECK(hipMemcpyAsync(hk.data(), okey, sizeof(u64) * V, hipMemcpyDeviceToHost, st));
    PCR_HIP_CHECK(hipStreamSynchronize(st));
    // per cloud: the map's iteration order (voxels in first-occurrence order);
    // clouds are independent, so their replays run on host threads
    const u64 mxk = (1ull << bx) - 1ull, myk = (1ull << by) - 1ull, mzk = (1ull << bz) - 1ull;
    std::vector<int> r0s;
    for (int r = 0; r < V; ++r)
        if (r == 0 || (bbat && (hk[r] >> a.sb) != (hk[r - 1] >> a.sb))) r0s.push_back(r);
    r0s.push_back(V);
    const int ncl = (int)r0s.size() - 1;
    std::vector<int> hout((size_t)V);
    auto replay = [&](int c) {
        const int r0 = r0s[c], cnt = r0s[c + 1] - r0;
        std::vector<int32_t> xyz(3 * (size_t)cnt), ord((size_t)cnt);
        for (int k = 0; k < cnt; ++k) {
            const u64 key = hk[r0 + k];
            xyz[3 * k] = (int32_t)((key >> a.sx) & mxk);
            xyz[3 * k + 1] = (int32_t)((key >> a.sy) & myk);
            xyz[3 * k + 2] = (int32_t)((key >> a.sz) & mzk);
        }
        voxel3i_map_order(xyz.data(), cnt, ord.data());
        for (int k = 0; k < cnt; ++k) hout[r0 + k] = r0 + ord[k];
    };
    const int nth = std::min(ncl, 16);
    if (nth <= 1 || V < 65536) {
        for (int c = 0; c < ncl; ++c) replay(c);
    } else {
        std::vector<std::thread> th;
        for (int t = 0; t < nth; ++t)
            th.emplace_back([&, t]() { for (int c = t; c < ncl; c += nth) replay(c); });
        for (auto &h : th) h.join();
    }
    for (int c = 0; c < ncl; ++c) {
        const u64 cb = bbat ? (hk[r0s[c]] >> a.sb) : 0ull;
        out_cloud_len[cb] = r0s[c + 1] - r0s[c];
    }
    const int total = (int)hout.size();
    PCR_HIP_CHECK(hipMemcpyAsync(outr, hout.data(), sizeof(int) * total, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(vd_emit, dim3((total + 255) / 256), blk, 0, st, a, outr, total, list, start, v,
                       out_points, normals ? out_normals : nullptr, colors ? out_colors : nullptr);
    PCR_LAUNCH_CHECK();
    PCR_HIP_CHECK(hipStreamSynchronize(st));  // hout is a host temporary
    *out_total = total;
    return PCR_OK;
}

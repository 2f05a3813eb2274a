/*
 * pcr_oracle.c -- CPU restatement of the reference's correspondence/alignment
 * hot path.  TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg as the CHECKER.  The product (libpcr.so) never
 * links, loads or calls anything in oracle/.
 *
 * Every function cites the reference file:line whose semantics it restates.
 * Compiled with -O2 -ffp-contract=off so every floating-point operation is
 * individually rounded in the order written (this is the bit-exact contract the
 * HIP kernels are tested against; see DESIGN.md "Numerical contract").
 *
 * Pinning (see tests/golden/README.md):
 *   nnd_*          pinned bit-exact against the compiled reference my_lib.cpp (oracle/_ref)
 *   procrustes     pinned against the reference's weighted_icp / rigid_fit (Python import)
 *   featnn         pinned against the reference's vote.get_coor_points semantics
 *   ransac / icp   Open3D is absent -> parity vs. reference UNPINNED; pinned only by
 *                  known-answer tests (ground-truth R,t) and GPU==CPU bit-exactness
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------- */
/* a1: brute-force 1-NN, restating dip/torch-nndistance/src/my_lib.cpp:3-25   */
/* (nnsearch) and :28-60 (nnd_forward: both directions).                      */
/*   d = (dx*dx + dy*dy) + dz*dz in fp32 with dx = b.x - a.x (my_lib.cpp:12-15)*/
/*   seed with k == 0, update on strict d < best (first index wins, :16)      */
/* ------------------------------------------------------------------------- */
static void nnsearch(int b, int n, int m, const float *xyz1, const float *xyz2,
                     float *dist, int32_t *idx)
{
    for (int i = 0; i < b; i++) {
        for (int j = 0; j < n; j++) {
            const float x1 = xyz1[((size_t)i * n + j) * 3 + 0];
            const float y1 = xyz1[((size_t)i * n + j) * 3 + 1];
            const float z1 = xyz1[((size_t)i * n + j) * 3 + 2];
            float best = 0.0f;
            int besti = 0;
            for (int k = 0; k < m; k++) {
                const float x2 = xyz2[((size_t)i * m + k) * 3 + 0] - x1;
                const float y2 = xyz2[((size_t)i * m + k) * 3 + 1] - y1;
                const float z2 = xyz2[((size_t)i * m + k) * 3 + 2] - z1;
                const float d = x2 * x2 + y2 * y2 + z2 * z2;
                if (k == 0 || d < best) { best = d; besti = k; }
            }
            dist[(size_t)i * n + j] = best;
            idx[(size_t)i * n + j] = besti;
        }
    }
}

void oracle_nnd_forward(const float *xyz1, const float *xyz2, int b, int n, int m,
                        float *dist1, float *dist2, int32_t *idx1, int32_t *idx2)
{
    nnsearch(b, n, m, xyz1, xyz2, dist1, idx1);
    nnsearch(b, m, n, xyz2, xyz1, dist2, idx2);
}

/* a2: restates my_lib.cpp:64-133 (nnd_backward), same accumulation order:   */
/* grads zeroed, loop 1 over xyz1 points (direct += then scatter -=), loop 2  */
/* over xyz2 points.  g = graddist*2 (fp32), term = g*(x1-x2).                */
void oracle_nnd_backward(const float *xyz1, const float *xyz2, const float *gd1,
                         const float *gd2, const int32_t *idx1, const int32_t *idx2,
                         int b, int n, int m, float *gxyz1, float *gxyz2)
{
    memset(gxyz1, 0, sizeof(float) * (size_t)b * n * 3);
    memset(gxyz2, 0, sizeof(float) * (size_t)b * m * 3);
    for (int i = 0; i < b; i++) {
        for (int j = 0; j < n; j++) {
            const float *p1 = xyz1 + ((size_t)i * n + j) * 3;
            const int j2 = idx1[(size_t)i * n + j];
            const float *p2 = xyz2 + ((size_t)i * m + j2) * 3;
            const float g = gd1[(size_t)i * n + j] * 2;
            float *g1 = gxyz1 + ((size_t)i * n + j) * 3;
            float *g2 = gxyz2 + ((size_t)i * m + j2) * 3;
            for (int c = 0; c < 3; c++) g1[c] += g * (p1[c] - p2[c]);
            for (int c = 0; c < 3; c++) g2[c] -= (g * (p1[c] - p2[c]));
        }
        for (int j = 0; j < m; j++) {
            const float *p1 = xyz2 + ((size_t)i * m + j) * 3;
            const int j2 = idx2[(size_t)i * m + j];
            const float *p2 = xyz1 + ((size_t)i * n + j2) * 3;
            const float g = gd2[(size_t)i * m + j] * 2;
            float *g1 = gxyz2 + ((size_t)i * m + j) * 3;
            float *g2 = gxyz1 + ((size_t)i * n + j2) * 3;
            for (int c = 0; c < 3; c++) g1[c] += g * (p1[c] - p2[c]);
            for (int c = 0; c < 3; c++) g2[c] -= (g * (p1[c] - p2[c]));
        }
    }
}

/* ========================================================================= */
/* Shared numerical helpers of the registration path (restated independently */
/* in the HIP code; DESIGN.md "Numerical contract" is the spec both follow).  */
/* ========================================================================= */

/* Philox4x32-10 counter-based RNG (Salmon et al. SC'11).  The reference's    */
/* hypothesis sampler (Open3D UniformIntGenerator, RANSAC.py:43-52) is not     */
/* user-seedable; the restatement keys the stream by (seed, pair, iteration)  */
/* so every hypothesis is reproducible independent of scheduling.            */
static void philox4x32(uint32_t c[4], uint32_t k0, uint32_t k1)
{
    for (int r = 0; r < 10; r++) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        const uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
        c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
}

void oracle_philox(uint64_t seed, uint32_t pair, uint32_t itr, uint32_t block, uint32_t out[4])
{
    uint32_t c[4] = {itr, pair, 0x52414E53u, block};
    philox4x32(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    memcpy(out, c, sizeof(c));
}

/* natural log for x in (0, +inf) from + - * / only (bit-identical on CPU and */
/* GPU, unlike libm/ocml log).  x = m * 2^e, m in [sqrt(.5), sqrt(2)),         */
/* log m = 2 atanh(z), z = (m-1)/(m+1).                                       */
double oracle_det_log(double x)
{
    if (!(x > 0.0)) return (x == 0.0) ? -INFINITY : NAN;
    if (x == INFINITY) return INFINITY;
    uint64_t bits;
    memcpy(&bits, &x, 8);
    int e = (int)((bits >> 52) & 0x7ff);
    if (e == 0) { /* subnormal: scale up */
        x *= 18014398509481984.0; /* 2^54 */
        memcpy(&bits, &x, 8);
        e = (int)((bits >> 52) & 0x7ff) - 54;
    }
    e -= 1023;
    bits = (bits & 0x000fffffffffffffull) | 0x3ff0000000000000ull;
    double m;
    memcpy(&m, &bits, 8); /* m in [1, 2) */
    if (m > 1.4142135623730951) { m = m * 0.5; e += 1; }
    const double z = (m - 1.0) / (m + 1.0);
    const double z2 = z * z;
    double term = z, sum = 0.0;
    for (int k = 1; k <= 41; k += 2) { sum = sum + term / (double)k; term = term * z2; }
    const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
    return ((double)e * ln2_hi + 2.0 * sum) + (double)e * ln2_lo;
}

/* deterministic sum: 256 lane partials (lane = i mod 256, increasing i),     */
/* then a fixed halving tree.  `skip` entries (mask==0) contribute nothing.  */
#define RED_LANES 256
static double det_sum(const double *v, const unsigned char *mask, int n)
{
    double p[RED_LANES];
    for (int l = 0; l < RED_LANES; l++) p[l] = 0.0;
    for (int i = 0; i < n; i++)
        if (!mask || mask[i]) p[i % RED_LANES] = p[i % RED_LANES] + v[i];
    for (int s = RED_LANES / 2; s >= 1; s >>= 1)
        for (int l = 0; l < s; l++) p[l] = p[l] + p[l + s];
    return p[0];
}

/* ------------------------------------------------------------------------- */
/* Largest-eigenvector of a symmetric 4x4 (cyclic Jacobi, + - * / sqrt only).  */
/* Mirrored bit for bit by horn_rotation (csrc/geom.h).                       */
/* ------------------------------------------------------------------------- */
static void jacobi4_max(double A[4][4], double q[4])
{
    double V[4][4] = {{1, 0, 0, 0}, {0, 1, 0, 0}, {0, 0, 1, 0}, {0, 0, 0, 1}};
    for (int sweep = 0; sweep < 16; sweep++) {
        double off = 0.0;
        for (int p = 0; p < 3; p++)
            for (int r = p + 1; r < 4; r++) off = off + A[p][r] * A[p][r];
        /* converged: off-diagonal mass below 2^-120 of the diagonal's (a further
         * sweep moves the eigenvector by ~1e-18 relative at most) */
        double dsq = 0.0;
        for (int k = 0; k < 4; k++) dsq = dsq + A[k][k] * A[k][k];
        if (off == 0.0 || off <= 0x1p-120 * dsq) break;
        for (int p = 0; p < 3; p++) {
            for (int r = p + 1; r < 4; r++) {
                const double apr = A[p][r];
                if (apr == 0.0) continue;
                const double theta = (A[r][r] - A[p][p]) / (2.0 * apr);
                double t = 1.0 / (fabs(theta) + sqrt(theta * theta + 1.0));
                if (theta < 0.0) t = -t;
                const double c = 1.0 / sqrt(t * t + 1.0);
                const double s = t * c;
                A[p][p] = A[p][p] - t * apr;
                A[r][r] = A[r][r] + t * apr;
                A[p][r] = 0.0;
                A[r][p] = 0.0;
                for (int k = 0; k < 4; k++) {
                    if (k == p || k == r) continue;
                    const double akp = A[k][p], akr = A[k][r];
                    A[k][p] = c * akp - s * akr;
                    A[p][k] = A[k][p];
                    A[k][r] = s * akp + c * akr;
                    A[r][k] = A[k][r];
                }
                for (int k = 0; k < 4; k++) {
                    const double vkp = V[k][p], vkr = V[k][r];
                    V[k][p] = c * vkp - s * vkr;
                    V[k][r] = s * vkp + c * vkr;
                }
            }
        }
    }
    int best = 0;
    for (int k = 1; k < 4; k++)
        if (A[k][k] > A[best][best]) best = k;
    double nrm = 0.0;
    for (int k = 0; k < 4; k++) nrm = nrm + V[k][best] * V[k][best];
    nrm = sqrt(nrm);
    for (int k = 0; k < 4; k++) q[k] = V[k][best] / nrm;
}

/* Horn 1987 closed form: the proper rotation maximising sum w s'.(R t')     */
/* given S[a][b] = sum w (s-mus)_a (t-mut)_b.  Same optimum as the Umeyama / */
/* Kabsch SVD with determinant fix used by the reference (Eigen::umeyama via */
/* Open3D TransformationEstimationPointToPoint, RANSAC.py:46;                */
/* ROPNet/src/models/model_utils.py:127-133; deformationpyramid/model/       */
/* geometry.py:24-31).                                                       */
void oracle_horn_rotation(const double S[9], double R[9])
{
    const double Sxx = S[0], Sxy = S[1], Sxz = S[2];
    const double Syx = S[3], Syy = S[4], Syz = S[5];
    const double Szx = S[6], Szy = S[7], Szz = S[8];
    double N[4][4];
    N[0][0] = (Sxx + Syy) + Szz;
    N[0][1] = Syz - Szy;
    N[0][2] = Szx - Sxz;
    N[0][3] = Sxy - Syx;
    N[1][1] = (Sxx - Syy) - Szz;
    N[1][2] = Sxy + Syx;
    N[1][3] = Szx + Sxz;
    N[2][2] = (Syy - Sxx) - Szz;
    N[2][3] = Syz + Szy;
    N[3][3] = (Szz - Sxx) - Syy;
    N[1][0] = N[0][1]; N[2][0] = N[0][2]; N[3][0] = N[0][3];
    N[2][1] = N[1][2]; N[3][1] = N[1][3]; N[3][2] = N[2][3];
    double q[4];
    jacobi4_max(N, q);
    const double w = q[0], x = q[1], y = q[2], z = q[3];
    R[0] = ((w * w + x * x) - y * y) - z * z;
    R[1] = 2.0 * (x * y - w * z);
    R[2] = 2.0 * (x * z + w * y);
    R[3] = 2.0 * (x * y + w * z);
    R[4] = ((w * w - x * x) + y * y) - z * z;
    R[5] = 2.0 * (y * z - w * x);
    R[6] = 2.0 * (x * z - w * y);
    R[7] = 2.0 * (y * z + w * x);
    R[8] = ((w * w - x * x) - y * y) + z * z;
}

/* p' = R p + t, fixed order */
static inline void xform(const double T[12], const double p[3], double o[3])
{
    o[0] = ((T[0] * p[0] + T[1] * p[1]) + T[2] * p[2]) + T[3];
    o[1] = ((T[4] * p[0] + T[5] * p[1]) + T[6] * p[2]) + T[7];
    o[2] = ((T[8] * p[0] + T[9] * p[1]) + T[10] * p[2]) + T[11];
}

static inline double d2_3(const double a[3], const double b[3])
{
    const double dx = b[0] - a[0], dy = b[1] - a[1], dz = b[2] - a[2];
    return (dx * dx + dy * dy) + dz * dz;
}

/* Umeyama (no scaling) for a small correspondence set, sequential sums     */
/* (the RANSAC minimal sample; Eigen::umeyama semantics, T = [R | t]).       */
void oracle_umeyama_small(const double *src, const double *tgt, int k, double T[12])
{
    double ms[3] = {0, 0, 0}, mt[3] = {0, 0, 0};
    for (int i = 0; i < k; i++)
        for (int c = 0; c < 3; c++) { ms[c] = ms[c] + src[3 * i + c]; mt[c] = mt[c] + tgt[3 * i + c]; }
    const double one_over_n = 1.0 / (double)k; /* Eigen::umeyama: sum * (1/n) */
    for (int c = 0; c < 3; c++) { ms[c] = ms[c] * one_over_n; mt[c] = mt[c] * one_over_n; }
    double S[9] = {0};
    for (int i = 0; i < k; i++)
        for (int a = 0; a < 3; a++)
            for (int b = 0; b < 3; b++)
                S[3 * a + b] = S[3 * a + b] + (src[3 * i + a] - ms[a]) * (tgt[3 * i + b] - mt[b]);
    double R[9];
    oracle_horn_rotation(S, R);
    for (int a = 0; a < 3; a++) {
        T[4 * a + 0] = R[3 * a + 0];
        T[4 * a + 1] = R[3 * a + 1];
        T[4 * a + 2] = R[3 * a + 2];
        T[4 * a + 3] = mt[a] - ((R[3 * a + 0] * ms[0] + R[3 * a + 1] * ms[1]) + R[3 * a + 2] * ms[2]);
    }
}

/* Weighted Procrustes over many points with the deterministic reduction.    */
/* Centroid = sum(w x) / (sum(w') + eps) where w' = |w| if absw else w:       */
/*   weighted_icp: absw=0, eps=1e-8 (ROPNet model_utils.py:120-122)           */
/*   rigid_fit:    absw=1, eps=1e-4 (deformationpyramid geometry.py:20-23)    */
/* H = sum w_norm (s-mus)(t-mut)^T, R = Horn(H), t = mut - R mus.             */
void oracle_procrustes(const double *src, const double *tgt, const double *w, int n,
                       int absw, double eps, double T[12])
{
    double *tmp = (double *)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
    for (int i = 0; i < n; i++) tmp[i] = absw ? fabs(w[i]) : w[i];
    const double W = det_sum(tmp, NULL, n) + eps;
    double ms[3], mt[3];
    for (int c = 0; c < 3; c++) {
        for (int i = 0; i < n; i++) tmp[i] = src[3 * i + c] * (w[i] / W);
        ms[c] = det_sum(tmp, NULL, n);
        for (int i = 0; i < n; i++) tmp[i] = tgt[3 * i + c] * (w[i] / W);
        mt[c] = det_sum(tmp, NULL, n);
    }
    double S[9];
    for (int a = 0; a < 3; a++)
        for (int b = 0; b < 3; b++) {
            for (int i = 0; i < n; i++)
                tmp[i] = ((src[3 * i + a] - ms[a]) * (w[i] / W)) * (tgt[3 * i + b] - mt[b]);
            S[3 * a + b] = det_sum(tmp, NULL, n);
        }
    free(tmp);
    double R[9];
    oracle_horn_rotation(S, R);
    for (int a = 0; a < 3; a++) {
        T[4 * a + 0] = R[3 * a + 0];
        T[4 * a + 1] = R[3 * a + 1];
        T[4 * a + 2] = R[3 * a + 2];
        T[4 * a + 3] = mt[a] - ((R[3 * a + 0] * ms[0] + R[3 * a + 1] * ms[1]) + R[3 * a + 2] * ms[2]);
    }
}

void oracle_procrustes_batch(const float *src, const float *tgt, const float *w, int b, int n,
                             int absw, double eps, double *T /* b x 12 */)
{
    double *s = (double *)malloc(sizeof(double) * 3 * (size_t)(n ? n : 1));
    double *t = (double *)malloc(sizeof(double) * 3 * (size_t)(n ? n : 1));
    double *ww = (double *)malloc(sizeof(double) * (size_t)(n ? n : 1));
    for (int p = 0; p < b; p++) {
        for (int i = 0; i < 3 * n; i++) {
            s[i] = src[(size_t)p * n * 3 + i];
            t[i] = tgt[(size_t)p * n * 3 + i];
        }
        for (int i = 0; i < n; i++) ww[i] = w[(size_t)p * n + i];
        oracle_procrustes(s, t, ww, n, absw, eps, T + 12 * (size_t)p);
    }
    free(s); free(t); free(ww);
}

/* ------------------------------------------------------------------------- */
/* a5: exact feature-space 1-NN (Open3D KDTreeFlann SearchKNN k=1 inside     */
/* registration_ransac_based_on_feature_matching; torch.cdist+min in         */
/* c2p-net/ngenet/models/vote.py:6-9).  D_ij = sum_k (f_ik - g_jk)^2 in f64, */
/* sequential over k, no FMA; argmin, lowest index on ties.                  */
/* ------------------------------------------------------------------------- */
void oracle_featnn(const float *F, const float *G, int n, int m, int d, int32_t *nn)
{
#pragma omp parallel for schedule(static)
    for (int i = 0; i < n; i++) {
        double best = INFINITY;
        int bi = 0;
        const float *f = F + (size_t)i * d;
        for (int j = 0; j < m; j++) {
            const float *g = G + (size_t)j * d;
            double acc = 0.0;
            for (int k = 0; k < d; k++) {
                const double df = (double)f[k] - (double)g[k];
                acc = acc + df * df;
            }
            if (acc < best) { best = acc; bi = j; }
        }
        nn[i] = bi;
    }
}

/* mutual filter + fallback (Open3D 0.13 RegistrationRANSACBasedOnFeature-   */
/* Matching: keep (i, nn12[i]) iff nn21[nn12[i]] == i; if fewer than          */
/* 3*ransac_n survive, use all (i, nn12[i])).  Returns count, fills corres.  */
int oracle_corres(const int32_t *nn12, const int32_t *nn21, int n, int mutual, int ransac_n,
                  int32_t *corres /* n x 2 */)
{
    int k = 0;
    if (mutual) {
        for (int i = 0; i < n; i++)
            if (nn21[nn12[i]] == i) { corres[2 * k] = i; corres[2 * k + 1] = nn12[i]; k++; }
        if (k >= 3 * ransac_n) return k;
    }
    for (int i = 0; i < n; i++) { corres[2 * i] = i; corres[2 * i + 1] = nn12[i]; }
    return n;
}

/* ------------------------------------------------------------------------- */
/* radius-limited 1-NN (Open3D KDTreeFlann::SearchHybrid(r, 1)): nearest     */
/* target with d2 < thr (strict), thr = (double)(float)(r*r) as FLANN takes  */
/* a float radius^2; lowest index on exact ties.  Brute force + a grid       */
/* variant (cells of 2r, sorted cell keys) with identical results.           */
/* ------------------------------------------------------------------------- */
double oracle_radius_thr(double r) { return (double)(float)(r * r); }

typedef struct {
    int n;
    double cell;
    int64_t *keys;   /* sorted cell keys */
    int32_t *order;  /* point index per sorted slot */
    const double *pts;
} ogrid;

static int64_t cell_key(int64_t x, int64_t y, int64_t z)
{
    return ((x + (1ll << 20)) << 42) | ((y + (1ll << 20)) << 21) | (z + (1ll << 20));
}

static const int64_t *g_sort_keys;
static int cmp_idx(const void *a, const void *b)
{
    const int32_t ia = *(const int32_t *)a, ib = *(const int32_t *)b;
    const int64_t ka = g_sort_keys[ia], kb = g_sort_keys[ib];
    if (ka != kb) return ka < kb ? -1 : 1;
    return ia < ib ? -1 : (ia > ib);
}

static void ogrid_build(ogrid *g, const double *pts, int n, double r)
{
    g->n = n;
    g->pts = pts;
    g->cell = 2.01 * r;
    int64_t *k = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n ? n : 1));
    g->order = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n ? n : 1));
    g->keys = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n ? n : 1));
    for (int i = 0; i < n; i++) {
        k[i] = cell_key((int64_t)floor(pts[3 * i] / g->cell), (int64_t)floor(pts[3 * i + 1] / g->cell),
                        (int64_t)floor(pts[3 * i + 2] / g->cell));
        g->order[i] = i;
    }
    g_sort_keys = k;   /* single-threaded use only */
    qsort(g->order, (size_t)n, sizeof(int32_t), cmp_idx);
    for (int i = 0; i < n; i++) g->keys[i] = k[g->order[i]];
    free(k);
}

static void ogrid_free(ogrid *g) { free(g->keys); free(g->order); }

static int lower_bound64(const int64_t *a, int n, int64_t v)
{
    int lo = 0, hi = n;
    while (lo < hi) { const int mid = (lo + hi) >> 1; if (a[mid] < v) lo = mid + 1; else hi = mid; }
    return lo;
}

/* returns index or -1; *d2out = distance^2 */
static int ogrid_query(const ogrid *g, const double p[3], double r, double thr, double *d2out)
{
    const double rr = 1.001 * r;
    int64_t lo[3], hi[3];
    for (int c = 0; c < 3; c++) {
        lo[c] = (int64_t)floor((p[c] - rr) / g->cell);
        hi[c] = (int64_t)floor((p[c] + rr) / g->cell);
    }
    double best = INFINITY;
    int bi = -1;
    for (int64_t x = lo[0]; x <= hi[0]; x++)
        for (int64_t y = lo[1]; y <= hi[1]; y++)
            for (int64_t z = lo[2]; z <= hi[2]; z++) {
                const int64_t key = cell_key(x, y, z);
                for (int s = lower_bound64(g->keys, g->n, key); s < g->n && g->keys[s] == key; s++) {
                    const int j = g->order[s];
                    const double d2 = d2_3(p, g->pts + 3 * j);
                    if (d2 < thr && (d2 < best || (d2 == best && j < bi))) { best = d2; bi = j; }
                }
            }
    *d2out = best;
    return bi;
}

int oracle_radius_nn_brute(const double *tgt, int m, const double p[3], double thr, double *d2out)
{
    double best = INFINITY;
    int bi = -1;
    for (int j = 0; j < m; j++) {
        const double d2 = d2_3(p, tgt + 3 * j);
        if (d2 < thr && d2 < best) { best = d2; bi = j; }
    }
    *d2out = best;
    return bi;
}

/* batch entry used by tests: queries (q x 3 f64) against tgt (m x 3 f64)     */
void oracle_radius_nn(const double *tgt, int m, const double *q, int nq, double r,
                      int use_grid, int32_t *idx, double *d2)
{
    const double thr = oracle_radius_thr(r);
    if (use_grid) {
        ogrid g;
        ogrid_build(&g, tgt, m, r);
        for (int i = 0; i < nq; i++) idx[i] = ogrid_query(&g, q + 3 * i, r, thr, d2 + i);
        ogrid_free(&g);
    } else {
        for (int i = 0; i < nq; i++) idx[i] = oracle_radius_nn_brute(tgt, m, q + 3 * i, thr, d2 + i);
    }
}

/* fixed-point error accumulator: q = (uint64)(d2 * 2^40 / thr), summed     */
/* exactly (order-independent).  inlier_rmse = sqrt((sum / scale) / count).  */
static inline double fx_scale(double thr) { return 1099511627776.0 / thr; }

/* Evaluate T on all source points: GetRegistrationResultAndCorrespondences */
/* (Open3D registration.cpp) restated.  Returns inlier count; fitness, rmse.  */
static int evaluate(const ogrid *g, const double *src, int n, const double T[12], double r,
                    double thr, double *fitness, double *rmse, int32_t *cj /* opt n */)
{
    const double scale = fx_scale(thr);
    uint64_t acc = 0;
    int cnt = 0;
    for (int i = 0; i < n; i++) {
        double p[3], d2;
        xform(T, src + 3 * i, p);
        const int j = ogrid_query(g, p, r, thr, &d2);
        if (cj) cj[i] = j;
        if (j >= 0) { cnt++; acc += (uint64_t)(d2 * scale); }
    }
    if (cnt > 0) {
        *fitness = (double)cnt / (double)n;
        *rmse = sqrt(((double)acc / scale) / (double)cnt);
    } else { *fitness = 0.0; *rmse = 0.0; }
    return cnt;
}

/* ------------------------------------------------------------------------- */
/* a6/a7: RANSAC hypothesize-and-verify, restating Open3D 0.13               */
/* RegistrationRANSACBasedOnCorrespondence as called from                    */
/* DataPreparation/RANSAC.py:43-52 (mutual, PointToPoint(False), n=3,        */
/* EdgeLength(0.9), Distance(d), RANSACConvergenceCriteria(100000, 0.999)),  */
/* run sequentially (OMP_NUM_THREADS=1 semantics) on the Philox stream:      */
/*   for itr < max_iter while itr < est_k:                                   */
/*     sample n corres (with replacement), T = Umeyama, run checkers;        */
/*     on pass evaluate all source points; if better (fitness up, or equal   */
/*     fitness and smaller rmse): keep, w = inlier ratio over corres (d2<d*d),*/
/*     est_k = min(est_k, ceil(log(1-conf)/log(1-w^n))).                     */
/* ------------------------------------------------------------------------- */
static void sample_indices(uint64_t seed, uint32_t pair, uint32_t itr, int n, int K, int32_t *out)
{
    uint32_t w[4];
    for (int j = 0; j < n; j++) {
        if ((j & 3) == 0) oracle_philox(seed, pair, itr, (uint32_t)(j >> 2), w);
        out[j] = (int32_t)(((uint64_t)w[j & 3] * (uint64_t)K) >> 32);
    }
}

double oracle_est_k(double w, int n, double confidence)
{
    double pw = 1.0;
    for (int j = 0; j < n; j++) pw = pw * w;
    if (!(pw > 0.0)) return INFINITY;
    if (pw >= 1.0) return 0.0;
    return oracle_det_log(1.0 - confidence) / oracle_det_log(1.0 - pw);
}

static void to_double3(const float *src, int n, double *dst)
{
    for (int i = 0; i < 3 * n; i++) dst[i] = (double)src[i];
}

typedef struct {
    double T[12];
    double fitness, rmse;
    int32_t iters;       /* iterations consumed (loop exit itr) */
    int32_t validated;   /* hypotheses that passed the checkers */
    int32_t best_itr;
} ransac_out;

static int ransac_core(const double *S, int n, const double *Tg, int m, const ogrid *g,
                       const int32_t *corres, int K, double d, int rn, double edge_ratio,
                       double dist_check, int max_iter, double conf, uint64_t seed,
                       uint32_t pair, ransac_out *o)
{
    const double thr = oracle_radius_thr(d);
    const double dd = d * d;
    double bestT[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
    double bfit = 0.0, brmse = 0.0;
    int est_k = max_iter, itr, validated = 0, best_itr = -1;
    int32_t samp[64];
    double ss[3 * 64], tt[3 * 64];
    for (itr = 0; itr < max_iter; itr++) {
        if (itr >= est_k) break;
        sample_indices(seed, pair, (uint32_t)itr, rn, K, samp);
        for (int j = 0; j < rn; j++) {
            const int c = samp[j];
            for (int a = 0; a < 3; a++) {
                ss[3 * j + a] = S[3 * corres[2 * c] + a];
                tt[3 * j + a] = Tg[3 * corres[2 * c + 1] + a];
            }
        }
        double T[12];
        oracle_umeyama_small(ss, tt, rn, T);
        int ok = 1;
        if (edge_ratio > 0.0) {
            for (int i = 0; i < rn && ok; i++)
                for (int j = i + 1; j < rn && ok; j++) {
                    const double ds = sqrt(d2_3(ss + 3 * i, ss + 3 * j));
                    const double dt = sqrt(d2_3(tt + 3 * i, tt + 3 * j));
                    if (ds < dt * edge_ratio || dt < ds * edge_ratio) ok = 0;
                }
        }
        if (ok && dist_check > 0.0) {
            for (int j = 0; j < rn && ok; j++) {
                double p[3];
                xform(T, ss + 3 * j, p);
                if (sqrt(d2_3(p, tt + 3 * j)) > dist_check) ok = 0;
            }
        }
        if (!ok) continue;
        validated++;
        double fit, rmse;
        evaluate(g, S, n, T, d, thr, &fit, &rmse, NULL);
        if (fit > bfit || (fit == bfit && rmse < brmse)) {
            bfit = fit; brmse = rmse; best_itr = itr;
            memcpy(bestT, T, sizeof(bestT));
            int cin = 0;
            for (int k = 0; k < K; k++) {
                double p[3];
                xform(T, S + 3 * corres[2 * k], p);
                if (d2_3(p, Tg + 3 * corres[2 * k + 1]) < dd) cin++;
            }
            const double kd = oracle_est_k((double)cin / (double)K, rn, conf);
            if (kd < (double)est_k) est_k = (int)ceil(kd);
        }
    }
    memcpy(o->T, bestT, sizeof(bestT));
    o->fitness = bfit; o->rmse = brmse; o->iters = itr; o->validated = validated;
    o->best_itr = best_itr;
    return best_itr >= 0;
}

static void t12_to_16(const double *T, double *M)
{
    for (int a = 0; a < 3; a++)
        for (int b = 0; b < 4; b++) M[4 * a + b] = T[4 * a + b];
    M[12] = 0; M[13] = 0; M[14] = 0; M[15] = 1;
}

/* returns number of correspondences of the best T (written to corr_out,   */
/* increasing source index, if non-NULL); stats[4] = {iters, validated,     */
/* best_itr, status(1 ok / 0 no result / -1 invalid input)}                 */
int oracle_ransac(const float *srcf, int n, const float *tgtf, int m, const int32_t *corres,
                  int K, double d, int rn, double edge_ratio, double dist_check, int max_iter,
                  double conf, uint64_t seed, uint32_t pair, double *T16, double *fit_rmse,
                  int32_t *corr_out, int32_t *stats)
{
    double I[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
    t12_to_16(I, T16);
    fit_rmse[0] = 0.0; fit_rmse[1] = 0.0;
    stats[0] = stats[1] = 0; stats[2] = -1; stats[3] = -1;
    if (rn < 3 || rn > 64 || K < rn || !(d > 0.0) || n <= 0 || m <= 0) return 0;
    double *S = (double *)malloc(sizeof(double) * 3 * (size_t)n);
    double *Tg = (double *)malloc(sizeof(double) * 3 * (size_t)m);
    to_double3(srcf, n, S);
    to_double3(tgtf, m, Tg);
    ogrid g;
    ogrid_build(&g, Tg, m, d);
    ransac_out o;
    const int found = ransac_core(S, n, Tg, m, &g, corres, K, d, rn, edge_ratio, dist_check,
                                  max_iter, conf, seed, pair, &o);
    t12_to_16(o.T, T16);
    fit_rmse[0] = o.fitness; fit_rmse[1] = o.rmse;
    stats[0] = o.iters; stats[1] = o.validated; stats[2] = o.best_itr; stats[3] = found;
    int nc = 0;
    if (found) {
        const double thr = oracle_radius_thr(d);
        for (int i = 0; i < n; i++) {
            double p[3], d2;
            xform(o.T, S + 3 * i, p);
            const int j = ogrid_query(&g, p, d, thr, &d2);
            if (j >= 0) {
                if (corr_out) { corr_out[2 * nc] = i; corr_out[2 * nc + 1] = j; }
                nc++;
            }
        }
    }
    ogrid_free(&g);
    free(S); free(Tg);
    return nc;
}

/* ------------------------------------------------------------------------- */
/* a8: point-to-point ICP, restating Open3D 0.13 RegistrationICP as called   */
/* from DataPreparation/RANSAC.py:61-63 (ICPConvergenceCriteria defaults:   */
/* 1e-6, 1e-6, 30).  Correspondences: radius-limited 1-NN; update = Umeyama  */
/* over all correspondences (1024 f64 lane partials, lane = source index    */
/* mod 1024, added exactly: xs_*); T <- update*T; points transformed in     */
/* place (f64).                                                             */
/* ------------------------------------------------------------------------- */
static void mat4_mul(const double A[16], const double B[16], double C[16])
{
    for (int a = 0; a < 4; a++)
        for (int b = 0; b < 4; b++)
            C[4 * a + b] = ((A[4 * a + 0] * B[b] + A[4 * a + 1] * B[4 + b]) + A[4 * a + 2] * B[8 + b]) +
                           A[4 * a + 3] * B[12 + b];
}

static int is_identity16(const double T[16])
{
    for (int a = 0; a < 4; a++)
        for (int b = 0; b < 4; b++)
            if (T[4 * a + b] != (a == b ? 1.0 : 0.0)) return 0;
    return 1;
}

/* Exact, order-independent sums (the ICP Umeyama step adds its 1024 lane    */
/* partials with them).  Every term (an f64 value)                           */
/* is taken to a signed 128-bit fixed-point integer with LSB 2^-80           */
/* (truncated toward zero below it; |term| saturates at 2^47), the integers  */
/* are added (associative: any split over lanes, waves or workgroups gives   */
/* the same total), and the total is rounded once to the nearest f64 (ties   */
/* to even).  The GPU kernel (csrc/xsum.h) does the same arithmetic, so ICP  */
/* results do not depend on how a pair's lanes are spread over workgroups.  */
typedef __int128 xs_t;
#define XS_FRAC 80

static xs_t xs_term(double x)
{
    uint64_t b;
    memcpy(&b, &x, 8);
    const int e = (int)((b >> 52) & 0x7ff);
    if (e == 0x7ff) return 0;                       /* non-finite: contributes 0 */
    const uint64_t f = b & 0x000fffffffffffffull;
    const uint64_t mant = e ? (f | 0x0010000000000000ull) : f;
    int s = (e ? e : 1) - 1075 + XS_FRAC;           /* value = mant * 2^(s - 80) */
    unsigned __int128 M = mant;
    if (s >= 0) {
        if (s > 74) { M = ((unsigned __int128)1 << 127) - 1; }   /* saturate */
        else M <<= s;
    } else {
        M = (-s >= 64) ? 0 : (M >> (-s));
    }
    const xs_t v = (xs_t)M;
    return (b >> 63) ? -v : v;
}

static double xs_to_double(xs_t v)
{
    const int neg = v < 0;
    unsigned __int128 u = neg ? (unsigned __int128)(-(v + 1)) + 1u : (unsigned __int128)v;
    if (u == 0) return 0.0;
    const uint64_t hi = (uint64_t)(u >> 64), lo = (uint64_t)u;
    const int msb = hi ? 127 - __builtin_clzll(hi) : 63 - __builtin_clzll(lo);
    uint64_t m;
    int sh = 0;
    if (msb <= 52) {
        m = (uint64_t)u;
    } else {
        sh = msb - 52;
        m = (uint64_t)(u >> sh);
        const unsigned __int128 rem = u & (((unsigned __int128)1 << sh) - 1u);
        const unsigned __int128 half = (unsigned __int128)1 << (sh - 1);
        if (rem > half || (rem == half && (m & 1u))) {
            m += 1u;
            if (m == (1ull << 53)) { m >>= 1; sh += 1; }
        }
    }
    /* m * 2^(sh - 80): m < 2^53 is exact in f64, the power of two is exact */
    const int k = sh - XS_FRAC;
    uint64_t pb = (uint64_t)(k + 1023) << 52;
    double p2;
    memcpy(&p2, &pb, 8);
    const double r = (double)m * p2;
    return neg ? -r : r;
}

double oracle_xs_sum(const double *v, int n)
{
    xs_t a = 0;
    for (int i = 0; i < n; i++) a += xs_term(v[i]);
    return xs_to_double(a);
}

/* Umeyama over the correspondences of an ICP iteration (round 3), one pass of   */
/* EXACT sums.  Per pair: a reference point c0 = the first target point and a   */
/* quantum 2^-k with k = 52 - e_n - e_max, where every inlier term below is at   */
/* most 2^e_max in magnitude (|s - c0|, |t - c0| <= B = max_j |t_j - c0|_inf +   */
/* 2d, since an inlier lies within d of its target; e_max = max(e_B, 2 e_B),     */
/* B < 2^e_B) and n <= 2^e_n.  Each term -- s' = s - c0, t' = t - c0 and the 9  */
/* products s'_a t'_b, all in f64 -- is truncated to a multiple of 2^-k; any    */
/* partial sum of them is then an integer multiple of 2^-k below 2^52 * 2^-k, so */
/* every f64 addition is exact and the sums do not depend on the order (the GPU  */
/* adds them in any split over threads, waves and workgroups).  Then            */
/*   ms' = Ss * (1/K), mt' = St * (1/K), C_ab = Sst_ab - ms'_a * St_b,          */
/*   ms = ms' + c0, mt = mt' + c0, R = Horn(C), t = mt - R ms.                  */
double oracle_icp_quantum(const double *Tg, int m, int n, double d, double c0[3])
{
    c0[0] = Tg[0]; c0[1] = Tg[1]; c0[2] = Tg[2];
    double bt = 0.0;
    for (int j = 0; j < m; j++)
        for (int a = 0; a < 3; a++) {
            const double v = fabs(Tg[3 * j + a] - c0[a]);
            if (v > bt) bt = v;
        }
    const double B = bt + 2.0 * d;
    int eb = 0;
    frexp(B, &eb);                        /* B < 2^eb */
    const int emax = eb > 2 * eb ? eb : 2 * eb;
    int en = 0;
    while ((1LL << en) < (long long)(n > 1 ? n : 1)) en++;
    int k = 52 - en - emax;
    if (k > 200) k = 200;
    if (k < -200) k = -200;
    return ldexp(1.0, k);                 /* 2^k */
}

static inline double icp_q(double x, double sk, double isk) { return trunc(x * sk) * isk; }

static void umeyama_masked(const double *P, const double *Tg, const int32_t *cj, int n,
                           const double c0[3], double sk, double T[12])
{
    const double isk = 1.0 / sk;  /* exact: a power of two */
    double Ss[3] = {0, 0, 0}, St[3] = {0, 0, 0}, Sst[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    int K = 0;
    for (int i = 0; i < n; i++) {
        if (cj[i] < 0) continue;
        K++;
        const double *p = P + 3 * i, *t = Tg + 3 * cj[i];
        double sp[3], tp[3];
        for (int a = 0; a < 3; a++) { sp[a] = p[a] - c0[a]; tp[a] = t[a] - c0[a]; }
        for (int a = 0; a < 3; a++) {
            Ss[a] = Ss[a] + icp_q(sp[a], sk, isk);
            St[a] = St[a] + icp_q(tp[a], sk, isk);
            for (int b = 0; b < 3; b++) Sst[3 * a + b] = Sst[3 * a + b] + icp_q(sp[a] * tp[b], sk, isk);
        }
    }
    const double one_over_n = 1.0 / (double)K;
    double ms[3], mt[3], msp[3], S[9];
    for (int c = 0; c < 3; c++) {
        msp[c] = Ss[c] * one_over_n;
        ms[c] = msp[c] + c0[c];
        mt[c] = St[c] * one_over_n + c0[c];
    }
    for (int a = 0; a < 3; a++)
        for (int b = 0; b < 3; b++) S[3 * a + b] = Sst[3 * a + b] - msp[a] * St[b];
    double R[9];
    oracle_horn_rotation(S, R);
    for (int a = 0; a < 3; a++) {
        T[4 * a + 0] = R[3 * a + 0];
        T[4 * a + 1] = R[3 * a + 1];
        T[4 * a + 2] = R[3 * a + 2];
        T[4 * a + 3] = mt[a] - ((R[3 * a + 0] * ms[0] + R[3 * a + 1] * ms[1]) + R[3 * a + 2] * ms[2]);
    }
}

/* returns #correspondences of the final result; out: T16, fit_rmse[2], iters. */
/* Trace (test infrastructure, may be NULL): for every iteration it the       */
/* working copy the estimate saw (P_tr[it*3n]) and its correspondences        */
/* (cj_tr[it*n], -1 = none), so an independent estimator can be run on the    */
/* very sets this loop estimated from.                                       */
static int icp_core(const float *srcf, int n, const float *tgtf, int m, const double *init16,
                    double d, int max_iter, double rel_fit, double rel_rmse, double *T16,
                    double *fit_rmse, int32_t *iters, double *P_tr, int32_t *cj_tr);

int oracle_icp(const float *srcf, int n, const float *tgtf, int m, const double *init16, double d,
               int max_iter, double rel_fit, double rel_rmse, double *T16, double *fit_rmse,
               int32_t *iters)
{
    return icp_core(srcf, n, tgtf, m, init16, d, max_iter, rel_fit, rel_rmse, T16, fit_rmse, iters,
                    NULL, NULL);
}

int oracle_icp_trace(const float *srcf, int n, const float *tgtf, int m, const double *init16,
                     double d, int max_iter, double rel_fit, double rel_rmse, double *T16,
                     double *fit_rmse, int32_t *iters, double *P_tr, int32_t *cj_tr)
{
    return icp_core(srcf, n, tgtf, m, init16, d, max_iter, rel_fit, rel_rmse, T16, fit_rmse, iters,
                    P_tr, cj_tr);
}

static int icp_core(const float *srcf, int n, const float *tgtf, int m, const double *init16,
                    double d, int max_iter, double rel_fit, double rel_rmse, double *T16,
                    double *fit_rmse, int32_t *iters, double *P_tr, int32_t *cj_tr)
{
    memcpy(T16, init16, sizeof(double) * 16);
    fit_rmse[0] = fit_rmse[1] = 0.0;
    *iters = 0;
    if (!(d > 0.0) || n <= 0 || m <= 0) return 0;
    double *P = (double *)malloc(sizeof(double) * 3 * (size_t)n);
    double *Tg = (double *)malloc(sizeof(double) * 3 * (size_t)m);
    int32_t *cj = (int32_t *)malloc(sizeof(int32_t) * (size_t)n);
    to_double3(srcf, n, P);
    to_double3(tgtf, m, Tg);
    const double thr = oracle_radius_thr(d);
    ogrid g;
    ogrid_build(&g, Tg, m, d);
    double T[16];
    memcpy(T, init16, sizeof(T));
    const double I12[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
    if (!is_identity16(T)) {
        double T12[12];
        for (int k = 0; k < 12; k++) T12[k] = T[k];
        for (int i = 0; i < n; i++) { double p[3]; xform(T12, P + 3 * i, p); memcpy(P + 3 * i, p, sizeof(p)); }
    }
    double fit, rmse, c0[3];
    const double sk = oracle_icp_quantum(Tg, m, n, d, c0);
    int cnt = evaluate(&g, P, n, I12, d, thr, &fit, &rmse, cj);
    int it;
    for (it = 0; it < max_iter; it++) {
        if (cnt == 0) break; /* Umeyama on an empty set is undefined in Eigen; stop */
        double U[12], U16[16], Tn[16];
        if (P_tr) memcpy(P_tr + (size_t)it * 3 * n, P, sizeof(double) * 3 * (size_t)n);
        if (cj_tr) memcpy(cj_tr + (size_t)it * n, cj, sizeof(int32_t) * (size_t)n);
        umeyama_masked(P, Tg, cj, n, c0, sk, U);
        t12_to_16(U, U16);
        mat4_mul(U16, T, Tn);
        memcpy(T, Tn, sizeof(T));
        for (int i = 0; i < n; i++) { double p[3]; xform(U, P + 3 * i, p); memcpy(P + 3 * i, p, sizeof(p)); }
        const double pf = fit, pr = rmse;
        cnt = evaluate(&g, P, n, I12, d, thr, &fit, &rmse, cj);
        if (fabs(pf - fit) < rel_fit && fabs(pr - rmse) < rel_rmse) { it++; break; }
    }
    memcpy(T16, T, sizeof(T));
    fit_rmse[0] = fit; fit_rmse[1] = rmse;
    *iters = it;
    ogrid_free(&g);
    free(P); free(Tg); free(cj);
    return cnt;
}

/* ------------------------------------------------------------------------- */
/* a4: DIP local reference frame, dip/lrf.py:19-78 (lrf.get).                 */
/*  - radius neighbours of pt: d2 = ((dx^2 + dy^2) + dz^2) < (double)(float)   */
/*    (r*r) (Open3D KDTreeFlann::SearchRadius passes float(r*r) to FLANN,     */
/*    strict <), sorted by (d2, index) (:21);                                  */
/*  - ptnn = all but the first (:23); cov = 1/len(ptnn) * A A^T where          */
/*    len(ptnn) == 3 (the array is 3 x k) (:27);                               */
/*  - np_hat = eigenvector of the smallest eigenvalue (:33-35), here cyclic    */
/*    Jacobi (first index on ties), normalised;                                */
/*  - zp sign (:38), xp from the alpha*beta weighted projections (:40-46),     */
/*    yp = xp x zp (:48), T = [[xp yp zp | pt]] (:50-61; det = -1);            */
/*  - patch rows lRg^T (p - pt) / kernel over ptall (incl. the first), zero    */
/*    padded to patch_size, rows picked by the caller's inds (:53-76; the      */
/*    np.random.choice draw stays with the caller).                            */
/* Sums use det_sum's 256-lane order so the GPU kernel matches bit for bit.   */
/* ------------------------------------------------------------------------- */
typedef struct { double d2; int idx; } lrf_hit;

static int cmp_hit(const void *a, const void *b)
{
    const lrf_hit *x = (const lrf_hit *)a, *y = (const lrf_hit *)b;
    if (x->d2 < y->d2) return -1;
    if (x->d2 > y->d2) return 1;
    return (x->idx > y->idx) - (x->idx < y->idx);
}

static void sym3_smallest(const double C[6], double v[3])
{
    /* C = xx xy xz yy yz zz; cyclic Jacobi, + - * / sqrt only */
    double A[3][3] = {{C[0], C[1], C[2]}, {C[1], C[3], C[4]}, {C[2], C[4], C[5]}};
    double V[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
    for (int sweep = 0; sweep < 32; sweep++) {
        const double off = (A[0][1] * A[0][1] + A[0][2] * A[0][2]) + A[1][2] * A[1][2];
        if (off == 0.0) break;
        for (int p = 0; p < 2; p++)
            for (int r = p + 1; r < 3; r++) {
                const double apr = A[p][r];
                if (apr == 0.0) continue;
                const double theta = (A[r][r] - A[p][p]) / (2.0 * apr);
                double t = 1.0 / (fabs(theta) + sqrt(theta * theta + 1.0));
                if (theta < 0.0) t = -t;
                const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
                A[p][p] = A[p][p] - t * apr;
                A[r][r] = A[r][r] + t * apr;
                A[p][r] = 0.0;
                A[r][p] = 0.0;
                for (int k = 0; k < 3; k++) {
                    if (k == p || k == r) continue;
                    const double akp = A[k][p], akr = A[k][r];
                    A[k][p] = c * akp - s * akr;
                    A[p][k] = A[k][p];
                    A[k][r] = s * akp + c * akr;
                    A[r][k] = A[k][r];
                }
                for (int k = 0; k < 3; k++) {
                    const double vkp = V[k][p], vkr = V[k][r];
                    V[k][p] = c * vkp - s * vkr;
                    V[k][r] = s * vkp + c * vkr;
                }
            }
    }
    int m = 0;
    for (int k = 1; k < 3; k++)
        if (A[k][k] < A[m][m]) m = k;
    const double n = sqrt((V[0][m] * V[0][m] + V[1][m] * V[1][m]) + V[2][m] * V[2][m]);
    for (int k = 0; k < 3; k++) v[k] = V[k][m] / n;
}

static int lrf_hits(const double *pts, int n, const double q[3], double kernel, lrf_hit *h)
{
    const double thr = (double)(float)(kernel * kernel);
    int k = 0;
    for (int i = 0; i < n; i++) {
        const double dx = pts[3 * i] - q[0], dy = pts[3 * i + 1] - q[1], dz = pts[3 * i + 2] - q[2];
        const double d2 = (dx * dx + dy * dy) + dz * dz;
        if (d2 < thr) { if (h) { h[k].d2 = d2; h[k].idx = i; } k++; }
    }
    return k;
}

int oracle_lrf_count(const double *pts, int n, const double q[3], double kernel)
{
    return lrf_hits(pts, n, q, kernel, NULL);
}

/* returns k; fills T (16, row-major 4x4) and patch (patch_size x 3) */
int oracle_lrf(const double *pts, int n, const double q[3], double kernel, int patch_size,
               const int32_t *inds, double *patch, double *T)
{
    lrf_hit *h = (lrf_hit *)malloc(sizeof(lrf_hit) * (size_t)(n > 0 ? n : 1));
    const int k = lrf_hits(pts, n, q, kernel, h);
    qsort(h, (size_t)k, sizeof(lrf_hit), cmp_hit);
    const int kn = k > 0 ? k - 1 : 0; /* ptnn = hits[1:] */
    double *v = (double *)malloc(sizeof(double) * (size_t)(kn > 0 ? kn : 1));
    double C[6];
    const int ca[6] = {0, 0, 0, 1, 1, 2}, cb[6] = {0, 1, 2, 1, 2, 2};
    for (int e = 0; e < 6; e++) {
        for (int i = 0; i < kn; i++) {
            const double *p = pts + 3 * h[i + 1].idx;
            v[i] = (p[ca[e]] - q[ca[e]]) * (p[cb[e]] - q[cb[e]]);
        }
        C[e] = (1.0 / 3.0) * det_sum(v, NULL, kn);
    }
    double nh[3];
    sym3_smallest(C, nh);
    for (int i = 0; i < kn; i++) {
        const double *p = pts + 3 * h[i + 1].idx;
        v[i] = (nh[0] * (q[0] - p[0]) + nh[1] * (q[1] - p[1])) + nh[2] * (q[2] - p[2]);
    }
    const double zs = det_sum(v, NULL, kn);
    double zp[3];
    for (int c = 0; c < 3; c++) zp[c] = zs > 0.0 ? nh[c] : -nh[c];
    double xs[3];
    for (int c = 0; c < 3; c++) {
        for (int i = 0; i < kn; i++) {
            const double *p = pts + 3 * h[i + 1].idx;
            const double dx = p[0] - q[0], dy = p[1] - q[1], dz = p[2] - q[2];
            const double proj = (dx * zp[0] + dy * zp[1]) + dz * zp[2];
            const double dc = c == 0 ? dx : (c == 1 ? dy : dz);
            const double vc = dc - proj * zp[c];
            const double ex = q[0] - p[0], ey = q[1] - p[1], ez = q[2] - p[2];
            const double nr = sqrt((ex * ex + ey * ey) + ez * ez);
            const double al = (kernel - nr) * (kernel - nr);
            const double be = proj * proj;
            v[i] = vc * (al * be);
        }
        xs[c] = det_sum(v, NULL, kn);
    }
    const double xn = 1.0 / sqrt((xs[0] * xs[0] + xs[1] * xs[1]) + xs[2] * xs[2]);
    double xp[3], yp[3];
    for (int c = 0; c < 3; c++) xp[c] = xn * xs[c];
    yp[0] = xp[1] * zp[2] - xp[2] * zp[1];
    yp[1] = xp[2] * zp[0] - xp[0] * zp[2];
    yp[2] = xp[0] * zp[1] - xp[1] * zp[0];
    for (int a = 0; a < 3; a++) {
        T[4 * a + 0] = xp[a];
        T[4 * a + 1] = yp[a];
        T[4 * a + 2] = zp[a];
        T[4 * a + 3] = q[a];
    }
    T[12] = 0.0; T[13] = 0.0; T[14] = 0.0; T[15] = 1.0;
    for (int i = 0; i < patch_size; i++) {
        const int s = inds[i];
        if (s < 0 || s >= k) { patch[3 * i] = 0.0; patch[3 * i + 1] = 0.0; patch[3 * i + 2] = 0.0; continue; }
        const double *p = pts + 3 * h[s].idx;
        const double dx = p[0] - q[0], dy = p[1] - q[1], dz = p[2] - q[2];
        patch[3 * i + 0] = ((xp[0] * dx + xp[1] * dy) + xp[2] * dz) / kernel;
        patch[3 * i + 1] = ((yp[0] * dx + yp[1] * dy) + yp[2] * dz) / kernel;
        patch[3 * i + 2] = ((zp[0] * dx + zp[1] * dy) + zp[2] * dz) / kernel;
    }
    free(v);
    free(h);
    return k;
}

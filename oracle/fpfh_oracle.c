/*
 * fpfh_oracle.c -- CPU restatement of SURVEY 8(f) row f1: normal estimation and
 * FPFH features, as DataPreparation/RANSAC.py:12-22 calls them:
 *     pcd.estimate_normals(KDTreeSearchParamHybrid(radius=4*voxel, max_nn=30))
 *     compute_fpfh_feature(pcd, KDTreeSearchParamHybrid(radius=7*voxel, max_nn=100))
 * TEST INFRASTRUCTURE ONLY (the checker of libpcr's fpfh.hip; never linked by
 * the product).
 *
 * The algorithm lives in Open3D (0.13.0 pinned, DataPreparation/requirements.txt:1),
 * which is absent from this image and not vendored.  What follows restates its
 * published algorithm (geometry/EstimateNormals.cpp, pipelines/registration/
 * Feature.cpp, geometry/KDTreeFlann.cpp of v0.13), recalled, NOT verified against
 * Open3D itself: PARITY VS THE REFERENCE IS UNPINNED for this row.  It is pinned
 * instead by known-answer properties (exact normals of planes and spheres, each
 * FPFH 11-bin group summing to 200, rigid-motion invariance) in
 * tests/test_oracle_fpfh.py, and the GPU kernels are tested bit-exact against it.
 *
 * Choices where Open3D's behaviour is implementation-defined:
 *   - SearchHybrid(r, max_nn) = the max_nn nearest points with d2 < (double)(float)(r*r)
 *     (FLANN takes a float radius^2, KNNRadiusResultSet rejects d >= worst), ordered
 *     by (d2, index): FLANN's order among equal distances is its tree-visit order;
 *   - d2 = (dx*dx + dy*dy) + dz*dz in f64 from the f32 coordinates (FLANN L2<double>);
 *   - acos / cos / atan2 are the det_* functions below (+ - * / sqrt only), so the
 *     GPU reproduces them bit for bit; they are within a few ulp of libm
 *     (tests/test_oracle_fpfh.py), which moves a histogram bin only for a pair
 *     feature within ulps of a bin edge.
 * Compiled -O2 -ffp-contract=off: every operation rounded in the order written.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define DPI 3.14159265358979311600   /* M_PI */
#define DPI_2 1.57079632679489655800
#define DPI_4 0.78539816339744827900
#define DPI_6 0.52359877559829892668
#define DSQRT3 1.73205080756887719318
#define DTAN_PI_12 0.26794919243112269546

/* ---- deterministic elementary functions (the GPU runs the same operations) -- */

/* atan on [0, 1]: one reduction by pi/6 above tan(pi/12), then the odd Taylor
 * series to t^29 in Horner form (|t| <= 0.268: truncation < 1e-18). */
static double det_atan_unit(double t)
{
    double off = 0.0;
    if (t > DTAN_PI_12) {
        t = (t * DSQRT3 - 1.0) / (t + DSQRT3);
        off = DPI_6;
    }
    const double t2 = t * t;
    double s = 1.0 / 29.0;
    for (int k = 13; k >= 0; k--) s = ((k & 1) ? -1.0 : 1.0) / (double)(2 * k + 1) + t2 * s;
    return off + t * s;
}

double oracle_det_atan2(double y, double x)
{
    const double ax = fabs(x), ay = fabs(y);
    double a;
    if (ax == 0.0 && ay == 0.0)
        a = signbit(x) ? DPI : 0.0;
    else {
        if (ay <= ax)
            a = det_atan_unit(ay / ax);
        else
            a = DPI_2 - det_atan_unit(ax / ay);
        if (signbit(x)) a = DPI - a;
    }
    return signbit(y) ? -a : a;
}

/* acos(x) = 2 atan2(sqrt(1 - x), sqrt(1 + x)); NaN outside [-1, 1] like libm */
double oracle_det_acos(double x)
{
    return 2.0 * oracle_det_atan2(sqrt(1.0 - x), sqrt(1.0 + x));
}

/* |x| <= pi/4, nested Taylor forms to x^20 (truncation < 1e-23) */
static double det_cos_poly(double x)
{
    const double x2 = x * x;
    double s = 1.0;
    for (int k = 10; k >= 1; k--) s = 1.0 - x2 / (double)((2 * k - 1) * (2 * k)) * s;
    return s;
}

static double det_sin_poly(double x)
{
    const double x2 = x * x;
    double s = 1.0;
    for (int k = 10; k >= 1; k--) s = 1.0 - x2 / (double)((2 * k) * (2 * k + 1)) * s;
    return x * s;
}

/* cos on [0, pi] (FastEigen3x3's angles); NaN in, NaN out */
double oracle_det_cos(double x)
{
    double sg = 1.0;
    if (x > DPI_2) {
        x = DPI - x;
        sg = -1.0;
    }
    if (x > DPI_4) return sg * det_sin_poly(DPI_2 - x);
    return sg * det_cos_poly(x);
}

/* ---- hybrid radius / max_nn search -------------------------------------- */

typedef struct { double d2; int idx; } nbr_t;

static int cmp_nbr(const void *a, const void *b)
{
    const nbr_t *x = (const nbr_t *)a, *y = (const nbr_t *)b;
    if (x->d2 < y->d2) return -1;
    if (x->d2 > y->d2) return 1;
    return (x->idx > y->idx) - (x->idx < y->idx);
}

/* KDTreeFlann::SearchHybrid(points[i], r, max_nn) for every point of the cloud:
 * idx/d2 (n, max_nn) row-major, cnt (n). */
void oracle_hybrid_search(const float *pts, int n, double r, int max_nn, int32_t *idx, double *d2,
                          int32_t *cnt)
{
    const double thr = (double)(float)(r * r);
    nbr_t *h = (nbr_t *)malloc(sizeof(nbr_t) * (n > 0 ? n : 1));
    for (int i = 0; i < n; i++) {
        const double qx = pts[3 * i], qy = pts[3 * i + 1], qz = pts[3 * i + 2];
        int k = 0;
        for (int j = 0; j < n; j++) {
            const double dx = qx - (double)pts[3 * j], dy = qy - (double)pts[3 * j + 1],
                         dz = qz - (double)pts[3 * j + 2];
            const double d = (dx * dx + dy * dy) + dz * dz;
            if (d < thr) { h[k].d2 = d; h[k].idx = j; k++; }
        }
        qsort(h, k, sizeof(nbr_t), cmp_nbr);
        if (k > max_nn) k = max_nn;
        cnt[i] = k;
        for (int t = 0; t < max_nn; t++) {
            idx[(size_t)i * max_nn + t] = t < k ? h[t].idx : -1;
            d2[(size_t)i * max_nn + t] = t < k ? h[t].d2 : 0.0;
        }
    }
    free(h);
}

/* ---- normals (EstimateNormals.cpp: ComputeCovariance + FastEigen3x3) ------ */

static void cross3(const double a[3], const double b[3], double o[3])
{
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}

static double dot3(const double a[3], const double b[3])
{
    return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2];
}

/* A row-major 3x3 symmetric */
static void eigvec0(const double A[9], double ev, double o[3])
{
    const double r0[3] = {A[0] - ev, A[1], A[2]};
    const double r1[3] = {A[1], A[4] - ev, A[5]};
    const double r2[3] = {A[2], A[5], A[8] - ev};
    double c01[3], c02[3], c12[3];
    cross3(r0, r1, c01);
    cross3(r0, r2, c02);
    cross3(r1, r2, c12);
    const double d0 = dot3(c01, c01), d1 = dot3(c02, c02), d2 = dot3(c12, c12);
    double dmax = d0;
    int imax = 0;
    if (d1 > dmax) { dmax = d1; imax = 1; }
    if (d2 > dmax) imax = 2;
    const double *c = imax == 0 ? c01 : (imax == 1 ? c02 : c12);
    const double s = sqrt(imax == 0 ? d0 : (imax == 1 ? d1 : d2));
    for (int k = 0; k < 3; k++) o[k] = c[k] / s;
}

static void eigvec1(const double A[9], const double e0[3], double ev, double o[3])
{
    double U[3], V[3];
    if (fabs(e0[0]) > fabs(e0[1])) {
        const double il = 1.0 / sqrt(e0[0] * e0[0] + e0[2] * e0[2]);
        U[0] = -e0[2] * il; U[1] = 0.0; U[2] = e0[0] * il;
    } else {
        const double il = 1.0 / sqrt(e0[1] * e0[1] + e0[2] * e0[2]);
        U[0] = 0.0; U[1] = e0[2] * il; U[2] = -e0[1] * il;
    }
    cross3(e0, U, V);
    const double AU[3] = {(A[0] * U[0] + A[1] * U[1]) + A[2] * U[2],
                          (A[1] * U[0] + A[4] * U[1]) + A[5] * U[2],
                          (A[2] * U[0] + A[5] * U[1]) + A[8] * U[2]};
    const double AV[3] = {(A[0] * V[0] + A[1] * V[1]) + A[2] * V[2],
                          (A[1] * V[0] + A[4] * V[1]) + A[5] * V[2],
                          (A[2] * V[0] + A[5] * V[1]) + A[8] * V[2]};
    double m00 = ((U[0] * AU[0] + U[1] * AU[1]) + U[2] * AU[2]) - ev;
    double m01 = (U[0] * AV[0] + U[1] * AV[1]) + U[2] * AV[2];
    double m11 = ((V[0] * AV[0] + V[1] * AV[1]) + V[2] * AV[2]) - ev;
    const double a00 = fabs(m00), a01 = fabs(m01), a11 = fabs(m11);
    if (a00 >= a11) {
        const double mx = a00 > a01 ? a00 : a01;
        if (mx > 0) {
            if (a00 >= a01) { m01 /= m00; m00 = 1.0 / sqrt(1.0 + m01 * m01); m01 *= m00; }
            else { m00 /= m01; m01 = 1.0 / sqrt(1.0 + m00 * m00); m00 *= m01; }
            for (int k = 0; k < 3; k++) o[k] = m01 * U[k] - m00 * V[k];
        } else
            for (int k = 0; k < 3; k++) o[k] = U[k];
    } else {
        const double mx = a11 > a01 ? a11 : a01;
        if (mx > 0) {
            if (a11 >= a01) { m01 /= m11; m11 = 1.0 / sqrt(1.0 + m01 * m01); m01 *= m11; }
            else { m11 /= m01; m01 = 1.0 / sqrt(1.0 + m11 * m11); m11 *= m01; }
            for (int k = 0; k < 3; k++) o[k] = m11 * U[k] - m01 * V[k];
        } else
            for (int k = 0; k < 3; k++) o[k] = U[k];
    }
}

/* FastEigen3x3 (Eberly's robust symmetric 3x3 solver): eigenvector of the
 * smallest eigenvalue, zero vector for the zero matrix. */
void oracle_fast_eigen3x3(const double C[9], double n[3])
{
    double mc = C[0];
    for (int k = 1; k < 9; k++) mc = C[k] > mc ? C[k] : mc;   /* Eigen maxCoeff */
    if (mc == 0.0) { n[0] = n[1] = n[2] = 0.0; return; }
    double A[9];
    for (int k = 0; k < 9; k++) A[k] = C[k] / mc;
    const double norm = (A[1] * A[1] + A[2] * A[2]) + A[5] * A[5];
    if (norm > 0) {
        const double q = ((A[0] + A[4]) + A[8]) / 3.0;
        const double b00 = A[0] - q, b11 = A[4] - q, b22 = A[8] - q;
        const double p = sqrt((((b00 * b00 + b11 * b11) + b22 * b22) + norm * 2.0) / 6.0);
        const double c00 = b11 * b22 - A[5] * A[5];
        const double c01 = A[1] * b22 - A[5] * A[2];
        const double c02 = A[1] * A[5] - b11 * A[2];
        const double det = ((b00 * c00 - A[1] * c01) + A[2] * c02) / ((p * p) * p);
        double hd = det * 0.5;
        hd = hd > -1.0 ? hd : -1.0;   /* std::min(std::max(hd, -1.0), 1.0) */
        hd = hd < 1.0 ? hd : 1.0;
        const double angle = oracle_det_acos(hd) / 3.0;
        const double beta2 = oracle_det_cos(angle) * 2.0;
        const double beta0 = oracle_det_cos(angle + 2.09439510239319549) * 2.0;
        const double beta1 = -(beta0 + beta2);
        const double e0 = q + p * beta0, e1 = q + p * beta1, e2 = q + p * beta2;
        double v0[3], v1[3], v2[3];
        if (hd >= 0) {
            eigvec0(A, e2, v2);
            if (e2 < e0 && e2 < e1) { memcpy(n, v2, sizeof(v2)); return; }
            eigvec1(A, v2, e1, v1);
            if (e1 < e0 && e1 < e2) { memcpy(n, v1, sizeof(v1)); return; }
            cross3(v1, v2, n);
        } else {
            eigvec0(A, e0, v0);
            if (e0 < e1 && e0 < e2) { memcpy(n, v0, sizeof(v0)); return; }
            eigvec1(A, v0, e1, v1);
            if (e1 < e0 && e1 < e2) { memcpy(n, v1, sizeof(v1)); return; }
            cross3(v0, v1, n);
        }
    } else {
        double B[9];
        for (int k = 0; k < 9; k++) B[k] = A[k] * mc;  /* A *= max_coeff */
        n[0] = n[1] = n[2] = 0.0;
        if (B[0] < B[4] && B[0] < B[8]) n[0] = 1.0;
        else if (B[4] < B[0] && B[4] < B[8]) n[1] = 1.0;
        else n[2] = 1.0;
    }
}

/* utility::ComputeCovariance over the neighbour list (cumulants in list order,
 * divided by the count, then E[xy] - E[x]E[y]) */
void oracle_covariance(const float *pts, const int32_t *nb, int k, double C[9])
{
    double c[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int t = 0; t < k; t++) {
        const double x = pts[3 * nb[t]], y = pts[3 * nb[t] + 1], z = pts[3 * nb[t] + 2];
        c[0] += x; c[1] += y; c[2] += z;
        c[3] += x * x; c[4] += x * y; c[5] += x * z;
        c[6] += y * y; c[7] += y * z; c[8] += z * z;
    }
    for (int t = 0; t < 9; t++) c[t] /= (double)k;
    C[0] = c[3] - c[0] * c[0];
    C[4] = c[6] - c[1] * c[1];
    C[8] = c[8] - c[2] * c[2];
    C[1] = C[3] = c[4] - c[0] * c[1];
    C[2] = C[6] = c[5] - c[0] * c[2];
    C[5] = C[7] = c[7] - c[1] * c[2];
}

/* PointCloud::EstimateNormals(KDTreeSearchParamHybrid(r, max_nn), fast=true):
 * fewer than 3 neighbours -> covariance I (-> (0,0,1)); zero normal -> prior or
 * (0,0,1); with prior normals (n_prior != NULL) flip to agree with them. */
void oracle_estimate_normals(const float *pts, int n, double r, int max_nn, const double *n_prior,
                             double *normals)
{
    int32_t *idx = (int32_t *)malloc(sizeof(int32_t) * (size_t)n * max_nn + 4);
    double *d2 = (double *)malloc(sizeof(double) * (size_t)n * max_nn + 8);
    int32_t *cnt = (int32_t *)malloc(sizeof(int32_t) * (size_t)n + 4);
    oracle_hybrid_search(pts, n, r, max_nn, idx, d2, cnt);
    for (int i = 0; i < n; i++) {
        double C[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, v[3];
        if (cnt[i] >= 3) oracle_covariance(pts, idx + (size_t)i * max_nn, cnt[i], C);
        oracle_fast_eigen3x3(C, v);
        if (sqrt(dot3(v, v)) == 0.0) {
            if (n_prior) memcpy(v, n_prior + 3 * i, sizeof(v));
            else { v[0] = 0.0; v[1] = 0.0; v[2] = 1.0; }
        }
        if (n_prior && dot3(v, n_prior + 3 * i) < 0.0)
            for (int k = 0; k < 3; k++) v[k] *= -1.0;
        memcpy(normals + 3 * i, v, sizeof(v));
    }
    free(idx); free(d2); free(cnt);
}

/* ---- FPFH (Feature.cpp: ComputePairFeatures, ComputeSPFHFeature,
 *      ComputeFPFHFeature) ---------------------------------------------------- */

/* (f0 = atan2 angle, f1, f2, f3 = |p2 - p1|) */
void oracle_pair_features(const double p1[3], const double n1[3], const double p2[3],
                          const double n2[3], double f[4])
{
    double dp[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
    f[3] = sqrt(dot3(dp, dp));
    if (f[3] == 0.0) { f[0] = f[1] = f[2] = f[3] = 0.0; return; }
    const double *a = n1, *b = n2;
    const double ang1 = dot3(n1, dp) / f[3];
    const double ang2 = dot3(n2, dp) / f[3];
    if (oracle_det_acos(fabs(ang1)) > oracle_det_acos(fabs(ang2))) {
        a = n2; b = n1;
        for (int k = 0; k < 3; k++) dp[k] *= -1.0;
        f[2] = -ang2;
    } else
        f[2] = ang1;
    double v[3], w[3];
    cross3(dp, a, v);
    const double vn = sqrt(dot3(v, v));
    if (vn == 0.0) { f[0] = f[1] = f[2] = f[3] = 0.0; return; }
    for (int k = 0; k < 3; k++) v[k] /= vn;
    cross3(a, v, w);
    f[1] = dot3(v, b);
    f[0] = oracle_det_atan2(dot3(w, b), dot3(a, b));
}

static int clamp_bin(int h) { return h < 0 ? 0 : (h >= 11 ? 10 : h); }

void oracle_pair_bins(const double f[4], int h[3])
{
    h[0] = clamp_bin((int)floor(11.0 * (f[0] + DPI) / (2.0 * DPI)));
    h[1] = clamp_bin((int)floor(11.0 * (f[1] + 1.0) * 0.5));
    h[2] = clamp_bin((int)floor(11.0 * (f[2] + 1.0) * 0.5));
}

/* ComputeFPFHFeature(input with normals, KDTreeSearchParamHybrid(r, max_nn)):
 * spfh / fpfh (n, 33) f64 = Open3D's Feature::data_ (33, n) column-major. */
void oracle_fpfh(const float *pts, const double *normals, int n, double r, int max_nn, double *spfh,
                 double *fpfh)
{
    int32_t *idx = (int32_t *)malloc(sizeof(int32_t) * (size_t)n * max_nn + 4);
    double *d2 = (double *)malloc(sizeof(double) * (size_t)n * max_nn + 8);
    int32_t *cnt = (int32_t *)malloc(sizeof(int32_t) * (size_t)n + 4);
    oracle_hybrid_search(pts, n, r, max_nn, idx, d2, cnt);
    memset(spfh, 0, sizeof(double) * (size_t)n * 33);
    memset(fpfh, 0, sizeof(double) * (size_t)n * 33);
    for (int i = 0; i < n; i++) {
        if (cnt[i] <= 1) continue;
        const double incr = 100.0 / (double)(cnt[i] - 1);
        const double p1[3] = {pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]};
        for (int k = 1; k < cnt[i]; k++) {
            const int j = idx[(size_t)i * max_nn + k];
            const double p2[3] = {pts[3 * j], pts[3 * j + 1], pts[3 * j + 2]};
            double f[4];
            int h[3];
            oracle_pair_features(p1, normals + 3 * i, p2, normals + 3 * j, f);
            oracle_pair_bins(f, h);
            spfh[(size_t)i * 33 + h[0]] += incr;
            spfh[(size_t)i * 33 + 11 + h[1]] += incr;
            spfh[(size_t)i * 33 + 22 + h[2]] += incr;
        }
    }
    for (int i = 0; i < n; i++) {
        if (cnt[i] <= 1) continue;
        double sum[3] = {0.0, 0.0, 0.0};
        double *F = fpfh + (size_t)i * 33;
        for (int k = 1; k < cnt[i]; k++) {
            const double dist = d2[(size_t)i * max_nn + k];
            if (dist == 0.0) continue;
            const double *S = spfh + (size_t)idx[(size_t)i * max_nn + k] * 33;
            for (int j = 0; j < 33; j++) {
                const double val = S[j] / dist;
                sum[j / 11] += val;
                F[j] += val;
            }
        }
        for (int g = 0; g < 3; g++)
            if (sum[g] != 0.0) sum[g] = 100.0 / sum[g];
        for (int j = 0; j < 33; j++) {
            F[j] *= sum[j / 11];
            F[j] += spfh[(size_t)i * 33 + j];
        }
    }
    free(idx); free(d2); free(cnt);
}

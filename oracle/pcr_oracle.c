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

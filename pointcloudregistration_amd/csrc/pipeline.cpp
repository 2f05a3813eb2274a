// Composite entry: feature matching -> correspondences -> RANSAC for P pairs.
#include "pcr_internal.h"

namespace pcr {
int feature_match_impl(const float *F, const float *G, int P, int Nmax, int Mmax, int D,
                       const int32_t *n_src, const int32_t *n_tgt, int32_t *nn12, int32_t *nn21,
                       hipStream_t s);
int feature_corres_impl(const float *F, const float *G, int P, int Nmax, int Mmax, int D,
                        const int32_t *n_src, const int32_t *n_tgt, int mutual, int ransac_n,
                        int32_t *nn12, int32_t *corres, int32_t *n_corres, hipStream_t s);
int corres_impl(const int32_t *nn12, const int32_t *nn21, const int32_t *n_src,
                const int32_t *n_tgt, int P, int Nmax, int Mmax, int mutual, int ransac_n,
                int32_t *corres, int32_t *n_corres, hipStream_t s);
int ransac_impl(const float *src, const float *tgt, int P, int Nmax, int Mmax,
                const int32_t *n_src, const int32_t *n_tgt, const int32_t *corres,
                const int32_t *n_corres, int Kmax, const uint32_t *pair_ids,
                const pcr_ransac_params *prm, double *T_out, double *fit_out, int32_t *stats,
                int32_t *corr_tgt, uint32_t *mask, hipStream_t s);
}  // namespace pcr

extern "C" int pcr_register_feature_ransac(const float *src_xyz, const float *tgt_xyz,
                                           const float *src_feat, const float *tgt_feat,
                                           int32_t P, int32_t Nmax, int32_t Mmax, int32_t D,
                                           const int32_t *n_src, const int32_t *n_tgt,
                                           const uint32_t *pair_ids,
                                           const pcr_ransac_params *params, double *T,
                                           double *fitness_rmse, int32_t *stats,
                                           int32_t *corr_tgt, uint32_t *inlier_mask,
                                           pcr_stream_t stream) {
    pcr::clear_error();
    PCR_REQUIRE(P >= 0 && Nmax >= 0 && Mmax >= 0, PCR_ERR_ARG, "register: negative size");
    if (P == 0) return PCR_OK;
    PCR_REQUIRE(src_xyz && tgt_xyz && src_feat && tgt_feat && params && T && fitness_rmse && stats,
                PCR_ERR_ARG, "register: null pointer");
    PCR_REQUIRE(P <= 65535, PCR_ERR_ARG, "register: P=%d > 65535", P);
    hipStream_t s = pcr::as_stream(stream);
    // nn12 | nn21 | corres | n_corres
    const size_t words = (size_t)P * Nmax + (size_t)P * Mmax + (size_t)P * Nmax * 2 + P;
    int32_t *ws = (int32_t *)pcr::workspace(9, words * sizeof(int32_t));
    PCR_REQUIRE(ws, PCR_ERR_NOMEM, "register: %s", pcr_last_error());
    int32_t *nn12 = ws, *nn21 = nn12 + (size_t)P * Nmax, *corres = nn21 + (size_t)P * Mmax;
    int32_t *n_corres = corres + (size_t)P * Nmax * 2;
    (void)nn21;
    int rc = PCR_OK;
    if (Mmax > 0 && Nmax > 0) {
        rc = pcr::feature_corres_impl(src_feat, tgt_feat, P, Nmax, Mmax, D, n_src, n_tgt,
                                      params->mutual_filter, params->ransac_n, nn12, corres, n_corres, s);
    } else {
        if (Nmax > 0) PCR_HIP_CHECK(hipMemsetAsync(nn12, 0, sizeof(int32_t) * (size_t)P * Nmax, s));
        rc = pcr::corres_impl(nn12, nn21, n_src, n_tgt, P, Nmax, Mmax, params->mutual_filter,
                              params->ransac_n, corres, n_corres, s);
    }
    if (rc != PCR_OK) return rc;
    return pcr::ransac_impl(src_xyz, tgt_xyz, P, Nmax, Mmax, n_src, n_tgt, corres, n_corres, Nmax,
                            pair_ids, params, T, fitness_rmse, stats, corr_tgt, inlier_mask, s);
}

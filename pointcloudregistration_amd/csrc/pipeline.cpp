// Composite entries: feature matching -> correspondences -> RANSAC for P pairs
// (pcr_register_feature_ransac), and the whole C4 pipeline step
// (pcr_pipeline_step) as one host call with no round trip -- the Python stage
// calls cost ~0.3 ms of host time per step, which a 32-pair shard (2.3 ms of
// kernels) could not hide.
#include "pcr_internal.h"
#include "grid.h"
#include <chrono>
#include <cstdio>
#include <cstdlib>

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
                int32_t *corr_tgt, uint32_t *mask, hipStream_t s, const int32_t **order_out,
                const GridBatch *grid_in, const int32_t *order_in, const float *perm_in);
int icp_impl(const float *src, const float *tgt, int P, int Nmax, int Mmax, const int32_t *n_src,
             const int32_t *n_tgt, const double *init, const pcr_icp_params *prm, double *T_out,
             double *fit_out, int32_t *stats, int32_t *corr_tgt, hipStream_t s, const int32_t *order_in,
             const GridBatch *grid_in, const float *perm_in);
int pipeline_records(const pcr_pipeline_io *io, hipStream_t s);
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
                            pair_ids, params, T, fitness_rmse, stats, corr_tgt, inlier_mask, s, nullptr,
                            nullptr, nullptr, nullptr);
}

static int io_check(const pcr_pipeline_io *io) {
    PCR_REQUIRE(io, PCR_ERR_ARG, "pipeline: null io");
    PCR_REQUIRE(io->P >= 0 && io->N >= 0 && io->M >= 0 && io->D >= 1, PCR_ERR_ARG, "pipeline: bad size");
    PCR_REQUIRE(io->P <= 65535, PCR_ERR_ARG, "pipeline: P=%d > 65535", io->P);
    PCR_REQUIRE(io->T_ransac && io->fit_ransac && io->stats_ransac && io->T_icp && io->fit_icp &&
                    io->stats_icp && io->n_corres && io->d1 && io->d2 && io->records,
                PCR_ERR_ARG, "pipeline: null buffer");
    return PCR_OK;
}

extern "C" int pcr_pipeline_step(const pcr_pipeline_io *io, const pcr_ransac_params *rp,
                                 const pcr_icp_params *ip, pcr_stream_t stream) {
    pcr::clear_error();
    int rc = io_check(io);
    if (rc != PCR_OK) return rc;
    PCR_REQUIRE(rp && ip && io->src_xyz && io->tgt_xyz && io->src_feat && io->tgt_feat && io->nn12 &&
                    io->corres && io->aligned && io->i1 && io->i2,
                PCR_ERR_ARG, "pipeline: null pointer");
    PCR_REQUIRE(io->N >= 1 && io->M >= 1, PCR_ERR_ARG, "pipeline: empty clouds");
    if (io->P == 0) return PCR_OK;
    hipStream_t s = pcr::as_stream(stream);
    const int P = io->P, N = io->N, M = io->M;
    // debug (PCR_HOST_TIMING): host time of each stage's calls, to stderr
    const bool ht = getenv("PCR_HOST_TIMING") != nullptr;
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto t_prev = now();
    auto lap = [&](const char *what) {
        if (!ht) return;
        const auto t = now();
        fprintf(stderr, "pipeline host %-10s %8.1f us\n", what,
                std::chrono::duration<double, std::micro>(t - t_prev).count());
        t_prev = t;
    };
    // RANSAC's and ICP's target grids and RANSAC's spatial order of the sources
    // depend on the clouds alone: they are built on a side stream while the
    // feature stage runs (one workgroup per pair each -- a small shard left
    // most of the chip idle for them), joined before RANSAC
    hipStream_t side = nullptr;
    hipEvent_t ev_in = nullptr, ev_prep = nullptr;
    rc = pcr::side_stream(&side, &ev_in, &ev_prep);
    if (rc != PCR_OK) return rc;
    // when the prep starts: 0 with the step (it then competes with the
    // bandwidth-bound descriptor pack), 1 / 2 once pass 1 of the feature screen
    // is done / launched (an event recorded inside the feature stage).  Measured
    // (round 4): 256 pairs 9.47 / 9.36 / 9.48 ms, 128 pairs 5.14 / 5.16 / 5.16,
    // 64 pairs 2.90 / 2.91 / 2.93, 32 pairs 1.84 / 1.83 / 1.81 ms.  D > 64 (no
    // hook in that screen): 0.  Round 5, with the feature stage's row rescan on
    // its own side stream beside pass 2: 256 pairs at 1 / 2 8.21 / 8.08 ms (one
    // box), 32 pairs 1.59 / 1.57, 64 and 128 pairs 0 / 1 / 2 within 0.03 ms
    int at = (P >= 192 || P <= 48) ? 2 : 0;
    if (const char *e = getenv("PCR_PREP_AT")) at = atoi(e);  // diagnostic override (0 / 1 / 2)
    if (io->D > 64) at = 0;
    pcr::GridBatch grid_r{}, grid_i{};
    const int32_t *order = nullptr;  // RANSAC's spatial order of the sources, reused by ICP
    const float *perm = nullptr;     // the sources in that order
    const bool gr = rp->max_correspondence_distance > 0.0, gi = ip->max_correspondence_distance > 0.0;
    auto prep = [&]() -> int {
        PCR_HIP_CHECK(hipStreamWaitEvent(side, ev_in, 0));
        if (gr) {
            int r = pcr::build_grids(io->tgt_xyz, nullptr, P, M, rp->max_correspondence_distance, side, 4, grid_r, 2.01, 3);
            if (r != PCR_OK) return r;
            r = pcr::spatial_order(io->src_xyz, nullptr, P, N, grid_r.cell, side, 13, &order, &perm, 36);
            if (r != PCR_OK) return r;
        }
        if (gi) {
            int r = pcr::build_grids(io->tgt_xyz, nullptr, P, M, ip->max_correspondence_distance, side, 7, grid_i);
            if (r != PCR_OK) return r;
        }
        PCR_HIP_CHECK(hipEventRecord(ev_prep, side));
        return PCR_OK;
    };
    if (at == 0) {
        PCR_HIP_CHECK(hipEventRecord(ev_in, s));
        rc = prep();
        if (rc != PCR_OK) return rc;
    }
    lap("prep");
    // at != 0: the feature stage enqueues the prep at its hook point (prep_fn),
    // ahead of its own side-stream work; if it took no hook, it runs here
    auto prep_tramp = [](void *c) -> int { return (*static_cast<decltype(prep) *>(c))(); };
    pcr::prep_event = at ? ev_in : nullptr;
    pcr::prep_at = at;
    pcr::prep_fn = at ? +prep_tramp : nullptr;
    pcr::prep_ctx = &prep;
    rc = pcr::feature_corres_impl(io->src_feat, io->tgt_feat, P, N, M, io->D, nullptr, nullptr,
                                  rp->mutual_filter, rp->ransac_n, io->nn12, io->corres, io->n_corres, s);
    const bool prep_left = pcr::prep_fn != nullptr;
    pcr::prep_event = nullptr;
    pcr::prep_at = 0;
    pcr::prep_fn = nullptr;
    pcr::prep_ctx = nullptr;
    if (rc != PCR_OK) return rc;
    if (at && prep_left) {
        PCR_HIP_CHECK(hipEventRecord(ev_in, s));
        rc = prep();
        if (rc != PCR_OK) return rc;
    }
    lap("features");
    PCR_HIP_CHECK(hipStreamWaitEvent(s, ev_prep, 0));
    rc = pcr::ransac_impl(io->src_xyz, io->tgt_xyz, P, N, M, nullptr, nullptr, io->corres, io->n_corres, N,
                          io->pair_ids, rp, io->T_ransac, io->fit_ransac, io->stats_ransac, nullptr,
                          io->inlier_mask, s, nullptr, gr ? &grid_r : nullptr, order, perm);
    if (rc != PCR_OK) return rc;
    lap("ransac");
    rc = pcr::icp_impl(io->src_xyz, io->tgt_xyz, P, N, M, nullptr, nullptr, io->T_ransac, ip, io->T_icp,
                       io->fit_icp, io->stats_icp, nullptr, s, order, gi ? &grid_i : nullptr, perm);
    if (rc != PCR_OK) return rc;
    lap("icp");
    if (pcr::nnd_uses_grid(P, N, M) && N <= 32768 && M <= 32768) {
        // the aligned sources formed inside the Chamfer's box pass (one launch fewer)
        rc = pcr::nnd_forward_grid_xf(io->aligned, io->src_xyz, io->T_icp, io->tgt_xyz, P, N, M, io->d1, io->d2,
                                      io->i1, io->i2, s);
    } else {
        rc = pcr_transform_batch(io->src_xyz, P, N, io->T_icp, io->aligned, stream);
        if (rc != PCR_OK) return rc;
        rc = pcr_nnd_forward(io->aligned, io->tgt_xyz, P, N, M, io->d1, io->d2, io->i1, io->i2, stream);
    }
    if (rc != PCR_OK) return rc;
    rc = pcr::pipeline_records(io, s);
    lap("chamfer");
    return rc;
}

extern "C" int pcr_pipeline_records(const pcr_pipeline_io *io, pcr_stream_t stream) {
    pcr::clear_error();
    int rc = io_check(io);
    if (rc != PCR_OK) return rc;
    if (io->P == 0) return PCR_OK;
    return pcr::pipeline_records(io, pcr::as_stream(stream));
}

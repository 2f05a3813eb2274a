/*
 * pcr_api.h -- C ABI of libpcr.so, the MI355X (gfx950) registration core.
 *
 * Plain pointers + sizes, no torch types.  Every pointer argument named as a
 * device buffer must be device (HBM) memory of the current HIP device; outputs
 * are caller-allocated (the reference's ownership rule,
 * dip/torch-nndistance/torch_nndistance/__init__.py:17-20,42-43).  Work is
 * enqueued on `stream` (a hipStream_t; NULL = legacy default stream, which is
 * what the reference launcher uses, nnd_cuda.cu:152-153) and is asynchronous
 * unless stated otherwise.
 *
 * Return value: PCR_OK (0) or a negative PCR_ERR_* code; pcr_last_error()
 * returns a thread-local message for the last failure.  (The reference CUDA
 * launcher prints and returns 0 / 1, nnd_cuda.cu:155-161; the Python layer
 * maps PCR_OK -> 1 and raises on failure.)
 *
 * Concurrency contract: scratch buffers come from a library-owned workspace
 * with one set of slots PER DEVICE (not per stream).  Calls for one device must
 * therefore be ordered: issue them on one stream at a time (or order the streams
 * with events), from any host thread.  Two libpcr calls running concurrently on
 * two streams of the same device would share scratch.  A slot that grows keeps
 * its previous buffer alive (HIP graphs captured earlier may still point at it);
 * pcr_workspace_release() frees every workspace buffer of the current device
 * after a device synchronize -- call it only when no captured graph that
 * contains libpcr kernels will be replayed again.
 */
#ifndef PCR_API_H
#define PCR_API_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PCR_OK 0
#define PCR_ERR_ARG (-1)
#define PCR_ERR_HIP (-2)
#define PCR_ERR_NOMEM (-3)

typedef void *pcr_stream_t; /* hipStream_t */

const char *pcr_last_error(void);
int pcr_version(void);
int pcr_workspace_release(void);
/* end of process: synchronise every device the library used and free its
 * workspace, retired buffers and pooled profiling events (idempotent; the
 * library stays usable; a device that cannot be synchronised keeps its
 * buffers).  A HIP graph captured before it records freed buffers and must not
 * be replayed after it.  The Python layer runs it from atexit. */
int pcr_shutdown(void);
/* Concurrent sub-batches.  pcr_set_workspace_context(ctx) (thread-local, 0..3)
 * selects which copy of the library's scratch the calling thread's next calls
 * use: calls that run concurrently on different streams must use different
 * contexts.  pcr_set_concurrency(k) (1..4): k launches share the device, so
 * cooperative grids (ICP's workgroups per pair and its tail launch) are sized
 * to CUs / k and k of them can be resident at once. */
int pcr_set_workspace_context(int32_t ctx);
int pcr_set_concurrency(int32_t k);
/* Diagnostics: one trivial launch of `blocks` (1..256) 256-thread blocks,
 * cooperative or plain, writing out[b] = b -- nothing else of the library
 * (tools/exit_probe.py isolates an exit-time fault under the profiler). */
int pcr_coop_probe(int32_t *out, int32_t blocks, int32_t cooperative, pcr_stream_t stream);

/* Optional per-kernel timing with HIP events recorded on the launch stream
 * around the hot kernels (id 0 feature screen (pass 1), 1 nnd forward, 2 RANSAC verify,
 * 3 ICP, 4 RANSAC hypotheses, 5 feature rescan, 6 feature pack, 7 nnd grid query,
 * 8 feature screen pass 2, 9 / 10 the 3-term screens behind passes 1 / 2, 11 the 1-term
 * screens' regroup and finish, featnn_regroup9 / featnn_finish9).  pcr_profile_read synchronizes the pending
 * events and returns the accumulated milliseconds and launch count. */
void pcr_profile_enable(int32_t on);
int pcr_profile_read(int32_t id, double *total_ms, int64_t *count, int32_t reset);

/* Diagnostic: rows (src->tgt, tgt->src) that the feature-NN screen could not
 * certify and sent to the exact f64 rescan since the last reset.  Synchronizes
 * the device. */
int pcr_featnn_rescan_rows(int64_t *rows12, int64_t *rows21, int32_t reset);
/* Diagnostic: source rows (pass 1) and target columns of J (pass 2) that the
 * 1-term f16 feature screens could not certify and left to the 3-term split
 * screen since the last reset.  Synchronizes the device. */
int pcr_featnn_fallback_rows(int64_t *rows12, int64_t *cols21, int32_t reset);
/* diagnostic: copy `bytes` of pcr_feature_correspondences' scratch from its
 * last call (device to device, on `stream`) */
int pcr_featmut_debug_copy(void *dst, int64_t bytes, pcr_stream_t stream);

/* ---------------------------------------------------------------------------
 * a1 -- brute-force bidirectional 1-NN ("nnd" / Chamfer building block).
 * Replaces nnd_forward_cuda (dip/torch-nndistance/src/my_lib_cuda.cpp:25-41)
 * -> NmDistanceKernelLauncher (nnd_cuda.cu:132-162).
 *   xyz1 (b,n,3) f32, xyz2 (b,m,3) f32, contiguous AoS, device.
 *   dist1 (b,n) f32 / idx1 (b,n) i32: for each xyz1 point, min over xyz2 of
 *   (dx*dx+dy*dy)+dz*dz in f32 (no FMA) and the FIRST index attaining it;
 *   dist2/idx2 the same from xyz2 to xyz1.  Bit-exact with my_lib.cpp:3-25.
 *   m == 0 (resp. n == 0) yields dist 0, idx 0 (my_lib.cpp seed values).
 * ------------------------------------------------------------------------- */
int pcr_nnd_forward(const float *xyz1, const float *xyz2, int32_t b, int32_t n, int32_t m,
                    float *dist1, float *dist2, int32_t *idx1, int32_t *idx2,
                    pcr_stream_t stream);

/* ---------------------------------------------------------------------------
 * a1/a3 -- the same search over RAGGED batches, and in f64.  Replaces
 * pytorch3d.knn_points(x, y, lengths1, lengths2, K=1) inside
 * compute_truncated_chamfer_distance (c2p-net/deformationpyramid/model/
 * loss.py:60-160: x_lengths / y_lengths, computed in the inputs' dtype).
 *   n1 (b) / n2 (b) i32 device: valid points of each cloud (NULL = n / m);
 *   rows i < n1[k] search the first n2[k] points of the other cloud with
 *   pcr_nnd_forward's contract (same formula and first-index rule, in f32 or
 *   f64); rows past a length, and rows whose other cloud is empty, get
 *   (0, 0).  Outputs are (b,n) / (b,m) like pcr_nnd_forward.
 * ------------------------------------------------------------------------- */
int pcr_nnd_forward_ragged(const float *xyz1, const float *xyz2, int32_t b, int32_t n, int32_t m,
                           const int32_t *n1, const int32_t *n2, float *dist1, float *dist2,
                           int32_t *idx1, int32_t *idx2, pcr_stream_t stream);
int pcr_nnd_forward_f64(const double *xyz1, const double *xyz2, int32_t b, int32_t n, int32_t m,
                        const int32_t *n1, const int32_t *n2, double *dist1, double *dist2,
                        int32_t *idx1, int32_t *idx2, pcr_stream_t stream);

/* ---------------------------------------------------------------------------
 * a2 -- gradient of (dist1, dist2) w.r.t. (xyz1, xyz2).
 * Replaces nnd_backward_cuda (my_lib_cuda.cpp:44-72) -> NmDistanceGradKernel
 * (nnd_cuda.cu:164-222).  gxyz1 (b,n,3), gxyz2 (b,m,3) are fully written (the
 * caller need not zero them).  Deterministic: the scatter terms are summed in
 * the exact order of the reference CPU loop (my_lib.cpp:93-130), so the result
 * is bitwise reproducible and bit-identical to the CPU reference (the CUDA
 * reference uses float atomics and is not).
 * ------------------------------------------------------------------------- */
int pcr_nnd_backward(const float *xyz1, const float *xyz2, const float *graddist1,
                     const float *graddist2, const int32_t *idx1, const int32_t *idx2,
                     int32_t b, int32_t n, int32_t m, float *gradxyz1, float *gradxyz2,
                     pcr_stream_t stream);


/* ===========================================================================
 * Registration path (batched over P cloud pairs).  Layout: pair p's source
 * points are src_xyz[p*Nmax*3 .. +n_src[p]*3) (f32, AoS), features
 * src_feat[p*Nmax*D ..] (f32, row-major); likewise tgt with Mmax.  n_src /
 * n_tgt may be NULL (= all Nmax / Mmax points valid).
 * ======================================================================== */

/* ---------------------------------------------------------------------------
 * a5 -- exact feature-space 1-NN, both directions.  Replaces the KD-tree
 * SearchKNN(k=1) loops inside Open3D registration_ransac_based_on_feature_matching
 * (called at DataPreparation/RANSAC.py:43, dip/demo.py:43,
 * c2p-net/ngenet/utils/o3d.py:174) and vote.get_coor_points
 * (c2p-net/ngenet/models/vote.py:6-9).  nn12 (P,Nmax): argmin_j |f_i-g_j|^2,
 * nn21 (P,Mmax): argmin_i; distances in f64, lowest index on ties.  1 <= D <= 128.
 * ------------------------------------------------------------------------- */
int pcr_feature_match(const float *src_feat, const float *tgt_feat, int32_t P, int32_t Nmax,
                      int32_t Mmax, int32_t D, const int32_t *n_src, const int32_t *n_tgt,
                      int32_t *nn12, int32_t *nn21, pcr_stream_t stream);

/* mutual filter + ordered compaction: corres (P,Nmax,2) = (i, nn12[i]) for i with
 * nn21[nn12[i]] == i in increasing i, or all (i, nn12[i]) when fewer than
 * 3*ransac_n survive or mutual_filter == 0 (Open3D 0.13 semantics). */
int pcr_correspondences(const int32_t *nn12, const int32_t *nn21, int32_t P, int32_t Nmax,
                        int32_t Mmax, const int32_t *n_src, const int32_t *n_tgt,
                        int32_t mutual_filter, int32_t ransac_n, int32_t *corres,
                        int32_t *n_corres, pcr_stream_t stream);

/* feature matching + mutual filter in one call: the correspondences the
 * two calls above produce (bit-identical corres / n_corres, and nn12), without
 * computing nn21 for every target -- the filter reads nn21 only at j = nn12[i]
 * (Open3D 0.13 RegistrationRANSACBasedOnFeatureMatching with mutual_filter,
 * DataPreparation/RANSAC.py:43-52).  The column direction is screened only for
 * the targets some source picked, and decided from certified screen values
 * (csrc/featnn.hip featnn_row7).  With mutual_filter == 0 only nn12 is
 * computed.  nn12 (P,Nmax) out; corres (P,Nmax,2), n_corres (P) out. */
int pcr_feature_correspondences(const float *src_feat, const float *tgt_feat, int32_t P,
                                int32_t Nmax, int32_t Mmax, int32_t D, const int32_t *n_src,
                                const int32_t *n_tgt, int32_t mutual_filter, int32_t ransac_n,
                                int32_t *nn12, int32_t *corres, int32_t *n_corres,
                                pcr_stream_t stream);

/* RANSAC parameters (Open3D names; RANSAC.py:43-52). */
typedef struct pcr_ransac_params {
    double max_correspondence_distance; /* verification radius d                         */
    double edge_length_ratio;           /* CorrespondenceCheckerBasedOnEdgeLength; <=0 off */
    double distance_check;              /* CorrespondenceCheckerBasedOnDistance;   <=0 off */
    double confidence;                  /* RANSACConvergenceCriteria.confidence            */
    int32_t max_iteration;              /* RANSACConvergenceCriteria.max_iteration          */
    int32_t ransac_n;                   /* 3..8                                            */
    int32_t mutual_filter;              /* used by pcr_register_feature_ransac             */
    int32_t reserved;
    uint64_t seed;                      /* Philox key; hypothesis = f(seed, pair_id, itr)  */
} pcr_ransac_params;

/* ---------------------------------------------------------------------------
 * a6/a7 -- RANSAC hypothesize-and-verify on given correspondences.
 * Replaces Open3D RegistrationRANSACBasedOnCorrespondence.  corres (P,Kmax,2)
 * with n_corres[p] valid rows; pair_ids (P) optional (default p) keys the
 * hypothesis stream.  Outputs: T (P,16) f64 row-major 4x4, fitness_rmse (P,2),
 * stats (P,5) = {iterations, validated, best_itr, status(1 ok/0 none/-1 bad
 * input), n_correspondences}, corr_tgt (P,Nmax) target index per source point
 * or -1 (optional), inlier_mask (P, ceil(Nmax/32)) bitset (optional).
 * Asynchronous on the stream (no host round trip): hypotheses run in two
 * rounds, [0,1024) and [1024, max_iteration), the second launched behind the
 * first and returning at once when no pair's bound est_k lies beyond 1024.
 * Verification runs speculatively on persistent workgroups, the sequential rule
 * is replayed afterwards: results do not depend on the scheduling or the round
 * split.  Workspace per pair: ~135 B per hypothesis slot of the larger round
 * (max_iteration - 1024 rounded up to 256, at least 1024: ~13 MB per pair at
 * max_iteration 100000), 2 x Nmax x 4 B of target buffers, plus up to 256 MB
 * per device of per-hypothesis target slots (fewer slots only add one sweep per
 * pair).  Past 2^26 slots in all (P x max_iteration), or with
 * PCR_RANSAC_SYNC=1, the host instead runs rounds of 4096 while a pair is
 * still active (one 32-byte readback per round, ~540 KB per pair).
 * ------------------------------------------------------------------------- */
int pcr_ransac_batch(const float *src_xyz, const float *tgt_xyz, int32_t P, int32_t Nmax,
                     int32_t Mmax, const int32_t *n_src, const int32_t *n_tgt,
                     const int32_t *corres, const int32_t *n_corres, int32_t Kmax,
                     const uint32_t *pair_ids, const pcr_ransac_params *params, double *T,
                     double *fitness_rmse, int32_t *stats, int32_t *corr_tgt,
                     uint32_t *inlier_mask, pcr_stream_t stream);

/* ---------------------------------------------------------------------------
 * a5+a6+a7 composite: feature matching -> (mutual) correspondences -> RANSAC.
 * Replaces registration_ransac_based_on_feature_matching (RANSAC.py:43-52) for
 * P pairs at once; outputs as pcr_ransac_batch.  `scratch` sizing is internal.
 * ------------------------------------------------------------------------- */
int pcr_register_feature_ransac(const float *src_xyz, const float *tgt_xyz,
                                const float *src_feat, const float *tgt_feat, int32_t P,
                                int32_t Nmax, int32_t Mmax, int32_t D, const int32_t *n_src,
                                const int32_t *n_tgt, const uint32_t *pair_ids,
                                const pcr_ransac_params *params, double *T,
                                double *fitness_rmse, int32_t *stats, int32_t *corr_tgt,
                                uint32_t *inlier_mask, pcr_stream_t stream);

/* ICP parameters (Open3D ICPConvergenceCriteria defaults 1e-6, 1e-6, 30). */
typedef struct pcr_icp_params {
    double max_correspondence_distance;
    double relative_fitness;
    double relative_rmse;
    int32_t max_iteration;
    int32_t reserved;
} pcr_icp_params;

/* ---------------------------------------------------------------------------
 * a8 -- point-to-point ICP.  Replaces Open3D registration_icp
 * (DataPreparation/RANSAC.py:61-63).  init (P,16) f64; outputs T (P,16),
 * fitness_rmse (P,2), stats (P,2) = {iterations, n_correspondences}, corr_tgt
 * (P,Nmax) optional: target index of each source point in the final
 * correspondence set (Open3D result.correspondence_set) or -1.
 * ------------------------------------------------------------------------- */
int pcr_icp_batch(const float *src_xyz, const float *tgt_xyz, int32_t P, int32_t Nmax,
                  int32_t Mmax, const int32_t *n_src, const int32_t *n_tgt, const double *init,
                  const pcr_icp_params *params, double *T, double *fitness_rmse, int32_t *stats,
                  int32_t *corr_tgt, pcr_stream_t stream);

/* ---------------------------------------------------------------------------
 * The C4 pipeline step (DataPreparation/RANSAC.py:109-122 per pair, with the
 * QualityCheck.py:25-31 Chamfer) for P resident pairs, no host round trip:
 * mutual feature correspondences (a5) -> RANSAC (a6/a7) -> ICP from the RANSAC
 * T (a8) -> aligned source (f64 T, f32 out) -> nnd both ways (a1) -> records.
 * Every buffer is device memory owned by the caller (inlier_mask optional).
 * records (P, 40) f64: [0,16) T_ransac, [16,32) T_icp, 32/33 RANSAC fitness /
 * rmse, 34/35 ICP fitness / rmse, 36 Chamfer = mean(d1) + mean(d2) (f64 sums
 * of the f32 distances in index order), 37 RANSAC iterations, 38 RANSAC
 * status, 39 correspondences after the mutual filter.
 * pcr_pipeline_records: the records alone, from buffers the stage calls filled.
 * Streams: the step forks once -- RANSAC's / ICP's target grids and the source
 * spatial order are built on a library-owned side stream of the calling
 * thread's (device, workspace context) while the feature stage runs on
 * `stream`, joined by an event before RANSAC -- and everything else, and the
 * completion, is on `stream` (a graph capture of the step sees the fork/join).
 * ------------------------------------------------------------------------- */
typedef struct pcr_pipeline_io {
    const float *src_xyz, *tgt_xyz;    /* (P,N,3), (P,M,3) */
    const float *src_feat, *tgt_feat;  /* (P,N,D), (P,M,D) */
    int32_t P, N, M, D;
    const uint32_t *pair_ids;          /* (P) or null */
    int32_t *nn12;                     /* (P,N) */
    int32_t *corres, *n_corres;        /* (P,N,2), (P) */
    double *T_ransac, *fit_ransac;     /* (P,16), (P,2) */
    int32_t *stats_ransac;             /* (P,5) */
    uint32_t *inlier_mask;             /* (P, ceil(N/32)) or null */
    double *T_icp, *fit_icp;           /* (P,16), (P,2) */
    int32_t *stats_icp;                /* (P,2) */
    float *aligned;                    /* (P,N,3) */
    float *d1, *d2;                    /* (P,N), (P,M) */
    int32_t *i1, *i2;                  /* (P,N), (P,M) */
    double *records;                   /* (P,40) */
} pcr_pipeline_io;
int pcr_pipeline_step(const pcr_pipeline_io *io, const pcr_ransac_params *ransac,
                      const pcr_icp_params *icp, pcr_stream_t stream);
int pcr_pipeline_records(const pcr_pipeline_io *io, pcr_stream_t stream);

/* ---------------------------------------------------------------------------
 * radius-limited 1-NN (Open3D KDTreeFlann::SearchHybrid(r, max_nn=1), used by
 * RANSAC verification / ICP): for each f64 query (P,Qmax,3) the nearest target
 * point with d^2 < float(r*r), lowest index on ties; idx -1 if none, d2 optional.
 * ------------------------------------------------------------------------- */
int pcr_radius_nn(const float *tgt_xyz, int32_t P, int32_t Mmax, const int32_t *n_tgt,
                  const double *queries, int32_t Qmax, const int32_t *n_q, double r,
                  int32_t *idx, double *d2, pcr_stream_t stream);

/* ---------------------------------------------------------------------------
 * a9 -- batched weighted Procrustes (B items of N points).  Replaces the
 * torch.svd Kabsch of ROPNet weighted_icp (model_utils.py:105-139; abs_weights=0,
 * eps=1e-8) and NDP rigid_fit (deformationpyramid/model/geometry.py:8-34;
 * abs_weights=1, eps=1e-4).  T (B,12) f64 = [R | t] row-major, tgt ~ R src + t.
 * ------------------------------------------------------------------------- */
int pcr_procrustes_batch(const float *src, const float *tgt, const float *weights, int32_t B,
                         int32_t N, int32_t abs_weights, double eps, double *T,
                         pcr_stream_t stream);
/* the same for f64 inputs (the reference functions are dtype-generic: f64
 * tensors run weighted_icp's torch.svd in f64, model_utils.py:120-133) */
int pcr_procrustes_batch_f64(const double *src, const double *tgt, const double *weights,
                             int32_t B, int32_t N, int32_t abs_weights, double eps, double *T,
                             pcr_stream_t stream);

/* out (B,N,3) f32 = (float)(R p + t) in f64 for each item's T (B,16) f64
 * row-major 4x4 (registration outputs).  Replaces the per-pair
 * source.transform(T) (Open3D PointCloud::Transform, RANSAC.py / QualityCheck.py)
 * before the Chamfer check. */
int pcr_transform_batch(const float *xyz, int32_t B, int32_t N, const double *T, float *out,
                        pcr_stream_t stream);

/* ---------------------------------------------------------------------------
 * a4 -- DIP local reference frames, batched.  Replaces lrf.get
 * (dip/lrf.py:19-78) called per sampled point by dip/demo.py:109-114.
 * Two phases so the reference's np.random.choice stream stays on the host:
 *   pcr_lrf_count   -> counts (P,Qmax): radius neighbours of each query
 *                      (d^2 < float(kernel^2), incl. the first hit);
 *   host            -> inds (P,Qmax,patch_size) = np.random.choice(
 *                      max(count, patch_size), patch_size, replace=False);
 *   pcr_lrf_compute -> patches (P,Qmax,patch_size,3) f64 (lRg^T (p - pt) /
 *                      kernel, zero rows past the count) and T (P,Qmax,16) f64
 *                      row-major [[xp yp zp | pt],[0 0 0 1]] (det -1, as the
 *                      reference).  max_count >= every count, <= 8192.
 * Points/queries f64 (Open3D stores double).  counts may be NULL in phase 2.
 * ------------------------------------------------------------------------- */
int pcr_lrf_count(const double *pts, int32_t P, int32_t Nmax, const int32_t *n_pts,
                  const double *queries, int32_t Qmax, const int32_t *n_q, double kernel,
                  int32_t *counts, pcr_stream_t stream);
int pcr_lrf_compute(const double *pts, int32_t P, int32_t Nmax, const int32_t *n_pts,
                    const double *queries, int32_t Qmax, const int32_t *n_q, double kernel,
                    int32_t patch_size, const int32_t *inds, int32_t max_count,
                    double *patches, double *T, int32_t *counts, pcr_stream_t stream);
/* Host only (no device work): the patch-index draws of dip/lrf.py:76,
 * np.random.choice(pop[c], k, replace=False) for c = 0..calls-1 in order, on the
 * caller's legacy RandomState MT19937 state (key[624], *pos as returned by
 * RandomState.get_state(); both updated as numpy would leave them).
 * out (calls, k) i32.  Fails with PCR_ERR_ARG when pop[c] < k, like numpy. */
int pcr_legacy_choice_batch(uint32_t *key, int32_t *pos, const int32_t *pop, int32_t calls,
                            int32_t k, int32_t *out);

/* ---------------------------------------------------------------------------
 * a10 -- NDP deformation-pyramid warp, all levels in one launch.  Replaces
 * Deformation_Pyramid.warp (c2p-net/deformationpyramid/model/nets.py:36-48)
 * over NDPLayer.forward (:111-140) with motion "SE3", rotation "axis_angle"
 * (the C5 configuration, config/NDP.yaml).  Weights in nn.Linear layout
 * (out, in) f32, device pointers; w_hid holds the depth-1 MLP layers
 * contiguously; w_nr/b_nr NULL for levels without the nonrigidity branch.
 * levels is a HOST array of n_levels (<= 16) entries.  x_levels (n_levels,N,3)
 * and nonrigidity (n_levels,N) are optional per-level outputs (data[i]).
 * ------------------------------------------------------------------------- */
typedef struct pcr_ndp_level {
    const float *w_in, *b_in;   /* (W,6), (W) */
    const float *w_hid, *b_hid; /* (depth-1,W,W), (depth-1,W) */
    const float *w_rot, *b_rot; /* (3,W), (3) */
    const float *w_trn, *b_trn; /* (3,W), (3) */
    const float *w_nr, *b_nr;   /* (1,W), (1) or NULL */
    int32_t m;                  /* level index + 1: omega = 2^(m + k0) */
    int32_t reserved;
} pcr_ndp_level;
int pcr_ndp_warp(const float *x, int32_t N, const pcr_ndp_level *levels, int32_t n_levels,
                 int32_t width, int32_t depth, int32_t k0, float *x_out, float *x_levels,
                 float *nonrigidity, pcr_stream_t stream);


/* ---------------------------------------------------------------------------
 * f2 -- KPConv input pyramid helpers (ngenet cpp_wrappers).
 *
 * pcr_grid_subsample replaces cpp_subsampling.subsample_batch
 * (c2p-net/ngenet/cpp_wrappers/cpp_subsampling/wrapper.cpp:59-330 ->
 * batch_grid_subsampling, grid_subsampling/grid_subsampling.cpp:109-211).
 *   points (n,3) f32 and features (n,fdim) f32 (or NULL, fdim 0) are device
 *   buffers; batch_len (nb) is a HOST array (cloud lengths, summing to <= n).
 *   Per cloud: voxels of side dl from the floor(min/dl)*dl corner, barycentre
 *   (f32 sums in input order, * (float)(1.0/count)) and mean features
 *   (f / (float)count), emitted in the reference's unordered_map iteration order
 *   and truncated to max_p per cloud (max_p < 1: n).  Writes out_points
 *   (capacity n*3), out_features (capacity n*fdim), out_batch_len (HOST, nb)
 *   and *out_total (HOST).  Bit-identical to the reference, order included.
 *   Synchronous (the emission order is replayed on the host).  Non-finite
 *   coordinates -> PCR_ERR_ARG (the reference's voxel index is undefined).
 *
 * pcr_voxel_map_order: host-only helper behind it -- the iteration order of a
 * std::unordered_map<size_t,...> after inserting the n distinct keys in order:
 * order[k] = insertion rank of the k-th visited key.
 *
 * pcr_radius_count / pcr_radius_neighbors replace cpp_neighbors.batch_query
 * (cpp_neighbors/wrapper.cpp:63-230 -> batch_nanoflann_neighbors,
 * neighbors/neighbors.cpp:211-332).
 *   queries (nq,3), supports (ns,3) f32 device; q_batches / s_batches (nb) HOST.
 *   Neighbours of a query: supports of its batch with f32
 *   (dx*dx + dy*dy) + dz*dz < radius*radius, by ascending distance (equal
 *   distances by ascending index), as global support indices.  counts (nq)
 *   device (optional) and *max_count (HOST) = the reference's row width.
 *   pcr_radius_neighbors writes out (nq,width) int32 device: the first `width`
 *   neighbours of each query, padded with ns (supports.size()); width =
 *   max_count is batch_query, min(max_count, max_nn) is dataloader.py
 *   batch_neighbors (:12-25).  Both synchronize the stream once.
 * ------------------------------------------------------------------------- */
int pcr_grid_subsample(const float *points, int32_t n, const int32_t *batch_len, int32_t nb,
                       const float *features, int32_t fdim, float dl, int32_t max_p,
                       float *out_points, float *out_features, int32_t *out_batch_len,
                       int32_t *out_total, pcr_stream_t stream);
int pcr_voxel_map_order(const uint64_t *keys, int32_t n, int32_t *order);
int pcr_radius_count(const float *queries, int32_t nq, const float *supports, int32_t ns,
                     const int32_t *q_batches, const int32_t *s_batches, int32_t nb, float radius,
                     int32_t *counts, int32_t *max_count, pcr_stream_t stream);
int pcr_radius_neighbors(const float *queries, int32_t nq, const float *supports, int32_t ns,
                         const int32_t *q_batches, const int32_t *s_batches, int32_t nb,
                         float radius, int32_t width, int32_t *out, int32_t *max_count,
                         pcr_stream_t stream);

/* ---------------------------------------------------------------------------
 * a5 (ii) -- the level voting of c2p-net/ngenet/models/vote.py:12-37 (after the
 * h / m / l feature-space 1-NN of get_coor_points, :6-9, on pcr_feature_match).
 *   tgt_xyz (m,3) f32, nn_h / nn_m / nn_l (n) i32 (source -> target at each
 *   level), feature rows (n,D) / (m,D) f32, all device.  For every source i:
 *   d12, d13, d23 = f32 Euclidean distances between its three targets (numpy's
 *   order, correctly rounded sqrt); sel_h = d12 < thr or d13 < thr, sel_m = d23
 *   < thr with thr = (float)(2 voxel_size); where !sel_h and sel_m the h rows
 *   are replaced in place: src_feat_h[i] <- src_feat_m[i] and
 *   tgt_feat_h[nn_m[i]] <- tgt_feat_m[nn_m[i]].  replaced (n) u8 optional.
 *   Asynchronous on `stream`.
 * ------------------------------------------------------------------------- */
int pcr_vote_apply(const float *tgt_xyz, int32_t m, const int32_t *nn_h, const int32_t *nn_m,
                   const int32_t *nn_l, int32_t n, double voxel_size, float *src_feat_h,
                   const float *src_feat_m, float *tgt_feat_h, const float *tgt_feat_m, int32_t D,
                   uint8_t *replaced, pcr_stream_t stream);

/* ---------------------------------------------------------------------------
 * f2 -- Open3D voxel down-sampling (dip/demo.py:73-74 pcd.voxel_down_sample,
 * Open3D 0.13 PointCloud::VoxelDownSample; oracle/voxel_oracle.cpp restates it).
 *   points (n,3) f64 device, optional normals / colors (n,3) f64 device (NULL:
 *   none); cloud_len (nb) HOST (lengths summing to <= n).  Per cloud: voxel
 *   min bound = min - voxel_size/2, voxel = int(floor((p - bound)/voxel_size)),
 *   per voxel the f64 sums in input order (normals with a NaN component
 *   skipped) divided by double(count), emitted in the iteration order of
 *   Open3D's unordered_map<Vector3i, ..., hash_eigen> (replayed on the host).
 *   Writes out_points / out_normals / out_colors (capacity n*3 each, device),
 *   out_cloud_len (HOST, nb) and *out_total (HOST).  Synchronous.  Errors as
 *   the reference: voxel_size <= 0, "voxel_size is too small"; non-finite
 *   coordinates -> PCR_ERR_ARG.
 * pcr_voxel3i_map_order: host-only helper behind it -- iteration order of that
 *   map after inserting the n distinct (x, y, z) int keys in order.
 * ------------------------------------------------------------------------- */
int pcr_voxel_down_sample(const double *points, int32_t n, const int32_t *cloud_len, int32_t nb,
                          double voxel_size, const double *normals, const double *colors,
                          double *out_points, double *out_normals, double *out_colors,
                          int32_t *out_cloud_len, int32_t *out_total, pcr_stream_t stream);
int pcr_voxel3i_map_order(const int32_t *xyz, int32_t n, int32_t *order);

/* ---------------------------------------------------------------------------
 * f1 -- normal estimation and FPFH, the preprocessing of
 * DataPreparation/RANSAC.py:12-22 (Open3D 0.13 PointCloud::estimate_normals
 * with KDTreeSearchParamHybrid(4 voxel, 30) and
 * pipelines.registration.compute_fpfh_feature with
 * KDTreeSearchParamHybrid(7 voxel, 100)), batched over P clouds.
 * Semantics restated in oracle/fpfh_oracle.c (Open3D absent: parity vs the
 * reference unpinned; GPU == restatement bit for bit).
 *
 * pcr_hybrid_search replaces KDTreeFlann::SearchHybrid(points[i], radius,
 *   max_nn) for every point of every cloud: the max_nn nearest points with
 *   f64 (dx*dx + dy*dy) + dz*dz < (double)(float)(radius^2), ascending
 *   (d2, index).  idx (P,Nmax,max_nn) local indices (-1 padded), d2 same shape
 *   f64, counts (P,Nmax).  1 <= max_nn <= 448.
 * pcr_estimate_normals: normals (P,Nmax,3) f64 (ComputeCovariance over the
 *   hybrid neighbourhood incl. the point, FastEigen3x3 smallest eigenvector;
 *   < 3 neighbours -> (0,0,1)).  prior_normals (P,Nmax,3) f64 or NULL: when
 *   given (the cloud already had normals) each result is flipped to agree
 *   with it, and a zero result takes it (EstimateNormals' has_normal branch).
 * pcr_compute_fpfh: fpfh (P,Nmax,33) f64 = Open3D's Feature::data_ (33, N)
 *   column-major; fpfh_f32 (optional) the same rounded to f32 (the input of
 *   pcr_feature_match); spfh (optional) the intermediate SPFH histograms.
 * Clouds are xyz (P,Nmax,3) f32 with n_pts (P) valid points (NULL = Nmax);
 * rows past a cloud's count are left untouched.
 * ------------------------------------------------------------------------- */
int pcr_hybrid_search(const float *xyz, int32_t P, int32_t Nmax, const int32_t *n_pts,
                      double radius, int32_t max_nn, int32_t *idx, double *d2, int32_t *counts,
                      pcr_stream_t stream);
int pcr_estimate_normals(const float *xyz, int32_t P, int32_t Nmax, const int32_t *n_pts,
                         double radius, int32_t max_nn, const double *prior_normals,
                         double *normals, pcr_stream_t stream);
int pcr_compute_fpfh(const float *xyz, const double *normals, int32_t P, int32_t Nmax,
                     const int32_t *n_pts, double radius, int32_t max_nn, double *fpfh,
                     float *fpfh_f32, double *spfh, pcr_stream_t stream);

/* ---------------------------------------------------------------------------
 * f4 -- device-side pieces of the NDP level optimisation
 * (c2p-net/deformationpyramid/model/registration.py:196-262), so one iteration
 * can be captured in a HIP graph and replayed without host round trips.
 *
 * pcr_ndp_control: the early-stop rule of :246-256 on the device (f64 on the f32
 *   loss, as Python evaluates loss.item()).  state (device f64[8]) =
 *   {active, break_count, loss_prev, steps, last_loss, step_flag, evaluated, 0},
 *   initialise to {1, 0, 1e6, 0, 0, 0, 0, 0} per level; stop_loss 1e-4.
 * pcr_adam_masked: torch.optim.Adam's update for n_tensors parameter tensors
 *   (a DEVICE table of pcr_adam_tensor), skipped when state[5] == 0; bias
 *   corrections from state[3] (steps taken, incremented by pcr_ndp_control).
 * ------------------------------------------------------------------------- */
typedef struct pcr_adam_tensor {
    float *param;
    const float *grad;
    float *exp_avg;
    float *exp_avg_sq;
    int32_t n;
    int32_t reserved;
} pcr_adam_tensor;
int pcr_ndp_control(const float *loss, double *state, double break_threshold_ratio,
                    int32_t max_break_count, double stop_loss, pcr_stream_t stream);
int pcr_adam_masked(const pcr_adam_tensor *tensors, int32_t n_tensors, int32_t max_numel,
                    const double *state, double lr, double beta1, double beta2, double eps,
                    pcr_stream_t stream);
/* pcr_set_gate: the early stop that stops the work (registration.py:250-256
 *   `break`s out of the level).  While a gate is set on the calling thread
 *   (gate = the level's state, a device pointer), every kernel that
 *   pcr_nnd_forward / pcr_nnd_backward / pcr_ndp_train_forward /
 *   pcr_ndp_train_backward / pcr_ndp_chamfer_glue launch reads gate[0] at entry
 *   and returns at once when it is 0 -- so the replays of a captured level graph
 *   left after the rule fired cost only their launches.  pcr_set_gate(NULL)
 *   restores ungated launches.  Thread-local; captured launches keep the pointer
 *   they were recorded with. */
int pcr_set_gate(const double *gate);

/* ---------------------------------------------------------------------------
 * f4 -- fused NDP level training step (one level of
 * registration.py:208-262 without PyTorch autograd).  One descriptor:
 *   x (N,3) level input; level weights in nn.Linear layout (level.w_hid /
 *   level.b_hid unused: the hidden layers are w_hid[k] / b_hid[k], k < depth-1,
 *   read in place so the optimizer updates them directly); width 128.
 *   Scratch (device, feature-major [F][N]): pe [6][N], H [depth][W][N],
 *   aux [8][N], dO [8][N], D [depth][W][N]; x_out (N,3) the warped points.
 *   g (N,3) = dL/dx_out (e.g. the Chamfer gradient), bce_scale = w_reg / N for
 *   a level with the nonrigidity branch (BCE(s, 0) mean), else 0.
 * pcr_ndp_train_forward: x_out, and the saved activations.
 * pcr_ndp_train_backward: the gradients of every parameter of the level into
 *   grads (HOST array of device pointers): {w_in, b_in, w_hid[0], b_hid[0], ...,
 *   w_branch (7 x W rows: rot 0-2, trn 3-5, nr 6), b_branch (7)}; part is
 *   scratch of pcr_ndp_train_partial_floats(N, width, depth, chunk) floats.
 * ------------------------------------------------------------------------- */
typedef struct pcr_ndp_train {
    const float *x;
    int32_t N, width, depth, k0;
    pcr_ndp_level level;
    const float *w_hid[4], *b_hid[4];
    float *pe, *H, *aux, *x_out;
    const float *g;
    double bce_scale;
    float *dO, *D;
    /* optional Chamfer subset (null = off): inv (N) = k where inds[k] == p for a
     * duplicate-free inds, else -1; the forward also writes x_out[inds] to xs (K,3)
     * and the backward takes dL/dx_out of p from gsub[inv[p]] (0 off the subset)
     * instead of g, i.e. g = index_add(zeros, inds, gsub) without materialising it */
    const int32_t *inv;
    float *xs;
    const float *gsub;
    /* optional (null = off): the subset gradient as pcr_ndp_chamfer_step leaves
     * it (pcr_ndp_chamfer_gacc_words(K) int64, layout there); read instead of
     * gsub; K = gacc_k */
    const long long *gacc;
    int32_t gacc_k, reserved;
} pcr_ndp_train;
int pcr_ndp_train_forward(const pcr_ndp_train *t, pcr_stream_t stream);
int pcr_ndp_train_backward(const pcr_ndp_train *t, float *part, int32_t chunk,
                           float *const *grads, pcr_stream_t stream);
int64_t pcr_ndp_train_partial_floats(int32_t N, int32_t width, int32_t depth, int32_t chunk);
/* pcr_ndp_chamfer_glue: the loss of registration.py:231-244 around the Chamfer
 *   pass, on the device, in a fixed reduction order:
 *   loss = sum(d1')/K + sum(d2')/M (+ w_reg * mean(-max(log(1 - s), -100)) when s
 *   is given), d' = d where d < trunc else 0; gd1 = 1/K and gd2 = 1/M where not
 *   truncated, else 0 (the dist gradients for pcr_nnd_backward; gd1 / gd2 may be
 *   null);
 *   log[min(*ctr, log_last)] = loss; ++*ctr (device int64). */
int pcr_ndp_chamfer_glue(const float *d1, int32_t K, const float *d2, int32_t M,
                         const float *s, int32_t N, double w_reg, double trunc,
                         float *gd1, float *gd2, float *loss, float *log, int64_t *ctr,
                         int32_t log_last, pcr_stream_t stream);

/* pcr_ndp_chamfer_*: the level's Chamfer pass with its gradient, specialised
 *   for the loop (csrc/ndp_chamfer.hip).  xs (K,3) = x_out[inds] (written by
 *   pcr_ndp_train_forward through inv), tgt (M,3) fixed for the level.
 *   d1/i1 (K), d2/i2 (M): pcr_nnd_forward's outputs bit for bit.  gacc
 *   (pcr_ndp_chamfer_gacc_words(K) = 1 + 6 K R int64, R =
 *   PCR_NDP_GACC_REPLICAS): the gradient of sum(d1')/K + sum(d2')/M w.r.t. xs
 *   (d' = d where d < trunc, else 0), each term exactly in a two-word fixed
 *   point whose exponent s follows the iteration's extents (every integer sum
 *   provably below 2^63): dL/dxs[k][c] = sum over r of
 *   hi[r][k][c] 2^-s + lo[r][k][c] 2^-(s+40), hi at gacc[1 + 3 (r K + k) + c],
 *   lo at gacc[1 + 3 K R + 3 (r K + k) + c]; gacc[0] = ((s + 2048) << 8) | f,
 *   f = 1 when a term was not finite -- consumed by pcr_ndp_train_backward
 *   (pcr_ndp_train.gacc).  K, M <= pcr_ndp_chamfer_max_points() (32768).
 *   scratch: pcr_ndp_chamfer_scratch_bytes(K, M) bytes, 256-byte aligned,
 *   owned by the caller for the level.
 * pcr_ndp_chamfer_prepare: the target grid and the subset cell (from xs0, the
 *   level's input subset) -- with the box path (default; PCR_NC_BOX=0: the grid
 *   path), both clouds' spatial orders and the target's leaf / group boxes;
 *   once per level, outside the captured graph.  The path is read from the
 *   environment by prepare and step alike: keep it unchanged between them.
 * pcr_ndp_chamfer_step: one iteration (gated like the other f4 launches).  The
 *   box path starts each query's search from its answer of the previous call,
 *   read from i1 / i2 before they are overwritten: any value is a valid start
 *   (out-of-range ones count as 0), the results are exact from every start,
 *   only the time depends on it. */
/* pcr_ndp_chamfer_loss: pcr_ndp_chamfer_glue's loss (no dist gradients: the
 *   Chamfer step made them) over 32 workgroups (fixed ranges, partials summed in
 *   block order), then -- when state is given -- pcr_ndp_control's rule on it,
 *   in one launch.  scratch: pcr_ndp_loss_scratch_bytes() bytes, zeroed once
 *   by the caller (the launch leaves it zeroed). */
int64_t pcr_ndp_loss_scratch_bytes(void);
int pcr_ndp_chamfer_loss(const float *d1, int32_t K, const float *d2, int32_t M, const float *s,
                         int32_t N, double w_reg, double trunc, float *loss, float *log, int64_t *ctr,
                         int32_t log_last, double *state, double break_threshold_ratio,
                         int32_t max_break_count, double stop_loss, void *scratch, pcr_stream_t stream);
#define PCR_NDP_GACC_REPLICAS 16
typedef struct pcr_ndp_chamfer {
    const float *xs;
    const float *tgt;
    int32_t K, M;
    double trunc;
    float *d1, *d2;
    int32_t *i1, *i2;
    long long *gacc;
    void *scratch;
} pcr_ndp_chamfer;
int64_t pcr_ndp_chamfer_scratch_bytes(int32_t K, int32_t M);
int64_t pcr_ndp_chamfer_gacc_words(int32_t K);
int32_t pcr_ndp_chamfer_max_points(void);
int pcr_ndp_chamfer_prepare(const pcr_ndp_chamfer *c, const float *xs0, pcr_stream_t stream);
int pcr_ndp_chamfer_step(const pcr_ndp_chamfer *c, pcr_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* PCR_API_H */

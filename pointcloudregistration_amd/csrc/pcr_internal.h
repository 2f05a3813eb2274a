// Internal helpers shared by the libpcr HIP translation units.
// gfx950 (MI355X) only: wave64, 160 KiB LDS/CU, 256 CUs in 8 XCDs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>
#include "../../include/pcr_api.h"

namespace pcr {

// thread-local last-error string, surfaced through pcr_last_error()
void set_error(const char *fmt, ...);
void clear_error();

// Per-device scratch owned by the library.  Grows on demand; superseded buffers
// stay allocated until process exit so kernels still in flight on another
// stream never see their scratch freed.  Mutex-guarded.  *fresh (optional) tells
// whether the buffer was (re)allocated by this call (contents undefined).
void *workspace(int slot, size_t bytes, bool *fresh = nullptr);
// a flag kept beside the calling thread's (device, context) buffer of `slot`
// (false at first): set by an owner whose launches may not all have gone in
bool *workspace_dirty(int slot);

// Chamfer NN (nnd.hip / nnd_grid.hip): the size rule of pcr_nnd_forward, and
// its grid path; _xf forms set 0 as T (x) src (transform_kernel's rounding),
// writing it to xyz1, inside the grid's box pass (max(n, m) <= 32768)
bool nnd_uses_grid(int b, int n, int m);

// pcr_pipeline_step's hook into the feature stage: when
// set, feature_corres_v5 records prep_event on its stream before (at = 2) or
// after (at = 1) the pass-1 launch and calls prep_fn(prep_ctx) there (then
// clears prep_fn), so the side stream's grid builds are enqueued -- and start
// -- at that point, ahead of the feature stage's own side-stream work
extern thread_local hipEvent_t prep_event;
extern thread_local int prep_at;
extern thread_local int (*prep_fn)(void *);
extern thread_local void *prep_ctx;
int nnd_forward_grid(const float *xyz1, const float *xyz2, int b, int n, int m, float *dist1,
                     float *dist2, int32_t *idx1, int32_t *idx2, hipStream_t s);
int nnd_forward_grid_xf(const float *xyz1, const float *src, const double *T, const float *xyz2, int b, int n,
                        int m, float *dist1, float *dist2, int32_t *idx1, int32_t *idx2, hipStream_t s);

inline hipStream_t as_stream(pcr_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

// The side stream of the calling thread's (device, workspace context) and a
// pair of events for fork / join with the caller's stream; created once,
// destroyed by pcr_shutdown.  which = the event pair: 0 the pipeline's grid
// prep, 1 the feature stage's exact row rescan (beside pass 2).  One stream for
// both: a second stream per context moved other streams' hardware queues (the
// process has 4) and cost the s8d job 18 %.  Pair 2 is on a second stream,
// created on its first use: the 3-term screens beside the 1-term regroups.
int side_stream(hipStream_t *s, hipEvent_t *e_in, hipEvent_t *e_out, int which = 0);

// per-kernel HIP-event timing on the launch stream (enabled by pcr_profile_enable)
enum ProfId { kProfFeatScreen = 0, kProfNndFwd = 1, kProfRansacValidate = 2, kProfIcp = 3,
              kProfRansacHyp = 4, kProfFeatRescan = 5, kProfFeatPack = 6, kProfNndGrid = 7,
              kProfFeatScreen2 = 8, kProfFeatScreen1b = 9, kProfFeatScreen2b = 10, kProfFeatRegroup = 11,
              kProfSlots = 12 };
void prof_begin(hipStream_t s, int id);
void prof_end(hipStream_t s, int id);

// f4 early stop: a thread-local gate pointer (pcr_set_gate).  Kernels that an
// NDP level graph captures carry it and return at entry once gate[0] == 0 (the
// level's early-stop rule fired, pcr_ndp_control's state[0]), so the replays
// left after the break do no work.  Null: ungated (every other caller).
const double *current_gate();
__device__ __forceinline__ bool gated_off(const double *g) { return g != nullptr && *g == 0.0; }

constexpr int kWave = 64;
constexpr int kCUs = 256;

}  // namespace pcr

#define PCR_HIP_CHECK(expr)                                                            \
    do {                                                                               \
        hipError_t e_ = (expr);                                                        \
        if (e_ != hipSuccess) {                                                        \
            pcr::set_error("%s failed at %s:%d: %s", #expr, __FILE__, __LINE__,       \
                           hipGetErrorString(e_));                                     \
            return PCR_ERR_HIP;                                                        \
        }                                                                              \
    } while (0)

#define PCR_REQUIRE(cond, code, ...)                                                   \
    do {                                                                               \
        if (!(cond)) {                                                                 \
            pcr::set_error(__VA_ARGS__);                                               \
            return (code);                                                             \
        }                                                                              \
    } while (0)

// PCR_SYNC_CHECK=1 (debug): also synchronise after every checked launch, so a
// kernel fault is reported at its own launch site
namespace pcr { bool sync_check(); }
#define PCR_LAUNCH_CHECK()                                                             \
    do {                                                                               \
        hipError_t e_ = hipGetLastError();                                             \
        if (e_ == hipSuccess && pcr::sync_check()) e_ = hipDeviceSynchronize();        \
        if (e_ != hipSuccess) {                                                        \
            pcr::set_error("kernel launch failed at %s:%d: %s", __FILE__, __LINE__,    \
                           hipGetErrorString(e_));                                     \
            return PCR_ERR_HIP;                                                        \
        }                                                                              \
    } while (0)

// libpcr runtime: thread-local error string, per-device workspace cache.
#include <hip/hip_runtime.h>
#include <cstdarg>
#include <cstdio>
#include <mutex>
#include <vector>
#include "pcr_internal.h"
#include "coop.h"
#include <cstdlib>

namespace pcr {

static thread_local char g_err[1024] = "";

void set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

void clear_error() { g_err[0] = '\0'; }

bool sync_check() {
    static const bool on = [] {
        const char *e = getenv("PCR_SYNC_CHECK");
        return e && e[0] == '1';
    }();
    return on;
}

namespace {
struct Slot {
    void *ptr = nullptr;
    size_t bytes = 0;
    bool dirty = false;  // workspace_dirty: the owner's last use did not complete
};
constexpr int kMaxDevices = 64;
constexpr int kMaxSlots = 40;
constexpr int kMaxCtx = 4;  // workspace contexts (pcr_set_workspace_context)
std::mutex g_mu;
Slot g_slots[kMaxDevices][kMaxCtx][kMaxSlots];
// the calling thread's workspace context: calls that may run concurrently on
// different streams (sub-batches of one step) use different contexts, so no
// scratch buffer is shared between them
thread_local int t_ctx = 0;
// launches sharing the device (pcr_set_concurrency): cooperative grids are sized
// to CUs / g_conc so concurrent ones can all be resident at once
int g_conc = 1;
// superseded buffers: kept until pcr_workspace_release (a graph captured before a
// slot grew still points at its old buffer)
std::vector<std::pair<int, void *>> g_retired;
}  // namespace

bool *workspace_dirty(int slot) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices || slot < 0 || slot >= kMaxSlots)
        return nullptr;
    std::lock_guard<std::mutex> lk(g_mu);
    return &g_slots[dev][t_ctx][slot].dirty;
}

void *workspace(int slot, size_t bytes, bool *fresh) {
    if (fresh) *fresh = false;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices || slot < 0 ||
        slot >= kMaxSlots) {
        set_error("workspace: bad device %d or slot %d", dev, slot);
        return nullptr;
    }
    if (bytes == 0) bytes = 16;
    std::lock_guard<std::mutex> lk(g_mu);
    Slot &s = g_slots[dev][t_ctx][slot];
    if (s.bytes >= bytes) return s.ptr;
    size_t want = bytes + bytes / 4;  // grow with headroom
    want = (want + 4095) & ~size_t(4095);
    void *p = nullptr;
    if (hipMalloc(&p, want) != hipSuccess) {
        (void)hipGetLastError();
        set_error("workspace: hipMalloc(%zu) failed", want);
        return nullptr;
    }
    if (s.ptr) g_retired.emplace_back(dev, s.ptr);
    s.ptr = p;
    s.bytes = want;
    if (fresh) *fresh = true;
    return p;
}

thread_local hipEvent_t prep_event = nullptr;
thread_local int prep_at = 0;
thread_local int (*prep_fn)(void *) = nullptr;
thread_local void *prep_ctx = nullptr;

// ---- side stream of a (device, workspace context) -------------------------
namespace {
struct Side {
    hipStream_t s = nullptr, s2 = nullptr;  // pairs 0, 1 on s; pair 2 on s2
    hipEvent_t e[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
};
Side g_side[kMaxDevices][kMaxCtx];
}  // namespace

int side_stream(hipStream_t *s, hipEvent_t *e_in, hipEvent_t *e_out, int which) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) {
        (void)hipGetLastError();
        set_error("side_stream: no current device");
        return PCR_ERR_HIP;
    }
    if (which < 0 || which > 2) {
        set_error("side_stream: no event pair %d", which);
        return PCR_ERR_ARG;
    }
    std::lock_guard<std::mutex> lk(g_mu);
    Side &d = g_side[dev][t_ctx];
    if (!d.s) {
        bool ok = hipStreamCreateWithFlags(&d.s, hipStreamNonBlocking) == hipSuccess;
        for (int i = 0; i < 6 && ok; ++i) ok = hipEventCreateWithFlags(&d.e[i], hipEventDisableTiming) == hipSuccess;
        if (!ok) {
            (void)hipGetLastError();
            set_error("side_stream: stream / event creation failed");
            return PCR_ERR_HIP;
        }
    }
    if (which == 2 && !d.s2 && hipStreamCreateWithFlags(&d.s2, hipStreamNonBlocking) != hipSuccess) {
        (void)hipGetLastError();
        set_error("side_stream: stream creation failed");
        return PCR_ERR_HIP;
    }
    *s = which == 2 ? d.s2 : d.s;
    *e_in = d.e[2 * which];
    *e_out = d.e[2 * which + 1];
    return PCR_OK;
}

// ---- several workgroups per pair (coop.h) ---------------------------------
int coop_groups(int P, int per_cu, int gmax) {
    if (const char *e = getenv("PCR_COOP_G")) {  // tests: force a split
        const int g = atoi(e);
        if (g >= 1 && g <= 16) return g;
    }
    int dev = 0, cus = 0;
    if (per_cu <= 0 || P <= 0 || hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) {
        (void)hipGetLastError();
        return 1;
    }
    const long cap = (long)per_cu * cus / (g_conc > 1 ? g_conc : 1);
    if ((long)P * 2 > cap) return 1;
    const long g = cap / P;
    return (int)(g > gmax ? gmax : g);
}

int coop_capacity(int per_cu) {
    int dev = 0, cus = 0;
    if (per_cu <= 0 || hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) {
        (void)hipGetLastError();
        return 0;
    }
    return per_cu * cus / (g_conc > 1 ? g_conc : 1);
}

hipError_t coop_launch(const void *fn, int P, int G, int threads, void **args, size_t lds,
                       hipStream_t s) {
    if (G <= 1) return hipLaunchKernel(fn, dim3(P), dim3(threads), args, lds, s);
    return hipLaunchCooperativeKernel(fn, dim3(P * G), dim3(threads), args, (unsigned)lds, s);
}

// ---- optional per-kernel HIP-event timing (pcr_profile_*) -----------------
namespace {
struct ProfRec {
    hipEvent_t b, e;
    int id;
};
std::mutex g_pmu;
bool g_prof_on = false;
std::vector<ProfRec> g_pending;
std::vector<hipEvent_t> g_free;
double g_total_ms[kProfSlots] = {0};
long g_count[kProfSlots] = {0};

hipEvent_t take_event() {
    if (!g_free.empty()) {
        hipEvent_t e = g_free.back();
        g_free.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}
thread_local hipEvent_t t_begin[kProfSlots];
}  // namespace

void prof_begin(hipStream_t s, int id) {
    if (!g_prof_on || id < 0 || id >= kProfSlots) return;
    std::lock_guard<std::mutex> lk(g_pmu);
    hipEvent_t e = take_event();
    if (e && hipEventRecord(e, s) == hipSuccess) t_begin[id] = e;
    else t_begin[id] = nullptr;
}

void prof_end(hipStream_t s, int id) {
    if (!g_prof_on || id < 0 || id >= kProfSlots || !t_begin[id]) return;
    std::lock_guard<std::mutex> lk(g_pmu);
    hipEvent_t e = take_event();
    if (e && hipEventRecord(e, s) == hipSuccess) g_pending.push_back({t_begin[id], e, id});
    t_begin[id] = nullptr;
}

namespace {
thread_local const double *t_gate = nullptr;
}
const double *current_gate() { return t_gate; }

}  // namespace pcr

extern "C" int pcr_set_workspace_context(int32_t ctx) {
    pcr::clear_error();
    PCR_REQUIRE(ctx >= 0 && ctx < pcr::kMaxCtx, PCR_ERR_ARG, "workspace context %d (0..%d)", ctx,
                pcr::kMaxCtx - 1);
    pcr::t_ctx = ctx;
    return PCR_OK;
}

extern "C" int pcr_set_concurrency(int32_t k) {
    pcr::clear_error();
    PCR_REQUIRE(k >= 1 && k <= pcr::kMaxCtx, PCR_ERR_ARG, "concurrency %d (1..%d)", k, pcr::kMaxCtx);
    std::lock_guard<std::mutex> lk(pcr::g_mu);
    pcr::g_conc = k;
    return PCR_OK;
}

extern "C" int pcr_set_gate(const double *gate) {
    pcr::t_gate = gate;
    return PCR_OK;
}

extern "C" void pcr_profile_enable(int32_t on) {
    std::lock_guard<std::mutex> lk(pcr::g_pmu);
    pcr::g_prof_on = on != 0;
}

extern "C" int pcr_profile_read(int32_t id, double *total_ms, int64_t *count, int32_t reset) {
    if (id < 0 || id >= pcr::kProfSlots) return PCR_ERR_ARG;
    std::lock_guard<std::mutex> lk(pcr::g_pmu);
    for (auto &r : pcr::g_pending) {
        float ms = 0.f;
        if (hipEventSynchronize(r.e) != hipSuccess || hipEventElapsedTime(&ms, r.b, r.e) != hipSuccess) {
            pcr::set_error("profile: event query failed");
            return PCR_ERR_HIP;
        }
        pcr::g_total_ms[r.id] += ms;
        pcr::g_count[r.id] += 1;
        pcr::g_free.push_back(r.b);
        pcr::g_free.push_back(r.e);
    }
    pcr::g_pending.clear();
    if (total_ms) *total_ms = pcr::g_total_ms[id];
    if (count) *count = pcr::g_count[id];
    if (reset) { pcr::g_total_ms[id] = 0.0; pcr::g_count[id] = 0; }
    return PCR_OK;
}

extern "C" int pcr_workspace_release(void) {
    pcr::clear_error();
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= pcr::kMaxDevices) {
        pcr::set_error("workspace_release: no current device");
        return PCR_ERR_HIP;
    }
    if (hipDeviceSynchronize() != hipSuccess) {
        pcr::set_error("workspace_release: device synchronize failed");
        return PCR_ERR_HIP;
    }
    std::lock_guard<std::mutex> lk(pcr::g_mu);
    for (auto &ctx : pcr::g_slots[dev])
        for (auto &s : ctx) {
            if (s.ptr) (void)hipFree(s.ptr);
            s.ptr = nullptr;
            s.bytes = 0;
        }
    std::vector<std::pair<int, void *>> keep;
    for (auto &r : pcr::g_retired) {
        if (r.first == dev) (void)hipFree(r.second);
        else keep.push_back(r);
    }
    pcr::g_retired.swap(keep);
    return PCR_OK;
}

// Process-end teardown (round 4): a profiled run (rocprofv3 --kernel-trace) of
// round 3 crashed inside exit() after its last output, in a library finaliser;
// the library's process-lifetime device objects -- workspace slots, retired
// buffers, pooled profiling events, side streams -- were never released and
// outlived the runtime's own teardown.  pcr_shutdown() releases all of them while the runtime
// is intact (Python's atexit runs it first; bench.py also calls it).  Idempotent;
// the library re-allocates on its next call.
extern "C" int pcr_shutdown(void) {
    pcr::clear_error();
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess) { (void)hipGetLastError(); return PCR_OK; }
    int rc = PCR_OK;
    {
        std::lock_guard<std::mutex> lk(pcr::g_pmu);
        pcr::g_prof_on = false;
        for (auto &r : pcr::g_pending) {
            (void)hipEventSynchronize(r.e);
            (void)hipEventDestroy(r.b);
            (void)hipEventDestroy(r.e);
        }
        pcr::g_pending.clear();
        for (hipEvent_t e : pcr::g_free) (void)hipEventDestroy(e);
        pcr::g_free.clear();
    }
    {
        std::lock_guard<std::mutex> lk(pcr::g_mu);
        // a device that cannot be synchronised may still run work on its
        // buffers: its slots and retired buffers are kept
        bool unsynced[pcr::kMaxDevices] = {};
        for (int dev = 0; dev < pcr::kMaxDevices; ++dev) {
            bool any = false;
            for (auto &ctx : pcr::g_slots[dev])
                for (auto &sl : ctx) any = any || sl.ptr;
            for (auto &r : pcr::g_retired) any = any || r.first == dev;
            if (!any) continue;
            if (hipSetDevice(dev) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
                (void)hipGetLastError();
                pcr::set_error("shutdown: device %d not synchronisable", dev);
                rc = PCR_ERR_HIP;
                unsynced[dev] = true;
                continue;
            }
            for (auto &ctx : pcr::g_slots[dev])
                for (auto &sl : ctx) {
                    if (sl.ptr) (void)hipFree(sl.ptr);
                    sl.ptr = nullptr;
                    sl.bytes = 0;
                }
        }
        for (int dev = 0; dev < pcr::kMaxDevices; ++dev)
            for (auto &sd : pcr::g_side[dev]) {
                if (!sd.s) continue;
                if (hipSetDevice(dev) == hipSuccess) {
                    (void)hipStreamSynchronize(sd.s);
                    (void)hipStreamDestroy(sd.s);
                    if (sd.s2) {
                        (void)hipStreamSynchronize(sd.s2);
                        (void)hipStreamDestroy(sd.s2);
                    }
                    for (hipEvent_t e : sd.e)
                        if (e) (void)hipEventDestroy(e);
                }
                sd = pcr::Side{};
            }
        std::vector<std::pair<int, void *>> keep;
        for (auto &r : pcr::g_retired) {
            if (!unsynced[r.first] && hipSetDevice(r.first) == hipSuccess) (void)hipFree(r.second);
            else keep.push_back(r);
        }
        pcr::g_retired.swap(keep);
    }
    (void)hipSetDevice(cur);
    (void)hipGetLastError();
    return rc;
}

extern "C" const char *pcr_last_error(void) { return pcr::g_err; }
extern "C" int pcr_version(void) { return 1; }

// libpcr runtime: thread-local error string, per-device workspace cache.
#include <hip/hip_runtime.h>
#include <cstdarg>
#include <cstdio>
#include <mutex>
#include <vector>
#include "pcr_internal.h"

namespace pcr {

static thread_local char g_err[1024] = "";

void set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

void clear_error() { g_err[0] = '\0'; }

namespace {
struct Slot {
    void *ptr = nullptr;
    size_t bytes = 0;
};
constexpr int kMaxDevices = 64;
constexpr int kMaxSlots = 32;
std::mutex g_mu;
Slot g_slots[kMaxDevices][kMaxSlots];
std::vector<void *> g_retired;  // superseded buffers, freed never (process lifetime)
}  // namespace

void *workspace(int slot, size_t bytes) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices || slot < 0 ||
        slot >= kMaxSlots) {
        set_error("workspace: bad device %d or slot %d", dev, slot);
        return nullptr;
    }
    if (bytes == 0) bytes = 16;
    std::lock_guard<std::mutex> lk(g_mu);
    Slot &s = g_slots[dev][slot];
    if (s.bytes >= bytes) return s.ptr;
    size_t want = bytes + bytes / 4;  // grow with headroom
    want = (want + 4095) & ~size_t(4095);
    void *p = nullptr;
    if (hipMalloc(&p, want) != hipSuccess) {
        (void)hipGetLastError();
        set_error("workspace: hipMalloc(%zu) failed", want);
        return nullptr;
    }
    if (s.ptr) g_retired.push_back(s.ptr);
    s.ptr = p;
    s.bytes = want;
    return p;
}

}  // namespace pcr

extern "C" const char *pcr_last_error(void) { return pcr::g_err; }
extern "C" int pcr_version(void) { return 1; }

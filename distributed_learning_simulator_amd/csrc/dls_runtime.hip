// Host-side runtime pieces of libdls_hip.so: error state, version, device query.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "dls_common.h"

namespace dls {

static thread_local std::string g_last_error;

void set_error(const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
}

int check_launch(const char *what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("%s: launch failed: %s", what, hipGetErrorString(e));
        return (int)e;
    }
    return DLS_OK;
}

int resident_blocks(const void *kernel, int block, size_t lds) {
    // (kernel, device) -> blocks per CU x CUs; cached: the occupancy query costs
    // microseconds and the launch functions run on every aggregation
    static std::mutex mu;
    static std::unordered_map<std::string, int> cache;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    char key[96];
    snprintf(key, sizeof(key), "%p/%d/%d/%zu", kernel, dev, block, lds);
    {
        std::lock_guard<std::mutex> g(mu);
        auto it = cache.find(key);
        if (it != cache.end()) return it->second;
    }
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, block, lds) != hipSuccess ||
        per_cu < 1)
        per_cu = 1;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus < 1)
        cus = 256;
    const int n = per_cu * cus;
    std::lock_guard<std::mutex> g(mu);
    cache[key] = n;
    return n;
}

int device_cus() {
    static std::mutex mu;
    static std::unordered_map<int, int> cache;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    std::lock_guard<std::mutex> g(mu);
    auto it = cache.find(dev);
    if (it != cache.end()) return it->second;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus < 1)
        cus = 256;
    cache[dev] = cus;
    return cus;
}

hipStream_t side_stream(hipStream_t parent, int idx) {
    // non-blocking streams per (device, idx), created on first use and kept for the
    // process (the library's launchers fork small concurrent kernels onto it and
    // join back to the caller's stream before returning).  The device is the
    // parent stream's, not the calling thread's current device: worker threads
    // may launch on tensors of another GPU than the one they have selected.
    static std::mutex mu;
    static std::unordered_map<int, hipStream_t> streams;
    int dev = 0;
    if (hipStreamGetDevice(parent, &dev) != hipSuccess) return nullptr;
    const int key = dev * 64 + idx;
    std::lock_guard<std::mutex> g(mu);
    auto it = streams.find(key);
    if (it != streams.end()) return it->second;
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess) return nullptr;
    if (cur != dev && hipSetDevice(dev) != hipSuccess) return nullptr;
    hipStream_t s = nullptr;
    const hipError_t e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    if (cur != dev) (void)hipSetDevice(cur);
    if (e != hipSuccess) return nullptr;
    streams[key] = s;
    return s;
}

hipEvent_t call_event(hipStream_t parent, int idx) {
    // keyed by the parent stream: calls on one stream are ordered, so re-recording
    // the same event for the next call is safe (a wait binds to the record that
    // precedes it); calls on different streams use different events
    static std::mutex mu;
    static std::unordered_map<std::string, hipEvent_t> events;
    char key[64];
    snprintf(key, sizeof(key), "%p/%d", (void *)parent, idx);
    std::lock_guard<std::mutex> g(mu);
    auto it = events.find(key);
    if (it != events.end()) return it->second;
    int dev = 0, cur = 0;
    if (hipStreamGetDevice(parent, &dev) != hipSuccess || hipGetDevice(&cur) != hipSuccess)
        return nullptr;
    if (cur != dev && hipSetDevice(dev) != hipSuccess) return nullptr;
    hipEvent_t e = nullptr;
    const hipError_t rc = hipEventCreateWithFlags(&e, hipEventDisableTiming);
    if (cur != dev) (void)hipSetDevice(cur);
    if (rc != hipSuccess) return nullptr;
    events[key] = e;
    return e;
}

// One block of mantissas; `target` lets the compiler vectorise the fma / div
// (the box's and this container's hosts are AVX-512 EPYC / Xeon parts).
__attribute__((target("avx2,fma"))) static bool two_constant_block(uint32_t m0, uint32_t n, float b,
                                                                  float yh, float yl) {
    int bad = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t u = 0x3f800000u | (m0 + i);
        float a;
        memcpy(&a, &u, 4);
        const float q = __builtin_fmaf(a, yh, a * yl);
        bad |= (q != a / b);
    }
    return bad == 0;
}

static std::mutex g_two_mu;
static std::unordered_map<uint32_t, bool> g_two_cache;

bool two_constant_exact(float b, float yh, float yl) {
    std::mutex &mu = g_two_mu;
    std::unordered_map<uint32_t, bool> &cache = g_two_cache;
    uint32_t key;
    memcpy(&key, &b, 4);
    {
        std::lock_guard<std::mutex> g(mu);
        auto it = cache.find(key);
        if (it != cache.end()) return it->second;
    }
    bool ok = true;
    for (uint32_t m0 = 0; ok && m0 < (1u << 23); m0 += 4096) ok = two_constant_block(m0, 4096, b, yh, yl);
    std::lock_guard<std::mutex> g(mu);
    cache[key] = ok;
    return ok;
}

void prove_two_constant(const float *b, int n) {
    std::vector<float> todo;
    {
        std::lock_guard<std::mutex> g(g_two_mu);
        for (int i = 0; i < n; ++i) {
            uint32_t key;
            memcpy(&key, &b[i], 4);
            const FastDiv d = make_fastdiv(b[i]);
            if (d.fast && g_two_cache.find(key) == g_two_cache.end()) todo.push_back(b[i]);
        }
    }
    if (todo.size() < 2) return;  // make_fastdiv2 does a single one itself
    const int nt = (int)std::min<size_t>(todo.size(), std::max(1u, std::thread::hardware_concurrency()));
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t)
        th.emplace_back([&, t] {
            for (size_t i = t; i < todo.size(); i += nt) (void)make_fastdiv2(todo[i]);
        });
    for (auto &x : th) x.join();
}

}  // namespace dls

extern "C" {

int dls_two_constant_division(float divisor) { return dls::make_fastdiv2(divisor).two; }


const char *dls_last_error(void) { return dls::g_last_error.c_str(); }

#ifndef DLS_SOURCE_HASH
#define DLS_SOURCE_HASH "unknown"
#endif
const char *dls_source_hash(void) { return DLS_SOURCE_HASH; }

int dls_abi_version(void) { return DLS_ABI_VERSION; }

int dls_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

}  // extern "C"

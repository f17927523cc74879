// Host-side runtime pieces of libdls_hip.so: error state, version, device query.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <mutex>
#include <string>
#include <unordered_map>

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

hipStream_t side_stream() {
    // one non-blocking stream per device, created on first use and kept for the
    // process (the library's launchers fork small concurrent kernels onto it and
    // join back to the caller's stream before returning)
    static std::mutex mu;
    static std::unordered_map<int, hipStream_t> streams;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> g(mu);
    auto it = streams.find(dev);
    if (it != streams.end()) return it->second;
    hipStream_t s = nullptr;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return nullptr;
    streams[dev] = s;
    return s;
}

}  // namespace dls

extern "C" {

const char *dls_last_error(void) { return dls::g_last_error.c_str(); }

int dls_abi_version(void) { return DLS_ABI_VERSION; }

int dls_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

}  // extern "C"

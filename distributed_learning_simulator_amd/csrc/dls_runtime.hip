// Host-side runtime pieces of libdls_hip.so: error state, version, device query.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <string>

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

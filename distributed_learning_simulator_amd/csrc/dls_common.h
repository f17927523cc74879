// Shared device/host helpers for libdls_hip.so (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdarg>
#include <cstdio>
#include <string>

#include "../../include/dls_hip.h"

namespace dls {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

// ------------------------------------------------------------------ errors
void set_error(const char *fmt, ...);

#define DLS_REQUIRE(cond, code, ...)        \
    do {                                    \
        if (!(cond)) {                      \
            ::dls::set_error(__VA_ARGS__);  \
            return (code);                  \
        }                                   \
    } while (0)

// Launch-error check after a hipLaunchKernelGGL (asynchronous errors surface
// at the caller's next synchronisation).
int check_launch(const char *what);

// Blocks of `kernel` resident on the whole device at once (occupancy x CUs),
// for persistent grids; cached per (kernel, device, block, lds).
int resident_blocks(const void *kernel, int block, size_t lds);
// Compute units of the current device (cached per device).
int device_cus();
// Auxiliary stream number idx (0..63) on `parent`'s device for fork/join inside
// one C-ABI call (nullptr on error).
hipStream_t side_stream(hipStream_t parent, int idx);
// Fork / join events of one C-ABI call on `parent` (idx 0: the fork, 1..: the
// joins), created on first use and kept per (parent stream, idx), so a call
// allocates nothing; nullptr on error.
hipEvent_t call_event(hipStream_t parent, int idx);
// FMA mode of dls_dequant_fedavg_mode: the tiles of table groups 0-9 in launch
// pieces of one wave per SIMD (quant_fma.hip; groups 8-9 exact).
int launch_dequant_fma_stream(const dls_qtile *tiles, const int32_t *nfast, const void *Q,
                              int64_t ldq, const float *F, int64_t ldf, const float *sz,
                              int64_t sz_row, int64_t sz_chan, const int32_t *rows, const float *w,
                              int32_t K, float N, float *out, hipStream_t st);

inline hipStream_t as_stream(dls_stream_t s) { return reinterpret_cast<hipStream_t>(s); }
inline bool aligned16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// --------------------------------------------------------- exact fp32 division
// The reference divides fl32(p*n) by fl32(N) (servers/fed_server.py:59-60) with
// one IEEE rounding.  On gfx950 the compiler's correctly rounded division is a
// ~10-instruction v_div_scale/v_rcp/v_fma/v_div_fmas/v_div_fixup sequence; the
// streaming kernels instead use Markstein's correction with y = RN(1/b):
//     q0 = a*y ; r = fma(-q0, b, a) ; q = fma(r, y, q0)
// which equals RN(a/b) whenever a, b and every intermediate stay in the normal
// range.  Floating-point ops are scale-invariant there, so checking every fp32
// mantissa of a in [1,2) proves it for one b; tests/test_oracle_golden.py does
// that exhaustively for adversarial divisors (and 6,000+ more were checked while
// building).  The kernels take the fast path for 2^-60 <= |a| <= 2^60 and
// 1 <= b <= 2^31 (host side: `fast`) and fall back to IEEE `/` otherwise
// (zeros incl. -0, denormals, inf, nan, huge values).
//
// Two-constant variant (Brisebarre, Muller & Raina, IEEE TC 2004): with
// yh = RN(1/b), yl = RN(1/b - yh),  q = fma(a, yh, RN(a*yl))  is RN(a/b) for
// every a for MOST divisors b (2 ops instead of 3).  Whether it holds for one b
// is decided on the host by the same exhaustive mantissa check
// (`two_constant_exact`, cached per b); `two` is set only when it passed and
// a*yl stays normal over the fast range.
struct FastDiv {
    float b;
    float y;
    int fast;
    float yl;
    int two;
};

inline FastDiv make_fastdiv(float b) {
    FastDiv d;
    d.b = b;
    d.y = (float)(1.0 / (double)b);  // RN(1/b): double rounding is innocuous for '/'
    d.fast = (b >= 1.0f && b <= 2147483648.0f) ? 1 : 0;
    d.yl = 0.f;
    d.two = 0;
    return d;
}

// Exhaustive check of the two-constant division for divisor b (every fp32
// mantissa of a in [1,2)); thread-safe, memoised per b (~ms on first use).
bool two_constant_exact(float b, float yh, float yl);
// Run the checks of the not yet memoised divisors among b[0..n) in parallel
// (host threads), so that make_fastdiv2 on each of them is then a cache hit.
void prove_two_constant(const float *b, int n);

inline FastDiv make_fastdiv2(float b) {
    FastDiv d = make_fastdiv(b);
    if (!d.fast) return d;
    d.yl = (float)(1.0 / (double)b - (double)d.y);
    // fast-range a >= 2^-60: a*yl normal needs |yl| >= 2^-66 (yl == 0: b = 2^k)
    const bool normal = d.yl == 0.f || (d.yl >= 0x1p-66f || d.yl <= -0x1p-66f);
    d.two = (normal && two_constant_exact(b, d.y, d.yl)) ? 1 : 0;
    return d;
}

__device__ __forceinline__ float div_two(float a, const FastDiv &d) {
    return __builtin_fmaf(a, d.y, a * d.yl);
}

__device__ __forceinline__ float markstein(float a, float b, float y) {
    const float q0 = a * y;
    const float r = __builtin_fmaf(-q0, b, a);
    return __builtin_fmaf(r, y, q0);
}

// 1 if 2^-60 <= |a| <= 2^60 (fast path valid), else 0.  Two VALU ops.
__device__ __forceinline__ bool in_fast_range(float a) {
    const uint32_t e = (__float_as_uint(a) >> 23) & 0xffu;  // biased exponent
    return (e - (127u - 60u)) <= 120u;
}

// Division with the rare-path fix-up hoisted out of the common case: returns
// false when the caller must redo the element with IEEE division.
__device__ __forceinline__ float div_fast(float a, const FastDiv &d) {
    return markstein(a, d.b, d.y);
}

__device__ __forceinline__ float div_ieee(float a, float b) {
    return a / b;  // hipcc default: correctly rounded fp32 division
}

// Guarded exact division (one element).
__device__ __forceinline__ float div_exact(float a, const FastDiv &d) {
    if (d.fast && in_fast_range(a)) return markstein(a, d.b, d.y);
    return a / d.b;
}

// ------------------------------------------------------------- misc device
__device__ __forceinline__ int lane_id() { return __lane_id(); }

template <typename T>
__device__ __forceinline__ T ldg_nt(const T *p) {
    return __builtin_nontemporal_load(p);
}

}  // namespace dls

// Exhaustive check (all 2^32 fp32 bit patterns) that gfx950's v_cvt_pk_bf16_f32
// (what __builtin_convertvector(float2 -> bf16x2) compiles to) equals the
// integer round-to-nearest-even of csrc/conv.hip's bf16_rne, which keeps a NaN's
// sign and top payload and sets the quiet bit.  Counts mismatches among non-NaN
// inputs and among NaN inputs (and NaN outputs that are not NaN).
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/bf16_cvt_probe.hip -o tools/_bf16_cvt_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
typedef __attribute__((ext_vector_type(2))) float f32x2;

__device__ __forceinline__ uint32_t rne_int(float x) {
    const uint32_t u = __float_as_uint(x);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (u >> 16) | 0x40u;
    return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}

__global__ void k_probe(unsigned long long *cnt, uint32_t *first) {
    unsigned long long bad_num = 0, bad_nan = 0, nan_not_nan = 0;
    const uint64_t n = 1ull << 32, step = (uint64_t)gridDim.x * blockDim.x * 2;
    for (uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 2; i < n; i += step) {
        const float a = __uint_as_float((uint32_t)i), b = __uint_as_float((uint32_t)(i + 1));
        const uint32_t hw = __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{a, b}, bf16x2));
        const uint32_t h0 = hw & 0xffffu, h1 = hw >> 16;
        const uint32_t r0 = rne_int(a), r1 = rne_int(b);
        const bool n0 = a != a, n1 = b != b;
        if (h0 != r0) {
            if (n0) ++bad_nan; else { ++bad_num; first[0] = (uint32_t)i; }
            if (n0 && ((h0 & 0x7fffu) <= 0x7f80u)) ++nan_not_nan;
        }
        if (h1 != r1) {
            if (n1) ++bad_nan; else { ++bad_num; first[1] = (uint32_t)(i + 1); }
            if (n1 && ((h1 & 0x7fffu) <= 0x7f80u)) ++nan_not_nan;
        }
    }
    atomicAdd(&cnt[0], bad_num);
    atomicAdd(&cnt[1], bad_nan);
    atomicAdd(&cnt[2], nan_not_nan);
}

int main() {
    unsigned long long *cnt;
    uint32_t *first;
    if (hipMalloc(&cnt, 3 * sizeof(unsigned long long)) != hipSuccess || hipMalloc(&first, 8) != hipSuccess) return 1;
    (void)hipMemset(cnt, 0, 3 * sizeof(unsigned long long));
    (void)hipMemset(first, 0xff, 8);
    hipLaunchKernelGGL(k_probe, dim3(4096), dim3(256), 0, 0, cnt, first);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    unsigned long long h[3];
    uint32_t f[2];
    (void)hipMemcpy(h, cnt, sizeof h, hipMemcpyDeviceToHost);
    (void)hipMemcpy(f, first, sizeof f, hipMemcpyDeviceToHost);
    printf("all 2^32 fp32 patterns: v_cvt_pk_bf16_f32 vs integer RNE: non-NaN mismatches %llu, NaN mismatches %llu "
           "(NaN -> non-NaN %llu); a non-NaN mismatch: 0x%08x 0x%08x\n", h[0], h[1], h[2], f[0], f[1]);
    (void)hipFree(cnt);
    (void)hipFree(first);
    return h[0] == 0 ? 0 : 3;
}

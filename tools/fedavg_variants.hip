// Development tool: time FedAvg-kernel variants on one MI355X (not product code).
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off tools/fedavg_variants.hip -o tools/fedavg_variants
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "../distributed_learning_simulator_amd/csrc/dls_common.h"

using namespace dls;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <bool NT> __device__ __forceinline__ f32x4 ld(const f32x4 *p) {
    if constexpr (NT) return __builtin_nontemporal_load(p); else return *p; }

__device__ __forceinline__ f32x4 term4(f32x4 x, float w, const FastDiv &d) {
    f32x4 t = x * w, q;
    for (int c = 0; c < 4; ++c) q[c] = markstein(t[c], d.b, d.y);
    bool ok = d.fast;
    for (int c = 0; c < 4; ++c) ok &= in_fast_range(t[c]);
    if (__builtin_expect(!ok, 0))
        for (int c = 0; c < 4; ++c) q[c] = (d.fast && in_fast_range(t[c])) ? q[c] : t[c] / d.b;
    return q;
}

// V (VEC float4 per thread, strided by blockDim), UNROLL clients in flight
template <int UNROLL, int VEC, bool NT, bool DIV>
__global__ __launch_bounds__(256) void kv(const f32x4 *__restrict__ U, int64_t ldu4, const int *__restrict__ rows,
                                          const float *__restrict__ w, int K, FastDiv d, int64_t P4, f32x4 *__restrict__ out) {
    const int64_t i0 = (int64_t)blockIdx.x * 256 * VEC + threadIdx.x;
    f32x4 acc[VEC];
    for (int v = 0; v < VEC; ++v) acc[v] = f32x4{0, 0, 0, 0};
    for (int j = 0; j < K; j += UNROLL) {
        f32x4 x[UNROLL][VEC];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
#pragma unroll
            for (int v = 0; v < VEC; ++v) {
                int64_t i = i0 + v * 256;
                x[u][v] = (j + u < K && i < P4) ? ld<NT>(U + (int64_t)rows[j + u] * ldu4 + i) : f32x4{0, 0, 0, 0};
            }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
#pragma unroll
            for (int v = 0; v < VEC; ++v) {
                if (DIV) acc[v] = (j + u == 0) ? term4(x[u][v], w[j + u], d) : acc[v] + term4(x[u][v], w[j + u], d);
                else acc[v] += x[u][v];
            }
    }
    for (int v = 0; v < VEC; ++v) { int64_t i = i0 + v * 256; if (i < P4) out[i] = acc[v]; }
}

template <int UNROLL, int VEC, bool NT, bool DIV>
void run(const char *name, const f32x4 *U, int64_t ldu4, const int *rows, const float *w, int K, FastDiv d, int64_t P4, f32x4 *out) {
    dim3 grid((unsigned)((P4 + 256 * VEC - 1) / (256 * VEC)));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((kv<UNROLL, VEC, NT, DIV>), grid, dim3(256), 0, 0, U, ldu4, rows, w, K, d, P4, out);
    CK(hipDeviceSynchronize());
    const int R = 20;
    CK(hipEventRecord(a));
    for (int i = 0; i < R; ++i) hipLaunchKernelGGL((kv<UNROLL, VEC, NT, DIV>), grid, dim3(256), 0, 0, U, ldu4, rows, w, K, d, P4, out);
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b)); ms /= R;
    double bytes = (double)K * P4 * 16 + P4 * 16;
    printf("%-34s %8.3f ms  %7.1f GB/s\n", name, ms, bytes / ms / 1e6);
}

int main() {
    const int K = 100; const int64_t P = 11174016, P4 = P / 4;
    f32x4 *U, *out; int *rows; float *w;
    CK(hipMalloc(&U, (size_t)K * P * 4)); CK(hipMalloc(&out, P * 4));
    CK(hipMalloc(&rows, K * 4)); CK(hipMalloc(&w, K * 4));
    std::vector<int> hr(K); std::vector<float> hw(K); double tot = 0;
    for (int k = 0; k < K; ++k) { hr[k] = k; hw[k] = 100 + 7 * k % 900; tot += hw[k]; }
    CK(hipMemcpy(rows, hr.data(), K * 4, hipMemcpyHostToDevice)); CK(hipMemcpy(w, hw.data(), K * 4, hipMemcpyHostToDevice));
    std::vector<float> hu(P); for (int64_t e = 0; e < P; ++e) hu[e] = 0.01f * (float)((e * 2654435761u) % 1000) - 5.f;
    for (int k = 0; k < K; ++k) CK(hipMemcpy((float *)U + (size_t)k * P, hu.data(), P * 4, hipMemcpyHostToDevice));
    FastDiv d = make_fastdiv((float)tot);
    run<8, 1, true, true>("exact u8 v1 nt (product)", U, P4, rows, w, K, d, P4, out);
    run<16, 1, true, true>("exact u16 v1 nt", U, P4, rows, w, K, d, P4, out);
    run<4, 1, true, true>("exact u4 v1 nt", U, P4, rows, w, K, d, P4, out);
    run<8, 1, false, true>("exact u8 v1 plain", U, P4, rows, w, K, d, P4, out);
    run<8, 2, true, true>("exact u8 v2 nt", U, P4, rows, w, K, d, P4, out);
    run<4, 2, true, true>("exact u4 v2 nt", U, P4, rows, w, K, d, P4, out);
    run<4, 4, true, true>("exact u4 v4 nt", U, P4, rows, w, K, d, P4, out);
    run<8, 1, true, false>("sum-only u8 v1 nt (read ceiling)", U, P4, rows, w, K, d, P4, out);
    run<16, 1, true, false>("sum-only u16 v1 nt", U, P4, rows, w, K, d, P4, out);
    run<8, 2, false, false>("sum-only u8 v2 plain", U, P4, rows, w, K, d, P4, out);
    run<8, 1, true, true>("exact u8 v1 nt (product, again)", U, P4, rows, w, K, d, P4, out);
    return 0;
}

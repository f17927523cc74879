// VALU issue-rate probe: packed fp32 (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32)
// vs scalar fp32 (v_fma_f32 ...) on gfx950, many independent chains per lane,
// every CU busy.  Prints lane-ops/s for each form; if a packed op issues at the
// same cost as one scalar op it doubles the fp32 rate, if at twice it is neutral.
//   hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize tools/valu_rate_probe.hip -o tools/_valu_rate_probe
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f32x2 __attribute__((ext_vector_type(2)));
constexpr int kChains = 8;
constexpr int kIters = 4096;

__global__ __launch_bounds__(256) void k_scalar_fma(float *out, float a, float b) {
    float x[2 * kChains];
#pragma unroll
    for (int c = 0; c < 2 * kChains; ++c) x[c] = threadIdx.x * 1e-3f + c;
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int c = 0; c < 2 * kChains; ++c) x[c] = __builtin_fmaf(x[c], a, b);
    }
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < 2 * kChains; ++c) s += x[c];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_pk_fma(float *out, float a, float b) {
    f32x2 x[kChains];
    const f32x2 a2 = {a, a}, b2 = {b, b};
#pragma unroll
    for (int c = 0; c < kChains; ++c) x[c] = f32x2{threadIdx.x * 1e-3f + c, threadIdx.x * 1e-3f - c};
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int c = 0; c < kChains; ++c) x[c] = __builtin_elementwise_fma(x[c], a2, b2);
    }
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < kChains; ++c) s += x[c].x + x[c].y;
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_pk_add(float *out, float a, float b) {
    f32x2 x[kChains];
    const f32x2 a2 = {a, a};
#pragma unroll
    for (int c = 0; c < kChains; ++c) x[c] = f32x2{threadIdx.x * 1e-3f + c, b - c};
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int c = 0; c < kChains; ++c) x[c] = x[c] + a2;
    }
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < kChains; ++c) s += x[c].x + x[c].y;
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_scalar_add(float *out, float a, float b) {
    float x[2 * kChains];
#pragma unroll
    for (int c = 0; c < 2 * kChains; ++c) x[c] = threadIdx.x * 1e-3f + c + b;
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int c = 0; c < 2 * kChains; ++c) x[c] = x[c] + a;
    }
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < 2 * kChains; ++c) s += x[c];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <class K>
static void run(const char *name, K kern, float *out, int blocks) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, 1.0000001f, 1e-7f);
    hipEventRecord(e0);
    const int reps = 5;
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, 1.0000001f, 1e-7f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    const double lane_ops = (double)reps * blocks * 256 * kIters * 2 * kChains;
    printf("%-12s %8.3f ms  %7.2f T lane-op/s (fma counted as 1 op)\n", name, ms / reps,
           lane_ops / (ms / 1e3) / 1e12);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int blocks = cus * 16;  // 16 waves... x4 per block: plenty per SIMD
    float *out = nullptr;
    if (hipMalloc(&out, (size_t)blocks * 256 * sizeof(float)) != hipSuccess) return 1;
    printf("CUs %d, blocks %d x 256 threads, %d independent chains x %d iters\n", cus, blocks,
           2 * kChains, kIters);
    for (int rep = 0; rep < 2; ++rep) {
        run("scalar_fma", k_scalar_fma, out, blocks);
        run("pk_fma", k_pk_fma, out, blocks);
        run("scalar_add", k_scalar_add, out, blocks);
        run("pk_add", k_pk_add, out, blocks);
    }
    hipFree(out);
    return 0;
}

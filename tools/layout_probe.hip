// Probe: HBM read rate of the fed_quant access pattern vs the payload layout.
//   client-major  Q[k][i]                      (the store's layout today)
//   blocked       Q[i / 4096][k][i % 4096]     (each wave's 4 KiB tile of all K
//                                               clients is one contiguous run)
// A wave owns one 4 KiB tile and walks the K clients (U clients in flight),
// xor-reducing the bytes (negligible VALU) — the memory stream of
// k_dequant_fast<4> without its arithmetic.
//   hipcc --offload-arch=gfx950 -O3 -o tools/_layout_probe tools/layout_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <bool BLOCKED, int U>
__global__ __launch_bounds__(256) void k_stream(const uint8_t *__restrict__ Q, int64_t ldq, int K,
                                                int ntiles, uint32_t *__restrict__ out) {
    const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (t >= ntiles) return;
    const int lane = threadIdx.x & 63;
    u32x4 acc = {0, 0, 0, 0};
    auto addr = [&](int k, int s) -> const u32x4 * {
        const int64_t off = BLOCKED ? ((int64_t)t * K + k) * 4096 : (int64_t)k * ldq + (int64_t)t * 4096;
        return reinterpret_cast<const u32x4 *>(Q + off + s * 1024 + lane * 16);
    };
    for (int k0 = 0; k0 < K; k0 += U) {
        u32x4 v[U][4];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int s = 0; s < 4; ++s) v[u][s] = __builtin_nontemporal_load(addr(min(k0 + u, K - 1), s));
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int s = 0; s < 4; ++s) acc ^= v[u][s];
    }
    out[(int64_t)t * 64 + lane] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
// The same stream with k_dequant_fast's per-element arithmetic (cvt, 4 packed
// fp32 ops + add per element pair) into G*16 fp32 accumulators per lane.
template <int G, int LDSKB>
__global__ __launch_bounds__(256) void k_compute(const uint8_t *__restrict__ Q, int64_t ldq, int K,
                                                 int ntiles, float s, float w, float y, float yl,
                                                 float *__restrict__ out) {
    extern __shared__ float pad[];
    const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (t >= ntiles * 4 / G) return;
    const int lane = threadIdx.x & 63;
    float acc[G][16];
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[g][e] = -0.f;
    const f32x2 s2 = {s, s}, w2 = {w, w}, y2 = {y, y}, yl2 = {yl, yl}, nz = {-s, -s};
    auto ld = [&](int k, u32x4 (&v)[G]) {
#pragma unroll
        for (int g = 0; g < G; ++g)
            v[g] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(
                Q + (int64_t)k * ldq + (int64_t)t * 1024 * G + g * 1024 + lane * 16));
    };
    auto step = [&](const u32x4 (&v)[G], float kk) {
        const f32x2 k2 = {kk, kk};
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int j = 0; j < 16; j += 2) {
                const f32x2 x = {(float)(int8_t)(v[g][j >> 2] >> (8 * (j & 3))),
                                 (float)(int8_t)(v[g][j >> 2] >> (8 * ((j + 1) & 3)))};
                const f32x2 d = __builtin_elementwise_fma(x, s2, nz);
                const f32x2 tt = d * (w2 + k2);
                const f32x2 q = __builtin_elementwise_fma(tt, y2, tt * yl2);
                const f32x2 r = f32x2{acc[g][j], acc[g][j + 1]} + q;
                acc[g][j] = r.x;
                acc[g][j + 1] = r.y;
                if ((j / 2) % 2 == 1) __builtin_amdgcn_sched_barrier(0);
            }
    };
    u32x4 a[G], b[G];
    ld(0, a);
    int k = 0;
    for (; k + 2 < K; k += 2) {
        ld(k + 1, b);
        step(a, (float)k);
        ld(k + 2, a);
        step(b, (float)k + 1);
    }
    for (; k < K; ++k) {
        ld(k, a);
        step(a, (float)k);
    }
    if (LDSKB) pad[threadIdx.x] = acc[0][0];
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int e = 0; e < 16; e += 4)
            *reinterpret_cast<float __attribute__((ext_vector_type(4))) *>(
                out + (int64_t)t * 1024 * G + g * 1024 + lane * 16 + e) =
                {acc[g][e], acc[g][e + 1], acc[g][e + 2], acc[g][e + 3]};
}

template <int G, int LDSKB>
float runc(const uint8_t *Q, int64_t ldq, int K, int ntiles, float *out) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int waves = ntiles * 4 / G;
    const dim3 grid((waves + 3) / 4);
    const size_t lds = LDSKB * 1024;
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((k_compute<G, LDSKB>), grid, dim3(256), lds, 0, Q, ldq, K, ntiles, 1e-3f, 500.f, 1.8e-5f, 1e-12f, out);
    hipEventRecord(a);
    const int reps = 10;
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((k_compute<G, LDSKB>), grid, dim3(256), lds, 0, Q, ldq, K, ntiles, 1e-3f, 500.f, 1.8e-5f, 1e-12f, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms / reps;
}

template <bool B, int U>
float run(const uint8_t *Q, int64_t ldq, int K, int ntiles, uint32_t *out) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const dim3 grid((ntiles + 3) / 4);
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((k_stream<B, U>), grid, dim3(256), 0, 0, Q, ldq, K, ntiles, out);
    hipEventRecord(a);
    const int reps = 10;
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((k_stream<B, U>), grid, dim3(256), 0, 0, Q, ldq, K, ntiles, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms / reps;
}

int main() {
    const int K = 100;
    const int ntiles = 33774;  // 138.3 MB per client
    const int64_t ldq = (int64_t)ntiles * 4096;
    uint8_t *Q;
    uint32_t *out;
    float *fo;
    if (hipMalloc(&Q, ldq * K) != hipSuccess || hipMalloc(&out, (size_t)ntiles * 256) != hipSuccess ||
        hipMalloc(&fo, (size_t)ntiles * 4096 * 4) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    hipMemset(Q, 1, ldq * K);
    const double bytes = (double)ldq * K;
    for (int rep = 0; rep < 2; ++rep) {
        float m;
        m = runc<4, 0>(Q, ldq, K, ntiles, fo); printf("compute G=4         %.3f ms %.0f GB/s\n", m, bytes / m / 1e6);
        m = runc<1, 0>(Q, ldq, K, ntiles, fo); printf("compute G=1         %.3f ms %.0f GB/s\n", m, bytes / m / 1e6);
        m = runc<2, 0>(Q, ldq, K, ntiles, fo); printf("compute G=2         %.3f ms %.0f GB/s\n", m, bytes / m / 1e6);
        m = runc<1, 36>(Q, ldq, K, ntiles, fo); printf("compute G=1 occ<=4  %.3f ms %.0f GB/s\n", m, bytes / m / 1e6);
        m = runc<1, 70>(Q, ldq, K, ntiles, fo); printf("compute G=1 occ<=2  %.3f ms %.0f GB/s\n", m, bytes / m / 1e6);
        m = run<false, 1>(Q, ldq, K, ntiles, out); printf("client-major U=1 %.3f ms %.0f GB/s\n", m, bytes / m / 1e6);
        m = run<true, 1>(Q, ldq, K, ntiles, out);  printf("blocked      U=1 %.3f ms %.0f GB/s\n", m, bytes / m / 1e6);
        m = run<false, 2>(Q, ldq, K, ntiles, out); printf("client-major U=2 %.3f ms %.0f GB/s\n", m, bytes / m / 1e6);
        m = run<true, 2>(Q, ldq, K, ntiles, out);  printf("blocked      U=2 %.3f ms %.0f GB/s\n", m, bytes / m / 1e6);
        m = run<false, 4>(Q, ldq, K, ntiles, out); printf("client-major U=4 %.3f ms %.0f GB/s\n", m, bytes / m / 1e6);
        m = run<true, 4>(Q, ldq, K, ntiles, out);  printf("blocked      U=4 %.3f ms %.0f GB/s\n", m, bytes / m / 1e6);
    }
    hipFree(Q);
    hipFree(out);
    return 0;
}

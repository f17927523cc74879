// Probe: HBM read ceiling of the fed_quant lane-tile access pattern.
// A wave owns a TKB-KiB tile of a client row and walks K client rows (U rows in
// flight), xor-reducing the bytes (negligible VALU) — the memory stream of
// k_dequant_lanes without its arithmetic.  Two questions:
//   1. does the payload's content matter?  (constant 0x01 bytes, as the round-3
//      layout probe used, vs hashed random bytes, as the bench stores hold)
//   2. at the ResNet-18 shape (11.2 MB rows, K = 1000) how do tile width and
//      rows in flight move the ceiling?
//   2b. tiles 1 KiB-aligned or not (the store aligns tensors to 256 B) and the
//      product lane kernel's pipeline shape: batches of 2 clients double-
//      buffered inside chunks of CH clients, drained at every chunk end (CH = 64
//      today), with global vs buffer loads; CH = K is one continuous pipeline.
//   3. the write side of the Shapley subset GEMM: 50 output rows of 44.7 MB, a
//      wave writing a CB-byte piece of every row (512 B today), vs contiguous
//      writes, and a 50/50 read+write copy.
//   hipcc --offload-arch=gfx950 -O3 -o tools/_stream_probe tools/stream_probe.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ void k_fill(uint32_t *p, int64_t n, int random) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t x = (uint64_t)i * 0x9E3779B97F4A7C15ull;
        x ^= x >> 31;
        x *= 0xBF58476D1CE4E5B9ull;
        x ^= x >> 27;
        p[i] = random ? (uint32_t)x : 0x01010101u;
    }
}

template <int TKB, int U>
__global__ __launch_bounds__(256) void k_stream(const uint8_t *__restrict__ Q, int64_t ldq, int K,
                                                int ntiles, uint32_t *__restrict__ out) {
    const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (t >= ntiles) return;
    const int lane = threadIdx.x & 63;
    u32x4 acc = {0, 0, 0, 0};
    for (int k0 = 0; k0 < K; k0 += U) {
        u32x4 v[U][TKB];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int s = 0; s < TKB; ++s)
                v[u][s] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(
                    Q + (int64_t)min(k0 + u, K - 1) * ldq + (int64_t)t * TKB * 1024 + s * 1024 + lane * 16));
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int s = 0; s < TKB; ++s) acc ^= v[u][s];
    }
    out[(int64_t)t * 64 + lane] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}


// wave t writes a CB-byte piece of each of R rows (row stride ldo bytes)
template <int CB>
__global__ __launch_bounds__(256) void k_write(uint8_t *__restrict__ O, int64_t ldo, int R, int ntiles) {
    const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (t >= ntiles) return;
    const int lane = threadIdx.x & 63;
    const u32x4 v = {(uint32_t)t, (uint32_t)lane, 7u, 9u};
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int s = 0; s < CB / 1024 + (CB < 1024); ++s) {
            if (CB < 1024 && lane * 16 >= CB) continue;
            __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(O + (int64_t)r * ldo + (int64_t)t * CB + s * 1024 + lane * 16));
        }
}

// read + write the same volume: wave t copies its 4 KiB tile of each row
__global__ __launch_bounds__(256) void k_copy(const uint8_t *__restrict__ Q, uint8_t *__restrict__ O, int64_t ld, int R, int ntiles) {
    const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (t >= ntiles) return;
    const int lane = threadIdx.x & 63;
    for (int r = 0; r < R; ++r) {
        u32x4 v[4];
#pragma unroll
        for (int s = 0; s < 4; ++s)
            v[s] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(Q + (int64_t)r * ld + (int64_t)t * 4096 + s * 1024 + lane * 16));
#pragma unroll
        for (int s = 0; s < 4; ++s)
            __builtin_nontemporal_store(v[s], reinterpret_cast<u32x4 *>(O + (int64_t)r * ld + (int64_t)t * 4096 + s * 1024 + lane * 16));
    }
}

template <typename F>
float time_it(F f) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int i = 0; i < 3; ++i) f();
    hipEventRecord(a);
    for (int i = 0; i < 10; ++i) f();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    hipEventDestroy(a);
    hipEventDestroy(b);
    return ms / 10;
}

// a wave owns one 1 KiB tile; batches of 2 clients double-buffered within chunks
// of CH clients (the pipeline drains at each chunk end, as chunk_pipeline_1tail)
template <int CH, bool BUF>
__global__ __launch_bounds__(256) void k_chunked(const uint8_t *__restrict__ Q, int64_t ldq, int K,
                                                 int ntiles, uint32_t *__restrict__ out, int mis) {
    const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (t >= ntiles) return;
    const int lane = threadIdx.x & 63;
    u32x4 acc = {0, 0, 0, 0};
    auto ld = [&](int k) -> u32x4 {
        if constexpr (BUF) {
            const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(Q + (int64_t)k * ldq), 0,
                                                              (int)0xffffffffu, 0x00020000);
            return __builtin_amdgcn_raw_buffer_load_b128(rs, t * 1024 + mis + lane * 16, 0, 2);
        } else {
            return __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(Q + (int64_t)k * ldq + (int64_t)t * 1024 + mis + lane * 16));
        }
    };
    struct Bt { u32x4 a, b; };
    auto load = [&](int k, Bt &x) { x.a = ld(k); x.b = ld(k + 1); };
    auto use = [&](const Bt &x) { acc ^= x.a; acc ^= x.b; };
    for (int base = 0; base < K; base += CH) {
        const int n = min(CH, K - base);
        const int nb = n / 2;
        Bt A, B;
        load(base, A);
        int b = 0;
        for (; b + 2 < nb; b += 2) {
            load(base + 2 * (b + 1), B);
            use(A);
            load(base + 2 * (b + 2), A);
            use(B);
        }
        const bool two = b + 1 < nb;
        if (two) load(base + 2 * (b + 1), B);
        use(A);
        if (two) use(B);
    }
    out[(int64_t)t * 64 + lane] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

template <int CH, bool BUF>
void runc(const uint8_t *Q, int64_t ldq, int K, int ntiles, uint32_t *out, int mis = 0) {
    const float ms = time_it([&] { hipLaunchKernelGGL((k_chunked<CH, BUF>), dim3((ntiles + 3) / 4), dim3(256), 0, 0, Q, ldq, K, ntiles, out, mis); });
    printf("chunked CH=%4d %s  tile offset +%4d B  waves %6d  %.3f ms  %.0f GB/s\n", CH, BUF ? "buffer" : "global", mis, ntiles, ms,
           (double)ntiles * 1024 * K / ms / 1e6);
}

template <int CB>
void runw(uint8_t *O, int64_t rowbytes, int R) {
    const int ntiles = (int)(rowbytes / CB);
    const float ms = time_it([&] { hipLaunchKernelGGL((k_write<CB>), dim3((ntiles + 3) / 4), dim3(256), 0, 0, O, rowbytes, R, ntiles); });
    const double bytes = (double)ntiles * CB * R;
    printf("write  piece %5d B  rows %2d  %.3f ms  %.0f GB/s\n", CB, R, ms, bytes / ms / 1e6);
}

template <int TKB, int U>
void run(const char *name, const uint8_t *Q, int64_t ldq, int K, int64_t rowbytes, uint32_t *out) {
    const int ntiles = (int)(rowbytes / (TKB * 1024));
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const dim3 grid((ntiles + 3) / 4);
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((k_stream<TKB, U>), grid, dim3(256), 0, 0, Q, ldq, K, ntiles, out);
    hipEventRecord(a);
    const int reps = 10;
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((k_stream<TKB, U>), grid, dim3(256), 0, 0, Q, ldq, K, ntiles, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    ms /= reps;
    const double bytes = (double)ntiles * TKB * 1024 * K;
    printf("%-6s tile %d KiB  U=%d  waves %6d  %.3f ms  %.0f GB/s\n", name, TKB, U, ntiles, ms, bytes / ms / 1e6);
    hipEventDestroy(a);
    hipEventDestroy(b);
}

int main() {
    const int64_t total = 14ll << 30;
    uint8_t *Q;
    uint32_t *out;
    if (hipMalloc(&Q, total) != hipSuccess || hipMalloc(&out, 64 << 20) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    // VGG-sized rows (138 MB, K = 100), the round-3 layout probe's shape
    const int64_t vgg_row = 33774ll * 4096, vgg_ld = vgg_row;
    // ResNet-18-sized rows (11.2M int8 parameters, K = 1000); ld padded like the store
    const int64_t r18_row = 11168ll * 1024, r18_ld = r18_row + 256;
    for (int random = 0; random < 2; ++random) {
        hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint32_t *>(Q), total / 4, random);
        if (hipDeviceSynchronize() != hipSuccess) return 2;
        const char *nm = random ? "random" : "const";
        printf("== payload %s\n", nm);
        run<4, 4>(nm, Q, vgg_ld, 100, vgg_row, out);
        run<1, 2>(nm, Q, r18_ld, 1000, r18_row, out);
        run<1, 4>(nm, Q, r18_ld, 1000, r18_row, out);
        run<1, 8>(nm, Q, r18_ld, 1000, r18_row, out);
        run<2, 4>(nm, Q, r18_ld, 1000, r18_row, out);
        run<4, 2>(nm, Q, r18_ld, 1000, r18_row, out);
        run<4, 4>(nm, Q, r18_ld, 1000, r18_row, out);
        if (random) {
            // the lane kernel's launch pieces: ~3,700 waves (one generation at 4 per SIMD)
            for (int nt : {11168, 3723})
                for (int mis : {0, 256, 512, 768}) {
                    runc<64, true>(Q, r18_ld, 1000, nt, out, mis);
                    runc<64, false>(Q, r18_ld, 1000, nt, out, mis);
                }
        }
    }
    // subset-GEMM output shape: 50 rows x 11,168,000 fp32 (44.7 MB)
    const int64_t orow = 11168000ll * 4;
    uint8_t *O = Q + (6ll << 30);
    runw<512>(O, orow, 50);
    runw<1024>(O, orow, 50);
    runw<4096>(O, orow, 50);
    runw<4096>(O, orow * 50, 1);
    {
        const int64_t half = 3ll << 30;
        const int ntiles = (int)(half / 4096);
        const float ms = time_it([&] { hipLaunchKernelGGL(k_copy, dim3((ntiles + 3) / 4), dim3(256), 0, 0, Q, Q + half, half, 1, ntiles); });
        printf("copy   3 GiB -> 3 GiB  %.3f ms  %.0f GB/s (read+write)\n", ms, 2.0 * half / ms / 1e6);
    }
    hipFree(Q);
    hipFree(out);
    return 0;
}

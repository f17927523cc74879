// FedAvg streaming reduction (servers/fed_server.py:44-66) for gfx950.
//
// One pass over the client rows: each lane owns 4 consecutive parameters per
// 1 KB slice of a row (one 16-byte load per client; a wave owns 1 slice, or 16
// or 22 consecutive slices on large models), walks the K clients in the reference's
// iteration order and keeps the running sum in registers, so every client byte
// is read once and the 4*P-byte result is written once.  HBM-bound: the
// algorithmic traffic of one call is K*P*4 + P*4 bytes.  The client rows and
// weights reach the wave through per-lane tables and v_readlane, and batches
// of clients are double-buffered (k_fedavg_exact_pipe).
//
// EXACT mode reproduces the reference op sequence bit-for-bit:
//     term_i = fl(fl(x * fl32(n_i)) / fl32(N)); acc = term_0; acc = fl(acc + term_i)
// (division: dls_common.h, Markstein fast path + IEEE fix-up for out-of-range).
// FMA mode computes acc = fma(x, fl(n_i/N), acc) (normwise ~1e-7).
#include "dls_common.h"

namespace dls {
namespace {

constexpr int kBlock = 256;
constexpr int kPipeBlock = 256;

template <bool NT>
__device__ __forceinline__ f32x4 load4(const f32x4 *p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    return *p;
}

// term = fl(fl(x*w)/N) for 4 lanes of a f32x4, exact.
__device__ __forceinline__ f32x4 term4(f32x4 x, float w, const FastDiv &d) {
    f32x4 t;
    t.x = x.x * w;
    t.y = x.y * w;
    t.z = x.z * w;
    t.w = x.w * w;
    f32x4 q;
    q.x = markstein(t.x, d.b, d.y);
    q.y = markstein(t.y, d.b, d.y);
    q.z = markstein(t.z, d.b, d.y);
    q.w = markstein(t.w, d.b, d.y);
    const bool ok = d.fast & in_fast_range(t.x) & in_fast_range(t.y) & in_fast_range(t.z) &
                    in_fast_range(t.w);
    if (__builtin_expect(!ok, 0)) {  // zeros, denormals, huge, inf/nan: IEEE division
        q.x = d.fast && in_fast_range(t.x) ? q.x : t.x / d.b;
        q.y = d.fast && in_fast_range(t.y) ? q.y : t.y / d.b;
        q.z = d.fast && in_fast_range(t.z) ? q.z : t.z / d.b;
        q.w = d.fast && in_fast_range(t.w) ? q.w : t.w / d.b;
    }
    return q;
}

__device__ __forceinline__ f32x4 add4(f32x4 a, f32x4 b) {
    return a + b;
}

// Software-pipelined form.  Clients are taken in chunks of 64: lane j holds
// client (base + j)'s row and weight (one coalesced vector load per field per
// chunk, the next chunk's fetched a whole chunk ahead) and every step reads them
// back as wave-uniform values with v_readlane, so no s_load -> s_waitcnt sits
// on the critical path.  Inside a chunk, batches of U clients are
// double-buffered: batch b+1's U loads are issued before batch b is reduced.
// Same op sequence as k_fedavg_exact.
template <int U, bool NT, int G>
__global__ __launch_bounds__(kPipeBlock) void k_fedavg_exact_pipe(const f32x4 *__restrict__ Uv,
                                                              int64_t ldu4,
                                                              const int32_t *__restrict__ rows,
                                                              const float *__restrict__ w, int K,
                                                              FastDiv d, int64_t P4,
                                                              f32x4 *__restrict__ out) {
    // a wave owns G KB of every client row: f32x4 slots wb + 64 q + lane, q < G
    const int lane = __lane_id();
    const int64_t wb = ((int64_t)blockIdx.x * (kPipeBlock / 64) + (threadIdx.x >> 6)) * 64 * G;
    int64_t iq[G];
#pragma unroll
    for (int q = 0; q < G; ++q) {
        const int64_t i0 = wb + 64 * q + lane;
        iq[q] = i0 < P4 ? i0 : P4 - 1;  // every lane stays: the table needs all 64
    }
    // -0 + t == t for every fp32 t (including -0 and NaN), so starting from -0
    // and always adding reproduces "the first client is assigned"
    // (servers/fed_server.py:62-65) without a special first step.
    f32x4 acc[G];
#pragma unroll
    for (int q = 0; q < G; ++q) acc[q] = f32x4{-0.f, -0.f, -0.f, -0.f};
    int nr = rows[min(lane, K - 1)];
    float nw = w[min(lane, K - 1)];
    for (int base = 0; base < K; base += 64) {
        const int tr = nr;
        const float tw = nw;
        const int kn = min(base + 64 + lane, K - 1);
        nr = rows[kn];  // next chunk, in flight behind this one's loads
        nw = w[kn];
        const int n = min(64, K - base);
        auto load = [&](int j0, f32x4 (&x)[U][G], float (&wk)[U]) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t r = __builtin_amdgcn_readlane(tr, j0 + u);
                wk[u] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(tw), j0 + u));
#pragma unroll
                for (int q = 0; q < G; ++q) x[u][q] = load4<NT>(Uv + r * ldu4 + iq[q]);
            }
        };
        auto consume = [&](const f32x4 (&x)[U][G], const float (&wk)[U]) {
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int q = 0; q < G; ++q) acc[q] = add4(acc[q], term4(x[u][q], wk[u], d));
        };
        // loads inside the steady-state loop are unconditional, so every consume
        // waits with an exact vmcnt (a conditional load would make the compiler's
        // merged count wait for the younger batch too)
        const int nb = n / U;
        int j = 0;
        if (nb > 0) {
            f32x4 xA[U][G], xB[U][G];
            float wA[U], wB[U];
            load(0, xA, wA);
            int b = 0;
            for (; b + 2 < nb; b += 2) {
                load((b + 1) * U, xB, wB);
                consume(xA, wA);
                load((b + 2) * U, xA, wA);
                consume(xB, wB);
            }
            if (b + 1 < nb) {
                load((b + 1) * U, xB, wB);
                consume(xA, wA);
                consume(xB, wB);
            } else {
                consume(xA, wA);
            }
            j = nb * U;
        }
        for (; j < n; ++j) {
            const int64_t r = __builtin_amdgcn_readlane(tr, j);
            const float wk = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(tw), j));
#pragma unroll
            for (int q = 0; q < G; ++q)
                acc[q] = add4(acc[q], term4(load4<NT>(Uv + r * ldu4 + iq[q]), wk, d));
        }
    }
#pragma unroll
    for (int q = 0; q < G; ++q)
        if (wb + 64 * q + lane < P4) out[iq[q]] = acc[q];
}

template <int UNROLL, bool NT>
__global__ __launch_bounds__(kBlock) void k_fedavg_fma(const f32x4 *__restrict__ U, int64_t ldu4,
                                                       const int32_t *__restrict__ rows,
                                                       const float *__restrict__ w, int K,
                                                       float total, int64_t P4,
                                                       f32x4 *__restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= P4) return;
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
    int j = 0;
    for (; j + UNROLL <= K; j += UNROLL) {
        f32x4 x[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) x[u] = load4<NT>(U + (int64_t)rows[j + u] * ldu4 + i);
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const float c = w[j + u] / total;
            acc.x = __builtin_fmaf(x[u].x, c, acc.x);
            acc.y = __builtin_fmaf(x[u].y, c, acc.y);
            acc.z = __builtin_fmaf(x[u].z, c, acc.z);
            acc.w = __builtin_fmaf(x[u].w, c, acc.w);
        }
    }
    for (; j < K; ++j) {
        const f32x4 x = load4<NT>(U + (int64_t)rows[j] * ldu4 + i);
        const float c = w[j] / total;
        acc.x = __builtin_fmaf(x.x, c, acc.x);
        acc.y = __builtin_fmaf(x.y, c, acc.y);
        acc.z = __builtin_fmaf(x.z, c, acc.z);
        acc.w = __builtin_fmaf(x.w, c, acc.w);
    }
    out[i] = acc;
}

// Batched reference-order subsets: blockIdx.y = subset.  Subsets of one GTG
// wave / multiround batch share client rows, which the 256 MiB Infinity Cache
// serves on re-read when the batch is processed column-tile by column-tile.
template <bool NT>
__global__ __launch_bounds__(kBlock) void k_subset_exact(const f32x4 *__restrict__ U,
                                                         int64_t ldu4,
                                                         const int32_t *__restrict__ sub_off,
                                                         const int32_t *__restrict__ sub_rows,
                                                         const float *__restrict__ sub_w,
                                                         const float *__restrict__ sub_total,
                                                         int S, int64_t P4,
                                                         f32x4 *__restrict__ out,
                                                         int64_t ldo4) {
    // subset-fastest block order: the S blocks of one column tile run together
    const int s = blockIdx.x % S;
    const int64_t tile = blockIdx.x / S;
    const int64_t i = tile * kBlock + threadIdx.x;
    if (i >= P4) return;
    const int beg = sub_off[s], end = sub_off[s + 1];
    const float b = sub_total[s];
    FastDiv d;
    d.b = b;
    d.y = (float)(1.0 / (double)b);
    d.fast = (b >= 1.0f && b <= 2147483648.0f) ? 1 : 0;
    f32x4 acc = term4(load4<NT>(U + (int64_t)sub_rows[beg] * ldu4 + i), sub_w[beg], d);
    for (int j = beg + 1; j < end; ++j)
        acc = add4(acc, term4(load4<NT>(U + (int64_t)sub_rows[j] * ldu4 + i), sub_w[j], d));
    out[(int64_t)s * ldo4 + i] = acc;
}

}  // namespace
}  // namespace dls

using namespace dls;

extern "C" int dls_fedavg_f32(const float *U, int64_t ldu, const int32_t *rows,
                              const float *weight, int32_t K, float total, int64_t P,
                              int32_t mode, float *out, dls_stream_t stream) {
    DLS_REQUIRE(U && rows && weight && out, DLS_EINVAL, "dls_fedavg_f32: null pointer");
    DLS_REQUIRE(K > 0 && P > 0, DLS_EINVAL, "dls_fedavg_f32: K=%d P=%lld", K, (long long)P);
    DLS_REQUIRE(P % 4 == 0 && ldu % 4 == 0 && ldu >= P, DLS_ELAYOUT,
                "dls_fedavg_f32: P=%lld and ldu=%lld must be multiples of 4, ldu >= P",
                (long long)P, (long long)ldu);
    DLS_REQUIRE(aligned16(U) && aligned16(out), DLS_ELAYOUT, "dls_fedavg_f32: 16-byte alignment");
    const int64_t P4 = P / 4;
    const dim3 grid((unsigned)((P4 + kBlock - 1) / kBlock));
    hipStream_t st = as_stream(stream);
    if (mode == DLS_FEDAVG_EXACT) {
        const FastDiv d = make_fastdiv(total);
        // Each wave streams G KB of every client row (one client per double-
        // buffered step); wide G beats 1 KB x 4 clients by 4-6 % at P = 11.2M.
        // A wave's work is K clients deep, so the grid is cut into pieces of at
        // most one generation of resident waves, launched back to back: a
        // second generation starting piecemeal behind the first, or a last
        // generation of a few waves running alone at latency-bound speed, costs
        // more than a kernel boundary (measured: G = 14 at P = 11.2M leaves 46
        // waves for a 4th generation, +13 %; two one-generation launches beat one
        // two-generation launch by 3 %).  Widest G that keeps >= kSat waves per
        // piece; the 1 KB kernel for small models.
        const f32x4 *Uv = reinterpret_cast<const f32x4 *>(U);
        f32x4 *ov = reinterpret_cast<f32x4 *>(out);
        constexpr int64_t kSat = 512;
        const int64_t ldu4 = ldu / 4;
        auto pieces = [&](const void *kern, int G, auto launch) {
            const int64_t waves = (P4 + 64 * G - 1) / (64 * G);
            const int64_t slots = (int64_t)resident_blocks(kern, kPipeBlock, 0) * (kPipeBlock / 64);
            const int64_t np = (waves + slots - 1) / slots;
            const int64_t per = (waves + np - 1) / np;  // waves per piece, <= slots
            if (per < kSat && G > 1) return false;
            for (int64_t w0 = 0; w0 < waves; w0 += per) {
                const int64_t c0 = w0 * 64 * G, c1 = min((w0 + per) * 64 * G, P4);  // f32x4 units
                launch(dim3((unsigned)((min(per, waves - w0) + 3) / 4)), c0, c1 - c0);
            }
            return true;
        };
#define DLS_PIPE_PIECES(U_, G_)                                                              \
    pieces(reinterpret_cast<const void *>(k_fedavg_exact_pipe<U_, true, G_>), G_,            \
           [&](dim3 grid, int64_t c0, int64_t n4) {                                          \
               hipLaunchKernelGGL((k_fedavg_exact_pipe<U_, true, G_>), grid, dim3(kPipeBlock), \
                                  0, st, Uv + c0, ldu4, rows, weight, (int)K, d, n4, ov + c0); \
           })
        if (!DLS_PIPE_PIECES(1, 22) && !DLS_PIPE_PIECES(1, 16)) DLS_PIPE_PIECES(4, 1);
#undef DLS_PIPE_PIECES
    } else if (mode == DLS_FEDAVG_FMA) {
        hipLaunchKernelGGL((k_fedavg_fma<8, true>), grid, dim3(kBlock), 0, st,
                           reinterpret_cast<const f32x4 *>(U), ldu / 4, rows, weight, (int)K, total,
                           P4, reinterpret_cast<f32x4 *>(out));
    } else {
        set_error("dls_fedavg_f32: unknown mode %d", mode);
        return DLS_EINVAL;
    }
    return check_launch("dls_fedavg_f32");
}

extern "C" int dls_subset_fedavg_f32(const float *U, int64_t ldu, const int32_t *sub_off,
                                     const int32_t *sub_rows, const float *sub_weight,
                                     const float *sub_total, int32_t S, int64_t P, float *out,
                                     int64_t ldo, dls_stream_t stream) {
    DLS_REQUIRE(U && sub_off && sub_rows && sub_weight && sub_total && out, DLS_EINVAL,
                "dls_subset_fedavg_f32: null pointer");
    DLS_REQUIRE(S > 0 && P > 0, DLS_EINVAL, "dls_subset_fedavg_f32: S=%d P=%lld", S,
                (long long)P);
    DLS_REQUIRE(P % 4 == 0 && ldu % 4 == 0 && ldo % 4 == 0 && ldu >= P && ldo >= P, DLS_ELAYOUT,
                "dls_subset_fedavg_f32: P, ldu, ldo must be multiples of 4");
    DLS_REQUIRE(aligned16(U) && aligned16(out), DLS_ELAYOUT,
                "dls_subset_fedavg_f32: 16-byte alignment");
    const int64_t P4 = P / 4;
    const int64_t tiles = (P4 + kBlock - 1) / kBlock;
    DLS_REQUIRE(tiles * S < (int64_t)1 << 31, DLS_EINVAL, "dls_subset_fedavg_f32: grid too large");
    hipLaunchKernelGGL((k_subset_exact<false>), dim3((unsigned)(tiles * S)), dim3(kBlock), 0,
                       as_stream(stream), reinterpret_cast<const f32x4 *>(U), ldu / 4, sub_off,
                       sub_rows, sub_weight, sub_total, (int)S, P4, reinterpret_cast<f32x4 *>(out),
                       ldo / 4);
    return check_launch("dls_subset_fedavg_f32");
}

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

// Batched reference-order subsets over a client "union" (the Shapley servers'
// default path, servers/GTG_shapley_value_server.py:56 and
// servers/multiround_shapley_value_server.py:37).  The batch's S coalitions are
// all made of the union's Ku clients, and walking the union in its order visits
// every coalition's members in that coalition's own order (the host orders the
// union so; sorted worker-id tuples always are).  So each client row is read
// from HBM once per batch instead of once per coalition containing it:
//   for client j of the union:  t = fl(x * fl32(n_j))
//       for every coalition s holding j (bit s of member[j]):  acc_s = fl(acc_s + fl(t / N_s))
// which is term for term the op sequence of servers/fed_server.py:57-65 for
// each coalition (acc_s starts at -0: -0 + q == q, "the first client is assigned").
//
// Block = one tile of 256 parameters (a lane owns 4), one wave per <= kSubsetSB
// coalitions (spread evenly): the waves of a block load the same 1 KiB of each client row at the
// same time (one HBM read, the others served by the CU's L1 / the XCD's L2) and
// each keeps its kSubsetSB accumulators in registers.  Membership is a
// wave-uniform bit test (SALU branch), so a coalition that does not hold client
// j costs nothing.  Algorithmic bytes: (Ku + S) * 4 per parameter; VALU: 4 per
// parameter per (client, coalition) membership (multiply-add Markstein division +
// add) + 4 per parameter per (client, wave) for t.  At S = Ku = 50 with
// coalitions half full the VALU issue, not HBM, is the roof.
#ifndef DLS_SUBSET_SB
#define DLS_SUBSET_SB 8  // coalitions per wave: 10 VGPRs each (SB 8 -> 135 VGPRs, 3 waves / SIMD)
#endif
#ifndef DLS_SUBSET_UB
#define DLS_SUBSET_UB 4  // clients per double-buffered batch
#endif
constexpr int kSubsetSB = DLS_SUBSET_SB;
constexpr int kSubsetUB = DLS_SUBSET_UB;
constexpr int kSubsetMaxBlock = 64 * ((DLS_SUBSET_UNION_MAX + kSubsetSB - 1) / kSubsetSB);

template <int SB, int UB>
__global__ __launch_bounds__(kSubsetMaxBlock) void k_subset_union(const f32x4 *__restrict__ Uv, int64_t ldu4,
                                                      const int32_t *__restrict__ urows,
                                                      const float *__restrict__ uw,
                                                      const uint64_t *__restrict__ member, int Ku,
                                                      const float *__restrict__ sub_total, int S,
                                                      int64_t P4, f32x4 *__restrict__ out,
                                                      int64_t ldo4) {
    const int lane = __lane_id();
    // the S coalitions are spread evenly over the block's waves (<= SB each)
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int nwv = blockDim.x >> 6;
    const int s0 = wv * S / nwv;
    const int ns = (wv + 1) * S / nwv - s0;  // wave-uniform, 1..SB by the launch geometry
    const int64_t i0 = (int64_t)blockIdx.x * 64 + lane;
    const int64_t iq = i0 < P4 ? i0 : P4 - 1;  // every lane stays: the tables need all 64
    // per-coalition divisor N_s and y_s = RN(1/N_s) (wave-uniform values, kept in
    // VGPRs: 2*SB SGPRs beside the client tables would spill)
    float bs[SB];
    f32x2 ys[SB];  // {y, y}: the packed multiply-adds take it as a register pair
    int allfast = 1;
#pragma unroll
    for (int s = 0; s < SB; ++s) {
        bs[s] = s < ns ? sub_total[s0 + s] : 1.f;
        const float y = (float)(1.0 / (double)bs[s]);
        ys[s] = f32x2{y, y};
        allfast &= (int)(bs[s] >= 1.0f && bs[s] <= 2147483648.0f);
    }
    f32x4 acc[SB];
#pragma unroll
    for (int s = 0; s < SB; ++s) acc[s] = f32x4{-0.f, -0.f, -0.f, -0.f};
    const uint32_t smask = (uint32_t)((1ull << ns) - 1ull);
    // client table: lane l holds client (chunk base + l); the next chunk is in flight
    auto fetch = [&](int k, int &r, float &w, uint32_t &m) {
        const int kk = min(k + lane, Ku - 1);
        r = urows[kk];
        w = uw[kk];
        m = k + lane < Ku ? (uint32_t)(member[kk] >> s0) & smask : 0u;  // past the end: no work
    };
    int nr;
    float nw;
    uint32_t nm;
    fetch(0, nr, nw, nm);
    // Common case only: every t of the wave in Markstein's range and every
    // divisor in [1, 2^31].  Otherwise (zeros, denormals, huge values, inf / nan)
    // the wave flags `redo` and recomputes its tile after the loop on a slow,
    // compact path, so the hot loop carries no fix-up code or registers.
    int redo = !allfast;
    auto one = [&](f32x4 x, float wk, uint32_t m) {
        f32x4 t;
        t.x = x.x * wk;
        t.y = x.y * wk;
        t.z = x.z * wk;
        t.w = x.w * wk;
        const int ok = (int)in_fast_range(t.x) & (int)in_fast_range(t.y) &
                       (int)in_fast_range(t.z) & (int)in_fast_range(t.w);
        redo |= (int)(__ballot(!ok) != 0);
#pragma unroll
        for (int s = 0; s < SB; ++s) {
            if (m & (1u << s)) {  // wave-uniform: a scalar branch
                // Markstein on element pairs (v_pk_mul / v_pk_fma: the scalar ops' roundings)
                const f32x2 b2 = f32x2{bs[s], bs[s]};
                const f32x2 tl = f32x2{t.x, t.y}, th = f32x2{t.z, t.w};
                const f32x2 ql0 = tl * ys[s], qh0 = th * ys[s];
                const f32x2 ql = __builtin_elementwise_fma(
                    __builtin_elementwise_fma(-ql0, b2, tl), ys[s], ql0);
                const f32x2 qh = __builtin_elementwise_fma(
                    __builtin_elementwise_fma(-qh0, b2, th), ys[s], qh0);
                acc[s] = add4(acc[s], f32x4{ql.x, ql.y, qh.x, qh.y});
            }
        }
    };
    for (int base = 0; base < Ku; base += 64) {
        const int tr = nr;
        const float tw = nw;
        const uint32_t tm = nm;
        fetch(base + 64, nr, nw, nm);
        // batches of UB clients, double-buffered; past the chunk's end a batch
        // loads a valid duplicate row with no membership (no work), so every load
        // is unconditional (exact vmcnt waits) and there is no tail loop
        const int nb = (min(64, Ku - base) + UB - 1) / UB;
        auto load = [&](int j0, f32x4 (&x)[UB], float (&wk)[UB], uint32_t (&mk)[UB]) {
#pragma unroll
            for (int u = 0; u < UB; ++u) {
                const int j = min(j0 + u, 63);
                const int64_t r = __builtin_amdgcn_readlane(tr, j);
                wk[u] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(tw), j));
                mk[u] = j0 + u < 64 ? (uint32_t)__builtin_amdgcn_readlane((int)tm, j) : 0u;
                x[u] = load4<false>(Uv + r * ldu4 + iq);
            }
        };
        f32x4 xA[UB], xB[UB];
        float wA[UB], wB[UB];
        uint32_t mA[UB], mB[UB];
        load(0, xA, wA, mA);
        for (int b = 0; b < nb; b += 2) {
            load((b + 1) * UB, xB, wB, mB);
#pragma unroll
            for (int u = 0; u < UB; ++u) one(xA[u], wA[u], mA[u]);
            load((b + 2) * UB, xA, wA, mA);
            if (b + 1 < nb) {
#pragma unroll
                for (int u = 0; u < UB; ++u) one(xB[u], wB[u], mB[u]);
            }
        }
    }
    if (__builtin_expect(!redo, 1)) {
        if (i0 < P4) {
#pragma unroll
            for (int s = 0; s < SB; ++s)
                if (s < ns) out[(int64_t)(s0 + s) * ldo4 + iq] = acc[s];
        }
        return;
    }
    // slow path (acc is dead here): one coalition at a time, guarded division
    for (int s = 0; s < ns; ++s) {
        FastDiv d;
        d.b = sub_total[s0 + s];
        d.y = (float)(1.0 / (double)d.b);
        d.fast = d.b >= 1.0f && d.b <= 2147483648.0f;
        f32x4 a = f32x4{-0.f, -0.f, -0.f, -0.f};
        for (int j = 0; j < Ku; ++j) {
            if (!((member[j] >> (s0 + s)) & 1u)) continue;
            const f32x4 x = load4<false>(Uv + (int64_t)urows[j] * ldu4 + iq);
            const float wk = uw[j];
#pragma unroll
            for (int e = 0; e < 4; ++e) a[e] += div_exact(x[e] * wk, d);
        }
        if (i0 < P4) out[(int64_t)(s0 + s) * ldo4 + iq] = a;
    }
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

extern "C" int dls_subset_fedavg_union_f32(const float *U, int64_t ldu, const int32_t *urows,
                                           const float *uweight, const uint64_t *member, int32_t Ku,
                                           const float *sub_total, int32_t S, int64_t P,
                                           float *out, int64_t ldo, dls_stream_t stream) {
    DLS_REQUIRE(U && urows && uweight && member && sub_total && out, DLS_EINVAL,
                "dls_subset_fedavg_union_f32: null pointer");
    DLS_REQUIRE(Ku > 0 && P > 0 && S > 0 && S <= DLS_SUBSET_UNION_MAX, DLS_EINVAL,
                "dls_subset_fedavg_union_f32: Ku=%d S=%d (1..%d) P=%lld", Ku, S,
                DLS_SUBSET_UNION_MAX, (long long)P);
    DLS_REQUIRE(P % 4 == 0 && ldu % 4 == 0 && ldo % 4 == 0 && ldu >= P && ldo >= P, DLS_ELAYOUT,
                "dls_subset_fedavg_union_f32: P, ldu, ldo must be multiples of 4");
    DLS_REQUIRE(aligned16(U) && aligned16(out), DLS_ELAYOUT,
                "dls_subset_fedavg_union_f32: 16-byte alignment");
    static_assert(kSubsetMaxBlock <= 1024, "at most 16 waves per block");
    const int64_t P4 = P / 4;
    const int64_t tiles = (P4 + 63) / 64;
    DLS_REQUIRE(tiles < (int64_t)1 << 31, DLS_EINVAL, "dls_subset_fedavg_union_f32: grid too large");
    const int waves = (S + kSubsetSB - 1) / kSubsetSB;
    hipLaunchKernelGGL((k_subset_union<kSubsetSB, kSubsetUB>), dim3((unsigned)tiles),
                       dim3(64 * waves), 0, as_stream(stream), reinterpret_cast<const f32x4 *>(U),
                       ldu / 4, urows, uweight, member, (int)Ku, sub_total, (int)S, P4,
                       reinterpret_cast<f32x4 *>(out), ldo / 4);
    return check_launch("dls_subset_fedavg_union_f32");
}

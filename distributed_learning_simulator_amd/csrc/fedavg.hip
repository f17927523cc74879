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
#include <cstring>
#include <type_traits>

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
//   t_j = fl(x_j * fl32(n_j)) once per client;
//   acc_s = fl(acc_s + fl(t_j / N_s)) for the members j of coalition s, in union order
// which is term for term the op sequence of servers/fed_server.py:57-65 for
// each coalition (acc_s starts at -0: -0 + q == q, "the first client is assigned").
// Algorithmic bytes: (Ku + S) * 4 per parameter; VALU: per parameter and
// membership the quotient (2 ops two-constant / 3 Markstein) + the add.
constexpr int kUnionChunk = 64;  // clients per launch (the host splits larger unions)

// in_fast_range (dls_common.h) of all four: 2^-60 <= |t| < 2^61 on the bit
// patterns (min / max of |bits|: zeros, denormals, inf and nan all fail)
__device__ __forceinline__ bool all_in_fast_range(f32x4 t) {
    const uint32_t a = __float_as_uint(t.x) & 0x7fffffffu, b = __float_as_uint(t.y) & 0x7fffffffu;
    const uint32_t c = __float_as_uint(t.z) & 0x7fffffffu, d = __float_as_uint(t.w) & 0x7fffffffu;
    const uint32_t mn = min(min(a, b), min(c, d)), mx = max(max(a, b), max(c, d));
    return mn >= (67u << 23) && mx < (188u << 23);
}

// Per-coalition division constants, computed on the host (dls_common.h FastDiv):
// {yh = RN(1/N), yl = RN(1/N - yh), N, flags}; flags bit 0: the two-constant
// quotient fma(t, yh, RN(t * yl)) is proven correctly rounded for this N (the
// host's exhaustive mantissa check), bit 1: N in Markstein's range [1, 2^31].
struct UnionDiv {
    f32x4 c[DLS_SUBSET_UNION_MAX];
};

// The kernel: TWO blocks of kUnionWaves = 8 waves per CU, persistent over
// 256-parameter tiles (a lane owns 4), so that one block's barriers, staging and
// load waits are filled by the other block's walks.  A block's LDS (< 80 KB) holds
// one tile's t_j of the <= 64 union clients (64 KiB) and the member lists as
// 16-bit offsets; per tile: walk the coalitions (each result stored as soon as
// it is summed), barrier, turn the next tile's rows — loaded during the walk —
// into t_j, issue the loads of the tile after, barrier.  The S coalitions are
// dealt to the waves once per block, longest first to the least loaded wave (a
// static LPT plan; 8 waves with ~6 coalitions each balance to ~1.05 x the mean).
// Per membership: one ds_read_b128 of t (4 parameters), the quotient (2 ops
// two-constant / 3 Markstein, element pairs packed) and the add.
// (Round 5 history, profiles/r05_union_ab.txt: one 16-wave block per CU with a
// double-buffered 128 KiB t took 1.77-1.79 ms at S = K = 50; its waves were
// parked on s_waitcnt / the barrier 60 % of their cycles.  Pairs of tiles per
// barrier interval in that kernel, for balance: 1.4 % slower; its member offsets
// read two groups ahead: 1.5 % faster; this kernel: 3 % faster, 1.745 vs 1.80
// ms.  Per membership it issues ~8 VALU instructions (the 6 packed ops, the t
// address, the offset unpack): at ~53 % VALU busy on every SIMD, 1.3 ms would
// take ~72 %.  Half-width tiles (2 parameters per lane: 32 KiB of t, 3 blocks
// and 24 waves per CU, 73 VGPRs): bit-identical and 1 % slower, 1.739 vs 1.722
// ms — more waves to hide the waits do not pay for the extra instructions.)
//
// f32x4 add as 2 v_pk_add_f32 (packed fp32 issues two lanes' elements at the
// cost of one scalar op: tools/valu_rate_probe.hip measured 75 vs 38 T lane-op/s)
__device__ __forceinline__ f32x4 addu(f32x4 a, f32x4 b) { return a + b; }
typedef __attribute__((ext_vector_type(2))) uint32_t u32x2;
constexpr int kUnionWaves = 8;
constexpr int kUnionKMax = DLS_SUBSET_UNION_MAX / kUnionWaves;  // coalitions per wave (the plan caps it)
constexpr int kUnionListRow = kUnionChunk + 8;  // + the offsets read ahead of a list's end

// acc = fl(acc + fl(t_l / N)) over a coalition's members l < n, in order: t at
// byte offset ml[l] from tb (this lane's 16 B of client 0); cc = the coalition's
// UnionDiv constants.  tile_fast: every t of the tile is in the fast range.
__device__ __forceinline__ f32x4 union_walk(f32x4 acc, const char *tb, const uint16_t *ml, int n, f32x4 cc,
                                            bool tile_fast) {
    auto tload = [&](int l) { return *reinterpret_cast<const f32x4 *>(tb + ml[l]); };
    if (__builtin_expect(tile_fast, 1)) {
        // the coalition's constants as SGPRs (pk ops take them with op_sel, no VGPR
        // pair copies)
        const float cy = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(cc.x)));
        const float cl = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(cc.y)));
        const float cb = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(cc.z)));
        const f32x2 y2 = f32x2{cy, cy}, l2 = f32x2{cl, cl};
        const f32x2 b2 = f32x2{cb, cb};
        // the division method is decided once per coalition (two copies of the
        // member loop), not per member
        auto walk = [&](auto two_c) {
            constexpr bool TWO = decltype(two_c)::value;
            auto quot = [&](f32x4 t) {
                const f32x2 tl = f32x2{t.x, t.y}, th = f32x2{t.z, t.w};
                f32x2 ql, qh;
                if constexpr (TWO) {
                    ql = __builtin_elementwise_fma(tl, y2, tl * l2);
                    qh = __builtin_elementwise_fma(th, y2, th * l2);
                } else {
                    const f32x2 ql0 = tl * y2, qh0 = th * y2;
                    ql = __builtin_elementwise_fma(__builtin_elementwise_fma(-ql0, b2, tl), y2, ql0);
                    qh = __builtin_elementwise_fma(__builtin_elementwise_fma(-qh0, b2, th), y2, qh0);
                }
                return f32x4{ql.x, ql.y, qh.x, qh.y};
            };
            // groups of 4 members, ping-pong between two register sets (the next
            // group's t are read from LDS while this group's 4 independent
            // quotients are computed; no register rotation).  A group's 4 member
            // offsets (one broadcast 8-byte read) are read two groups ahead of its
            // t: the t reads depend on them, and read just before, their latency
            // would stall the wave once per group.
            auto offs = [&](int l0) { return *reinterpret_cast<const u32x2 *>(ml + l0); };
            auto tfetch = [&](u32x2 o, f32x4 (&x)[4]) {
                x[0] = *reinterpret_cast<const f32x4 *>(tb + (o.x & 0xffffu));
                x[1] = *reinterpret_cast<const f32x4 *>(tb + (o.x >> 16));
                x[2] = *reinterpret_cast<const f32x4 *>(tb + (o.y & 0xffffu));
                x[3] = *reinterpret_cast<const f32x4 *>(tb + (o.y >> 16));
            };
            auto group = [&](const f32x4 (&x)[4]) {
                const f32x4 q0 = quot(x[0]), q1 = quot(x[1]), q2 = quot(x[2]), q3 = quot(x[3]);
                acc = addu(addu(addu(addu(acc, q0), q1), q2), q3);
            };
            int l = 0;
            const int ng = n >> 2;  // whole groups
            if (ng > 0) {
                f32x4 xa[4], xb[4];
                u32x2 oa = offs(0), ob = offs(4);  // past the list: read, never used
                tfetch(oa, xa);
                oa = offs(8);
                int g = 0;
                for (; g + 2 < ng; g += 2) {
                    tfetch(ob, xb);
                    ob = offs(4 * (g + 3));
                    group(xa);
                    tfetch(oa, xa);
                    oa = offs(4 * (g + 4));
                    group(xb);
                }
                if (g + 1 < ng) {
                    tfetch(ob, xb);
                    group(xa);
                    group(xb);
                } else {
                    group(xa);
                }
                l = 4 * ng;
            }
            for (; l < n; ++l) acc = addu(acc, quot(tload(l)));
        };
        if ((__float_as_uint(cc.w) & 1u) != 0)  // wave-uniform
            walk(std::true_type{});
        else
            walk(std::false_type{});
    } else {  // zeros, denormals, huge values, inf / nan, divisors out of range
        FastDiv d;
        d.b = cc.z;
        d.y = cc.x;
        d.fast = (__float_as_uint(cc.w) & 2u) != 0;
        for (int l = 0; l < n; ++l) {
            const f32x4 t = tload(l);
            for (int e = 0; e < 4; ++e)
                acc[e] += (d.fast && in_fast_range(t[e])) ? markstein(t[e], d.b, d.y) : t[e] / d.b;
        }
    }
    return acc;
}

template <bool ACC>
__global__ __launch_bounds__(64 * kUnionWaves, 4) void k_subset_union(
    const f32x4 *__restrict__ Uv, int64_t ldu4, const int32_t *__restrict__ urows,
    const float *__restrict__ uw, const uint64_t *__restrict__ member, int Ku, UnionDiv dv, int S,
    int64_t P4, int64_t ntiles, f32x4 *__restrict__ out, int64_t ldo4) {
    constexpr int W = kUnionWaves, NL = kUnionChunk / kUnionWaves;
    static_assert(kUnionWaves * kUnionKMax >= DLS_SUBSET_UNION_MAX, "plan capacity");
    __shared__ f32x4 ts[kUnionChunk * 64];  // 64 KiB: one tile's t
    // member byte offsets in ts (client j: j * 1 KiB < 2^16), per coalition; a wave
    // reads 4 at a time as one broadcast 8-byte read (no readlane per member)
    __shared__ __attribute__((aligned(16))) uint16_t lst[DLS_SUBSET_UNION_MAX][kUnionListRow];
    __shared__ f32x4 cst[DLS_SUBSET_UNION_MAX];  // UnionDiv, per coalition
    __shared__ int lens[DLS_SUBSET_UNION_MAX];
    __shared__ int plan[W][kUnionKMax + 1];  // [0] = count, then coalitions
    __shared__ uint32_t tbad[W];
    const int64_t G = gridDim.x;
    int64_t tile = blockIdx.x;
    if (tile >= ntiles) return;  // block-uniform
    const int lane = __lane_id();
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int kk = min(lane, Ku - 1);
    const int tr = urows[kk];
    const float tw = uw[kk];
    const uint64_t mj = lane < Ku ? member[kk] : 0ull;
    // member lists (wave w builds coalitions w, w + W, ...)
    for (int c = wv; c < S; c += W) {
        const uint64_t in = __ballot((mj >> c) & 1ull);
        if ((mj >> c) & 1ull)
            lst[c][__builtin_amdgcn_mbcnt_hi((uint32_t)(in >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)in, 0u))] =
                (uint16_t)(lane << 10);
        if (lane == 0) {
            lens[c] = __popcll(in);
            cst[c] = dv.c[c];
        }
    }
    int fast = (int)(__ballot(!(tw >= 1.0f && tw <= 16777216.0f)) == 0);  // 1 <= n_j <= 2^24
    __syncthreads();
    if (wv == 0 && lane == 0) {  // LPT: longest coalition first, to the least loaded wave
        int load[W];
        for (int w = 0; w < W; ++w) {
            load[w] = 0;
            plan[w][0] = 0;
        }
        uint64_t done = 0;
        for (int it = 0; it < S; ++it) {
            int best = -1;
            for (int c = 0; c < S; ++c)
                if (!((done >> c) & 1ull) && (best < 0 || lens[c] > lens[best])) best = c;
            done |= 1ull << best;
            int bw = -1;
            for (int w = 0; w < W; ++w)
                if (plan[w][0] < kUnionKMax && (bw < 0 || load[w] < load[bw])) bw = w;
            plan[bw][1 + plan[bw][0]++] = best;
            load[bw] += lens[best] + 2;  // + the coalition's fixed cost
        }
    }
    // loader slots: wave wv stages clients wv + W l (l < NL) that exist; R holds
    // the loads of the next tile while this one is walked
    f32x4 R[NL];
    auto issue = [&](int64_t t) {
        const int64_t i0 = t * 64 + lane;
        const int64_t iq = i0 < P4 ? i0 : P4 - 1;
#pragma unroll
        for (int l = 0; l < NL; ++l) {
            const int j = wv + W * l;
            if (j < Ku) {
                const int64_t r = __builtin_amdgcn_readlane(tr, j);
                R[l] = load4<false>(Uv + r * ldu4 + iq);
            }
        }
    };
    auto stage = [&]() {  // t_j = fl(x_j * n_j) into ts; out-of-range flag
        uint32_t bad = 0;
#pragma unroll
        for (int l = 0; l < NL; ++l) {
            const int j = wv + W * l;
            if (j < Ku) {
                const float wk = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(tw), j));
                f32x4 t;
                t.x = R[l].x * wk;
                t.y = R[l].y * wk;
                t.z = R[l].z * wk;
                t.w = R[l].w * wk;
                ts[j * 64 + lane] = t;
                bad |= (uint32_t)(__ballot(!all_in_fast_range(t)) != 0);
            }
        }
        if (lane == 0) tbad[wv] = bad;
    };
    issue(tile);
    stage();
    if (tile + G < ntiles) issue(tile + G);
    __syncthreads();  // the first tile's t and the plan are ready
    const int nk = __builtin_amdgcn_readfirstlane(plan[wv][0]);
    int cid[kUnionKMax];
#pragma unroll
    for (int k = 0; k < kUnionKMax; ++k)
        cid[k] = __builtin_amdgcn_readfirstlane(plan[wv][1 + (k < nk ? k : 0)]);
#pragma unroll
    for (int k = 0; k < kUnionKMax; ++k)
        if (k < nk) fast &= (int)((__float_as_uint(cst[cid[k]].w) & 2u) != 0);
    const char *tb = reinterpret_cast<const char *>(ts) + 16 * lane;
    for (;;) {
        const int64_t i0 = tile * 64 + lane;
        const int64_t iq = i0 < P4 ? i0 : P4 - 1;
        uint32_t anybad = 0;
#pragma unroll
        for (int w = 0; w < W; ++w) anybad |= tbad[w];
        const bool tile_fast = fast && anybad == 0;
#pragma unroll
        for (int k = 0; k < kUnionKMax; ++k) {
            if (k >= nk) break;  // wave-uniform
            const int c = cid[k];
            f32x4 *dst = out + (int64_t)c * ldo4;
            const f32x4 acc = union_walk(ACC ? dst[iq] : f32x4{-0.f, -0.f, -0.f, -0.f}, tb, lst[c], lens[c],
                                         cst[c], tile_fast);
            if (i0 < P4) dst[i0] = acc;
        }
        const int64_t next = tile + G;
        if (next >= ntiles) break;  // block-uniform
        __syncthreads();  // every wave is done with this tile's t
        stage();           // the next tile's (its loads have landed by now)
        if (next + G < ntiles) issue(next + G);
        __syncthreads();
        tile = next;
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
    const int64_t P4 = P / 4;
    const int64_t ntiles = (P4 + 63) / 64;
    hipStream_t st = as_stream(stream);
    // division constants per coalition (host array sub_total): the exhaustive
    // two-constant checks of new divisors run in parallel, then cached
    UnionDiv dv;
    prove_two_constant(sub_total, S);
    for (int c = 0; c < S; ++c) {
        const FastDiv d = make_fastdiv2(sub_total[c]);
        const uint32_t flags = (d.two ? 1u : 0u) | (d.fast ? 2u : 0u);
        float f;
        memcpy(&f, &flags, 4);
        dv.c[c] = f32x4{d.y, d.yl, d.b, f};
    }
    for (int c = S; c < DLS_SUBSET_UNION_MAX; ++c) dv.c[c] = f32x4{1.f, 0.f, 1.f, 0.f};
    // unions of more than 64 clients: one launch per 64-client chunk, each
    // continuing the running sums in `out` (the same fp32 additions, in order)
    for (int32_t c0 = 0; c0 < Ku; c0 += kUnionChunk) {
        const int kc = Ku - c0 < kUnionChunk ? Ku - c0 : kUnionChunk;
        const int64_t blocks = resident_blocks(reinterpret_cast<const void *>(k_subset_union<false>),
                                               64 * kUnionWaves, 0);
        const dim3 grid((unsigned)(ntiles < blocks ? ntiles : blocks));
        auto launch = [&](auto kern) {
            hipLaunchKernelGGL(kern, grid, dim3(64 * kUnionWaves), 0, st,
                               reinterpret_cast<const f32x4 *>(U), ldu / 4, urows + c0,
                               uweight + c0, member + c0, kc, dv, (int)S, P4, ntiles,
                               reinterpret_cast<f32x4 *>(out), ldo / 4);
        };
        if (c0 == 0)
            launch(k_subset_union<false>);
        else  // a later chunk continues the running sums in `out`
            launch(k_subset_union<true>);
        const int rc = check_launch("dls_subset_fedavg_union_f32");
        if (rc != DLS_OK) return rc;
    }
    return DLS_OK;
}

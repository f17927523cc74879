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
//
// Persistent blocks of kUnionWaves waves walk 256-parameter tiles (a lane owns 4
// parameters).  Per tile the waves stage t_j of the <= 64 clients in LDS (each
// wave a few clients, register-staged: the NEXT tile's rows are loaded while
// this tile is computed, so HBM latency hides behind a whole tile of work);
// then wave w computes its coalitions (w, w + W, ...) coalition-major: it walks
// the coalition's member list (built once per block in LDS from the member
// masks) with 4 independent Markstein quotients in flight and the adds in list
// order.  No per-membership branches; a wave's results are stored at the start
// of the next tile, just before that tile's loads are issued, so the loads never
// wait behind younger stores (vmcnt counts both, in order).
// Algorithmic bytes: (Ku + S) * 4 per parameter.  VALU per parameter: 4 per
// (client, coalition) membership (Markstein's 3 + the add) + 1 per client for t;
// at S = Ku = 50 with half-full coalitions the VALU issue, not HBM, is the roof
// (DESIGN.md §4).
constexpr int kUnionChunk = 64;  // clients per launch (the host splits larger unions)

// in_fast_range (dls_common.h) of all four: 2^-60 <= |t| < 2^61 on the bit
// patterns (min / max of |bits|: zeros, denormals, inf and nan all fail)
__device__ __forceinline__ bool all_in_fast_range(f32x4 t) {
    const uint32_t a = __float_as_uint(t.x) & 0x7fffffffu, b = __float_as_uint(t.y) & 0x7fffffffu;
    const uint32_t c = __float_as_uint(t.z) & 0x7fffffffu, d = __float_as_uint(t.w) & 0x7fffffffu;
    const uint32_t mn = min(min(a, b), min(c, d)), mx = max(max(a, b), max(c, d));
    return mn >= (67u << 23) && mx < (188u << 23);
}
constexpr int kUnionWaves = 8;   // waves per block: <= 8 clients staged, <= KW coalitions each

// KW = ceil(S / 8) coalitions per wave (a template parameter, so that every wave
// issues exactly KW stores and NL loads per tile: the compiler's vmcnt waits
// are then exact, and waiting for the next tile's loads never waits for this
// tile's younger stores).
// Per-coalition division constants, computed on the host (dls_common.h FastDiv):
// {yh = RN(1/N), yl = RN(1/N - yh), N, flags}; flags bit 0: the two-constant
// quotient fma(t, yh, RN(t * yl)) is proven correctly rounded for this N (the
// host's exhaustive mantissa check), bit 1: N in Markstein's range [1, 2^31].
struct UnionDiv {
    f32x4 c[DLS_SUBSET_UNION_MAX];
};

template <int KW, bool ACC>
__global__ __launch_bounds__(64 * kUnionWaves) void k_subset_union(
    const f32x4 *__restrict__ Uv, int64_t ldu4, const int32_t *__restrict__ urows,
    const float *__restrict__ uw, const uint64_t *__restrict__ member, int Ku, UnionDiv dv, int S,
    int64_t P4, int64_t ntiles, f32x4 *__restrict__ out, int64_t ldo4) {
    constexpr int W = kUnionWaves, NL = kUnionChunk / kUnionWaves;
    // 69 KiB in all, so two blocks (16 waves) share a CU
    __shared__ f32x4 ts[kUnionChunk * 64];                    // 64 KiB: t_j of this tile
    __shared__ uint8_t lst[DLS_SUBSET_UNION_MAX][kUnionChunk];  // member positions, per coalition
    __shared__ f32x4 cst[DLS_SUBSET_UNION_MAX];               // UnionDiv, per coalition
    __shared__ uint32_t tbad[W];                              // per loader wave: t out of range
    int64_t tile = blockIdx.x;
    if (tile >= ntiles) return;  // block-uniform
    const int lane = __lane_id();
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    // client table: lane j holds client j's row and weight
    const int kk = min(lane, Ku - 1);
    const int tr = urows[kk];
    const float tw = uw[kk];
    const uint64_t mj = lane < Ku ? member[kk] : 0ull;
    // this wave's coalitions: wv + W k (k < nk); a wave without one (S < 8)
    // recomputes coalition S - 1 (the same bits, stored twice)
    int nk = (S - wv + W - 1) / W;
    const int cdup = nk > 0 ? -1 : S - 1;
    nk = nk > 0 ? nk : 1;
    auto coal = [&](int k) { return cdup >= 0 ? cdup : wv + W * k; };
    int len[KW];
    int fast = (int)(__ballot(!(tw >= 1.0f && tw <= 16777216.0f)) == 0);  // 1 <= n_j <= 2^24
#pragma unroll
    for (int k = 0; k < KW; ++k) {
        len[k] = 0;
        if (k < nk) {
            const int c = coal(k);
            const uint64_t in = __ballot((mj >> c) & 1ull);
            len[k] = __popcll(in);
            if (cdup < 0) {  // one wave builds each coalition's tables
                if ((mj >> c) & 1ull)
                    lst[c][__builtin_amdgcn_mbcnt_hi((uint32_t)(in >> 32),
                                                     __builtin_amdgcn_mbcnt_lo((uint32_t)in, 0u))] =
                        (uint8_t)lane;
                if (lane == 0) cst[c] = dv.c[c];
            }
            fast &= (int)((__float_as_uint(dv.c[c].w) & 2u) != 0);
        }
    }
    // loader slots: wave wv stages clients wv + W l, l < NL (past Ku: a duplicate
    // row, loaded but never staged, so the load count is static)
    f32x4 R[NL];
    auto issue = [&](int64_t t) {
        const int64_t i0 = t * 64 + lane;
        const int64_t iq = i0 < P4 ? i0 : P4 - 1;
#pragma unroll
        for (int l = 0; l < NL; ++l) {
            const int j = min(wv + W * l, Ku - 1);
            const int64_t r = __builtin_amdgcn_readlane(tr, j);
            R[l] = load4<false>(Uv + r * ldu4 + iq);
        }
    };
    f32x4 ain[KW];  // ACC: running sums of a previous 64-client chunk
    auto load_acc = [&](int64_t t) {
        const int64_t i0 = t * 64 + lane;
        const int64_t iq = i0 < P4 ? i0 : P4 - 1;
#pragma unroll
        for (int k = 0; k < KW; ++k)
            ain[k] = out[(int64_t)coal(k < nk ? k : nk - 1) * ldo4 + iq];
    };
    if (ACC) load_acc(tile);
    issue(tile);
    for (; tile < ntiles; tile += gridDim.x) {
        const int64_t i0 = tile * 64 + lane;
        const int64_t iq = i0 < P4 ? i0 : P4 - 1;
        __syncthreads();  // every wave is done reading the previous tile's t (and the tables)
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
        f32x4 acc_in[KW];
#pragma unroll
        for (int k = 0; k < KW; ++k)
            acc_in[k] = ACC ? ain[k] : f32x4{-0.f, -0.f, -0.f, -0.f};
        // the next tile's rows (the last tile reloads itself: a static load count)
        const int64_t next = tile + gridDim.x < ntiles ? tile + gridDim.x : tile;
        if (ACC) load_acc(next);
        issue(next);  // in flight during this tile's compute
        __syncthreads();
        uint32_t anybad = 0;
#pragma unroll
        for (int w = 0; w < W; ++w) anybad |= tbad[w];
        // Common case: every t of the tile in Markstein's range and every divisor in
        // [1, 2^31].  Otherwise (zeros, denormals, huge values, inf / nan) a compact
        // slow path with guarded division.  Both issue exactly KW stores.
        const bool tile_fast = fast && anybad == 0;
        f32x4 last = acc_in[0];
        int64_t lrow = (int64_t)coal(0) * ldo4;
#pragma unroll
        for (int k = 0; k < KW; ++k) {
            if (k < nk) {  // wave-uniform
                const int c = coal(k);
                f32x4 acc = acc_in[k];
                if (__builtin_expect(tile_fast, 1)) {
                    const f32x4 cc = cst[c];
                    const f32x2 y2 = f32x2{cc.x, cc.x}, l2 = f32x2{cc.y, cc.y};
                    const f32x2 b2 = f32x2{cc.z, cc.z};
                    const bool two = (__float_as_uint(cc.w) & 1u) != 0;  // wave-uniform
                    const uint32_t vl = (uint32_t)lst[c][lane] << 10;  // lane l: member l's offset
                    const int n = len[k];
                    // q = RN(t / N): two-constant (2 ops) when proven for N, else
                    // Markstein (3 ops); element pairs in v_pk_* (the scalar roundings)
                    auto quot = [&](f32x4 t) {
                        const f32x2 tl = f32x2{t.x, t.y}, th = f32x2{t.z, t.w};
                        f32x2 ql, qh;
                        if (two) {
                            ql = __builtin_elementwise_fma(tl, y2, tl * l2);
                            qh = __builtin_elementwise_fma(th, y2, th * l2);
                        } else {
                            const f32x2 ql0 = tl * y2, qh0 = th * y2;
                            ql = __builtin_elementwise_fma(__builtin_elementwise_fma(-ql0, b2, tl),
                                                           y2, ql0);
                            qh = __builtin_elementwise_fma(__builtin_elementwise_fma(-qh0, b2, th),
                                                           y2, qh0);
                        }
                        return f32x4{ql.x, ql.y, qh.x, qh.y};
                    };
                    auto tload = [&](int l) {
                        const uint32_t off = (uint32_t)__builtin_amdgcn_readlane((int)vl, l);
                        return *reinterpret_cast<const f32x4 *>(
                            reinterpret_cast<const char *>(ts) + off + 16 * lane);
                    };
                    int l = 0;
                    if (n >= 4) {
                        // groups of 4 members: the next group's t are read from LDS
                        // while this group's 4 independent quotients are computed;
                        // the adds stay in member order
                        f32x4 x0 = tload(0), x1 = tload(1), x2 = tload(2), x3 = tload(3);
                        for (; l + 8 <= n; l += 4) {
                            const f32x4 z0 = tload(l + 4), z1 = tload(l + 5);
                            const f32x4 z2 = tload(l + 6), z3 = tload(l + 7);
                            const f32x4 q0 = quot(x0), q1 = quot(x1), q2 = quot(x2), q3 = quot(x3);
                            acc = add4(add4(add4(add4(acc, q0), q1), q2), q3);
                            x0 = z0;
                            x1 = z1;
                            x2 = z2;
                            x3 = z3;
                        }
                        const f32x4 q0 = quot(x0), q1 = quot(x1), q2 = quot(x2), q3 = quot(x3);
                        acc = add4(add4(add4(add4(acc, q0), q1), q2), q3);
                        l += 4;
                    }
                    for (; l < n; ++l) acc = add4(acc, quot(tload(l)));
                } else {
                    const f32x4 cc = cst[c];
                    FastDiv d;
                    d.b = cc.z;
                    d.y = cc.x;
                    d.fast = (__float_as_uint(cc.w) & 2u) != 0;
                    for (int j = 0; j < Ku; ++j) {
                        if (!__builtin_amdgcn_readlane((int)((mj >> c) & 1ull), j)) continue;
                        const f32x4 t = ts[j * 64 + lane];
                        for (int e = 0; e < 4; ++e)
                            acc[e] += (d.fast && in_fast_range(t[e])) ? markstein(t[e], d.b, d.y)
                                                                      : t[e] / d.b;
                    }
                }
                last = acc;
                lrow = (int64_t)c * ldo4;
            }
            // exactly KW stores per wave and tile (past nk: the last one again; lanes
            // past P hold column P-1's value, iq: the same bits stored twice)
            out[lrow + iq] = last;
        }
    }
}

// Register-resident form: one wave per tile of 64*V parameters (a lane owns V
// consecutive ones), no LDS and no barriers.  The wave loads the tile's slice of
// all Ku client rows into registers (t[j], V*KU VGPRs), forms t_j = fl(x_j * n_j)
// in place, then walks the S coalitions one after another: coalition s's member
// mask over the union (a wave-uniform 64-bit ballot of the per-client coalition
// masks) drives a statically unrolled j loop whose scalar branches skip the
// non-members, so t[j] stays a static register and the adds follow union order.
// Per membership and element: the quotient (2 ops two-constant / 3 Markstein)
// and the add, nothing else; per (coalition, client) pair one scalar test.
// A tile with any t outside Markstein's range, or a coalition whose divisor is
// outside [1, 2^31], takes IEEE division for that coalition.
#ifndef DLS_UNION_REG
#define DLS_UNION_REG 2
#endif
#ifndef DLS_UNION_V
#define DLS_UNION_V 2
#endif
#ifndef DLS_UNION_SEL
#define DLS_UNION_KEEP_BRANCH asm volatile("")
#else
#define DLS_UNION_KEEP_BRANCH
#endif
constexpr int kUnionRegBlock = 256;

template <int V, int KU, bool ACC>
__global__ __launch_bounds__(kUnionRegBlock) void k_subset_union_reg(
    const float *__restrict__ U, int64_t ldu, const int32_t *__restrict__ urows,
    const float *__restrict__ uw, const uint64_t *__restrict__ member, int Ku, UnionDiv dv, int S,
    int64_t PV, float *__restrict__ out, int64_t ldo) {
    typedef float vf __attribute__((ext_vector_type(V)));
    const vf *__restrict__ Uv = reinterpret_cast<const vf *>(U);
    vf *__restrict__ ov = reinterpret_cast<vf *>(out);
    const int64_t ldv = ldu / V, ldov = ldo / V;
    const int lane = __lane_id();
    const int64_t tile = (int64_t)blockIdx.x * (kUnionRegBlock / 64) + (threadIdx.x >> 6);
    if (tile * 64 >= PV) return;  // wave-uniform
    const int64_t i0 = tile * 64 + lane;
    const int64_t iq = i0 < PV ? i0 : PV - 1;
    const int kk = min(lane, Ku - 1);
    const int tr = urows[kk];
    const float tw = uw[kk];
    const uint64_t mj = lane < Ku ? member[kk] : 0ull;
    // wave-uniform row base in a buffer descriptor (SALU) + the lane's 32-bit
    // byte offset: no 64-bit address VGPRs per client
    const int boff = (int)((uint32_t)iq * (uint32_t)sizeof(vf));
    vf t[KU];
#pragma unroll
    for (int j = 0; j < KU; ++j) {
        // past Ku: client Ku-1's slice again (same lines, a static load count)
        const int64_t r = __builtin_amdgcn_readlane(tr, j < Ku ? j : Ku - 1);
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<vf *>(Uv + r * ldv), 0,
                                                          (int)0xffffffffu, 0x00020000);
        if constexpr (V == 2)
            t[j] = __builtin_bit_cast(vf, __builtin_amdgcn_raw_buffer_load_b64(rs, boff, 0, 0));
        else
            t[j] = __builtin_bit_cast(vf, __builtin_amdgcn_raw_buffer_load_b128(rs, boff, 0, 0));
    }
    // min / max of |t| bit patterns over the tile: 2^-60 <= |t| < 2^61 for the
    // fast quotients (zeros, denormals, inf and nan all fail)
    uint32_t mn = 0xffffffffu, mx = 0;
#pragma unroll
    for (int j = 0; j < KU; ++j) {
        const float wk = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(tw), j < Ku ? j : Ku - 1));
#pragma unroll
        for (int e = 0; e < V; ++e) {
            t[j][e] = t[j][e] * wk;
            const uint32_t a = __float_as_uint(t[j][e]) & 0x7fffffffu;
            mn = min(mn, a);
            mx = max(mx, a);
        }
    }
    const bool tile_slow = __ballot(mn < (67u << 23) || mx >= (188u << 23)) != 0;  // wave-uniform
    for (int s = 0; s < S; ++s) {
        const uint64_t m = __ballot((mj >> s) & 1ull);  // coalition s's clients (bit j)
        const f32x4 cc = dv.c[s];
        const uint32_t flags = __float_as_uint(cc.w);
        vf acc;
        if (ACC)
            acc = ov[(int64_t)s * ldov + iq];
        else
#pragma unroll
            for (int e = 0; e < V; ++e) acc[e] = -0.f;
        if (!tile_slow && (flags & 3u) == 3u) {  // two-constant: q = fma(t, yh, RN(t*yl))
            const float yh = cc.x, yl = cc.y;
#pragma unroll
            for (int j = 0; j < KU; ++j)
                if ((m >> j) & 1ull) {
                    // an empty volatile asm keeps the branch (no if-conversion into
                    // selects, which would compute every pair)
                    DLS_UNION_KEEP_BRANCH;
#pragma unroll
                    for (int e = 0; e < V; ++e)
                        acc[e] = acc[e] + __builtin_fmaf(t[j][e], yh, t[j][e] * yl);
                }
        } else if (!tile_slow && (flags & 2u)) {  // Markstein
            const float y = cc.x, b = cc.z;
#pragma unroll
            for (int j = 0; j < KU; ++j)
                if ((m >> j) & 1ull) {
                    DLS_UNION_KEEP_BRANCH;
#pragma unroll
                    for (int e = 0; e < V; ++e) acc[e] = acc[e] + markstein(t[j][e], b, y);
                }
        } else {  // zeros, denormals, huge values, inf / nan, divisors out of range
            const float b = cc.z;
            for (int j = 0; j < Ku; ++j)
                if ((m >> j) & 1ull) {
                    // dynamic j: the row again from memory (L2-warm), t recomputed
                    const int64_t r = __builtin_amdgcn_readlane(tr, j);
                    const float wk = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(tw), j));
                    const vf x = Uv[r * ldv + iq];
#pragma unroll
                    for (int e = 0; e < V; ++e) acc[e] = acc[e] + (x[e] * wk) / b;
                }
        }
        if (i0 < PV) ov[(int64_t)s * ldov + i0] = acc;
    }
}


// Double-buffered LDS form (DLS_UNION_REG == 2).  One block of kU2Waves waves per
// CU, persistent over 256-parameter tiles (a lane owns 4).  The tile's t_j of
// the <= 64 union clients live in LDS, double-buffered: while the block computes
// tile i from one buffer, each wave's loads of tile i+1's rows are in flight, and
// after its coalitions it turns them into t_j in the other buffer — one barrier
// per tile.  The S coalitions are dealt to the waves once per block, longest
// first to the least loaded wave (a static LPT plan, so the per-tile barrier
// waits for a balanced set); a wave holds its coalitions' results in registers
// and stores them after staging the next tile, so its next loads never wait
// behind its stores.  Per membership: one ds_read_b128 of t (4 parameters), the
// quotient (2 ops two-constant / 3 Markstein, element pairs packed) and the add.
#ifndef DLS_UNION_SCALAR
#define DLS_UNION_SCALAR 0
#endif
// f32x4 add as 4 scalar v_add_f32 (DLS_UNION_SCALAR) or 2 v_pk_add_f32
__device__ __forceinline__ f32x4 addu(f32x4 a, f32x4 b) {
#if DLS_UNION_SCALAR
    f32x4 r;
    r.x = a.x + b.x;
    r.y = a.y + b.y;
    r.z = a.z + b.z;
    r.w = a.w + b.w;
    return r;
#else
    return a + b;
#endif
}
constexpr int kU2Waves = 16;
constexpr int kU2KMax = 8;   // coalitions per wave (the plan caps it; 16 x 8 >= 64)

template <bool ACC>
__global__ __launch_bounds__(64 * kU2Waves) void k_subset_union2(
    const f32x4 *__restrict__ Uv, int64_t ldu4, const int32_t *__restrict__ urows,
    const float *__restrict__ uw, const uint64_t *__restrict__ member, int Ku, UnionDiv dv, int S,
    int64_t P4, int64_t ntiles, f32x4 *__restrict__ out, int64_t ldo4) {
    constexpr int W = kU2Waves, NL = kUnionChunk / kU2Waves;
    __shared__ f32x4 ts[2][kUnionChunk * 64];                   // 2 x 64 KiB
    __shared__ uint8_t lst[DLS_SUBSET_UNION_MAX][kUnionChunk];  // member positions, per coalition
    __shared__ f32x4 cst[DLS_SUBSET_UNION_MAX];                 // UnionDiv, per coalition
    __shared__ int lens[DLS_SUBSET_UNION_MAX];
    __shared__ int plan[W][kU2KMax + 1];                        // [0] = count, then coalitions
    __shared__ uint32_t tbad[2][W];
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
            lst[c][__builtin_amdgcn_mbcnt_hi((uint32_t)(in >> 32),
                                             __builtin_amdgcn_mbcnt_lo((uint32_t)in, 0u))] =
                (uint8_t)lane;
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
                if (plan[w][0] < kU2KMax && (bw < 0 || load[w] < load[bw])) bw = w;
            plan[bw][1 + plan[bw][0]++] = best;
            load[bw] += lens[best] + 2;  // + the coalition's fixed cost
        }
    }
    // loader slots: wave wv stages clients wv + W l (l < NL) that exist
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
    auto stage = [&](int b) {  // t_j = fl(x_j * n_j) into buffer b; out-of-range flag
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
                ts[b][j * 64 + lane] = t;
                bad |= (uint32_t)(__ballot(!all_in_fast_range(t)) != 0);
            }
        }
        if (lane == 0) tbad[b][wv] = bad;
    };
    issue(tile);
    stage(0);
    __syncthreads();  // buffer 0 and the plan are ready
    const int nk = __builtin_amdgcn_readfirstlane(plan[wv][0]);
    int cid[kU2KMax];
#pragma unroll
    for (int k = 0; k < kU2KMax; ++k)
        cid[k] = __builtin_amdgcn_readfirstlane(plan[wv][1 + (k < nk ? k : 0)]);
#pragma unroll
    for (int k = 0; k < kU2KMax; ++k)
        if (k < nk) fast &= (int)((__float_as_uint(cst[cid[k]].w) & 2u) != 0);
    int b = 0;
    for (; tile < ntiles; tile += gridDim.x, b ^= 1) {
        const int64_t i0 = tile * 64 + lane;
        const int64_t iq = i0 < P4 ? i0 : P4 - 1;
        const int64_t next = tile + gridDim.x;
        f32x4 res[kU2KMax];
#pragma unroll
        for (int k = 0; k < kU2KMax; ++k)
            if (ACC && k < nk) res[k] = out[(int64_t)cid[k] * ldo4 + iq];
        if (next < ntiles) issue(next);  // in flight during this tile's coalitions
        uint32_t anybad = 0;
#pragma unroll
        for (int w = 0; w < W; ++w) anybad |= tbad[b][w];
        const bool tile_fast = fast && anybad == 0;
        const char *tb = reinterpret_cast<const char *>(ts[b]) + 16 * lane;
#pragma unroll
        for (int k = 0; k < kU2KMax; ++k) {
            if (k >= nk) break;  // wave-uniform
            const int c = cid[k];
            f32x4 acc = ACC ? res[k] : f32x4{-0.f, -0.f, -0.f, -0.f};
            const f32x4 cc = cst[c];
            const int n = lens[c];
            const uint32_t vl = (uint32_t)lst[c][lane] << 10;  // lane l: member l's offset
            auto tload = [&](int l) {
                const uint32_t off = (uint32_t)__builtin_amdgcn_readlane((int)vl, l);
                return *reinterpret_cast<const f32x4 *>(tb + off);
            };
            if (__builtin_expect(tile_fast, 1)) {
                const f32x2 y2 = f32x2{cc.x, cc.x}, l2 = f32x2{cc.y, cc.y};
                const f32x2 b2 = f32x2{cc.z, cc.z};
                // the division method is decided once per coalition (two copies of
                // the member loop), not per member
                auto walk = [&](auto two_c) {
                    constexpr bool TWO = decltype(two_c)::value;
                    auto quot = [&](f32x4 t) {
#if DLS_UNION_SCALAR
                        f32x4 q;
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            if constexpr (TWO) {
                                q[e] = __builtin_fmaf(t[e], cc.x, t[e] * cc.y);
                            } else {
                                const float q0 = t[e] * cc.x;
                                q[e] = __builtin_fmaf(__builtin_fmaf(-q0, cc.z, t[e]), cc.x, q0);
                            }
                        }
                        return q;
#endif
                        const f32x2 tl = f32x2{t.x, t.y}, th = f32x2{t.z, t.w};
                        f32x2 ql, qh;
                        if constexpr (TWO) {
                            ql = __builtin_elementwise_fma(tl, y2, tl * l2);
                            qh = __builtin_elementwise_fma(th, y2, th * l2);
                        } else {
                            const f32x2 ql0 = tl * y2, qh0 = th * y2;
                            ql = __builtin_elementwise_fma(__builtin_elementwise_fma(-ql0, b2, tl),
                                                           y2, ql0);
                            qh = __builtin_elementwise_fma(__builtin_elementwise_fma(-qh0, b2, th),
                                                           y2, qh0);
                        }
                        return f32x4{ql.x, ql.y, qh.x, qh.y};
                    };
                    int l = 0;
                    if (n >= 4) {
                        f32x4 x0 = tload(0), x1 = tload(1), x2 = tload(2), x3 = tload(3);
                        for (; l + 8 <= n; l += 4) {
                            const f32x4 z0 = tload(l + 4), z1 = tload(l + 5);
                            const f32x4 z2 = tload(l + 6), z3 = tload(l + 7);
                            const f32x4 q0 = quot(x0), q1 = quot(x1), q2 = quot(x2), q3 = quot(x3);
                            acc = addu(addu(addu(addu(acc, q0), q1), q2), q3);
                            x0 = z0;
                            x1 = z1;
                            x2 = z2;
                            x3 = z3;
                        }
                        const f32x4 q0 = quot(x0), q1 = quot(x1), q2 = quot(x2), q3 = quot(x3);
                        acc = addu(addu(addu(addu(acc, q0), q1), q2), q3);
                        l += 4;
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
                        acc[e] += (d.fast && in_fast_range(t[e])) ? markstein(t[e], d.b, d.y)
                                                                  : t[e] / d.b;
                }
            }
            res[k] = acc;
        }
        if (next < ntiles) stage(b ^ 1);  // the next tile's t (its loads have landed by now)
#pragma unroll
        for (int k = 0; k < kU2KMax; ++k)
            if (k < nk && i0 < P4) out[(int64_t)cid[k] * ldo4 + i0] = res[k];
        __syncthreads();  // buffer b ^ 1 is complete; buffer b free for the tile after next
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
#if DLS_UNION_REG == 2
        {
            auto launch2 = [&](auto kern) {
                const int64_t blocks =
                    resident_blocks(reinterpret_cast<const void *>(kern), 64 * kU2Waves, 0);
                const dim3 grid((unsigned)(ntiles < blocks ? ntiles : blocks));
                hipLaunchKernelGGL(kern, grid, dim3(64 * kU2Waves), 0, st,
                                   reinterpret_cast<const f32x4 *>(U), ldu / 4, urows + c0,
                                   uweight + c0, member + c0, kc, dv, (int)S, P4, ntiles,
                                   reinterpret_cast<f32x4 *>(out), ldo / 4);
            };
            if (c0 == 0)
                launch2(k_subset_union2<false>);
            else  // a later chunk continues the running sums in `out`
                launch2(k_subset_union2<true>);
            const int rc = check_launch("dls_subset_fedavg_union_f32");
            if (rc != DLS_OK) return rc;
            continue;
        }
#elif DLS_UNION_REG
        {
            constexpr int V = DLS_UNION_V;
            const int64_t PV = P / V;
            const int64_t waves = (PV + 63) / 64;
            const dim3 grid((unsigned)((waves + kUnionRegBlock / 64 - 1) / (kUnionRegBlock / 64)));
            auto launch = [&](auto kern) {
                hipLaunchKernelGGL(kern, grid, dim3(kUnionRegBlock), 0, st, U, ldu, urows + c0,
                                   uweight + c0, member + c0, kc, dv, (int)S, PV, out, ldo);
            };
            // KU = the chunk's client count rounded up to 8 (V*KU registers of t)
#define DLS_UNION_REG_KU(K_)                                          \
    case K_ / 8:                                                      \
        if (c0 == 0)                                                  \
            launch(k_subset_union_reg<V, K_, false>);                 \
        else /* a later chunk continues the running sums in `out` */ \
            launch(k_subset_union_reg<V, K_, true>);                  \
        break;
            switch ((kc + 7) / 8) {
                DLS_UNION_REG_KU(8)
                DLS_UNION_REG_KU(16)
                DLS_UNION_REG_KU(24)
                DLS_UNION_REG_KU(32)
                DLS_UNION_REG_KU(40)
                DLS_UNION_REG_KU(48)
                DLS_UNION_REG_KU(56)
                DLS_UNION_REG_KU(64)
            }
#undef DLS_UNION_REG_KU
            const int rc = check_launch("dls_subset_fedavg_union_f32");
            if (rc != DLS_OK) return rc;
            continue;
        }
#endif
        auto launch = [&](auto kern) {
            const int64_t blocks =
                resident_blocks(reinterpret_cast<const void *>(kern), 64 * kUnionWaves, 0);
            const dim3 grid((unsigned)(ntiles < blocks ? ntiles : blocks));
            hipLaunchKernelGGL(kern, grid, dim3(64 * kUnionWaves), 0, st,
                               reinterpret_cast<const f32x4 *>(U), ldu / 4, urows + c0,
                               uweight + c0, member + c0, kc, dv, (int)S, P4, ntiles,
                               reinterpret_cast<f32x4 *>(out), ldo / 4);
        };
        const int kw = (S + kUnionWaves - 1) / kUnionWaves;
        static_assert(DLS_SUBSET_UNION_MAX == 8 * kUnionWaves, "KW instances 1..8");
#define DLS_UNION_KW(K_)                                                 \
    case K_:                                                             \
        if (c0 == 0)                                                     \
            launch(k_subset_union<K_, false>);                           \
        else /* a later chunk continues the running sums in `out` */    \
            launch(k_subset_union<K_, true>);                            \
        break;
        switch (kw) {
            DLS_UNION_KW(1)
            DLS_UNION_KW(2)
            DLS_UNION_KW(3)
            DLS_UNION_KW(4)
            DLS_UNION_KW(5)
            DLS_UNION_KW(6)
            DLS_UNION_KW(7)
            DLS_UNION_KW(8)
        }
#undef DLS_UNION_KW
        const int rc = check_launch("dls_subset_fedavg_union_f32");
        if (rc != DLS_OK) return rc;
    }
    return DLS_OK;
}

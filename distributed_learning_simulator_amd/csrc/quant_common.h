// Client-walk helpers of the fused dequant-FedAvg kernels (quant.hip,
// quant_fma.hip) and the walks of the two small tile groups both modes share:
// fp32 tensors and int tensors with short channel rows (bit-exact reference
// arithmetic in either mode).
#pragma once

#include "dls_common.h"

namespace dls {
namespace quant {

__device__ __forceinline__ bool scale_fast(float sw) {
    // |q - zp| in [1, 383]: fl(deq*n) then lies in [2^-60, 2^60] (dls_common.h)
    return sw >= 0x1p-59f && sw <= 0x1p50f;
}

__device__ __forceinline__ int readlane_i(int v, int j) { return __builtin_amdgcn_readlane(v, j); }
__device__ __forceinline__ float readlane_f(float v, int j) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), j));
}

// (scale, zero point) pairs: pair of (client row r, channel c) at
// sz[r * row + c * chan] (strides in pairs).  The store keeps them channel-major
// (chan = capacity, row = 1), so a wave's per-chunk table load for its channel
// reads 64 consecutive pairs instead of 64 lines 107 KB apart.
struct SzLayout {
    int64_t row, chan;
};

// --------------------------------------------------------- client pipeline
// Clients are walked in chunks of 64.  Lane j holds client (base + j)'s row
// and weight (one coalesced vector load per field and chunk, fetched a chunk
// ahead), read back as wave-uniform values with v_readlane, so no scalar load
// sits on the streaming loop's critical path.  Within a chunk, batches of U
// clients are double-buffered: batch b+1's loads are issued before batch b is
// reduced.  Loads inside the steady-state loop are unconditional, so every
// reduction waits with an exact vmcnt.  All 64 lanes must run this (no lane
// may have exited early).
template <int U, class Batch, class Load, class Consume, class Single>
__device__ __forceinline__ void chunk_pipeline(int n, Load load, Consume consume, Single single) {
    const int nb = n / U;
    int j = 0;
    if (nb > 0) {
        Batch A, B;
        load(0, A);
        int b = 0;
        for (; b + 2 < nb; b += 2) {
            load((b + 1) * U, B);
            consume(A);
            load((b + 2) * U, A);
            consume(B);
        }
        if (b + 1 < nb) {
            load((b + 1) * U, B);
            consume(A);
            consume(B);
        } else {
            consume(A);
        }
        j = nb * U;
    }
    for (; j < n; ++j) single(j);
}

// The same walk with the drain written so that no batch's code appears in both
// arms of a branch (the compiler hoists such a common prefix, and with it every
// conversion of the batch, above the first scheduling barrier).
template <int U, class Batch, class Load, class Consume, class Single>
__device__ __forceinline__ void chunk_pipeline_1tail(int n, Load load, Consume consume,
                                                     Single single) {
    const int nb = n / U;
    if (nb > 0) {
        Batch A, B;
        load(0, A);
        int b = 0;
        for (; b + 2 < nb; b += 2) {
            load((b + 1) * U, B);
            consume(A);
            load((b + 2) * U, A);
            consume(B);
        }
        const bool two = b + 1 < nb;
        if (two) load((b + 1) * U, B);
        consume(A);
        if (two) consume(B);
    }
    for (int j = nb * U; j < n; ++j) single(j);
}

struct ChunkRows {
    int r0, r1, r2;   // rows of chunks c, c+1, c+2 (lane j: client 64c + j)
    float w0, w1, w2;
    __device__ __forceinline__ void fetch(const int32_t *rows, const float *w, int K, int k,
                                          int &r, float &wk) {
        const int kk = min(k + __lane_id(), K - 1);  // past the end: harmless duplicates
        r = rows[kk];
        wk = w[kk];
    }
    __device__ __forceinline__ void init(const int32_t *rows, const float *w, int K) {
        fetch(rows, w, K, 0, r0, w0);
        fetch(rows, w, K, 64, r1, w1);
        fetch(rows, w, K, 128, r2, w2);
    }
    __device__ __forceinline__ void advance(const int32_t *rows, const float *w, int K, int base) {
        r0 = r1;
        w0 = w1;
        r1 = r2;
        w1 = w2;
        fetch(rows, w, K, base + 192, r2, w2);
    }
};

// fp32 tensors (biases, norm weights) as their own group: tiles of <= 256
// elements, a lane owning 4, walked like dls_fedavg_f32's pipelined kernel —
// batches of kF32U clients double-buffered — so that the few waves of a small
// tensor keep 2 * kF32U client rows in flight instead of one dependent load per
// client (with K = 1000 clients the unpipelined loop is a ~2 ms latency chain).
constexpr int kF32U = 16;
template <int U = kF32U>
__device__ __forceinline__ void f32_side_tile(const dls_qtile &t, const float *__restrict__ F,
                                              int64_t ldf, const int32_t *__restrict__ rows,
                                              const float *__restrict__ w, int K, const FastDiv &d,
                                              float *__restrict__ out) {
    const int e0 = 4 * __lane_id();
    const int lenpad = (t.len + 63) & ~63;
    const int ec = e0 < lenpad ? e0 : lenpad - 4;  // idle lanes load a valid duplicate
    const float *src = F + t.src + ec;
    f32x4 acc = f32x4{-0.f, -0.f, -0.f, -0.f};
    auto term = [&](f32x4 x, float wk) {
        f32x4 t, q;
#pragma unroll
        for (int c = 0; c < 4; ++c) t[c] = x[c] * wk;
        const bool ok = d.fast && in_fast_range(t.x) && in_fast_range(t.y) && in_fast_range(t.z) &&
                        in_fast_range(t.w);
        if (__builtin_expect(__ballot(!ok) == 0, 1)) {  // wave-uniform common case
#pragma unroll
            for (int c = 0; c < 4; ++c) q[c] = markstein(t[c], d.b, d.y);
        } else {
#pragma unroll
            for (int c = 0; c < 4; ++c) q[c] = div_exact(t[c], d);
        }
        return q;
    };
    struct Batch {
        f32x4 x[U];
        float wk[U];
    };
    ChunkRows cr;
    cr.init(rows, w, K);
    for (int base = 0; base < K; base += 64) {
        const int tr = cr.r0;
        const float tw = cr.w0;
        cr.advance(rows, w, K, base);
        auto fetch = [&](int j, f32x4 &x, float &wk) {
            const int64_t r = readlane_i(tr, j);
            x = __builtin_nontemporal_load(reinterpret_cast<const f32x4 *>(src + r * ldf));
            wk = readlane_f(tw, j);
        };
        chunk_pipeline<U, Batch>(
            min(64, K - base),
            [&](int j0, Batch &b) {
#pragma unroll
                for (int u = 0; u < U; ++u) fetch(j0 + u, b.x[u], b.wk[u]);
            },
            [&](const Batch &b) {
#pragma unroll
                for (int u = 0; u < U; ++u) acc = acc + term(b.x[u], b.wk[u]);
            },
            [&](int j) {
                f32x4 x;
                float wk;
                fetch(j, x, wk);
                acc = acc + term(x, wk);
            });
    }
    if (e0 < lenpad) {
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[c] = e0 + c < t.len ? acc[c] : 0.f;  // keep padding zero
        *reinterpret_cast<f32x4 *>(out + t.dst + e0) = acc;
    }
}

// int tensors whose channel rows are not a multiple of 16 elements (the first
// conv of a CIFAR ResNet: rows of 27): tiles of <= 256 elements, a lane owning 4
// consecutive elements, which span at most two channels when rows are >= 4
// long; the reference formula fl(fl(fl(q - zp) * s) * n) / N per element, the
// pipelined client walk of k_dequant_f32.  Few waves, each a long client chain:
// kept small so that it neither starves nor thrashes the instruction cache.
template <bool SIGNED>
__device__ __forceinline__ float small_byte(uint32_t w, int k) {
    return SIGNED ? (float)(int8_t)(w >> (8 * k)) : (float)((w >> (8 * k)) & 0xffu);
}

__device__ __forceinline__ void small_side_tile(const dls_qtile &t, const uint8_t *__restrict__ Q,
                                                int64_t ldq, const f32x2 *__restrict__ sz, SzLayout L,
                                                const int32_t *__restrict__ rows,
                                                const float *__restrict__ w, int K, const FastDiv &d,
                                                float *__restrict__ out) {
    const bool sgn = t.kind == 1;
    const int e0 = 4 * __lane_id();
    const int lenpad = (t.len + 3) & ~3;
    const int ec = e0 < lenpad ? e0 : lenpad - 4;  // idle lanes load a valid duplicate
    const int p = t.row_pos + ec;
    const int c = min(t.chan0 + p / t.row_len, t.chan_end - 1);
    const int split = t.row_len - p % t.row_len;  // elements of this lane in channel c
    const int64_t ca = (int64_t)c * L.chan;
    const int64_t cb = (int64_t)min(c + 1, t.chan_end - 1) * L.chan;
    const uint8_t *src = Q + t.src + ec;
    f32x4 acc = f32x4{-0.f, -0.f, -0.f, -0.f};
    struct One {
        uint32_t q;
        f32x2 a, b;
        float wk;
    };
    constexpr int U = 8;
    struct Batch {
        One c[U];
    };
    auto step = [&](const One &o) {
        const bool fast = d.fast && scale_fast(o.a.x * o.wk) && scale_fast(o.b.x * o.wk);
        f32x4 tt;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const bool second = e >= split;
            const float x = sgn ? small_byte<true>(o.q, e) : small_byte<false>(o.q, e);
            tt[e] = ((x - (second ? o.b.y : o.a.y)) * (second ? o.b.x : o.a.x)) * o.wk;
        }
        if (__builtin_expect(__ballot(!fast) == 0, 1)) {
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[e] += markstein(tt[e], d.b, d.y);
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[e] += fast ? markstein(tt[e], d.b, d.y) : tt[e] / d.b;
        }
    };
    ChunkRows cr;
    cr.init(rows, w, K);
    for (int base = 0; base < K; base += 64) {
        const int tr = cr.r0;
        const float tw = cr.w0;
        cr.advance(rows, w, K, base);
        auto fetch = [&](int j, One &o) {
            const int64_t r = readlane_i(tr, j);
            o.q = __builtin_nontemporal_load(reinterpret_cast<const uint32_t *>(src + r * ldq));
            o.a = sz[ca + r * L.row];
            o.b = sz[cb + r * L.row];
            o.wk = readlane_f(tw, j);
        };
        chunk_pipeline<U, Batch>(
            min(64, K - base),
            [&](int j0, Batch &b) {
#pragma unroll
                for (int u = 0; u < U; ++u) fetch(j0 + u, b.c[u]);
            },
            [&](const Batch &b) {
#pragma unroll
                for (int u = 0; u < U; ++u) step(b.c[u]);
            },
            [&](int j) {
                One o;
                fetch(j, o);
                step(o);
            });
    }
    // tiles start 64-aligned in the output row: lanes up to the tensor's 64-element
    // row padding store, so the padding reads as zero (the re-quantization's
    // segment min / max spans it)
    if (e0 < ((t.len + 63) & ~63)) {
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[e] = e0 + e < t.len ? acc[e] : 0.f;  // keep padding zero
        *reinterpret_cast<f32x4 *>(out + t.dst + e0) = acc;
    }
}

}  // namespace quant
}  // namespace dls

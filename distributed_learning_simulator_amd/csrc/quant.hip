// fed_quant server path for gfx950: fused per-channel dequant + FedAvg,
// segmented min/max, MinMax qparams, affine (deterministic / stochastic) quantize.
//
// Reference: FedQuantServer._process_client_parameter (servers/fed_quant_server.py:25-33)
// dequantizes every client's int tensors to fp32 in a Python loop over output
// channels, then FedServer.get_subset_model (servers/fed_server.py:44-66) averages
// them.  Here one pass reads the int8 payloads once (1 B/param/client) and never
// materialises the fp32 client tensors:
//     out[e] (+)= fl(fl(fl(fl(q - zp[c]) * fl32(scale[c])) * fl32(n_i)) / fl32(N))
// bit-exact in client order.  Algorithmic bytes: K*(Pq + 4*Pf + 8*C) + 4*P.
#include <algorithm>
#include <type_traits>

#include "dls_common.h"
#include "quant_common.h"

namespace dls {
namespace {

using namespace quant;

constexpr int kBlock = 256;
constexpr int kQuantU = 2;      // clients per batch (1 KiB tiles); two batches in flight per lane
constexpr int kQuantUG = 1;     // clients per batch on multi-KiB tiles
constexpr int kQuantSched = 2;  // element pairs between scheduling barriers
#ifndef DLS_LANE_US
#define DLS_LANE_US 2
#endif
constexpr int kLaneUS = DLS_LANE_US;  // clients per batch on lane-channel tiles (staged path)
#ifndef DLS_LANE_USG
#define DLS_LANE_USG 1
#endif
constexpr int kLaneUSG = DLS_LANE_USG;  // the same on multi-KiB lane tiles
#ifndef DLS_LANE_SCHED
#define DLS_LANE_SCHED 2
#endif
constexpr int kLaneSched = DLS_LANE_SCHED;  // element pairs between scheduling barriers

__device__ __forceinline__ float byte_f32(uint32_t w, int k) {
    return (float)((w >> (8 * k)) & 0xffu);  // selects v_cvt_f32_ubyte{k}
}

__device__ __forceinline__ f32x2 pk_fma(f32x2 a, f32x2 b, f32x2 c) {
    return __builtin_elementwise_fma(a, b, c);
}

// ------------------------------------------------------------ int8 tiles
// One client's contribution to a lane's 16 consecutive elements of ONE channel
// (wave-uniform scale s and zero point z, already offset by 128 for int8 read
// as q ^ 0x80).  Packed fp32: every op below is a v_pk_*_f32 over two
// elements with the scalar ops' IEEE roundings.  When fl(z*s) is exact (always
// for symmetric int8, z = 128), fl((x - z)*s) == fma(x, s, -z*s): one op.
// Byte k of a dword as fp32: the unsigned value (v_cvt_f32_ubyteK) or, for
// int8, the sign-extended one (v_cvt_f32_i32 with an SDWA sext byte select):
// one VALU op either way.
template <bool SEXT>
__device__ __forceinline__ float byte_val(uint32_t w, int k) {
    if (SEXT) return (float)(int8_t)(w >> (8 * k));
    return (float)((w >> (8 * k)) & 0xffu);
}

// TWO: the two-constant division q = fma(t, yh, RN(t*yl)) (dls_common.h), valid
// for this divisor when the host's exhaustive check passed (d.two): 2 packed ops
// per element pair instead of Markstein's 3.
template <bool ZFMA, bool FAST, bool SEXT = false, bool TWO = false, int SCHED = kQuantSched>
__device__ __forceinline__ void accum16_one(float (&acc)[16], u32x4 qv, float s, float zs, float z,
                                            float wk, const FastDiv &d) {
    const f32x2 s2 = f32x2{s, s}, w2 = f32x2{wk, wk};
    const f32x2 nzs = f32x2{-zs, -zs}, z2 = f32x2{z, z};
    const f32x2 b2 = f32x2{d.b, d.b}, y2 = f32x2{d.y, d.y}, yl2 = f32x2{d.yl, d.yl};
#pragma unroll
    for (int j = 0; j < 16; j += 2) {
        const f32x2 x = f32x2{byte_val<SEXT>(qv[j >> 2], j & 3),
                              byte_val<SEXT>(qv[j >> 2], (j + 1) & 3)};
        const f32x2 deq = ZFMA ? pk_fma(x, s2, nzs) : (x - z2) * s2;
        const f32x2 t = deq * w2;
        f32x2 q;
        if (FAST && TWO) {
            q = pk_fma(t, y2, t * yl2);
        } else if (FAST) {
            const f32x2 q0 = t * y2;
            q = pk_fma(pk_fma(-q0, b2, t), y2, q0);
        } else {
            q = f32x2{t.x / d.b, t.y / d.b};
        }
        const f32x2 r = f32x2{acc[j], acc[j + 1]} + q;
        acc[j] = r.x;
        acc[j + 1] = r.y;
        // keep the scheduler from widening the chain over all 16 elements of
        // every in-flight client (that costs ~60 VGPRs and waves per SIMD)
        if (SCHED > 0 && (j / 2) % SCHED == SCHED - 1) __builtin_amdgcn_sched_barrier(0);
    }
}

// The common path of the lane tiles: sz = (s, -fl(z*s)) from the wave's LDS
// table.  Per step two element pairs, (j, j+1) and (j+8, j+9), as independent
// chains interleaved by hand: a packed op that reads the result of the packed op
// issued just before it costs an s_nop (4 cycles, as much as the op itself), and
// the compiler's schedule serialised the two chains (a third of the issue slots
// were s_nops).  The two-constant division (TWO) runs in the asm block;
// Markstein's (its rare fallback divisors) in plain code.  Each step ends in a
// scheduling barrier so that no later conversion is hoisted above it (hoisting
// all of a batch's conversions cost ~40 VGPRs).
template <bool SEXT, bool TWO>
__device__ __forceinline__ void accum16_pk(float (&acc)[16], u32x4 qv, f32x2 sz, float wk,
                                           const FastDiv &d) {
    const f32x2 w2 = f32x2{wk, wk};
    const f32x2 b2 = f32x2{d.b, d.b}, y2 = f32x2{d.y, d.y}, yl2 = f32x2{d.yl, d.yl};
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
        const int k = j & 3;
        const f32x2 xa = f32x2{byte_val<SEXT>(qv[j >> 2], k), byte_val<SEXT>(qv[j >> 2], k + 1)};
        const f32x2 xb = f32x2{byte_val<SEXT>(qv[(j >> 2) + 2], k),
                               byte_val<SEXT>(qv[(j >> 2) + 2], k + 1)};
        f32x2 ra = f32x2{acc[j], acc[j + 1]}, rb = f32x2{acc[j + 8], acc[j + 9]};
        if constexpr (TWO) {
            f32x2 ta, tb, la, lb;
            asm volatile(
                "v_pk_fma_f32 %[ta], %[xa], %[sz], %[sz] op_sel:[0,0,1] op_sel_hi:[1,0,1]\n\t"
                "v_pk_fma_f32 %[tb], %[xb], %[sz], %[sz] op_sel:[0,0,1] op_sel_hi:[1,0,1]\n\t"
                "v_pk_mul_f32 %[ta], %[w], %[ta]\n\t"
                "v_pk_mul_f32 %[tb], %[w], %[tb]\n\t"
                "v_pk_mul_f32 %[la], %[yl], %[ta]\n\t"
                "v_pk_mul_f32 %[lb], %[yl], %[tb]\n\t"
                "v_pk_fma_f32 %[ta], %[ta], %[y], %[la]\n\t"
                "v_pk_fma_f32 %[tb], %[tb], %[y], %[lb]\n\t"
                "v_pk_add_f32 %[ra], %[ra], %[ta]\n\t"
                "v_pk_add_f32 %[rb], %[rb], %[tb]"
                : [ra] "+v"(ra), [rb] "+v"(rb), [ta] "=&v"(ta), [tb] "=&v"(tb), [la] "=&v"(la),
                  [lb] "=&v"(lb)
                : [xa] "v"(xa), [xb] "v"(xb), [sz] "v"(sz), [w] "s"(w2), [yl] "s"(yl2),
                  [y] "s"(y2));
        } else {
            auto term = [&](f32x2 x) {
                const f32x2 t = pk_fma(x, sz.xx, sz.yy) * w2;
                const f32x2 q0 = t * y2;
                return pk_fma(pk_fma(-q0, b2, t), y2, q0);
            };
            ra = ra + term(xa);
            rb = rb + term(xb);
            asm volatile("" : "+v"(ra), "+v"(rb));
        }
        acc[j] = ra.x;
        acc[j + 1] = ra.y;
        acc[j + 8] = rb.x;
        acc[j + 9] = rb.y;
        __builtin_amdgcn_sched_barrier(0);
    }
}

// DLS_FEDAVG_FMA (zero point 0): acc = fma(q, c, acc), c = fl(fl(s * n_i) / N) of
// the (client, channel): 2 conversions + 1 packed fma per element pair; cz.x
// holds c (op_sel_hi reads it for both halves).  Two independent pairs per step.
template <bool SEXT>
__device__ __forceinline__ void accum16_fma(float (&acc)[16], u32x4 qv, f32x2 cz) {
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
        const int k = j & 3;
        const f32x2 xa = f32x2{byte_val<SEXT>(qv[j >> 2], k), byte_val<SEXT>(qv[j >> 2], k + 1)};
        const f32x2 xb = f32x2{byte_val<SEXT>(qv[(j >> 2) + 2], k),
                               byte_val<SEXT>(qv[(j >> 2) + 2], k + 1)};
        f32x2 ra = f32x2{acc[j], acc[j + 1]}, rb = f32x2{acc[j + 8], acc[j + 9]};
        asm volatile(
            "v_pk_fma_f32 %[ra], %[xa], %[cz], %[ra] op_sel_hi:[1,0,1]\n\t"
            "v_pk_fma_f32 %[rb], %[xb], %[cz], %[rb] op_sel_hi:[1,0,1]"
            : [ra] "+v"(ra), [rb] "+v"(rb)
            : [xa] "v"(xa), [xb] "v"(xb), [cz] "v"(cz));
        acc[j] = ra.x;
        acc[j + 1] = ra.y;
        acc[j + 8] = rb.x;
        acc[j + 9] = rb.y;
        // no later conversion is hoisted above this step (hoisting every in-flight
        // client's conversions costs registers, and with them waves per SIMD)
        __builtin_amdgcn_sched_barrier(0);
    }
}

// FMA-mode constant of a (client, channel): fl(fl(s * n_i) / N) (IEEE division,
// once per chunk and channel)
__device__ __forceinline__ float fma_coef(float s, float wk, float N) { return (s * wk) / N; }

// FMA mode: every lane-tile width in one launch (k_dequant_lanes_fma_any); 0: one
// launch per width, the narrower ones on side streams (A/B knob)
#ifndef DLS_QUANT_FMA_ANY
#define DLS_QUANT_FMA_ANY 1
#endif
constexpr bool kQuantFmaAny = DLS_QUANT_FMA_ANY != 0;
// FMA mode: groups 0-7 on the one-wave-per-SIMD kernel (quant_fma.hip); 0: the round-4
// launches (k_dequant_fast_fma pieces + k_dequant_lanes_fma_any), an A/B knob
#ifndef DLS_QUANT_FMA_STREAM
#define DLS_QUANT_FMA_STREAM 1
#endif
constexpr bool kQuantFmaStream = DLS_QUANT_FMA_STREAM != 0;
#ifndef DLS_QUANT_PIECE_WPS
#define DLS_QUANT_PIECE_WPS 0  // > 0: the grouped kernels' launch pieces of this many waves per SIMD
#endif
constexpr int kQuantPieceWps = DLS_QUANT_PIECE_WPS;
#ifndef DLS_QUANT_NTSTORE
#define DLS_QUANT_NTSTORE 0  // 1: non-temporal output stores in store_tile (A/B knob)
#endif

#ifndef DLS_QUANT_PROBE
#define DLS_QUANT_PROBE 0  // 1: stream-only timing probe (loads + a xor per dword; wrong output)
// 2: as 1, and lane_tile skips its per-chunk scale staging (no sz gathers, LDS table, ballot)
// 3: as 2, and lane_tile addresses client j of a chunk as row base + j (no v_readlane)
#endif

template <int U, int GN>
struct QBatch {
    u32x4 qv[U][GN];
    float s[U], z[U], wk[U];
};

template <bool SIGNED, int G, bool TWO>
__device__ __forceinline__ void int_one_channel(float (&acc)[G][16], const uint8_t *__restrict__ Q,
                                                const uint32_t (&qoff)[G], int64_t ldq,
                                                const f32x2 *__restrict__ szc, SzLayout L,
                                                const int32_t *__restrict__ rows,
                                                const float *__restrict__ w, int K,
                                                const FastDiv &d) {
    // int8 bytes convert sign-extended (value q, zero point zp); uint8 bytes
    // unsigned.  The payload address is (Q + row*ldq) [wave-uniform, SALU] +
    // qoff[g] [this lane's 32-bit offset in KiB slice g of the tile].
    ChunkRows cr;
    cr.init(rows, w, K);
    f32x2 nsz = szc[(int64_t)cr.r0 * L.row];  // this wave's channel, client 64c + lane
    for (int base = 0; base < K; base += 64) {
        const int tr = cr.r0;
        const float tw = cr.w0;
        const f32x2 tsz = nsz;
        nsz = szc[(int64_t)cr.r1 * L.row];  // next chunk (its rows landed a chunk ago)
        cr.advance(rows, w, K, base);
        const int n = min(64, K - base);
        // one wave-uniform decision per chunk: if every client of the chunk takes
        // the common path (exact fl(z*s) and the fast division), the streaming loop
        // carries that path alone, reading (scale, -fl(z*s)) straight from the table
        const float ls = tsz.x, lz = tsz.y, lzs = lz * ls;
        const bool lfast = __builtin_fmaf(lz, ls, -lzs) == 0.f && d.fast && scale_fast(ls * tw);
        const bool allfast = __ballot(!lfast && __lane_id() < n) == 0;
        const float tnzs = -lzs;
        // slices [G0, G0 + GN) of the tile, clients of this chunk
        auto run = [&](auto common_only, auto g0, auto gn) {
            constexpr bool COMMON = decltype(common_only)::value;
            constexpr int G0 = decltype(g0)::value, GN = decltype(gn)::value;
            constexpr int U = GN > 1 ? kQuantUG : kQuantU;  // clients per batch
            auto fetch = [&](int j, u32x4 (&qv)[GN], float &sc, float &zz, float &wk) {
                const int64_t r = readlane_i(tr, j);
                // wave-uniform row base in a buffer descriptor (SALU), lane offset in
                // a VGPR: buffer_load ... offen nt, no VALU address arithmetic per client
                const auto rs = __builtin_amdgcn_make_buffer_rsrc(
                    const_cast<uint8_t *>(Q + r * ldq), 0, (int)0xffffffffu, 0x00020000);  // 4 GiB
#pragma unroll
                for (int g = 0; g < GN; ++g)
                    qv[g] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)qoff[G0 + g], 0, 2 /* nt */);
                wk = readlane_f(tw, j);
                sc = readlane_f(tsz.x, j);
                zz = COMMON ? readlane_f(tnzs, j) : readlane_f(tsz.y, j);  // -z*s or z
            };
            auto step = [&](const u32x4 (&qv)[GN], float sc, float zz, float wk) {
                if constexpr (COMMON) {
#pragma unroll
                    for (int g = 0; g < GN; ++g)
                        accum16_one<true, true, SIGNED, TWO>(acc[G0 + g], qv[g], sc, -zz, 0.f, wk, d);
                } else {
                    const float zs = zz * sc;
                    const bool zfma = __builtin_fmaf(zz, sc, -zs) == 0.f;  // fl(z*s) exact
                    const bool fast = d.fast && scale_fast(sc * wk);
                    // client-uniform path choice, outside the slice loop
                    if (__builtin_expect(zfma && fast, 1)) {
#pragma unroll
                        for (int g = 0; g < GN; ++g)
                            accum16_one<true, true, SIGNED>(acc[G0 + g], qv[g], sc, zs, zz, wk, d);
                    } else if (fast) {
#pragma unroll
                        for (int g = 0; g < GN; ++g)
                            accum16_one<false, true, SIGNED>(acc[G0 + g], qv[g], sc, zs, zz, wk, d);
                    } else {
#pragma unroll
                        for (int g = 0; g < GN; ++g)
                            accum16_one<false, false, SIGNED>(acc[G0 + g], qv[g], sc, zs, zz, wk, d);
                    }
                }
            };
            chunk_pipeline<U, QBatch<U, GN>>(
                n,
                [&](int j0, QBatch<U, GN> &bt) {
#pragma unroll
                    for (int u = 0; u < U; ++u) fetch(j0 + u, bt.qv[u], bt.s[u], bt.z[u], bt.wk[u]);
                },
                [&](const QBatch<U, GN> &bt) {
#pragma unroll
                    for (int u = 0; u < U; ++u) step(bt.qv[u], bt.s[u], bt.z[u], bt.wk[u]);
                },
                [&](int j) {
                    u32x4 qv[GN];
                    float sc, zz, wk;
                    fetch(j, qv, sc, zz, wk);
                    step(qv, sc, zz, wk);
                });
        };
        using I0 = std::integral_constant<int, 0>;
        using IG = std::integral_constant<int, G>;
        using I1 = std::integral_constant<int, 1>;
        if (allfast) {
            run(std::true_type{}, I0{}, IG{});
        } else {
            // rare chunks (inexact fl(z*s), out-of-range scales): one slice at a
            // time, so that this path's registers stay within the common path's
            run(std::false_type{}, I0{}, I1{});
            if constexpr (G > 1) run(std::false_type{}, std::integral_constant<int, 1>{}, I1{});
            if constexpr (G > 2) run(std::false_type{}, std::integral_constant<int, 2>{}, I1{});
            if constexpr (G > 3) run(std::false_type{}, std::integral_constant<int, 3>{}, I1{});
        }
    }
}

// Lanes of the wave in different channels (and a lane possibly straddling a
// channel boundary at `split`): per-lane (scale, zero point) loads.
template <bool SIGNED>
__device__ __forceinline__ void int_lane_channels(float (&acc)[16], const uint8_t *__restrict__ Qt,
                                                  int64_t ldq, const f32x2 *__restrict__ szc,
                                                  SzLayout L, int split,
                                                  const int32_t *__restrict__ rows,
                                                  const float *__restrict__ w, int K,
                                                  const FastDiv &d) {
    ChunkRows cr;
    cr.init(rows, w, K);
    const float zadj = SIGNED ? 128.f : 0.f;
    const bool two = split < 16;
    struct One {
        u32x4 qv;
        f32x2 a, b;
        float wk;
    };
    constexpr int U = 8;  // clients per batch, double-buffered: a few waves walk all K clients, so
                          // the loads of 2U clients in flight set the time (a latency chain)
    struct Batch {
        One c[U];
    };
    for (int base = 0; base < K; base += 64) {
        const int tr = cr.r0;
        const float tw = cr.w0;
        cr.advance(rows, w, K, base);
        auto fetch = [&](int j, One &o) {
            const int64_t r = readlane_i(tr, j);
            o.wk = readlane_f(tw, j);
            o.qv = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(Qt + r * ldq));
            o.a = szc[r * L.row];
            o.b = two ? szc[r * L.row + L.chan] : o.a;
        };
        auto step = [&](One o) {
            if (SIGNED) o.qv ^= 0x80808080u;
            const float za = o.a.y + zadj, zb = o.b.y + zadj;
            const bool fast = d.fast && scale_fast(o.a.x * o.wk) && scale_fast(o.b.x * o.wk);
            // wave-uniform: the common client carries Markstein only (a per-lane
            // select would compute both divisions for every element)
            if (__builtin_expect(__ballot(!fast) == 0, 1)) {
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                    const bool second = e >= split;
                    const float s = second ? o.b.x : o.a.x;
                    const float z = second ? zb : za;
                    const float t = ((byte_f32(o.qv[e >> 2], e & 3) - z) * s) * o.wk;
                    acc[e] += markstein(t, d.b, d.y);
                }
            } else {
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                    const bool second = e >= split;
                    const float s = second ? o.b.x : o.a.x;
                    const float z = second ? zb : za;
                    const float t = ((byte_f32(o.qv[e >> 2], e & 3) - z) * s) * o.wk;
                    acc[e] += fast ? markstein(t, d.b, d.y) : t / d.b;
                }
            }
        };
        chunk_pipeline<U, Batch>(
            min(64, K - base),
            [&](int j0, Batch &bt) {
#pragma unroll
                for (int u = 0; u < U; ++u) fetch(j0 + u, bt.c[u]);
            },
            [&](const Batch &bt) {
#pragma unroll
                for (int u = 0; u < U; ++u) step(bt.c[u]);
            },
            [&](int j) {
                One o;
                fetch(j, o);
                step(o);
            });
    }
}

// Lanes in different channels but none straddling a channel boundary (channel
// rows a multiple of 16 long, e.g. every 3x3 conv weight of VGG-16 / ResNet):
// the one-channel pipeline with each lane's (scale, zero point) loaded per
// client next to its payload (8 bytes, a handful of distinct lines per wave).
template <bool SIGNED>
__device__ __forceinline__ void int_lane_pipelined(float (&acc)[16], const uint8_t *__restrict__ Qt,
                                                   int64_t ldq, const f32x2 *__restrict__ szl,
                                                   SzLayout L, const int32_t *__restrict__ rows,
                                                   const float *__restrict__ w, int K,
                                                   const FastDiv &d) {
    constexpr int U = kQuantU;
    struct Batch {
        u32x4 qv[U];
        f32x2 sz[U];
        float wk[U];
    };
    const float zadj = SIGNED ? 128.f : 0.f;
    ChunkRows cr;
    cr.init(rows, w, K);
    auto one = [&](const u32x4 qv, f32x2 sz, float wk) {
        const float sc = sz.x, z = sz.y + zadj, zs = z * sc;
        const bool zfma = __builtin_fmaf(z, sc, -zs) == 0.f;  // fl(z*s) exact
        const bool fast = d.fast && scale_fast(sc * wk);
        if (__ballot(!(zfma && fast)) == 0) {  // wave-uniform common case
            accum16_one<true, true>(acc, qv, sc, zs, z, wk, d);
        } else if (zfma && fast) {
            accum16_one<true, true>(acc, qv, sc, zs, z, wk, d);
        } else if (fast) {
            accum16_one<false, true>(acc, qv, sc, zs, z, wk, d);
        } else {
            accum16_one<false, false>(acc, qv, sc, zs, z, wk, d);
        }
    };
    for (int base = 0; base < K; base += 64) {
        const int tr = cr.r0;
        const float tw = cr.w0;
        cr.advance(rows, w, K, base);
        auto fetch = [&](int j, u32x4 &qv, f32x2 &sz, float &wk) {
            const int64_t r = readlane_i(tr, j);
            qv = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(Qt + r * ldq));
            if (SIGNED) qv ^= 0x80808080u;  // int8 q read as the unsigned byte q + 128
            sz = szl[r * L.row];
            wk = readlane_f(tw, j);
        };
        chunk_pipeline<U, Batch>(
            min(64, K - base),
            [&](int j0, Batch &bt) {
#pragma unroll
                for (int u = 0; u < U; ++u) fetch(j0 + u, bt.qv[u], bt.sz[u], bt.wk[u]);
            },
            [&](const Batch &bt) {
#pragma unroll
                for (int u = 0; u < U; ++u) one(bt.qv[u], bt.sz[u], bt.wk[u]);
            },
            [&](int j) {
                u32x4 qv;
                f32x2 sz;
                float wk;
                fetch(j, qv, sz, wk);
                one(qv, sz, wk);
            });
    }
}

// Channel rows shorter than 16 elements: per-element channel lookup.
template <bool SIGNED>
__device__ __forceinline__ void int_tiny_rows(float (&acc)[16], const uint8_t *__restrict__ Qt,
                                              int64_t ldq, const f32x2 *__restrict__ sz,
                                              SzLayout L, const int (&cj)[16],
                                              const int32_t *__restrict__ rows,
                                              const float *__restrict__ w, int K,
                                              const FastDiv &d) {
    const float zadj = SIGNED ? 128.f : 0.f;
    for (int k = 0; k < K; ++k) {
        const int64_t row = rows[k];
        u32x4 qv = *reinterpret_cast<const u32x4 *>(Qt + row * ldq);
        if (SIGNED) qv ^= 0x80808080u;
        const float wk = w[k];
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const f32x2 a = sz[row * L.row + cj[e] * L.chan];
            const float t = ((byte_f32(qv[e >> 2], e & 3) - (a.y + zadj)) * a.x) * wk;
            acc[e] += (d.fast && scale_fast(a.x * wk)) ? markstein(t, d.b, d.y) : t / d.b;
        }
    }
}

__device__ __forceinline__ float fp_term(float x, float wk, const FastDiv &d) {
    const float tn = x * wk;
    return (d.fast && in_fast_range(tn)) ? markstein(tn, d.b, d.y) : tn / d.b;
}

__device__ __forceinline__ void f32_chunk(float (&acc)[16], const float *__restrict__ Ft,
                                          int64_t ldf, const int32_t *__restrict__ rows,
                                          const float *__restrict__ w, int K, const FastDiv &d) {
    for (int k = 0; k < K; ++k) {
        const f32x4 *src = reinterpret_cast<const f32x4 *>(Ft + (int64_t)rows[k] * ldf);
        const float wk = w[k];
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const f32x4 x = src[v];
#pragma unroll
            for (int c = 0; c < 4; ++c) acc[4 * v + c] += fp_term(x[c], wk, d);
        }
    }
}

// Tiles are wave tiles inside one tensor; wave w of block b takes tile 4b + w.
// The host sorts the table so that the first tiles are int tiles inside ONE
// channel (the bulk of every large-row weight), grouped by their number of
// 1 KiB slices (4, 3, 2, 1): one k_dequant_fast<G> launch per group runs only
// that path, so its register budget is set neither by a wider G nor by the
// rare paths of k_dequant_general (<= 1024 elements, a lane owns 16).
// -0 + t == t for every fp32 t, so every accumulator starts at -0 and the
// first client "is assigned" (servers/fed_server.py:62-65).
struct WaveTile {
    dls_qtile t;
    int lenpad, e0, ec;
    bool active;
};

__device__ __forceinline__ bool wave_tile(const dls_qtile *__restrict__ tiles, int ntiles,
                                          WaveTile &wt) {
    const int idx = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    if (idx >= ntiles) return false;  // wave-uniform
    wt.t = tiles[idx];
    wt.lenpad = (wt.t.len + 63) & ~63;  // chunks up to the 64-element row padding
    wt.e0 = 16 * __lane_id();
    wt.active = wt.e0 < wt.lenpad;
    wt.ec = wt.active ? wt.e0 : wt.lenpad - 16;  // idle lanes load a valid duplicate
    return true;
}

__device__ __forceinline__ void store16(const WaveTile &wt, float (&acc)[16],
                                        float *__restrict__ out) {
    if (!wt.active) return;
    if (wt.e0 + 16 > wt.t.len) {  // tensor tail: keep the row padding zero
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[e] = (wt.e0 + e < wt.t.len) ? acc[e] : 0.f;
    }
    f32x4 *o = reinterpret_cast<f32x4 *>(out + wt.t.dst + wt.e0);
#pragma unroll
    for (int v = 0; v < 4; ++v)
        o[v] = f32x4{acc[4 * v], acc[4 * v + 1], acc[4 * v + 2], acc[4 * v + 3]};
}

template <int G, bool EXT = false>
__device__ __forceinline__ void store_tile(const WaveTile &wt, float (&acc)[G][16],
                                           float *__restrict__ out, float *mine = nullptr);

// One-channel tiles of up to 4 KiB: slice g of the tile is lanes'
// 16-element chunks 1024 g + 16 lane; the wave walks the clients once for all
// its slices (per-client table reads and readlanes amortised over G KiB).
template <bool SIGNED, int G, bool TWO>
__device__ __forceinline__ void fast_tile(const WaveTile &wt, const uint8_t *__restrict__ Q,
                                          int64_t ldq, const f32x2 *__restrict__ sz, SzLayout L,
                                          const int32_t *__restrict__ rows,
                                          const float *__restrict__ w, int K, const FastDiv &d,
                                          float *__restrict__ out) {
    float acc[G][16];
    uint32_t qoff[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[g][e] = -0.f;
        const int e0 = 1024 * g + 16 * __lane_id();
        // idle lanes load a valid duplicate (loads stay unconditional)
        qoff[g] = (uint32_t)(wt.t.src + (e0 < wt.lenpad ? e0 : wt.lenpad - 16));  // ldq < 4 GiB
    }
    int_one_channel<SIGNED, G, TWO>(acc, Q, qoff, ldq, sz + wt.t.chan0 * L.chan, L, rows, w, K, d);
    store_tile<G>(wt, acc, out);
}

// Multi-channel tiles of 1 KiB (every int tensor whose channel rows are a
// multiple of 16 elements, so no lane's 16-element chunk straddles two channels:
// the 3x3 convs of ResNet-18 / VGG-16, 576-4608-element rows).  Slice g of the
// tile is lanes' chunks 1024 g + 16 lane, each lane in its own channel; the wave
// walks the clients once for all its slices, double-buffered like the
// one-channel tiles.
//
// Per-lane (scale, zero point): a tile spans `span` consecutive channels.  When
// span <= kSpanMax the wave stages them once per 64-client chunk: lane j loads
// client j's pairs of those channels (a chunk ahead, coalesced: the table is
// channel-major), checks the fast-path conditions for all of them at once (one
// ballot per chunk) and writes (s, s, -fl(z*s), -fl(z*s)) to the wave's LDS
// table; every client step then reads the lane's constants with one broadcast
// ds_read_b128 per slice instead of a per-lane 8-byte global gather (which
// doubled the vector-memory instructions and the texture data path's load)
// and the per-client check.  Chunks that fail the check, and tiles spanning
// more channels, take the per-client path: (scale, zero point) gathered per
// lane with each client's payload and the check per client.
constexpr int kSpanMax = 4;

template <bool SIGNED, int G, bool TWO>
__device__ __forceinline__ void lane_tile(const WaveTile &wt, const uint8_t *__restrict__ Q,
                                          int64_t ldq, const f32x2 *__restrict__ sz, SzLayout L,
                                          const int32_t *__restrict__ rows,
                                          const float *__restrict__ w, int K, const FastDiv &d,
                                          float *__restrict__ out) {
    __shared__ __attribute__((aligned(16))) f32x2 stab[kBlock / 64][kSpanMax][64];
    f32x2(*tab)[64] = stab[threadIdx.x >> 6];
    float acc[G][16];
    uint32_t qoff[G];
    int64_t coff[G];  // the lane's channel in slice g, in (scale, zp) pairs
    uint32_t toff[G];  // its row of the LDS table, in pairs
    const int span = (wt.t.row_pos + wt.t.len - 1) / wt.t.row_len + 1;  // wave-uniform
    const bool staged = span <= kSpanMax;
#pragma unroll
    for (int g = 0; g < G; ++g) {
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[g][e] = -0.f;
        const int e0 = 1024 * g + 16 * __lane_id();
        const int ec = e0 < wt.lenpad ? e0 : wt.lenpad - 16;  // idle lanes: a valid duplicate
        qoff[g] = (uint32_t)(wt.t.src + ec);
        const int crel = min((wt.t.row_pos + ec) / wt.t.row_len, span - 1);
        const int c = min(wt.t.chan0 + crel, wt.t.chan_end - 1);
        coff[g] = (int64_t)c * L.chan;
        toff[g] = (uint32_t)min(crel, kSpanMax - 1) * 64;
    }
    // channel c of the tile (clamped into the tensor), client row r
    auto tab_load = [&](int r, f32x2 (&v)[kSpanMax]) {
#pragma unroll
        for (int c = 0; c < kSpanMax; ++c)
            v[c] = sz[(int64_t)min(wt.t.chan0 + c, wt.t.chan_end - 1) * L.chan + (int64_t)r * L.row];
    };
    struct One1 {
        u32x4 qv;
        f32x2 s;
        float wk;
    };
    struct SOne {
        u32x4 qv[G];
        float wk;
        int j;
    };
    // clients per batch: kLaneUS on 1 KiB tiles, kLaneUSG on wider ones (G KiB
    // per client already; two batches in flight per wave either way)
    constexpr int US = G > 1 ? kLaneUSG : kLaneUS;
    struct SBatch {
        SOne c[US];
    };
    ChunkRows cr;
    cr.init(rows, w, K);
    f32x2 nsz[kSpanMax];
    if (staged && DLS_QUANT_PROBE < 2) tab_load(cr.r0, nsz);
    for (int base = 0; base < K; base += 64) {
        const int tr = cr.r0;
        const float tw = cr.w0;
        f32x2 tsz[kSpanMax];
#pragma unroll
        for (int c = 0; c < kSpanMax; ++c) tsz[c] = nsz[c];
        if (staged && DLS_QUANT_PROBE < 2) tab_load(cr.r1, nsz);  // next chunk (its rows landed a chunk ago)
        cr.advance(rows, w, K, base);
        const int n = min(64, K - base);
        bool allfast = DLS_QUANT_PROBE >= 2;
        if (staged && DLS_QUANT_PROBE < 2) {
            // every (client, channel) of the chunk on the common path: exact fl(z*s)
            // and the fast division range (always, for symmetric int8)
            int ok = d.fast;
#pragma unroll
            for (int c = 0; c < kSpanMax; ++c) {
                const float s = tsz[c].x, zs = tsz[c].y * s;
                ok &= (int)(c >= span) |
                      ((int)(__builtin_fmaf(tsz[c].y, s, -zs) == 0.f) & (int)scale_fast(s * tw));
                tab[c][__lane_id()] = f32x2{s, -zs};
            }
            allfast = __ballot(!ok && __lane_id() < n) == 0;
        }
        if (allfast) {
            auto sfetch = [&](int j, SOne &b) {
                const int64_t r = DLS_QUANT_PROBE >= 3 ? (int64_t)(base + j) : readlane_i(tr, j);
                const auto rs = __builtin_amdgcn_make_buffer_rsrc(
                    const_cast<uint8_t *>(Q + r * ldq), 0, (int)0xffffffffu, 0x00020000);  // 4 GiB
#pragma unroll
                for (int g = 0; g < G; ++g)
                    b.qv[g] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)qoff[g], 0, 2 /* nt */);
                b.wk = DLS_QUANT_PROBE >= 3 ? 1.f : readlane_f(tw, j);
                b.j = j;
            };
            auto sstep = [&](const SOne &b) {
                // the lane's (s, -zs): a broadcast LDS read (<= kSpanMax addresses per wave)
#pragma unroll
                for (int g = 0; g < G; ++g) {
                    if constexpr (DLS_QUANT_PROBE >= 1)
                        acc[g][g] += __uint_as_float((b.qv[g].x ^ b.qv[g].y ^ b.qv[g].z ^ b.qv[g].w) &
                                                     0x3fffffffu);
                    else
                        accum16_pk<SIGNED, TWO>(acc[g], b.qv[g], tab[0][toff[g] + b.j], b.wk, d);
                }
            };
            chunk_pipeline_1tail<US, SBatch>(
                n,
                [&](int j0, SBatch &b) {
#pragma unroll
                    for (int u = 0; u < US; ++u) sfetch(j0 + u, b.c[u]);
                },
                [&](const SBatch &b) {
#pragma unroll
                    for (int u = 0; u < US; ++u) sstep(b.c[u]);
                },
                [&](int j) {
                    SOne b;
                    sfetch(j, b);
                    sstep(b);
                });
            continue;
        }
        // per-client path (chunks that fail the check, tiles over more than
        // kSpanMax channels): the lane's (scale, zero point) gathered with each
        // client's payload, one wave-uniform decision per client (exact fl(zp * s)
        // and the fast division range on every lane).  One KiB slice at a time, so
        // that this path's registers stay within the staged path's.
        auto rare = [&](auto g_c) {
            constexpr int g = decltype(g_c)::value;
            auto fetch = [&](int j, One1 &b) {
                const int64_t r = readlane_i(tr, j);
                const auto rs = __builtin_amdgcn_make_buffer_rsrc(
                    const_cast<uint8_t *>(Q + r * ldq), 0, (int)0xffffffffu, 0x00020000);  // 4 GiB
                b.qv = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)qoff[g], 0, 2 /* nt */);
                b.s = sz[coff[g] + r * L.row];
                b.wk = readlane_f(tw, j);
            };
            auto step = [&](const One1 &b) {
                const float zs = b.s.y * b.s.x;
                const int ok = d.fast & (int)(__builtin_fmaf(b.s.y, b.s.x, -zs) == 0.f) &
                               (int)scale_fast(b.s.x * b.wk);
                if (__builtin_expect(__ballot(!ok) == 0, 1))
                    accum16_one<true, true, SIGNED, TWO, kLaneSched>(acc[g], b.qv, b.s.x, zs, 0.f,
                                                                     b.wk, d);
                else  // rare clients: the reference's formula with IEEE division
                    accum16_one<false, false, SIGNED>(acc[g], b.qv, b.s.x, 0.f, b.s.y, b.wk, d);
            };
            chunk_pipeline<1, One1>(
                n, [&](int j0, One1 &bb) { fetch(j0, bb); }, [&](const One1 &bb) { step(bb); },
                [&](int j) {
                    One1 bb;
                    fetch(j, bb);
                    step(bb);
                });
        };
        rare(std::integral_constant<int, 0>{});
        if constexpr (G > 1) rare(std::integral_constant<int, 1>{});
        if constexpr (G > 2) rare(std::integral_constant<int, 2>{});
        if constexpr (G > 3) rare(std::integral_constant<int, 3>{});
    }
    store_tile<G>(wt, acc, out);
}

// Write a wave tile's G slices of accumulators, transposed through LDS so that
// each store instruction writes 1 KiB contiguous.
// EXT: mine is the wave's 4 KiB of LDS from the caller (a kernel running several
// tile widths holds ONE buffer); else the function's own
template <int G, bool EXT>
__device__ __forceinline__ void store_tile(const WaveTile &wt, float (&acc)[G][16],
                                           float *__restrict__ out, float *mine) {
    if constexpr (!EXT) {
        __shared__ __attribute__((aligned(16))) float xs[kBlock / 64][1024];
        mine = xs[threadIdx.x >> 6];
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const int e0 = 1024 * g + 16 * __lane_id();
        if (e0 + 16 > wt.t.len) {  // tensor tail: keep the row padding zero
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[g][e] = (e0 + e < wt.t.len) ? acc[g][e] : 0.f;
        }
#pragma unroll
        for (int v = 0; v < 4; ++v)
            *reinterpret_cast<f32x4 *>(mine + 16 * __lane_id() + 4 * v) =
                f32x4{acc[g][4 * v], acc[g][4 * v + 1], acc[g][4 * v + 2], acc[g][4 * v + 3]};
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const int e = 256 * v + 4 * __lane_id();
            const f32x4 x = *reinterpret_cast<const f32x4 *>(mine + e);
            if (1024 * g + e < wt.lenpad) {
                f32x4 *o = reinterpret_cast<f32x4 *>(out + wt.t.dst + 1024 * g + e);
                if constexpr (DLS_QUANT_NTSTORE)
                    __builtin_nontemporal_store(x, o);
                else
                    *o = x;
            }
        }
    }
}

template <int G, bool TWO>
__global__ __launch_bounds__(kBlock, 1) void k_dequant_fast(
    const dls_qtile *__restrict__ tiles, int ntiles, const uint8_t *__restrict__ Q, int64_t ldq,
    const f32x2 *__restrict__ sz, SzLayout L, const int32_t *__restrict__ rows,
    const float *__restrict__ w, int K, FastDiv d, float *__restrict__ out) {
    // one launch per (slice count G, division method): each instance has its
    // own register budget
    WaveTile wt;
    if (!wave_tile(tiles, ntiles, wt)) return;
    if (wt.t.kind == 1)
        fast_tile<true, G, TWO>(wt, Q, ldq, sz, L, rows, w, K, d, out);
    else
        fast_tile<false, G, TWO>(wt, Q, ldq, sz, L, rows, w, K, d, out);
}

// ------------------------------------------------------------ FMA mode
// DLS_FEDAVG_FMA (north-star FedAvg tolerance, not bit-exact): every int
// element accumulates fma(q - z, c, acc) with one constant per (client,
// channel) c = fl(fl(s * n_i) / N) (q - z is exact in fp32).  None of the exact
// path's rounding sequence, range checks or fallbacks is needed, so these
// kernels are lean (no rare path in the register budget): more waves per SIMD,
// more bytes in flight.  Zero points are almost always 0 (symmetric qint8, the
// QAT worker's format): a chunk whose zero points are all 0 skips the
// subtraction (one wave-uniform test per 64-client chunk).
template <bool SEXT>
__device__ __forceinline__ void accum16_fmaz(float (&acc)[16], u32x4 qv, f32x2 cz) {
    // cz = (c, -z): x + (-z) exact, then fma(x, c, acc)
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
        const int k = j & 3;
        f32x2 xa = f32x2{byte_val<SEXT>(qv[j >> 2], k), byte_val<SEXT>(qv[j >> 2], k + 1)};
        f32x2 xb = f32x2{byte_val<SEXT>(qv[(j >> 2) + 2], k), byte_val<SEXT>(qv[(j >> 2) + 2], k + 1)};
        f32x2 ra = f32x2{acc[j], acc[j + 1]}, rb = f32x2{acc[j + 8], acc[j + 9]};
        asm volatile(
            "v_pk_add_f32 %[xa], %[xa], %[cz] op_sel:[0,1] op_sel_hi:[1,1]\n\t"
            "v_pk_add_f32 %[xb], %[xb], %[cz] op_sel:[0,1] op_sel_hi:[1,1]\n\t"
            "v_pk_fma_f32 %[ra], %[xa], %[cz], %[ra] op_sel_hi:[1,0,1]\n\t"
            "v_pk_fma_f32 %[rb], %[xb], %[cz], %[rb] op_sel_hi:[1,0,1]"
            : [ra] "+v"(ra), [rb] "+v"(rb), [xa] "+v"(xa), [xb] "+v"(xb)
            : [cz] "v"(cz));
        acc[j] = ra.x;
        acc[j + 1] = ra.y;
        acc[j + 8] = rb.x;
        acc[j + 9] = rb.y;
        __builtin_amdgcn_sched_barrier(0);
    }
}

template <bool SEXT>
__device__ __forceinline__ void accum16_fma_any(float (&acc)[16], u32x4 qv, f32x2 cz, bool allz) {
    if (allz)
        accum16_fma<SEXT>(acc, qv, cz);
    else
        accum16_fmaz<SEXT>(acc, qv, cz);
}

// One-channel tiles (groups 0-3) in FMA mode: one (c, -z) per client, read back
// as wave-uniform values; G KiB slices per client.
template <bool SIGNED, int G>
__device__ __forceinline__ void fma_one_channel_tile(const WaveTile &wt, const uint8_t *__restrict__ Q,
                                                     int64_t ldq, const f32x2 *__restrict__ sz,
                                                     SzLayout L, const int32_t *__restrict__ rows,
                                                     const float *__restrict__ w, int K, float N,
                                                     float *__restrict__ out) {
    float acc[G][16];
    uint32_t qoff[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[g][e] = 0.f;
        const int e0 = 1024 * g + 16 * __lane_id();
        qoff[g] = (uint32_t)(wt.t.src + (e0 < wt.lenpad ? e0 : wt.lenpad - 16));
    }
    const f32x2 *szc = sz + wt.t.chan0 * L.chan;
    ChunkRows cr;
    cr.init(rows, w, K);
    f32x2 nsz = szc[(int64_t)cr.r0 * L.row];
    constexpr int U = G > 1 ? kQuantUG : kQuantU;
    struct B {
        u32x4 qv[U][G];
        float c[U], z[U];
    };
    for (int base = 0; base < K; base += 64) {
        const int tr = cr.r0;
        const float coef = fma_coef(nsz.x, cr.w0, N), nz = -nsz.y;
        const bool allz = __ballot(nsz.y != 0.f && __lane_id() < K - base) == 0;
        nsz = szc[(int64_t)cr.r1 * L.row];  // next chunk (its rows landed a chunk ago)
        cr.advance(rows, w, K, base);
        const int n = min(64, K - base);
        auto fetch = [&](int j, u32x4 (&qv)[G], float &c, float &z) {
            const int64_t r = readlane_i(tr, j);
            const auto rs = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<uint8_t *>(Q + r * ldq), 0, (int)0xffffffffu, 0x00020000);  // 4 GiB
#pragma unroll
            for (int g = 0; g < G; ++g)
                qv[g] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)qoff[g], 0, 2 /* nt */);
            c = readlane_f(coef, j);
            z = readlane_f(nz, j);
        };
        auto step = [&](const u32x4 (&qv)[G], float c, float z) {
#pragma unroll
            for (int g = 0; g < G; ++g) accum16_fma_any<SIGNED>(acc[g], qv[g], f32x2{c, z}, allz);
        };
        chunk_pipeline<U, B>(
            n,
            [&](int j0, B &b) {
#pragma unroll
                for (int u = 0; u < U; ++u) fetch(j0 + u, b.qv[u], b.c[u], b.z[u]);
            },
            [&](const B &b) {
#pragma unroll
                for (int u = 0; u < U; ++u) step(b.qv[u], b.c[u], b.z[u]);
            },
            [&](int j) {
                u32x4 qv[G];
                float c, z;
                fetch(j, qv, c, z);
                step(qv, c, z);
            });
    }
    store_tile<G>(wt, acc, out);
}

// Multi-channel (lane) tiles (groups 4-7) in FMA mode: the channels' (c, -z) of
// the chunk's 64 clients staged in the wave's LDS table (lane j computes client
// j's), one broadcast ds_read_b64 per slice and client.  A tile over more than
// kSpanMax channels is walked in ceil(span / kSpanMax) passes of kSpanMax
// channels; a lane outside the pass's channels reads the table's zero row
// (c = 0: fma(x, 0, acc) leaves acc), so there is ONE walk loop.  A second loop
// (the per-client gather path of round 3), or a per-chunk choice between the
// zero-point forms, made the register allocator keep two copies of the
// accumulators: 234 VGPRs at G = 4 (2 waves per SIMD, the group in two launch
// pieces of 1.2 waves per SIMD) against 156 with one loop (3 waves per SIMD,
// one piece).  The zero point is always subtracted: x + (-z) is exact and
// x + (-0) == x, so a chunk of zero points 0 gives the bits of the
// subtraction-free form.
template <bool SIGNED, int G, bool EXT = false>
__device__ __forceinline__ void fma_lane_tile(const WaveTile &wt, const uint8_t *__restrict__ Q,
                                              int64_t ldq, const f32x2 *__restrict__ sz, SzLayout L,
                                              const int32_t *__restrict__ rows,
                                              const float *__restrict__ w, int K, float N,
                                              float *__restrict__ out,
                                              f32x2 (*tab)[64] = nullptr, float *xsw = nullptr) {
    if constexpr (!EXT) {  // else the caller's (k_dequant_lanes_fma_any)
        __shared__ __attribute__((aligned(16))) f32x2 ftab[kBlock / 64][kSpanMax + 1][64];
        tab = ftab[threadIdx.x >> 6];
    }
    tab[kSpanMax][__lane_id()] = f32x2{0.f, 0.f};  // the zero row
    float acc[G][16];
    uint32_t qoff[G];
    int crel[G];  // the lane's channel in slice g, relative to the tile's first
    const int span = (wt.t.row_pos + wt.t.len - 1) / wt.t.row_len + 1;  // wave-uniform
#pragma unroll
    for (int g = 0; g < G; ++g) {
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[g][e] = 0.f;
        const int e0 = 1024 * g + 16 * __lane_id();
        const int ec = e0 < wt.lenpad ? e0 : wt.lenpad - 16;
        qoff[g] = (uint32_t)(wt.t.src + ec);
        crel[g] = min((wt.t.row_pos + ec) / wt.t.row_len, span - 1);
    }
    constexpr int US = G > 1 ? kLaneUSG : kLaneUS;
    struct SOne {
        u32x4 qv[G];
        int j;
    };
    struct SBatch {
        SOne c[US];
    };
    // passes x chunks as ONE loop (a loop over passes around the chunk loop cost
    // 24 VGPRs at G = 4); almost every tile has one pass
    const int npass = (span + kSpanMax - 1) / kSpanMax;
    const int nch = (K + 63) / 64;
    int c0 = wt.t.chan0;  // the pass's first channel
    uint32_t toff[G];     // the lane's table row, in pairs
    auto pass_rows = [&](int p) {
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const int c = crel[g] - kSpanMax * p;
            toff[g] = (uint32_t)(c >= 0 && c < kSpanMax ? c : kSpanMax) * 64;
        }
    };
    auto tab_load = [&](int r, f32x2 (&v)[kSpanMax]) {
#pragma unroll
        for (int c = 0; c < kSpanMax; ++c)
            v[c] = sz[(int64_t)min(c0 + c, wt.t.chan_end - 1) * L.chan + (int64_t)r * L.row];
    };
    pass_rows(0);
    ChunkRows cr;
    cr.init(rows, w, K);
    f32x2 nsz[kSpanMax];
    tab_load(cr.r0, nsz);
    for (int it = 0, p = 0, base = 0; it < npass * nch; ++it) {
        const int tr = cr.r0;
        const float tw = cr.w0;
        const int n = min(64, K - base);
#pragma unroll
        for (int c = 0; c < kSpanMax; ++c)
            tab[c][__lane_id()] = f32x2{fma_coef(nsz[c].x, tw, N), -nsz[c].y};
        tab_load(cr.r1, nsz);  // next chunk (its rows landed a chunk ago)
        cr.advance(rows, w, K, base);
        auto sfetch = [&](int j, SOne &b) {
            const int64_t r = readlane_i(tr, j);
            const auto rs = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<uint8_t *>(Q + r * ldq), 0, (int)0xffffffffu, 0x00020000);  // 4 GiB
#pragma unroll
            for (int g = 0; g < G; ++g)
                b.qv[g] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)qoff[g], 0, 2 /* nt */);
            b.j = j;
        };
        auto sstep = [&](const SOne &b) {
#pragma unroll
            for (int g = 0; g < G; ++g) {
                if constexpr (DLS_QUANT_PROBE == 1)
                    acc[g][g] += __uint_as_float((b.qv[g].x ^ b.qv[g].y ^ b.qv[g].z ^ b.qv[g].w) &
                                                 0x3fffffffu);
                else
                    accum16_fmaz<SIGNED>(acc[g], b.qv[g], tab[0][toff[g] + b.j]);
            }
        };
        chunk_pipeline_1tail<US, SBatch>(
            n,
            [&](int j0, SBatch &b) {
#pragma unroll
                for (int u = 0; u < US; ++u) sfetch(j0 + u, b.c[u]);
            },
            [&](const SBatch &b) {
#pragma unroll
                for (int u = 0; u < US; ++u) sstep(b.c[u]);
            },
            [&](int j) {
                SOne b;
                sfetch(j, b);
                sstep(b);
            });
        base += 64;
        if (base >= K && p + 1 < npass) {  // the next pass: its channels, the clients again
            ++p;
            base = 0;
            c0 += kSpanMax;
            pass_rows(p);
            cr.init(rows, w, K);
            tab_load(cr.r0, nsz);
        }
    }
    store_tile<G, EXT>(wt, acc, out, xsw);
}

template <int G>
__global__ __launch_bounds__(kBlock) void k_dequant_fast_fma(
    const dls_qtile *__restrict__ tiles, int ntiles, const uint8_t *__restrict__ Q, int64_t ldq,
    const f32x2 *__restrict__ sz, SzLayout L, const int32_t *__restrict__ rows,
    const float *__restrict__ w, int K, FastDiv d, float *__restrict__ out) {
    WaveTile wt;
    if (!wave_tile(tiles, ntiles, wt)) return;
    if (wt.t.kind == 1)
        fma_one_channel_tile<true, G>(wt, Q, ldq, sz, L, rows, w, K, d.b, out);
    else
        fma_one_channel_tile<false, G>(wt, Q, ldq, sz, L, rows, w, K, d.b, out);
}

template <int G>
__global__ __launch_bounds__(kBlock) void k_dequant_lanes_fma(
    const dls_qtile *__restrict__ tiles, int ntiles, const uint8_t *__restrict__ Q, int64_t ldq,
    const f32x2 *__restrict__ sz, SzLayout L, const int32_t *__restrict__ rows,
    const float *__restrict__ w, int K, FastDiv d, float *__restrict__ out) {
    WaveTile wt;
    if (!wave_tile(tiles, ntiles, wt)) return;
    if (wt.t.kind == 1)
        fma_lane_tile<true, G>(wt, Q, ldq, sz, L, rows, w, K, d.b, out);
    else
        fma_lane_tile<false, G>(wt, Q, ldq, sz, L, rows, w, K, d.b, out);
}

// Every lane-tile group (4, 3, 2 and 1 KiB tiles, the table's groups 4-7, which
// are contiguous) in ONE launch: a wave takes its tile's width (wave-uniform),
// one LDS table and store buffer per wave serve every width, so the kernel's
// registers and LDS are those of the widest.  The bulk of the FMA call then has
// no side-stream lane kernels beside it, and no fork / join for them.
__global__ __launch_bounds__(kBlock) void k_dequant_lanes_fma_any(
    const dls_qtile *__restrict__ tiles, int ntiles, const uint8_t *__restrict__ Q, int64_t ldq,
    const f32x2 *__restrict__ sz, SzLayout L, const int32_t *__restrict__ rows,
    const float *__restrict__ w, int K, FastDiv d, float *__restrict__ out) {
    __shared__ __attribute__((aligned(16))) f32x2 ftab[kBlock / 64][kSpanMax + 1][64];
    __shared__ __attribute__((aligned(16))) float xs[kBlock / 64][1024];
    WaveTile wt;
    if (!wave_tile(tiles, ntiles, wt)) return;
    f32x2(*tab)[64] = ftab[threadIdx.x >> 6];
    float *mine = xs[threadIdx.x >> 6];
    const int slices = __builtin_amdgcn_readfirstlane((wt.t.len + 1023) >> 10);
    auto run = [&](auto sgn_c, auto g_c) {
        constexpr bool SG = decltype(sgn_c)::value;
        constexpr int G = decltype(g_c)::value;
        fma_lane_tile<SG, G, true>(wt, Q, ldq, sz, L, rows, w, K, d.b, out, tab, mine);
    };
    auto by_width = [&](auto sgn_c) {
        if (slices >= 4)
            run(sgn_c, std::integral_constant<int, 4>{});
        else if (slices == 3)
            run(sgn_c, std::integral_constant<int, 3>{});
        else if (slices == 2)
            run(sgn_c, std::integral_constant<int, 2>{});
        else
            run(sgn_c, std::integral_constant<int, 1>{});
    };
    if (wt.t.kind == 1)
        by_width(std::true_type{});
    else
        by_width(std::false_type{});
}

// The fp32 and small-int groups (quant_common.h walks), a wave per tile.  A few
// waves that walk all K clients beside the bulk kernel's: without priority they
// get a fifth of their SIMD's issue slots and finish last.
__global__ __launch_bounds__(kBlock) void k_dequant_f32(const dls_qtile *__restrict__ tiles,
                                                        int ntiles, const float *__restrict__ F,
                                                        int64_t ldf,
                                                        const int32_t *__restrict__ rows,
                                                        const float *__restrict__ w, int K,
                                                        FastDiv d, float *__restrict__ out) {
    const int idx = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    if (idx >= ntiles) return;  // wave-uniform
    __builtin_amdgcn_s_setprio(3);
    f32_side_tile(tiles[idx], F, ldf, rows, w, K, d, out);
}

__global__ __launch_bounds__(kBlock) void k_dequant_small(const dls_qtile *__restrict__ tiles,
                                                          int ntiles, const uint8_t *__restrict__ Q,
                                                          int64_t ldq, const f32x2 *__restrict__ sz,
                                                          SzLayout L,
                                                          const int32_t *__restrict__ rows,
                                                          const float *__restrict__ w, int K,
                                                          FastDiv d, float *__restrict__ out) {
    const int idx = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    if (idx >= ntiles) return;  // wave-uniform
    __builtin_amdgcn_s_setprio(3);
    small_side_tile(tiles[idx], Q, ldq, sz, L, rows, w, K, d, out);
}

template <int G, bool TWO>
__global__ __launch_bounds__(kBlock, 1) void k_dequant_lanes(
    const dls_qtile *__restrict__ tiles, int ntiles, const uint8_t *__restrict__ Q, int64_t ldq,
    const f32x2 *__restrict__ sz, SzLayout L, const int32_t *__restrict__ rows,
    const float *__restrict__ w, int K, FastDiv d, float *__restrict__ out) {
    WaveTile wt;
    if (!wave_tile(tiles, ntiles, wt)) return;
    if (wt.t.kind == 1)
        lane_tile<true, G, TWO>(wt, Q, ldq, sz, L, rows, w, K, d, out);
    else
        lane_tile<false, G, TWO>(wt, Q, ldq, sz, L, rows, w, K, d, out);
}

__global__ __launch_bounds__(kBlock) void k_dequant_general(
    const dls_qtile *__restrict__ tiles, int ntiles, const uint8_t *__restrict__ Q, int64_t ldq,
    const float *__restrict__ F, int64_t ldf, const f32x2 *__restrict__ sz, SzLayout L,
    const int32_t *__restrict__ rows, const float *__restrict__ w, int K, FastDiv d,
    float *__restrict__ out) {
    WaveTile wt;
    if (!wave_tile(tiles, ntiles, wt)) return;
    __builtin_amdgcn_s_setprio(3);  // few long waves beside the bulk kernel's (cf. k_dequant_f32)
    const dls_qtile &t = wt.t;
    float acc[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = -0.f;
    if (t.kind == 0) {
        f32_chunk(acc, F + t.src + wt.ec, ldf, rows, w, K, d);
    } else {
        const bool sgn = t.kind == 1;
        const uint8_t *Qt = Q + t.src + wt.ec;
        const int p = t.row_pos + wt.ec;
        const int c = t.chan0 + p / t.row_len;
        if (t.row_len >= 16) {
            const int split = t.row_len - p % t.row_len;  // [0, split) in c, rest in c + 1
            if (__ballot(split < 16) == 0) {  // wave-uniform: no lane straddles a channel
                if (sgn)
                    int_lane_pipelined<true>(acc, Qt, ldq, sz + c * L.chan, L, rows, w, K, d);
                else
                    int_lane_pipelined<false>(acc, Qt, ldq, sz + c * L.chan, L, rows, w, K, d);
            } else if (sgn) {
                int_lane_channels<true>(acc, Qt, ldq, sz + c * L.chan, L, split, rows, w, K, d);
            } else {
                int_lane_channels<false>(acc, Qt, ldq, sz + c * L.chan, L, split, rows, w, K, d);
            }
        } else {
            const int r = p % t.row_len;
            int cj[16];
#pragma unroll
            for (int e = 0; e < 16; ++e) cj[e] = min(c + (r + e) / t.row_len, t.chan_end - 1);
            if (sgn)
                int_tiny_rows<true>(acc, Qt, ldq, sz, L, cj, rows, w, K, d);
            else
                int_tiny_rows<false>(acc, Qt, ldq, sz, L, cj, rows, w, K, d);
        }
    }
    store16(wt, acc, out);
}

// ------------------------------------------------------------- min / max
__device__ __forceinline__ void atomic_min_f32(float *a, float v) {
    if (v >= 0.f)
        atomicMin(reinterpret_cast<int *>(a), __float_as_int(v));
    else
        atomicMax(reinterpret_cast<unsigned int *>(a), __float_as_uint(v));
}
__device__ __forceinline__ void atomic_max_f32(float *a, float v) {
    if (v >= 0.f)
        atomicMax(reinterpret_cast<int *>(a), __float_as_int(v));
    else
        atomicMin(reinterpret_cast<unsigned int *>(a), __float_as_uint(v));
}

__global__ void k_minmax_init(float *mins, float *maxs, int nseg) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s < nseg) {
        mins[s] = __builtin_inff();
        maxs[s] = -__builtin_inff();
    }
}

__device__ __forceinline__ int find_segment(const int64_t *seg_off, int nseg, int64_t e) {
    int lo = 0, hi = nseg - 1;  // last s with seg_off[s] <= e
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (seg_off[mid] <= e)
            lo = mid;
        else
            hi = mid - 1;
    }
    return lo;
}

template <typename T>
__device__ __forceinline__ T wave_reduce(T v, bool is_min) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const T u = __shfl_xor(v, o);
        v = is_min ? fminf(v, u) : fmaxf(v, u);
    }
    return v;
}

constexpr int kMinmaxChunk = kBlock * 4 * 8;  // 8192 elements per block

__global__ __launch_bounds__(kBlock) void k_segment_minmax(const float *__restrict__ x,
                                                           const int64_t *__restrict__ seg_off,
                                                           int nseg, float *mins, float *maxs) {
    __shared__ int s_seg[2];
    __shared__ float s_red[2][kBlock / 64];
    const int64_t total = seg_off[nseg];
    const int64_t c0 = (int64_t)blockIdx.x * kMinmaxChunk;
    const int64_t c1 = c0 + kMinmaxChunk < total ? c0 + kMinmaxChunk : total;
    if (threadIdx.x == 0) {
        s_seg[0] = find_segment(seg_off, nseg, c0);
        s_seg[1] = find_segment(seg_off, nseg, c1 - 1);
    }
    __syncthreads();
    const int sa = s_seg[0], sb = s_seg[1];
    if (sa == sb) {
        float lo = __builtin_inff(), hi = -__builtin_inff();
        for (int64_t e = c0 + 4 * threadIdx.x; e < c1; e += 4 * kBlock) {
            if (e + 4 <= c1 && ((reinterpret_cast<uintptr_t>(x + e) & 15u) == 0)) {
                const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4 *>(x + e));
                lo = fminf(lo, fminf(fminf(v.x, v.y), fminf(v.z, v.w)));
                hi = fmaxf(hi, fmaxf(fmaxf(v.x, v.y), fmaxf(v.z, v.w)));
            } else {
                for (int t = 0; t < 4 && e + t < c1; ++t) {
                    lo = fminf(lo, x[e + t]);
                    hi = fmaxf(hi, x[e + t]);
                }
            }
        }
        lo = wave_reduce(lo, true);
        hi = wave_reduce(hi, false);
        const int wv = threadIdx.x >> 6;
        if (__lane_id() == 0) {
            s_red[0][wv] = lo;
            s_red[1][wv] = hi;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int i = 1; i < kBlock / 64; ++i) {
                lo = fminf(lo, s_red[0][i]);
                hi = fmaxf(hi, s_red[1][i]);
            }
            atomic_min_f32(mins + sa, lo);
            atomic_max_f32(maxs + sa, hi);
        }
    } else {  // chunk crosses segment boundaries (at most nseg such chunks)
        for (int64_t e = c0 + threadIdx.x; e < c1; e += kBlock) {
            const float v = x[e];
            if (v != v) continue;  // NaNs are ignored, as fminf / fmaxf do on the bulk path
            const int s = find_segment(seg_off, nseg, e);
            atomic_min_f32(mins + s, v);
            atomic_max_f32(maxs + s, v);
        }
    }
}

__global__ void k_qparams(const float *mins, const float *maxs, int nseg, int qmin, int qmax,
                          int symmetric, float *scale, int32_t *zp) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nseg) return;
    // torch.ao MinMaxObserver._calculate_qparams, fp32 tensor math
    const float eps = 1.1920928955078125e-07f;  // torch.finfo(float32).eps
    const float lo = fminf(mins[s], 0.f), hi = fmaxf(maxs[s], 0.f);
    if (symmetric) {  // per_tensor/per_channel_symmetric
        float sc = fmaxf(-lo, hi) / ((float)(qmax - qmin) / 2.f);
        scale[s] = fmaxf(sc, eps);
        zp[s] = qmin < 0 ? 0 : (qmin + qmax + 1) / 2;
        return;
    }
    float sc = (hi - lo) / (float)(qmax - qmin);
    sc = fmaxf(sc, eps);
    float z = (float)qmin - rintf(lo / sc);
    z = fminf(fmaxf(z, (float)qmin), (float)qmax);
    scale[s] = sc;
    zp[s] = (int32_t)z;
}

// counter-based uniform in [0,1): splitmix64 of (seed, element)
__device__ __forceinline__ float uniform01(uint64_t seed, uint64_t e) {
    uint64_t z = seed + 0x9E3779B97F4A7C15ull * (e + 1);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (float)(uint32_t)(z >> 40) * 0x1p-24f;
}

__global__ __launch_bounds__(kBlock) void k_quantize(const float *__restrict__ x,
                                                     const int64_t *__restrict__ seg_off, int nseg,
                                                     const float *__restrict__ scale,
                                                     const int32_t *__restrict__ zp, float qmin,
                                                     float qmax, uint8_t *__restrict__ q,
                                                     float *__restrict__ deq, int stochastic,
                                                     uint64_t seed) {
    __shared__ int s_seg;
    const int64_t total = seg_off[nseg];
    const int64_t e0 = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * 4;
    if (threadIdx.x == 0) s_seg = find_segment(seg_off, nseg, (int64_t)blockIdx.x * kBlock * 4);
    __syncthreads();
    if (e0 >= total) return;
    int s = s_seg;
    uint32_t packed = 0;
    float dq[4];
    for (int t = 0; t < 4; ++t) {
        const int64_t e = e0 + t;
        if (e >= total) break;
        while (seg_off[s + 1] <= e) ++s;
        const float sc = scale[s];
        const float inv = 1.0f / sc;  // torch: inv_scale = 1.0f / (float)scale
        const float z = (float)zp[s];
        const float v = x[e] * inv;
        const float r = stochastic ? floorf(v + uniform01(seed, (uint64_t)e)) : rintf(v);
        const float qf = fminf(fmaxf(r + z, qmin), qmax);  // nan -> qmin
        packed |= ((uint32_t)(int32_t)qf & 0xffu) << (8 * t);
        dq[t] = (qf - z) * sc;
    }
    const int64_t n = total - e0 < 4 ? total - e0 : 4;
    if (n == 4 && ((reinterpret_cast<uintptr_t>(q + e0) & 3u) == 0)) {
        *reinterpret_cast<uint32_t *>(q + e0) = packed;
    } else {
        for (int t = 0; t < n; ++t) q[e0 + t] = (uint8_t)(packed >> (8 * t));
    }
    if (deq)
        for (int t = 0; t < n; ++t) deq[e0 + t] = dq[t];
}

}  // namespace
}  // namespace dls

using namespace dls;

extern "C" int dls_dequant_fedavg(const dls_qtile *tiles, int32_t ntiles, const int32_t *nfast,
                                  const void *Q, int64_t ldq, const float *F, int64_t ldf,
                                  const float *sz, int64_t sz_row, int64_t sz_chan,
                                  const int32_t *rows,
                                  const float *weight, int32_t K, float total, float *out,
                                  dls_stream_t stream) {
    return dls_dequant_fedavg_mode(tiles, ntiles, nfast, Q, ldq, F, ldf, sz, sz_row, sz_chan, rows,
                                   weight, K, total, DLS_FEDAVG_EXACT, out, stream);
}

extern "C" int dls_dequant_fedavg_mode(const dls_qtile *tiles, int32_t ntiles,
                                       const int32_t *nfast, const void *Q, int64_t ldq,
                                       const float *F, int64_t ldf, const float *sz,
                                       int64_t sz_row, int64_t sz_chan, const int32_t *rows,
                                       const float *weight, int32_t K, float total, int32_t mode,
                                       float *out, dls_stream_t stream) {
    DLS_REQUIRE(tiles && nfast && rows && weight && out && sz, DLS_EINVAL,
                "dls_dequant_fedavg: null pointer");
    DLS_REQUIRE(mode == DLS_FEDAVG_EXACT || mode == DLS_FEDAVG_FMA, DLS_EINVAL,
                "dls_dequant_fedavg: mode=%d", mode);
    int64_t nf = 0;
    for (int g = 0; g < DLS_QTILE_GROUPS; ++g) {
        DLS_REQUIRE(nfast[g] >= 0, DLS_EINVAL, "dls_dequant_fedavg: nfast[%d]=%d", g, nfast[g]);
        nf += nfast[g];
    }
    DLS_REQUIRE(ntiles > 0 && K > 0 && nf <= ntiles, DLS_EINVAL,
                "dls_dequant_fedavg: ntiles=%d grouped tiles=%lld K=%d", ntiles, (long long)nf, K);
    DLS_REQUIRE(ldq % 16 == 0 && ldf % 4 == 0 && aligned16(out) && (!Q || aligned16(Q)) &&
                    (!F || aligned16(F)),
                DLS_ELAYOUT, "dls_dequant_fedavg: ldq %% 16, ldf %% 4, 16-byte alignment");
    DLS_REQUIRE(ldq < ((int64_t)1 << 32), DLS_ELAYOUT,
                "dls_dequant_fedavg: ldq=%lld must be < 2^32 (32-bit lane offsets)",
                (long long)ldq);
    // two-constant division when proven exact for this N, else Markstein (the
    // FMA-mode bulk kernels divide once per (client, channel) with IEEE '/')
    const FastDiv d = mode == DLS_FEDAVG_FMA ? make_fastdiv(total) : make_fastdiv2(total);
    const SzLayout L{sz_row, sz_chan};
    hipStream_t st = as_stream(stream);
    constexpr int wpb = kBlock / 64;
    // Groups: 0-3 one-channel tiles of 4/3/2/1 KiB slices, 4-7 lane-channel tiles
    // of 4/3/2/1 KiB, 8 fp32 tiles, 9 small int tiles, then the general tiles.  The group with
    // the most bytes runs on the caller's stream; every other non-empty group on a
    // side stream of its own, concurrently (their waves walk all K clients, so a
    // small group is a long latency chain, not a small amount of work), and the
    // caller's stream joins them all.
    const dls_qtile *tg[DLS_QTILE_GROUPS];
    const dls_qtile *t = tiles;
    int big = -1;
    auto bytes = [&](int g) {  // ~ bytes per client of group g
        return g < 8 ? (int64_t)nfast[g] * 1024 * (4 - g % 4) : (int64_t)nfast[g] * 256;
    };
    for (int g = 0; g < DLS_QTILE_GROUPS; ++g) {
        tg[g] = t;
        t += nfast[g];
        if (nfast[g] > 0 && (big < 0 || bytes(g) > bytes(big))) big = g;
    }
    // FMA mode: the lane groups (4-7, contiguous in the table) as ONE launch of
    // k_dequant_lanes_fma_any, on the caller's stream when their bytes are the most
    const bool any = mode == DLS_FEDAVG_FMA && kQuantFmaAny;
    int lanes_n = 0;
    int64_t lanes_bytes = 0;
    bool big_lanes = false;
    if (any) {
        for (int g = 4; g < 8; ++g) {
            lanes_n += nfast[g];
            lanes_bytes += bytes(g);
        }
        big = -1;
        for (int g = 0; g < DLS_QTILE_GROUPS; ++g)
            if ((g < 4 || g > 7) && nfast[g] > 0 && (big < 0 || bytes(g) > bytes(big))) big = g;
        if (lanes_n > 0 && (big < 0 || lanes_bytes >= bytes(big))) {
            big_lanes = true;
            big = -1;
        }
    }
    // FMA mode: groups 0-9 on quant_fma.hip's kernel on the caller's stream (the
    // fp32 and small-int tiles exact, in the first launch piece); only general
    // tiles (channel rows < 4 elements) still go to a side stream
    const bool stream_fma = mode == DLS_FEDAVG_FMA && kQuantFmaStream;
    if (stream_fma) {
        big = -1;
        big_lanes = false;
    }
    const int ngen = ntiles - (int)nf;
    // fork / join events cached per caller stream (dls_runtime.hip call_event):
    // a call creates and destroys nothing
    hipEvent_t fork = nullptr;
    hipStream_t sides[DLS_QTILE_GROUPS + 1] = {};
    int nside = 0;
    bool forked = false;
    auto stream_for = [&](bool empty) -> hipStream_t {  // a fresh side stream, else st
        if (empty) return st;
        if (!forked) {
            forked = true;
            fork = call_event(st, 0);
            if (fork && hipEventRecord(fork, st) != hipSuccess) fork = nullptr;
        }
        if (!fork) return st;
        hipStream_t s2 = side_stream(st, nside);
        if (!s2 || hipStreamWaitEvent(s2, fork, 0) != hipSuccess) return st;
        sides[nside++] = s2;
        return s2;
    };
    using Kfn = void (*)(const dls_qtile *, int, const uint8_t *, int64_t, const f32x2 *, SzLayout,
                         const int32_t *, const float *, int, FastDiv, float *);
    // [group][0: Markstein, 1: two-constant division, 2: FMA mode]
    static const Kfn kgroup[8][3] = {
        {k_dequant_fast<4, false>, k_dequant_fast<4, true>, k_dequant_fast_fma<4>},
        {k_dequant_fast<3, false>, k_dequant_fast<3, true>, k_dequant_fast_fma<3>},
        {k_dequant_fast<2, false>, k_dequant_fast<2, true>, k_dequant_fast_fma<2>},
        {k_dequant_fast<1, false>, k_dequant_fast<1, true>, k_dequant_fast_fma<1>},
        {k_dequant_lanes<4, false>, k_dequant_lanes<4, true>, k_dequant_lanes_fma<4>},
        {k_dequant_lanes<3, false>, k_dequant_lanes<3, true>, k_dequant_lanes_fma<3>},
        {k_dequant_lanes<2, false>, k_dequant_lanes<2, true>, k_dequant_lanes_fma<2>},
        {k_dequant_lanes<1, false>, k_dequant_lanes<1, true>, k_dequant_lanes_fma<1>}};
    // A wave walks all K clients, so waves are long and equal: a group is launched
    // in pieces of at most one generation of resident waves (a last generation of
    // a few waves would run alone at latency-bound speed; cf. dls_fedavg_f32).
    auto launch_group = [&](int g, hipStream_t s) {
        const int n = nfast[g];
        if (n == 0) return;
        if (g == 8) {
            hipLaunchKernelGGL(k_dequant_f32, dim3((unsigned)((n + wpb - 1) / wpb)), dim3(kBlock),
                               0, s, tg[g], n, F, ldf, rows, weight, (int)K, d, out);
            return;
        }
        if (g == 9) {
            hipLaunchKernelGGL(k_dequant_small, dim3((unsigned)((n + wpb - 1) / wpb)),
                               dim3(kBlock), 0, s, tg[g], n, reinterpret_cast<const uint8_t *>(Q),
                               ldq, reinterpret_cast<const f32x2 *>(sz), L, rows, weight, (int)K, d,
                               out);
            return;
        }
        const Kfn kern = kgroup[g][mode == DLS_FEDAVG_FMA ? 2 : (d.two ? 1 : 0)];
        int64_t slots = (int64_t)resident_blocks(reinterpret_cast<const void *>(kern), kBlock, 0) * wpb;
        if (kQuantPieceWps > 0)  // pieces of this many waves per SIMD (A/B knob)
            slots = std::min<int64_t>(slots, (int64_t)device_cus() * 4 * kQuantPieceWps);
        const int64_t np = (n + slots - 1) / slots;
        const int64_t per = (n + np - 1) / np;  // tiles per piece, <= slots
        for (int64_t t0 = 0; t0 < n; t0 += per) {
            const int m = (int)(n - t0 < per ? n - t0 : per);
            hipLaunchKernelGGL(kern, dim3((unsigned)((m + wpb - 1) / wpb)), dim3(kBlock), 0, s,
                               tg[g] + t0, m, reinterpret_cast<const uint8_t *>(Q), ldq,
                               reinterpret_cast<const f32x2 *>(sz), L, rows, weight, (int)K, d, out);
        }
    };
    auto launch_lanes_any = [&](hipStream_t s) {  // pieces of at most one generation
        const void *kern = reinterpret_cast<const void *>(k_dequant_lanes_fma_any);
        const int64_t slots = (int64_t)resident_blocks(kern, kBlock, 0) * wpb;
        const int64_t np = (lanes_n + slots - 1) / slots;
        const int64_t per = (lanes_n + np - 1) / np;
        for (int64_t t0 = 0; t0 < lanes_n; t0 += per) {
            const int m = (int)(lanes_n - t0 < per ? lanes_n - t0 : per);
            hipLaunchKernelGGL(k_dequant_lanes_fma_any, dim3((unsigned)((m + wpb - 1) / wpb)),
                               dim3(kBlock), 0, s, tg[4] + t0, m,
                               reinterpret_cast<const uint8_t *>(Q), ldq,
                               reinterpret_cast<const f32x2 *>(sz), L, rows, weight, (int)K, d, out);
        }
    };
    for (int g = 0; g < DLS_QTILE_GROUPS; ++g) {
        if ((any || stream_fma) && g >= 4 && g < 8) continue;
        if (stream_fma && (g < 4 || g == 8 || g == 9)) continue;  // all on the FMA kernel
        if (g != big && nfast[g] > 0) launch_group(g, stream_for(false));
    }
    if (any && !stream_fma && lanes_n > 0 && !big_lanes) launch_lanes_any(stream_for(false));
    if (ngen > 0)
        hipLaunchKernelGGL(k_dequant_general, dim3((unsigned)((ngen + wpb - 1) / wpb)),
                           dim3(kBlock), 0, stream_for(false), t, ngen,
                           reinterpret_cast<const uint8_t *>(Q), ldq, F, ldf,
                           reinterpret_cast<const f32x2 *>(sz), L, rows, weight, (int)K, d, out);
    int rc = DLS_OK;
    if (stream_fma)
        rc = launch_dequant_fma_stream(tiles, nfast, Q, ldq, F, ldf, sz, sz_row, sz_chan, rows,
                                       weight, K, total, out, st);
    else if (big_lanes)
        launch_lanes_any(st);
    else if (big >= 0)
        launch_group(big, st);
    if (rc == DLS_OK) rc = check_launch("dls_dequant_fedavg");
    for (int i = 0; i < nside; ++i) {
        hipEvent_t join = call_event(st, 1 + i);
        hipError_t e = join ? hipEventRecord(join, sides[i]) : hipErrorOutOfMemory;
        if (e == hipSuccess) e = hipStreamWaitEvent(st, join, 0);
        if (e != hipSuccess) {  // the caller's stream must not run ahead of the side work
            (void)hipStreamSynchronize(sides[i]);
            set_error("dls_dequant_fedavg: stream join failed: %s", hipGetErrorString(e));
            rc = (int)e;
        }
    }
    return rc;
}

extern "C" int dls_segment_minmax_f32(const float *x, const int64_t *seg_off, int32_t nseg,
                                      float *mins, float *maxs, int64_t total,
                                      dls_stream_t stream) {
    DLS_REQUIRE(x && seg_off && mins && maxs, DLS_EINVAL, "dls_segment_minmax_f32: null pointer");
    DLS_REQUIRE(nseg > 0 && total > 0, DLS_EINVAL, "dls_segment_minmax_f32: nseg=%d total=%lld",
                nseg, (long long)total);
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(k_minmax_init, dim3((unsigned)((nseg + 255) / 256)), dim3(256), 0, st, mins,
                       maxs, (int)nseg);
    const int64_t blocks = (total + kMinmaxChunk - 1) / kMinmaxChunk;
    hipLaunchKernelGGL(k_segment_minmax, dim3((unsigned)blocks), dim3(kBlock), 0, st, x, seg_off,
                       (int)nseg, mins, maxs);
    return check_launch("dls_segment_minmax_f32");
}

extern "C" int dls_qparams_minmax(const float *mins, const float *maxs, int32_t nseg, int32_t qmin,
                                  int32_t qmax, int32_t symmetric, float *scale, int32_t *zp,
                                  dls_stream_t stream) {
    DLS_REQUIRE(mins && maxs && scale && zp && nseg > 0 && qmax > qmin, DLS_EINVAL,
                "dls_qparams_minmax: bad arguments");
    hipLaunchKernelGGL(k_qparams, dim3((unsigned)((nseg + 255) / 256)), dim3(256), 0,
                       as_stream(stream), mins, maxs, (int)nseg, (int)qmin, (int)qmax,
                       (int)symmetric, scale, zp);
    return check_launch("dls_qparams_minmax");
}

extern "C" int dls_quantize_affine(const float *x, const int64_t *seg_off, int32_t nseg,
                                   const float *scale, const int32_t *zp, int32_t qmin,
                                   int32_t qmax, void *q, float *deq, int32_t stochastic,
                                   uint64_t seed, int64_t total, dls_stream_t stream) {
    DLS_REQUIRE(x && seg_off && scale && zp && q && nseg > 0 && total > 0, DLS_EINVAL,
                "dls_quantize_affine: bad arguments");
    DLS_REQUIRE(qmin >= -128 && qmax <= 255 && qmax > qmin && qmax - qmin <= 255, DLS_EINVAL,
                "dls_quantize_affine: [qmin, qmax] = [%d, %d] must fit one byte", qmin, qmax);
    const int64_t threads = (total + 3) / 4;
    hipLaunchKernelGGL(k_quantize, dim3((unsigned)((threads + kBlock - 1) / kBlock)), dim3(kBlock),
                       0, as_stream(stream), x, seg_off, (int)nseg, scale, zp, (float)qmin,
                       (float)qmax, reinterpret_cast<uint8_t *>(q), deq, (int)stochastic, seed);
    return check_launch("dls_quantize_affine");
}

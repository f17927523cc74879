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
#include "dls_common.h"

namespace dls {
namespace {

constexpr int kBlock = 256;
#ifndef DLS_QUANT_U
#define DLS_QUANT_U 2  // A/B on MI355X: 2 > 3 > 4 clients per batch (tools/ab_bench.py)
#endif
#ifndef DLS_QUANT_SCALAR_SZ
#define DLS_QUANT_SCALAR_SZ 1
#endif

__device__ __forceinline__ float byte_f32(uint32_t w, int k) {
    return (float)((w >> (8 * k)) & 0xffu);  // selects v_cvt_f32_ubyte{k}
}

__device__ __forceinline__ bool scale_fast(float sw) {
    // |q - zp| in [1, 383]: fl(deq*n) then lies in [2^-60, 2^60] (dls_common.h)
    return sw >= 0x1p-59f && sw <= 0x1p50f;
}

// One client's contribution to a lane's 16 consecutive elements.  TWO: the
// chunk straddles a channel boundary at `split` (elements [split,16) use the
// next channel's (scale, zero point)); FIRST: assign instead of accumulate
// (servers/fed_server.py:62-65).  The exact-division fast path is decided once
// per client from the channel scale (scale_fast), not per element.
template <bool SIGNED, bool TWO, bool FIRST>
__device__ __forceinline__ void accum16(float (&acc)[16], u32x4 qv, f32x2 a, f32x2 b, float wk,
                                        int split, const FastDiv &d) {
    if (SIGNED) qv ^= 0x80808080u;  // int8 q read as the unsigned byte q + 128
    const float zadj = SIGNED ? 128.f : 0.f;
    const float za = a.y + zadj, zb = b.y + zadj;
    const bool fast = d.fast && scale_fast(a.x * wk) && (!TWO || scale_fast(b.x * wk));
    if (__builtin_expect(fast, 1)) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const bool second = TWO && j >= split;
            const float s = second ? b.x : a.x;
            const float z = second ? zb : za;
            const float x = byte_f32(qv[j >> 2], j & 3);
            const float q = markstein(((x - z) * s) * wk, d.b, d.y);
            acc[j] = FIRST ? q : acc[j] + q;
        }
    } else {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const bool second = TWO && j >= split;
            const float s = second ? b.x : a.x;
            const float z = second ? zb : za;
            const float x = byte_f32(qv[j >> 2], j & 3);
            const float q = (((x - z) * s) * wk) / d.b;
            acc[j] = FIRST ? q : acc[j] + q;
        }
    }
}

template <bool SIGNED, bool TWO>
__device__ __forceinline__ void int_chunk_loop(float (&acc)[16], const uint8_t *__restrict__ Qt,
                                               int64_t ldq, const f32x2 *__restrict__ szc,
                                               int64_t ldc, const int32_t *__restrict__ rows,
                                               const float *__restrict__ w, int K, int split,
                                               const FastDiv &d) {
    constexpr int U = DLS_QUANT_U;  // clients per batch (two batches in flight per lane)
    const f32x2 zero2 = f32x2{0.f, 0.f};
    {
        const int64_t row = rows[0];
        const u32x4 qv = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(Qt + row * ldq));
        const f32x2 a = szc[row * ldc];
        const f32x2 b = TWO ? szc[row * ldc + 1] : zero2;
        accum16<SIGNED, TWO, true>(acc, qv, a, b, w[0], split, d);
    }
    // batches of U clients, double-buffered: batch b+1 loads while batch b computes
    struct Batch {
        u32x4 qv[U];
        f32x2 a[U], b[U];
    };
    auto load = [&](int k0, Batch &bt) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t row = rows[k0 + u];
            bt.qv[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(Qt + row * ldq));
            bt.a[u] = szc[row * ldc];
            bt.b[u] = TWO ? szc[row * ldc + 1] : zero2;
        }
    };
    auto consume = [&](int k0, const Batch &bt) {
#pragma unroll
        for (int u = 0; u < U; ++u)
            accum16<SIGNED, TWO, false>(acc, bt.qv[u], bt.a[u], bt.b[u], w[k0 + u], split, d);
    };
    int k = 1;
    const int nfull = (K - 1) / U;  // full batches after the peeled first client
    if (nfull > 0) {
        Batch A, B;
        load(k, A);
        for (int bi = 0; bi < nfull; bi += 2) {
            if (bi + 1 < nfull) load(k + U, B);
            consume(k, A);
            k += U;
            if (bi + 1 >= nfull) break;
            if (bi + 2 < nfull) load(k + U, A);
            consume(k, B);
            k += U;
        }
    }
    for (; k < K; ++k) {
        const int64_t row = rows[k];
        const u32x4 qv = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(Qt + row * ldq));
        const f32x2 a = szc[row * ldc];
        const f32x2 b = TWO ? szc[row * ldc + 1] : zero2;
        accum16<SIGNED, TWO, false>(acc, qv, a, b, w[k], split, d);
    }
}

// Integer (per-channel) tile: 16 consecutive elements per lane.
template <bool SIGNED>
__device__ __forceinline__ void int_tile(const dls_qtile &t, const uint8_t *__restrict__ Q,
                                         int64_t ldq, const f32x2 *__restrict__ sz, int64_t ldc,
                                         const int32_t *__restrict__ rows,
                                         const float *__restrict__ w, int K, const FastDiv &d,
                                         float *__restrict__ out, int e0) {
    const int p = t.row_pos + e0;
    const int c = t.chan0 + p / t.row_len;
    const int r = p % t.row_len;
    float acc[16];
    if (t.row_len >= 16) {
        const int split = t.row_len - r;  // elements [0, split) in channel c, rest in c + 1
        // wave-uniform choice: most waves of a large-row tensor never straddle a channel
        if (__ballot(split < 16) == 0) {
            const int c0 = __builtin_amdgcn_readfirstlane(c);
            if (DLS_QUANT_SCALAR_SZ && __ballot(c != c0) == 0)  // one channel for the whole
                // wave: (scale, zp) become scalar loads and the fast-path test a uniform branch
                int_chunk_loop<SIGNED, false>(acc, Q + t.src + e0, ldq, sz + c0, ldc, rows, w, K,
                                              16, d);
            else
                int_chunk_loop<SIGNED, false>(acc, Q + t.src + e0, ldq, sz + c, ldc, rows, w, K,
                                              16, d);
        } else
            int_chunk_loop<SIGNED, true>(acc, Q + t.src + e0, ldq, sz + c, ldc, rows, w, K, split, d);
    } else {  // tiny channel rows: per-element channel lookup
        const float zadj = SIGNED ? 128.f : 0.f;
        int cj[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) cj[j] = min(c + (r + j) / t.row_len, t.chan_end - 1);
        for (int k = 0; k < K; ++k) {
            const int64_t row = rows[k];
            u32x4 qv = *reinterpret_cast<const u32x4 *>(Q + row * ldq + t.src + e0);
            if (SIGNED) qv ^= 0x80808080u;
            const float wk = w[k];
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const f32x2 a = sz[row * ldc + cj[j]];
                const float x = byte_f32(qv[j >> 2], j & 3);
                const float deq = (x - (a.y + zadj)) * a.x;
                const float tn = deq * wk;
                const float q = (d.fast && scale_fast(a.x * wk)) ? markstein(tn, d.b, d.y)
                                                                : tn / d.b;
                acc[j] = (k == 0) ? q : acc[j] + q;
            }
        }
    }
    if (e0 + 16 > t.len) {  // tensor tail: keep the row padding zero
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[j] = (e0 + j < t.len) ? acc[j] : 0.f;
    }
    f32x4 *o = reinterpret_cast<f32x4 *>(out + t.dst + e0);
#pragma unroll
    for (int v = 0; v < 4; ++v)
        o[v] = f32x4{acc[4 * v], acc[4 * v + 1], acc[4 * v + 2], acc[4 * v + 3]};
}

__device__ __forceinline__ float fp_term(float x, float wk, const FastDiv &d) {
    const float tn = x * wk;
    return (d.fast && in_fast_range(tn)) ? markstein(tn, d.b, d.y) : tn / d.b;
}

__device__ __forceinline__ void f32_tile(const dls_qtile &t, const float *__restrict__ F,
                                         int64_t ldf, const int32_t *__restrict__ rows,
                                         const float *__restrict__ w, int K, const FastDiv &d,
                                         float *__restrict__ out, int e0) {
    f32x4 acc[4];
    for (int k = 0; k < K; ++k) {
        const f32x4 *src = reinterpret_cast<const f32x4 *>(F + (int64_t)rows[k] * ldf + t.src + e0);
        const float wk = w[k];
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const f32x4 x = src[v];
            f32x4 q;
#pragma unroll
            for (int c = 0; c < 4; ++c) q[c] = fp_term(x[c], wk, d);
            acc[v] = (k == 0) ? q : acc[v] + q;
        }
    }
    if (e0 + 16 > t.len) {
#pragma unroll
        for (int v = 0; v < 4; ++v)
#pragma unroll
            for (int c = 0; c < 4; ++c) acc[v][c] = (e0 + 4 * v + c < t.len) ? acc[v][c] : 0.f;
    }
    f32x4 *o = reinterpret_cast<f32x4 *>(out + t.dst + e0);
#pragma unroll
    for (int v = 0; v < 4; ++v) o[v] = acc[v];
}

__global__ __launch_bounds__(kBlock) void k_dequant_fedavg(
    const dls_qtile *__restrict__ tiles, const uint8_t *__restrict__ Q, int64_t ldq,
    const float *__restrict__ F, int64_t ldf, const f32x2 *__restrict__ sz, int64_t ldc,
    const int32_t *__restrict__ rows, const float *__restrict__ w, int K, FastDiv d,
    float *__restrict__ out) {
    const dls_qtile t = tiles[blockIdx.x];
    const int e0 = 16 * threadIdx.x;
    if (e0 >= ((t.len + 63) & ~63)) return;  // chunks up to the 64-element row padding
    if (t.kind == 1)
        int_tile<true>(t, Q, ldq, sz, ldc, rows, w, K, d, out, e0);
    else if (t.kind == 2)
        int_tile<false>(t, Q, ldq, sz, ldc, rows, w, K, d, out, e0);
    else
        f32_tile(t, F, ldf, rows, w, K, d, out, e0);
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
            const int s = find_segment(seg_off, nseg, e);
            atomic_min_f32(mins + s, x[e]);
            atomic_max_f32(maxs + s, x[e]);
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

extern "C" int dls_dequant_fedavg(const dls_qtile *tiles, int32_t ntiles, const void *Q,
                                  int64_t ldq, const float *F, int64_t ldf, const float *sz,
                                  int64_t ldc, const int32_t *rows, const float *weight, int32_t K,
                                  float total, float *out, dls_stream_t stream) {
    DLS_REQUIRE(tiles && rows && weight && out && sz, DLS_EINVAL,
                "dls_dequant_fedavg: null pointer");
    DLS_REQUIRE(ntiles > 0 && K > 0, DLS_EINVAL, "dls_dequant_fedavg: ntiles=%d K=%d", ntiles, K);
    DLS_REQUIRE(ldq % 16 == 0 && ldf % 4 == 0 && aligned16(out) && (!Q || aligned16(Q)) &&
                    (!F || aligned16(F)),
                DLS_ELAYOUT, "dls_dequant_fedavg: ldq %% 16, ldf %% 4, 16-byte alignment");
    const FastDiv d = make_fastdiv(total);
    hipLaunchKernelGGL(k_dequant_fedavg, dim3((unsigned)ntiles), dim3(kBlock), 0,
                       as_stream(stream), tiles, reinterpret_cast<const uint8_t *>(Q), ldq, F, ldf,
                       reinterpret_cast<const f32x2 *>(sz), ldc, rows, weight, (int)K, d, out);
    return check_launch("dls_dequant_fedavg");
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

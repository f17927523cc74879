// FMA mode (DLS_FEDAVG_FMA) of the fused dequant-FedAvg: every int tile of the
// table's groups 0-7 (one-channel and lane-channel tiles, 1-4 KiB slices) on one
// kernel, in launch pieces of exactly one wave per SIMD.
//
// Reference: FedQuantServer._process_client_parameter (servers/fed_quant_server.py:25-33)
// dequantizes each client's int tensors channel by channel, FedServer.get_subset_model
// (servers/fed_server.py:44-66) averages them.  FMA mode folds the per-(client,
// channel) constants into one c = fl(fl(scale * n_i) / N) and accumulates
//     out[e] = fma(q - zp, c, out[e])          (q - zp exact in fp32)
// which is the north-star's 1e-6 (normwise) FedAvg tolerance, not bit-exact; the
// bits equal the round-4 FMA kernels' (the same terms in the same client order).
// Algorithmic bytes per call: K*(Pq + 8*C) for these tiles + 4*Pq written.
//
// What sets the stream rate here (round 5, profiles/r05_quant_fma_ab.txt, the
// same payloads in one process): every wave of a launch piece walks the K
// client rows of its tile in the same order, so while the piece's waves stay in
// step they read one contiguous window of one client row at a time.  Waves that
// share a SIMD do not stay in step (the older one issues first), so the pieces
// hold ONE wave per SIMD (4-wave blocks, one per CU: 1,024 waves), with only 2
// clients in flight per wave and non-temporal output stores:
//   100 x VGG-16 2.19-2.22 ms (6.5-6.6 TB/s), 1000 x ResNet-18 1.71-1.73 ms,
// against 2.43 / 1.82 ms for the round-4 kernels (2-3 waves per SIMD, one
// generation per piece).  Measured worse, same session: 2-3 waves per SIMD
// (+8-11 %), 4 / 8 / 16 clients in flight (+7 / +12 / +20 %), a persistent grid
// pulling tiles from a device queue (+24 %), one oversubscribed launch (+23 %),
// pieces alternating between two streams (+20 %), runs of 2-4 tiles per wave with
// the ring carried across them (+1-3 % VGG, +8-24 % ResNet-18), 8 KiB tiles (+3 %),
// plain stores (+4 %).
//
// The client walk is one ring of D clients in flight per wave that runs across
// the 64-client chunk boundaries: client rows and weights come from per-lane
// chunk tables read back with v_readlane (lane j = client 64c + j; chunks c, c+1
// in registers, c+2 in flight), and each chunk's (c, -zp) of the tile's <= 4
// channels are staged in the wave's LDS table at the chunk start (lane j computes
// client j's), read per client with one broadcast ds_read_b64 per slice.  Clients
// past K get c = 0 (their loads are clamped duplicates), so the ring needs no
// tail code.
#include <algorithm>
#include <type_traits>

#include "dls_common.h"
#include "quant_common.h"

namespace dls {
namespace {

using namespace quant;

constexpr int kFmaBlock = 256;  // 4 waves: a piece places one block per CU, one wave per SIMD
constexpr int kFmaSpan = 4;     // channels per staged table (a tile over more: passes)

#ifndef DLS_FMA_D
#define DLS_FMA_D 2
#endif
constexpr int kFmaD = DLS_FMA_D;  // clients in flight per wave
static_assert(kFmaD >= 1 && kFmaD <= 64, "the ring depth");
#ifndef DLS_FMA_GMAX
#define DLS_FMA_GMAX 4
#endif
constexpr int kFmaGMax = DLS_FMA_GMAX;  // widest tile (KiB slices) the kernel instantiates
#ifndef DLS_FMA_T
#define DLS_FMA_T 0
#endif
// tiles per wave per launch piece; 0: 2 for short client walks (K <= 256: the
// pieces' fixed start and drain are a larger share of a 100-client walk), else 1
constexpr int kFmaT = DLS_FMA_T;
#ifndef DLS_FMA_WPS
#define DLS_FMA_WPS 1
#endif
constexpr int kFmaWps = DLS_FMA_WPS;  // waves per SIMD per launch piece
#ifndef DLS_FMA_NTSTORE
#define DLS_FMA_NTSTORE 1  // non-temporal output stores (0: plain, A/B knob)
#endif
#ifndef DLS_FMA_SIDE_PRIO
#define DLS_FMA_SIDE_PRIO 0  // issue priority of the fp32 / small-int side waves (3: +1 %)
#endif
// A piece with fewer than 80 % of its waves on 3-4 KiB tiles (ResNet-18's last:
// 766 of 994, the rest 1x1-conv tiles of <= 1 KiB that finish early) leaves SIMDs
// without a stream; its waves keep DS x the clients in flight: 1000 x ResNet-18
// 1.717-1.727 -> 1.665-1.668 ms (DS 3: 1.728-1.734), VGG-16 unchanged, the same
// bits (profiles/r05_quant_fma_ab.txt, r05p2).
#ifndef DLS_FMA_SPARSE_DS
#define DLS_FMA_SPARSE_DS 2
#endif
#ifndef DLS_FMA_F32U
#define DLS_FMA_F32U 16  // clients per batch of the fp32 side walk (two batches in flight)
#endif
#ifndef DLS_FMA_PROBE
#define DLS_FMA_PROBE 0  // 1: stream-only timing probe (loads + a xor per dword; wrong output)
#endif

// The tile order: segment s (widest tiles first: table groups 0, 4, 1, 5, 2, 6,
// 3, 7) holds indices [cum[s], cum[s+1]), table indices start[s] + i.
struct FmaPlan {
    int cum[9];
    int start[8];
};

// Bytes HI*2, HI*2+1 of w as two fp32 values (sign-extended for int8: SDWA byte
// select; unsigned: v_cvt_f32_ubyteN).  In volatile asm so that the conversions
// stay in program order with the accumulation steps: as plain code the compiler
// converted all 16 bytes of every in-flight client up front.
template <bool SEXT, int HI>
__device__ __forceinline__ f32x2 cvt2(uint32_t w) {
    float lo, hi;
    if constexpr (SEXT && HI == 0)
        asm volatile(
            "v_cvt_f32_i32_sdwa %0, sext(%2) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0\n\t"
            "v_cvt_f32_i32_sdwa %1, sext(%2) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1"
            : "=v"(lo), "=v"(hi) : "v"(w));
    else if constexpr (SEXT)
        asm volatile(
            "v_cvt_f32_i32_sdwa %0, sext(%2) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2\n\t"
            "v_cvt_f32_i32_sdwa %1, sext(%2) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3"
            : "=v"(lo), "=v"(hi) : "v"(w));
    else if constexpr (HI == 0)
        asm volatile("v_cvt_f32_ubyte0 %0, %2\n\tv_cvt_f32_ubyte1 %1, %2"
                     : "=v"(lo), "=v"(hi) : "v"(w));
    else
        asm volatile("v_cvt_f32_ubyte2 %0, %2\n\tv_cvt_f32_ubyte3 %1, %2"
                     : "=v"(lo), "=v"(hi) : "v"(w));
    return f32x2{lo, hi};
}

// acc[0..16) += (x - z) * c for the lane's 16 bytes, cz = (c, -z): x + (-z) is
// exact (x + (-0) == x, so zero points 0 give the subtraction-free bits), then one
// packed fma per element pair.  Two independent pairs per step, interleaved by
// hand (a packed op reading the packed result issued just before it waits a
// cycle group).
template <bool SEXT>
__device__ __forceinline__ void fma16(float (&acc)[16], u32x4 qv, f32x2 cz) {
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
        f32x2 xa, xb;
        if ((j & 3) == 0) {
            xa = cvt2<SEXT, 0>(qv[j >> 2]);
            xb = cvt2<SEXT, 0>(qv[(j >> 2) + 2]);
        } else {
            xa = cvt2<SEXT, 1>(qv[j >> 2]);
            xb = cvt2<SEXT, 1>(qv[(j >> 2) + 2]);
        }
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

// Wave-level arguments that stay fixed over the call.
struct FmaCall {
    const uint8_t *Q;
    int64_t ldq;
    const f32x2 *sz;
    SzLayout L;
    const int32_t *rows;
    const float *w;
    int K;
    float N;
    float *out;
};

// The tile descriptor in scalar registers (every field wave-uniform), so that
// the walk's per-tile constants (channel offsets, lengths) are SGPRs.
__device__ __forceinline__ dls_qtile uniform_tile(const dls_qtile *p) {
    const int32_t *w = reinterpret_cast<const int32_t *>(p);
    int32_t v[10];
#pragma unroll
    for (int i = 0; i < 10; ++i) v[i] = __builtin_amdgcn_readfirstlane(w[i]);
    dls_qtile t;
    t.dst = (int64_t)(((uint64_t)(uint32_t)v[1] << 32) | (uint32_t)v[0]);
    t.src = (int64_t)(((uint64_t)(uint32_t)v[3] << 32) | (uint32_t)v[2]);
    t.len = v[4];
    t.kind = v[5];
    t.chan0 = v[6];
    t.row_len = v[7];
    t.row_pos = v[8];
    t.chan_end = v[9];
    return t;
}

// One tile of G KiB slices (lane l of slice g: elements 1024 g + 16 l .. +16),
// walked over all K clients with D in flight.  rf0/wf0, rf1/wf1: the chunk
// tables of clients 0-63 and 64-127 (call-wide, loaded once per wave).  buf: the
// wave's 4 KiB of LDS (coefficient table while walking, store transpose at the end).
// Clients in flight per wave for G KiB slices: kFmaD at 3-4 KiB, more for narrower
// tiles (DLS_FMA_DN: about the same bytes in flight; 0: kFmaD at every width).  A
// 1 KiB tile of a 1000-client walk at 2 in flight is a ~1,000 x latency chain
// that outlasts the launch piece's 4 KiB tiles.
#ifndef DLS_FMA_DN
#define DLS_FMA_DN 1
#endif
// DS: x DS clients in flight, for a piece whose wide tiles leave SIMDs without a
// stream (DLS_FMA_SPARSE_DS, the launcher's choice per piece)
template <int G, int DS = 1>
constexpr int ring_depth() {
    return DS * ((DLS_FMA_DN == 0 || G >= 3) ? kFmaD : (G == 2 ? 2 * kFmaD : 4 * kFmaD));
}

template <int G, bool SIGNED, int DS = 1>
__device__ __forceinline__ void fma_tile(const dls_qtile &t, const FmaCall &a, int rf0, float wf0,
                                         int rf1, float wf1, float *buf) {
    constexpr int D = ring_depth<G, DS>();
    f32x2(*tab)[64] = reinterpret_cast<f32x2(*)[64]>(buf);  // [kFmaSpan + 1][64]
    const int lane = __lane_id();
    const int K = a.K;
    const int Kpad = (K + D - 1) / D * D;
    const int lenpad = (t.len + 63) & ~63;                    // chunks up to the row padding
    const int span = (t.row_pos + t.len - 1) / t.row_len + 1;  // channels of the tile
    const int npass = (span + kFmaSpan - 1) / kFmaSpan;
    uint32_t qoff[G];  // the lane's byte offset in slice g (ldq < 4 GiB)
    int crel[G];       // its channel in slice g, relative to chan0
    float acc[G][16];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const int e0 = 1024 * g + 16 * lane;
        const int ec = e0 < lenpad ? e0 : lenpad - 16;  // idle lanes load a valid duplicate
        qoff[g] = (uint32_t)(t.src + ec);
        crel[g] = min((t.row_pos + ec) / t.row_len, span - 1);
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[g][e] = 0.f;
    }
    tab[kFmaSpan][lane] = f32x2{0.f, 0.f};  // the zero row (lanes outside the pass)
    auto fetch = [&](u32x4 (&v)[G], int row) {
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint8_t *>(a.Q + (int64_t)row * a.ldq), 0, (int)0xffffffffu, 0x00020000);
#pragma unroll
        for (int g = 0; g < G; ++g)
            v[g] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)qoff[g], 0, 2 /* nt */);
    };
    for (int p = 0; p < npass; ++p) {
        uint32_t toff[G];  // the lane's table row in this pass, in pairs
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const int c = crel[g] - kFmaSpan * p;
            toff[g] = (uint32_t)(c >= 0 && c < kFmaSpan ? c : kFmaSpan) * 64;
        }
        int64_t choff[kFmaSpan];  // the pass's channels (clamped into the tensor), in pairs
#pragma unroll
        for (int c = 0; c < kFmaSpan; ++c)
            choff[c] = (int64_t)min(t.chan0 + kFmaSpan * p + c, t.chan_end - 1) * a.L.chan;
        int r0 = rf0, r1 = rf1, r2;
        float w0 = wf0, w1 = wf1, w2;
        {
            const int kk = min(128 + lane, K - 1);
            r2 = a.rows[kk];
            w2 = a.w[kk];
        }
        f32x2 szn[kFmaSpan];
#pragma unroll
        for (int c = 0; c < kFmaSpan; ++c) szn[c] = a.sz[choff[c] + (int64_t)r0 * a.L.row];
        u32x4 slot[D][G];
#pragma unroll
        for (int u = 0; u < D; ++u) fetch(slot[u], readlane_i(r0, u));  // lanes >= K hold row K-1
        auto chunk_start = [&](int k) {  // wave-uniform
            if (k > 0) {
                r0 = r1;
                w0 = w1;
                r1 = r2;
                w1 = w2;
                const int kk = min(k + 128 + lane, K - 1);
                r2 = a.rows[kk];
                w2 = a.w[kk];
            }
            const bool live = lane < K - k;  // lanes past K: c = 0
#pragma unroll
            for (int c = 0; c < kFmaSpan; ++c)  // c = fl(fl(s * n_i) / N), IEEE division
                tab[c][lane] = live ? f32x2{(szn[c].x * w0) / a.N, -szn[c].y} : f32x2{0.f, 0.f};
#pragma unroll
            for (int c = 0; c < kFmaSpan; ++c)  // the next chunk's (its rows landed a chunk ago)
                szn[c] = a.sz[choff[c] + (int64_t)r1 * a.L.row];
        };
        for (int k = 0; k < Kpad; k += D) {
            if constexpr (64 % D == 0)
                if ((k & 63) == 0) chunk_start(k);
#pragma unroll
            for (int u = 0; u < D; ++u) {
                const int kk = k + u;
                if constexpr (64 % D != 0)
                    if ((kk & 63) == 0) chunk_start(kk);
                const int j = kk & 63;
#pragma unroll
                for (int g = 0; g < G; ++g) {
                    if constexpr (DLS_FMA_PROBE == 1)
                        acc[g][g] += __uint_as_float(
                            (slot[u][g].x ^ slot[u][g].y ^ slot[u][g].z ^ slot[u][g].w) & 0x3fffffffu);
                    else
                        fma16<SIGNED>(acc[g], slot[u][g], tab[0][toff[g] + j]);
                }
                const int f = kk + D, cb = kk & ~63;  // f < cb + 128: in chunk cb or the next
                fetch(slot[u], f - cb < 64 ? readlane_i(r0, f & 63) : readlane_i(r1, f & 63));
            }
        }
    }
    // store: transposed through LDS so that each store instruction writes 1 KiB
    // contiguous; lanes past len write 0 (the output's row padding stays zero).
    // One slice at a time (scheduling barriers); len and lane laundered through
    // asm: the compiler hoisted the 64 element indices of the masks and addresses
    // out of the walk (~80 VGPRs live across it)
    int len = t.len, ln = lane;
    asm volatile("" : "+v"(len), "+v"(ln));
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const int e0 = 1024 * g + 16 * ln;
#pragma unroll
        for (int v = 0; v < 8; ++v) {  // element pairs: the packed accumulators' register pairs
            f32x2 x;
#pragma unroll
            for (int c = 0; c < 2; ++c) x[c] = (e0 + 2 * v + c < len) ? acc[g][2 * v + c] : 0.f;
            *reinterpret_cast<f32x2 *>(buf + 16 * ln + 2 * v) = x;
        }
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const int e = 256 * v + 4 * ln;
            const f32x4 x = *reinterpret_cast<const f32x4 *>(buf + e);
            if (1024 * g + e < lenpad) {
                f32x4 *o = reinterpret_cast<f32x4 *>(a.out + t.dst + 1024 * g + e);
                if constexpr (DLS_FMA_NTSTORE)
                    __builtin_nontemporal_store(x, o);
                else
                    *o = x;
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    }
}

// The fp32 and small-int tiles of the call (table groups 8 and 9), walked by the
// first launch piece's extra blocks with the exact arithmetic (quant_common.h):
// no side streams, so no fork / join between calls (~20 us each).
struct FmaSide {
    const dls_qtile *f32;
    int nf32;
    const dls_qtile *small;
    int nsmall;
    const float *F;
    int64_t ldf;
    FastDiv d;
    int main_blocks;  // blocks of the piece's main tiles; the side tiles' follow
};

// One launch piece: wave w of the piece walks tiles qbase + w + i * nwaves < qend
// (T tiles per wave, the launcher sizes the piece so).
template <int DS>
__global__ __launch_bounds__(kFmaBlock) void k_dequant_fma_stream(const dls_qtile *__restrict__ tiles,
                                                                  FmaPlan plan, FmaCall a, int qbase,
                                                                  int qend, FmaSide side) {
    __shared__ __attribute__((aligned(16))) float sbuf[kFmaBlock / 64][1024];
    float *buf = sbuf[threadIdx.x >> 6];
    const int lane = __lane_id();
    if ((int)blockIdx.x >= side.main_blocks) {  // block-uniform
        const int i = ((int)blockIdx.x - side.main_blocks) * (kFmaBlock / 64) + (int)(threadIdx.x >> 6);
        __builtin_amdgcn_s_setprio(DLS_FMA_SIDE_PRIO);  // few long client walks beside the stream
        if (i < side.nf32)
            f32_side_tile<DLS_FMA_F32U>(side.f32[i], side.F, side.ldf, a.rows, a.w, a.K, side.d,
                                        a.out);
        else if (i < side.nf32 + side.nsmall)
            small_side_tile(side.small[i - side.nf32], a.Q, a.ldq, a.sz, a.L, a.rows, a.w, a.K,
                            side.d, a.out);
        return;
    }
    const int nwaves = side.main_blocks * (kFmaBlock / 64);
    // chunk tables of clients 0-63 and 64-127 (the same for every tile)
    const int rf0 = a.rows[min(lane, a.K - 1)];
    const float wf0 = a.w[min(lane, a.K - 1)];
    const int rf1 = a.rows[min(64 + lane, a.K - 1)];
    const float wf1 = a.w[min(64 + lane, a.K - 1)];
    for (int q = qbase + (int)blockIdx.x * (kFmaBlock / 64) + (int)(threadIdx.x >> 6); q < qend;
         q += nwaves) {
        int s = 0;
#pragma unroll
        for (int i = 1; i < 8; ++i) s += (q >= plan.cum[i]) ? 1 : 0;
        const dls_qtile t = uniform_tile(tiles + plan.start[s] + (q - plan.cum[s]));
        const int slices = (t.len + 1023) >> 10;
        auto by_width = [&](auto sgn) {
            constexpr bool SG = decltype(sgn)::value;
            if (kFmaGMax >= 4 && slices >= 4)
                fma_tile<(kFmaGMax >= 4 ? 4 : 1), SG, DS>(t, a, rf0, wf0, rf1, wf1, buf);
            else if (kFmaGMax >= 3 && slices == 3)
                fma_tile<(kFmaGMax >= 3 ? 3 : 1), SG, DS>(t, a, rf0, wf0, rf1, wf1, buf);
            else if (kFmaGMax >= 2 && slices == 2)
                fma_tile<(kFmaGMax >= 2 ? 2 : 1), SG, DS>(t, a, rf0, wf0, rf1, wf1, buf);
            else
                fma_tile<1, SG, DS>(t, a, rf0, wf0, rf1, wf1, buf);
        };
        if (t.kind == 1)
            by_width(std::true_type{});
        else
            by_width(std::false_type{});
    }
}

}  // namespace

// Groups 0-7 of an FMA-mode call (quant.hip dls_dequant_fedavg_mode).
int launch_dequant_fma_stream(const dls_qtile *tiles, const int32_t *nfast, const void *Q,
                              int64_t ldq, const float *F, int64_t ldf, const float *sz,
                              int64_t sz_row, int64_t sz_chan, const int32_t *rows, const float *w,
                              int32_t K, float N, float *out, hipStream_t st) {
    static const int order[8] = {0, 4, 1, 5, 2, 6, 3, 7};  // widest tiles first
    int gstart[8];
    for (int g = 0, s = 0; g < 8; ++g) {
        gstart[g] = s;
        s += nfast[g];
    }
    FmaPlan plan;
    plan.cum[0] = 0;
    for (int s = 0; s < 8; ++s) {
        plan.start[s] = gstart[order[s]];
        plan.cum[s + 1] = plan.cum[s] + nfast[order[s]];
    }
    const int ntotal = plan.cum[8];
    FmaSide side{tiles + gstart[7] + nfast[7], nfast[8], tiles + gstart[7] + nfast[7] + nfast[8],
                 nfast[9], F, ldf, make_fastdiv(N), 0};
    const int nside = nfast[8] + nfast[9];
    if (ntotal == 0 && nside == 0) return DLS_OK;
    for (int g = 0; g < 8; ++g)  // groups g % 4 hold tiles of 4 - g % 4 slices
        DLS_REQUIRE(nfast[g] == 0 || 4 - g % 4 <= kFmaGMax, DLS_EINVAL,
                    "dls_dequant_fedavg_mode: group %d tiles are wider than this build's %d KiB",
                    g, kFmaGMax);
    constexpr int wpb = kFmaBlock / 64;
    // a piece: kFmaWps waves per SIMD (one 4-wave block per CU at 1), at most what
    // the kernel's registers allow resident; pieces of equal size (a part-filled
    // last piece would stream at part rate)
    const int64_t resident = std::min<int64_t>(
        (int64_t)resident_blocks(reinterpret_cast<const void *>(k_dequant_fma_stream<1>), kFmaBlock, 0) *
            wpb,
        (int64_t)device_cus() * 4 * kFmaWps);
    const int T = kFmaT > 0 ? kFmaT : (K <= 256 ? 2 : 1);
    const int64_t cap = (int64_t)T * resident;
    const int64_t npieces = std::max<int64_t>(1, (ntotal + cap - 1) / cap);
    const int64_t per = std::max<int64_t>(1, (ntotal + npieces - 1) / npieces);
    FmaCall a{reinterpret_cast<const uint8_t *>(Q), ldq, reinterpret_cast<const f32x2 *>(sz),
              SzLayout{sz_row, sz_chan}, rows, w, (int)K, N, out};
    const int side_blocks = (nside + wpb - 1) / wpb;  // with the first piece
    for (int64_t q0 = 0; q0 < std::max(ntotal, 1); q0 += per) {
        const int m = (int)(ntotal - q0 < per ? ntotal - q0 : per);
        const int64_t waves = std::min<int64_t>(resident, (m + T - 1) / T);  // T tiles per wave
        side.main_blocks = (int)((waves + wpb - 1) / wpb);
        const int extra = q0 == 0 ? side_blocks : 0;
        // tiles of 3-4 KiB slices in this piece (the plan runs widest first)
        int64_t wide = 0;
        for (int s = 0; s < 8; ++s)
            if (4 - order[s] % 4 >= 3)
                wide += std::max<int64_t>(0, std::min<int64_t>(q0 + m, plan.cum[s + 1]) -
                                                 std::max<int64_t>(q0, plan.cum[s]));
        const bool sparse = DLS_FMA_SPARSE_DS > 1 && T == 1 && wide * 5 < waves * 4;
        if (sparse)
            hipLaunchKernelGGL(k_dequant_fma_stream<DLS_FMA_SPARSE_DS>, dim3((unsigned)(side.main_blocks + extra)),
                               dim3(kFmaBlock), 0, st, tiles, plan, a, (int)q0, (int)q0 + m, side);
        else
            hipLaunchKernelGGL(k_dequant_fma_stream<1>, dim3((unsigned)(side.main_blocks + extra)),
                               dim3(kFmaBlock), 0, st, tiles, plan, a, (int)q0, (int)q0 + m, side);
    }
    return check_launch("dls_dequant_fedavg_mode (fma)");
}

}  // namespace dls

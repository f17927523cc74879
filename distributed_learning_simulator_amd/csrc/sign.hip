// signSGD: 2-bit sign planes, majority vote and worker step, for gfx950.
//
// Wire format (include/dls_hip.h): per group of 64 parameters two uint64
// words [pos, neg], bit j = parameter 64g + j; NaN sets both bits.  A client's
// fp32 sign vector (4 B/param, workers/sign_sgd_worker.py:44) becomes 2 bits/param.
//
// Vote (servers/sign_sgd_server.py:12-21): counts = #pos - #neg per parameter,
// accumulated with bit-sliced ("vertical") counters: one 64-bit word per
// counter bit holds that bit of 64 parameters' counts, fed by a carry-save
// (Harley-Seal) adder tree, so 8 clients cost 7 CSAs (5 bitwise ops each)
// per plane word and no per-parameter unpacking; the counters are unpacked
// once at the end.  Exact in any order.
#include "dls_common.h"

namespace dls {
namespace {

constexpr int kBlock = 256;

__device__ __forceinline__ uint64_t spread16(uint64_t x) {
    // bit k of a 16-bit value -> bit 4k
    x &= 0xFFFFull;
    x = (x | (x << 24)) & 0x000000FF000000FFull;
    x = (x | (x << 12)) & 0x000F000F000F000Full;
    x = (x | (x << 6)) & 0x0303030303030303ull;
    x = (x | (x << 3)) & 0x1111111111111111ull;
    return x;
}

// One wavefront packs one 256-parameter tile: lane l loads parameters 4l..4l+3
// (16 B); one 64-lane ballot per component c gives bit l = parameter 4l + c.
// Output word m (parameters 64m..64m+63) takes bit j from ballot_{j&3} bit
// 16m + (j>>2): lanes 0..7 each build one word (m = lane/2, pos/neg = lane&1)
// with a 4-way bit interleave in VALU, in parallel.
__device__ __forceinline__ void pack_tile(f32x4 v, uint64_t *dst_tile, int32_t *nonternary,
                                          int valid_words = 8) {
    const int lane = __lane_id();
    uint64_t pos[4], neg[4];
    int nbad = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const float x = v[c];
        const bool nan = x != x;
        pos[c] = __ballot(x > 0.f || nan);
        neg[c] = __ballot(x < 0.f || nan);
        if (nonternary) nbad += __popcll(__ballot(!(x == 0.f || x == 1.f || x == -1.f || nan)));
    }
    if (nonternary && nbad && lane == 0) atomicAdd(nonternary, nbad);
    const int m = (lane >> 1) & 3;
    const bool isneg = lane & 1;
    uint64_t w = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) w |= spread16((isneg ? neg[c] : pos[c]) >> (16 * m)) << c;
    if (lane < valid_words) dst_tile[lane] = w;  // a tensor's last tile may end early
}

// The client-side pack (dls_sign_pack_f32) in the wire's own bit order: in step c
// (0..3) lane l holds parameter 64c + l of the tile (4-byte loads, each
// wave-instruction 256 contiguous bytes), so the 64-lane ballot of step c IS the
// tile's word c (bit j = parameter 64c + j) and no bit interleave is needed:
// 2 compares per 64 parameters and plane, plus the 8 words' store.  (pack_tile's
// 16-byte loads need a 4-way bit interleave of the ballots in VALU: 31 VALU
// instructions per 64 parameters, issue-bound at 0.757 of HBM, profiles/r05_pmc_summary.txt.)
__device__ __forceinline__ void pack_tile_nat(const float (&x)[4], uint64_t *dst_tile, int32_t *nonternary) {
    const int lane = __lane_id();
    uint64_t pos[4], neg[4];
    int nbad = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const bool nan = x[c] != x[c];
        pos[c] = __ballot(x[c] > 0.f || nan);
        neg[c] = __ballot(x[c] < 0.f || nan);
        if (nonternary) nbad += __popcll(__ballot(!(x[c] == 0.f || x[c] == 1.f || x[c] == -1.f || nan)));
    }
    if (nonternary && nbad && lane == 0) atomicAdd(nonternary, nbad);
    // lane 2c + q stores word [pos_c, neg_c][q]
    const int m = (lane >> 1) & 3;
    const bool isneg = lane & 1;
    uint64_t w = isneg ? neg[0] : pos[0];
#pragma unroll
    for (int c = 1; c < 4; ++c) w = m == c ? (isneg ? neg[c] : pos[c]) : w;
    if (lane < 8) dst_tile[lane] = w;
}

// grid: x = blocks of 4 waves x kPackTPW tiles, y = client.  Each wave issues
// the loads of its kPackTPW tiles before packing any (memory-level parallelism).
// (2, 8, 16 tiles per wave: 0.133, 0.125, 0.132 vs 0.122 ms for 16 ResNet-18 clients,
// profiles/r05_pack_tpw.txt)
constexpr int kPackTPW = 4;

__global__ __launch_bounds__(kBlock) void k_sign_pack(const float *__restrict__ X, int64_t ldx,
                                                      int64_t P, uint64_t *__restrict__ planes,
                                                      int64_t ldp, int64_t ntiles,
                                                      int32_t *nonternary) {
    const int64_t t0 = ((int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)) * kPackTPW;
    if (t0 >= ntiles) return;  // wave-uniform
    const int64_t k = blockIdx.y;
    const int lane = __lane_id();
    const float *row = X + k * ldx;
    float v[kPackTPW][4];
#pragma unroll
    for (int i = 0; i < kPackTPW; ++i) {
        const int64_t e0 = (t0 + i) * 256 + lane;
        if ((t0 + i + 1) * 256 <= P) {  // wave-uniform: a whole tile
#pragma unroll
            for (int c = 0; c < 4; ++c) v[i][c] = __builtin_nontemporal_load(row + e0 + 64 * c);
        } else {
#pragma unroll
            for (int c = 0; c < 4; ++c) v[i][c] = e0 + 64 * c < P ? row[e0 + 64 * c] : 0.f;
        }
    }
#pragma unroll
    for (int i = 0; i < kPackTPW; ++i)
        if (t0 + i < ntiles) pack_tile_nat(v[i], planes + k * ldp + (t0 + i) * 8, nonternary);
}

// ---------------------------------------------------------------- vote
// Carry-save (Harley-Seal) accumulation of 8 one-bit planes: ones/twos/fours
// are carry-save partial counts, every 8 inputs emit an "eights" word that
// ripples into the CB-bit counter c (in units of 8).  7 CSAs of 5 ops per 8
// clients instead of 8 ripple increments of 2*B ops.
__device__ __forceinline__ void csa(uint64_t &h, uint64_t &l, uint64_t a, uint64_t b, uint64_t c) {
    const uint64_t u = a ^ b;
    h = (a & b) | (u & c);
    l = u ^ c;
}

template <int CB>
struct HSCounter {
    // carry-save partial counts (ones/twos/fours) + CB-bit counter of eights
    uint64_t ones = 0, twos = 0, fours = 0;
    uint64_t c[CB];
    __device__ __forceinline__ HSCounter() {
#pragma unroll
        for (int b = 0; b < CB; ++b) c[b] = 0;
    }
    __device__ __forceinline__ void add8(const uint64_t (&x)[8]) {
        uint64_t twosA, twosB, foursA, foursB, eights;
        csa(twosA, ones, ones, x[0], x[1]);
        csa(twosB, ones, ones, x[2], x[3]);
        csa(foursA, twos, twos, twosA, twosB);
        csa(twosA, ones, ones, x[4], x[5]);
        csa(twosB, ones, ones, x[6], x[7]);
        csa(foursB, twos, twos, twosA, twosB);
        csa(eights, fours, fours, foursA, foursB);
        ripple(eights);  // c += eights
    }
    __device__ __forceinline__ void ripple(uint64_t eights) {
#pragma unroll
        for (int b = 0; b < CB; ++b) {
            const uint64_t t = c[b] & eights;
            c[b] ^= eights;
            eights = t;
        }
    }
    __device__ __forceinline__ int count(int j) const {
        int v = (int)((ones >> j) & 1u) | ((int)((twos >> j) & 1u) << 1) |
                ((int)((fours >> j) & 1u) << 2);
#pragma unroll
        for (int b = 0; b < CB; ++b) v |= (int)((c[b] >> j) & 1u) << (3 + b);
        return v;
    }
};

// Vote kernel: wave w of nw owns the contiguous range of groups (64 parameters
// each) [w VG / nw, (w+1) VG / nw) (VG = vote groups; sizes differ by at most
// one); lane l owns groups wlo + l + 64 q, q < G = ceil(range / 64),
// and walks all K clients: one 16-byte [pos, neg] load per client and group,
// batches of 8 clients through the carry-save counters.  The grid is one
// generation of resident waves sweeping the client rows in step.  On large
// models nw = kVoteWPC x CUs, a whole number of waves per CU: every CU then
// streams the same number of bytes — with 256 groups per wave (682 waves on
// ResNet-18) a third of the CUs held 3 waves and the rest 2.  Epilogue: the counters are already
// bit-sliced (bit b of parameter j's count = bit j of word b), so the fp32 sign
// needs no unpacking: a bit-sliced comparison of the pos / neg counters gives
// two words (gt, lt) per group.  Those words (or, when the int32 counts are
// wanted, the 2B counter words) go through the wave's LDS slice and the wave
// writes its outputs coalesced, a 16-lane group per 64-parameter group,
// instead of 64 lanes each scattering 256 bytes.
constexpr int kVoteWPBMax = 4;  // waves per block
#ifndef DLS_VOTE_WPC
#define DLS_VOTE_WPC 4
#endif
#ifndef DLS_VOTE_WPB
#define DLS_VOTE_WPB 4
#endif
constexpr int kVoteWPC = DLS_VOTE_WPC;  // waves per CU on large models (0: 256 groups per wave)
constexpr int kVoteWPB = DLS_VOTE_WPB;
static_assert(kVoteWPB >= 1 && kVoteWPB <= kVoteWPBMax, "DLS_VOTE_WPB");
constexpr int kVoteG = 4;    // widest G (registers: single-buffered 8-client batches)
constexpr int kVoteDbG = 1;  // widest G whose 8-client batches are double-buffered

// LDS is per wave and the epilogue trip counts differ between the waves of a
// block, so the epilogue synchronises the wave only (LDS ops of one wave
// execute in order; the fences keep the compiler from moving them).
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int CB, bool ROWS, int G>
__device__ __forceinline__ void wave_counts(const uint64_t *__restrict__ planes, int64_t ldp,
                                            const int32_t *__restrict__ rows, int K, int64_t g,
                                            int64_t gend, HSCounter<CB> (&cp)[G],
                                            HSCounter<CB> (&cn)[G], uint64_t (&nan)[G]) {
    // lane's groups: g + 64 q, q < G (each load instruction covers up to 1 KB of
    // a row); groups past the wave's range (or the model) re-read group g (in
    // bounds) and are never written
    const u64x2 *base = reinterpret_cast<const u64x2 *>(planes) + g;
    int qoff[G];
#pragma unroll
    for (int q = 0; q < G; ++q) qoff[q] = g + 64 * q < gend ? 64 * q : 0;
    const int64_t ldp2 = ldp / 2;
    constexpr int B8 = 8;
    auto row = [&](int k) -> int64_t { return ROWS ? (int64_t)rows[k] : (int64_t)k; };
    auto load8 = [&](int j, u64x2 (&w8)[G][B8]) {
#pragma unroll
        for (int u = 0; u < B8; ++u) {
            const u64x2 *r = base + row(j + u) * ldp2;
#pragma unroll
            for (int q = 0; q < G; ++q) w8[q][u] = __builtin_nontemporal_load(r + qoff[q]);
        }
    };
    auto consume8 = [&](const u64x2 (&w8)[G][B8]) {
#pragma unroll
        for (int q = 0; q < G; ++q) {
            uint64_t xp[B8], xn[B8];
#pragma unroll
            for (int u = 0; u < B8; ++u) {
                xp[u] = w8[q][u][0];
                xn[u] = w8[q][u][1];
                nan[q] |= xp[u] & xn[u];
            }
            cp[q].add8(xp);
            cn[q].add8(xn);
        }
    };
    // batches of 8 clients, double-buffered; loads inside the steady-state loop
    // are unconditional so every consume waits with an exact vmcnt
    const int nb = K / B8;
    if (G > kVoteDbG) {  // one batch (8 clients x G KB) in flight per wave: register budget
        for (int b = 0; b < nb; ++b) {
            u64x2 wa[G][B8];
            load8(b * B8, wa);
            // all 8 x G loads issue before the batch is reduced (without this the
            // scheduler sinks them next to their uses once the reduction is short)
            __builtin_amdgcn_sched_barrier(0);
            consume8(wa);
        }
    } else if (nb > 0) {
        u64x2 wa[G][B8], wb[G][B8];
        load8(0, wa);
        int b = 0;
        for (; b + 2 < nb; b += 2) {
            load8((b + 1) * B8, wb);
            consume8(wa);
            load8((b + 2) * B8, wa);
            consume8(wb);
        }
        if (b + 1 < nb) {
            load8((b + 1) * B8, wb);
            consume8(wa);
            consume8(wb);
        } else {
            consume8(wa);
        }
    }
    if (nb * B8 < K) {  // tail: missing clients count as zero planes
        u64x2 w8[G][B8];
#pragma unroll
        for (int u = 0; u < B8; ++u) {
            const int k = nb * B8 + u;
#pragma unroll
            for (int q = 0; q < G; ++q)
                w8[q][u] = k < K ? __builtin_nontemporal_load(base + row(k) * ldp2 + qoff[q]) : u64x2{0, 0};
        }
        consume8(w8);
    }
}

// Bit-sliced B-bit counter from the carry-save form: ones / twos / fours have
// weights 1, 2, 4 and the CB-bit counter counts eights.
template <int CB>
__device__ __forceinline__ void sliced(const HSCounter<CB> &h, uint64_t (&x)[CB + 3]) {
    x[0] = h.ones;
    x[1] = h.twos;
    x[2] = h.fours;
#pragma unroll
    for (int b = 0; b < CB; ++b) x[3 + b] = h.c[b];
}

template <int CB, bool COUNTS, int G>
__global__ __launch_bounds__(64 * kVoteWPBMax) void k_sign_vote(
    const uint64_t *__restrict__ planes, int64_t ldp, const int32_t *__restrict__ rows, int K,
    int64_t P, int64_t ngroups, int32_t *__restrict__ counts, float *__restrict__ sign_out,
    uint64_t *__restrict__ vote_planes, int64_t vote_groups, int64_t nwaves) {
    constexpr int B = CB + 3;
    constexpr int NW = COUNTS ? 2 * B + 1 : 3;  // words per group through LDS
    extern __shared__ uint64_t xws[];  // [waves per block][NW][64] (launch: vote_lds)
    uint64_t(*xw)[64] = reinterpret_cast<uint64_t(*)[64]>(xws + (threadIdx.x >> 6) * NW * 64);
    const int lane = __lane_id();
    // the wave's group range [wlo, whi); groups >= ngroups are the zero padding of
    // the last 256-parameter tile (vote 0)
    const int64_t wave = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (wave >= nwaves) return;  // wave-uniform
    // nwaves near-equal ranges (sizes differ by at most one group; with G > 1, by
    // up to 8: every range starts on a multiple of 8 groups = 128 bytes, so on rows
    // whose pitch is a multiple of 128 bytes (_native.sign_row_pitch) no line is
    // fetched by two waves: HBM reads 1.028 -> 1.016 x the algorithmic bytes even
    // with the 64-byte pitch, -1.2 % time, profiles/r06_sign_vote_pmc.txt; the host
    // sizes G for ranges up to 7 groups longer)
    int64_t wlo = wave * vote_groups / nwaves;
    int64_t whi = (wave + 1) * vote_groups / nwaves;
    if (G > 1) {
        wlo &= ~(int64_t)7;
        whi = wave + 1 == nwaves ? vote_groups : whi & ~(int64_t)7;
    }
    const int64_t gend = min(whi, ngroups);
    HSCounter<CB> cpa[G], cna[G];
    uint64_t nana[G];
#pragma unroll
    for (int q = 0; q < G; ++q) nana[q] = 0;
    if (wlo + lane < gend) {
        if (rows)
            wave_counts<CB, true, G>(planes, ldp, rows, K, wlo + lane, gend, cpa, cna, nana);
        else
            wave_counts<CB, false, G>(planes, ldp, rows, K, wlo + lane, gend, cpa, cna, nana);
    }
#pragma unroll
    for (int q = 0; q < G; ++q) {
        const int64_t g0 = wlo + 64 * q;
        if (g0 >= whi) break;  // wave-uniform
        const int64_t g = g0 + lane;
        const HSCounter<CB> &cp = cpa[q], &cn = cna[q];
        const bool live = g < gend;  // padding groups (q > 0 lanes re-read group g) vote 0
        const uint64_t nan = live ? nana[q] : 0;
        uint64_t xp[B], xn[B];
        sliced<CB>(cp, xp);
        sliced<CB>(cn, xn);
    #pragma unroll
        for (int b = 0; b < B; ++b) {
            xp[b] = live ? xp[b] : 0;
            xn[b] = live ? xn[b] : 0;
        }
        // bit-sliced compare, MSB first: gt = pos > neg, lt = pos < neg
        uint64_t gt = 0, lt = 0, eq = ~0ull;
    #pragma unroll
        for (int b = B - 1; b >= 0; --b) {
            gt |= eq & xp[b] & ~xn[b];
            lt |= eq & ~xp[b] & xn[b];
            eq &= ~(xp[b] ^ xn[b]);
        }
        // the vote in the wire format (16 coalesced bytes per lane); NaN-poisoned
        // and tied parameters vote 0 (neither bit)
        if (vote_planes && g < whi)
            reinterpret_cast<u64x2 *>(vote_planes)[g] = u64x2{gt & ~nan, lt & ~nan};
        if (COUNTS) {
    #pragma unroll
            for (int b = 0; b < B; ++b) {
                xw[b][lane] = xp[b];
                xw[B + b][lane] = xn[b];
            }
            xw[NW - 1][lane] = nan;
        } else {
            xw[0][lane] = gt;
            xw[1][lane] = lt;
            xw[2][lane] = nan;
        }
        if (!sign_out && !COUNTS) continue;  // wave-uniform: the packed vote was all
        wave_sync();
        // a 16-lane group writes one group's 64 parameters, 4 per lane
        const int jb = 4 * (lane & 15);
    #pragma unroll 4
        for (int it = 0; it < 16; ++it) {
            const int gl = it * 4 + (lane >> 4);
            const int64_t e = (g0 + gl) * 64 + jb;
            if (g0 + gl >= whi || e >= P) continue;  // P % 4 == 0: all four or none
            f32x4 s4;
            if (COUNTS) {
                int pc[4] = {0, 0, 0, 0}, nc[4] = {0, 0, 0, 0};
    #pragma unroll
                for (int b = 0; b < B; ++b) {
                    const uint32_t pw = (uint32_t)(xw[b][gl] >> jb);
                    const uint32_t nw = (uint32_t)(xw[B + b][gl] >> jb);
    #pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        pc[t] |= (int)((pw >> t) & 1u) << b;
                        nc[t] |= (int)((nw >> t) & 1u) << b;
                    }
                }
                const uint32_t nn = (uint32_t)(xw[NW - 1][gl] >> jb);
                int32_t c4[4];
    #pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const bool poisoned = (nn >> t) & 1u;
                    const int c = pc[t] - nc[t];
                    c4[t] = poisoned ? c + DLS_SIGN_NAN_MARK : c;
                    s4[t] = poisoned ? 0.f : (c > 0 ? 1.f : (c < 0 ? -1.f : 0.f));
                }
                *reinterpret_cast<int4 *>(counts + e) = make_int4(c4[0], c4[1], c4[2], c4[3]);
                if (!sign_out) continue;
            } else {
                const uint32_t gt = (uint32_t)(xw[0][gl] >> jb);
                const uint32_t lt = (uint32_t)(xw[1][gl] >> jb);
                const uint32_t nn = (uint32_t)(xw[2][gl] >> jb);
    #pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const uint32_t m = 1u << t;
                    s4[t] = (nn & m) ? 0.f : ((gt & m) ? 1.f : ((lt & m) ? -1.f : 0.f));
                }
            }
            if (sign_out) *reinterpret_cast<f32x4 *>(sign_out + e) = s4;
        }
        wave_sync();  // xw is rewritten for the next q
    }
}

__device__ __forceinline__ float vote_of(int32_t c) {
    if (c >= DLS_SIGN_NAN_MARK / 2) return 0.f;
    return c > 0 ? 1.f : (c < 0 ? -1.f : 0.f);
}

// counts -> fp32 sign + optional packed vote (one wave per 256-param tile).
__global__ __launch_bounds__(kBlock) void k_sign_from_counts(const int32_t *__restrict__ counts,
                                                             int64_t P, int64_t ntiles,
                                                             float *__restrict__ sign_out,
                                                             uint64_t *__restrict__ vote_planes) {
    const int64_t tile = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    if (tile >= ntiles) return;
    const int lane = __lane_id();
    const int64_t e = tile * 256 + 4 * lane;
    f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
    if (e + 4 <= P) {
        const int4 c = *reinterpret_cast<const int4 *>(counts + e);
        v = f32x4{vote_of(c.x), vote_of(c.y), vote_of(c.z), vote_of(c.w)};
        if (sign_out) *reinterpret_cast<f32x4 *>(sign_out + e) = v;
    } else {
        for (int t = 0; t < 4; ++t)
            if (e + t < P) {
                v[t] = vote_of(counts[e + t]);
                if (sign_out) sign_out[e + t] = v[t];
            }
    }
    if (vote_planes) pack_tile(v, vote_planes + tile * 8, nullptr);
}

// --------------------------------------------------------------- worker
// workers/sign_sgd_worker.py:32-44 fused: momentum/dampening/nesterov, sign,
// pack.  buf.mul_(m).add_(g, alpha=a) == fma(g, a, buf*m); g.add(buf, alpha=m)
// == fma(buf, m, g) (torch CPU semantics, pinned by the golden vectors).
__global__ __launch_bounds__(kBlock) void k_sign_sgd_direction(
    const float *__restrict__ grad, float *__restrict__ buf, int64_t P, int64_t ntiles,
    float momentum, float a, int nesterov, int first, uint64_t *__restrict__ planes,
    float *__restrict__ sign_out) {
    const int64_t tile = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    if (tile >= ntiles) return;
    const int lane = __lane_id();
    const int64_t e = tile * 256 + 4 * lane;
    f32x4 g = f32x4{0.f, 0.f, 0.f, 0.f}, b = g;
    const bool full = e + 4 <= P;
    if (full) {
        g = *reinterpret_cast<const f32x4 *>(grad + e);
        if (momentum != 0.f && !first) b = *reinterpret_cast<const f32x4 *>(buf + e);
    } else {
        for (int t = 0; t < 4; ++t)
            if (e + t < P) {
                g[t] = grad[e + t];
                if (momentum != 0.f && !first) b[t] = buf[e + t];
            }
    }
    f32x4 d = g;
    if (momentum != 0.f) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            b[t] = first ? g[t] : __builtin_fmaf(g[t], a, b[t] * momentum);
            d[t] = nesterov ? __builtin_fmaf(b[t], momentum, g[t]) : b[t];
        }
        if (full) {
            *reinterpret_cast<f32x4 *>(buf + e) = b;
        } else {
            for (int t = 0; t < 4; ++t)
                if (e + t < P) buf[e + t] = b[t];
        }
    }
    f32x4 s;
#pragma unroll
    for (int t = 0; t < 4; ++t) s[t] = d[t] > 0.f ? 1.f : (d[t] < 0.f ? -1.f : 0.f);  // nan -> 0
    if (sign_out) {
        if (full) {
            *reinterpret_cast<f32x4 *>(sign_out + e) = s;
        } else {
            for (int t = 0; t < 4; ++t)
                if (e + t < P) sign_out[e + t] = s[t];
        }
    }
    if (!full) {
        for (int t = 0; t < 4; ++t)
            if (e + t >= P) s[t] = 0.f;
    }
    const int64_t words_left = 2 * ((P + 63) / 64) - tile * 8;
    pack_tile(s, planes + tile * 8, nullptr, words_left < 8 ? (int)words_left : 8);
}

// workers/sign_sgd_worker.py:48-57: d = vote (+ fma(p, wd, vote)); p = fma(d, -lr, p).
__global__ __launch_bounds__(kBlock) void k_sign_sgd_apply(float *__restrict__ param,
                                                           const uint64_t *__restrict__ vote,
                                                           int64_t P, float neg_lr, float wd) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;  // 4 params each
    const int64_t e = i * 4;
    if (e >= P) return;
    const int64_t g = e >> 6;
    const int sh = (int)(e & 63);
    const uint64_t pw = vote[2 * g], nw = vote[2 * g + 1];
    for (int t = 0; t < 4 && e + t < P; ++t) {
        const int pb = (int)((pw >> (sh + t)) & 1u), nb = (int)((nw >> (sh + t)) & 1u);
        float d = (pb && !nb) ? 1.f : ((nb && !pb) ? -1.f : 0.f);
        float p = param[e + t];
        if (wd != 0.f) d = __builtin_fmaf(p, wd, d);
        param[e + t] = __builtin_fmaf(d, neg_lr, p);
    }
}

template <int CB>
int launch_vote(const uint64_t *planes, int64_t ldp, const int32_t *rows, int K, int64_t P,
                int32_t *counts, float *sign_out, uint64_t *vote_planes, hipStream_t st) {
    const int64_t ngroups = (P + 63) / 64;
    const int64_t vote_groups = DLS_SIGN_WORDS(P) / 2;  // whole 256-parameter tiles
    // Large models: kVoteWPC waves per CU, each a contiguous range of R groups,
    // 2-4 groups per lane (each wave streams R x 16 B of every client row:
    // multi-KB pieces measured 12 % faster than 1 KB at P = 11.2M).  Small
    // models: R = 64, 1 group per lane, double-buffered batches.
    int64_t nwaves = (vote_groups + 63) / 64;
    int G = 1, wpb = 1;
    if (CB <= 12) {
        if (kVoteWPC > 0) {
            // exactly kVoteWPC waves per CU, near-equal ranges of up to 64 G groups
            int64_t waves = (int64_t)kVoteWPC * device_cus();
            int64_t r = (vote_groups + waves - 1) / waves + 7;  // + the range alignment
            if (r > 64 * kVoteG) {
                // models past 64 kVoteG groups per wave (P > ~16.7M on 256 CUs, e.g.
                // VGG-16): a multiple of kVoteWPC waves per CU, so that every wave
                // keeps the wide layout (G = kVoteG at most) instead of G = 1
                waves *= (r + 64 * kVoteG - 1) / (64 * kVoteG);
                r = (vote_groups + waves - 1) / waves + 7;
            }
            if (r > 64) {
                nwaves = waves;
                G = (int)((r + 63) / 64);
                wpb = kVoteWPB;
            }
        } else if ((vote_groups + 64 * kVoteG - 1) / (64 * kVoteG) >= 512) {
            // the round-3 form: 256 groups per wave, one wave per block
            nwaves = (vote_groups + 64 * kVoteG - 1) / (64 * kVoteG);
            G = kVoteG;
        }
    }
    const dim3 grid((unsigned)((nwaves + wpb - 1) / wpb));
    const size_t lds = (size_t)wpb * (counts ? 2 * (CB + 3) + 1 : 3) * 64 * sizeof(uint64_t);
#define DLS_VOTE_LAUNCH(C_, G_)                                                                  \
    hipLaunchKernelGGL((k_sign_vote<CB, C_, G_>), grid, dim3(64 * wpb), lds, st, planes, ldp, rows, \
                       K, P, ngroups, counts, sign_out, vote_planes, vote_groups, nwaves)
#define DLS_VOTE_BY_G(C_)                     \
    switch (G) {                              \
        case 1: DLS_VOTE_LAUNCH(C_, 1); break; \
        case 2: DLS_VOTE_LAUNCH(C_, 2); break; \
        case 3: DLS_VOTE_LAUNCH(C_, 3); break; \
        default: DLS_VOTE_LAUNCH(C_, 4); break; \
    }
    if constexpr (CB > 12) {  // wide counters: 1 group per lane only (registers)
        if (counts) DLS_VOTE_LAUNCH(true, 1);
        else DLS_VOTE_LAUNCH(false, 1);
    } else {
        if (counts) {
            DLS_VOTE_BY_G(true)
        } else {
            DLS_VOTE_BY_G(false)
        }
    }
#undef DLS_VOTE_BY_G
#undef DLS_VOTE_LAUNCH
    return check_launch("dls_sign_vote");
}

int vote_dispatch(const uint64_t *planes, int64_t ldp, const int32_t *rows, int32_t K, int64_t P,
                  int32_t *counts, float *sign_out, uint64_t *vote_planes, hipStream_t st) {
    // counts reach 8*c + 7 with c <= ceil(K/8) < 2^CB (fewer bits = fewer ops/registers)
    const int64_t c_max = (K + 7) / 8;
    if (c_max < (1 << 2)) return launch_vote<2>(planes, ldp, rows, K, P, counts, sign_out, vote_planes, st);
    if (c_max < (1 << 4)) return launch_vote<4>(planes, ldp, rows, K, P, counts, sign_out, vote_planes, st);
    if (c_max < (1 << 6)) return launch_vote<6>(planes, ldp, rows, K, P, counts, sign_out, vote_planes, st);
    if (c_max < (1 << 8)) return launch_vote<8>(planes, ldp, rows, K, P, counts, sign_out, vote_planes, st);
    if (c_max < (1 << 12)) return launch_vote<12>(planes, ldp, rows, K, P, counts, sign_out, vote_planes, st);
    if (K < (1 << 20)) return launch_vote<16>(planes, ldp, rows, K, P, counts, sign_out, vote_planes, st);
    set_error("dls_sign_vote: K=%d exceeds 2^20-1 clients", K);
    return DLS_EINVAL;
}

}  // namespace
}  // namespace dls

using namespace dls;

extern "C" int dls_sign_pack_f32(const float *X, int64_t ldx, int32_t K, int64_t P,
                                 uint64_t *planes, int64_t ldp, int32_t *nonternary,
                                 dls_stream_t stream) {
    DLS_REQUIRE(X && planes, DLS_EINVAL, "dls_sign_pack_f32: null pointer");
    DLS_REQUIRE(K > 0 && P > 0 && K < 65536, DLS_EINVAL, "dls_sign_pack_f32: K=%d P=%lld", K,
                (long long)P);
    DLS_REQUIRE(ldx >= P && ldp >= DLS_SIGN_WORDS(P) && ldx % 4 == 0 && aligned16(X), DLS_ELAYOUT,
                "dls_sign_pack_f32: ldx=%lld (multiple of 4, >= P) ldp=%lld (>= %lld)",
                (long long)ldx, (long long)ldp, (long long)DLS_SIGN_WORDS(P));
    const int64_t ntiles = (P + 255) / 256;
    const int64_t per_block = (kBlock / 64) * kPackTPW;
    const dim3 grid((unsigned)((ntiles + per_block - 1) / per_block), (unsigned)K);
    hipLaunchKernelGGL(k_sign_pack, grid, dim3(kBlock), 0, as_stream(stream), X, ldx, P, planes,
                       ldp, ntiles, nonternary);
    return check_launch("dls_sign_pack_f32");
}

extern "C" int dls_sign_vote_count(const uint64_t *planes, int64_t ldp, const int32_t *rows,
                                   int32_t K, int64_t P, int32_t *counts, dls_stream_t stream) {
    DLS_REQUIRE(planes && counts, DLS_EINVAL, "dls_sign_vote_count: null pointer");
    DLS_REQUIRE(K > 0 && P > 0, DLS_EINVAL, "dls_sign_vote_count: K=%d P=%lld", K, (long long)P);
    DLS_REQUIRE(ldp >= DLS_SIGN_WORDS(P) && ldp % 2 == 0 && aligned16(planes) && P % 4 == 0 &&
                    aligned16(counts),
                DLS_ELAYOUT, "dls_sign_vote_count: layout (ldp=%lld, P=%lld)", (long long)ldp,
                (long long)P);
    return vote_dispatch(planes, ldp, rows, K, P, counts, nullptr, nullptr, as_stream(stream));
}

extern "C" int dls_sign_vote(const uint64_t *planes, int64_t ldp, const int32_t *rows, int32_t K,
                             int64_t P, int32_t *counts, float *sign_out, uint64_t *vote_planes,
                             dls_stream_t stream) {
    DLS_REQUIRE(planes && (sign_out || vote_planes || counts), DLS_EINVAL,
                "dls_sign_vote: null pointer");
    DLS_REQUIRE(K > 0 && P > 0, DLS_EINVAL, "dls_sign_vote: K=%d P=%lld", K, (long long)P);
    DLS_REQUIRE(ldp >= DLS_SIGN_WORDS(P) && ldp % 2 == 0 && aligned16(planes) && P % 4 == 0 &&
                    (!sign_out || aligned16(sign_out)) && (!counts || aligned16(counts)) &&
                    (!vote_planes || aligned16(vote_planes)),
                DLS_ELAYOUT, "dls_sign_vote: layout (ldp=%lld, P=%lld)", (long long)ldp,
                (long long)P);
    return vote_dispatch(planes, ldp, rows, K, P, counts, sign_out, vote_planes,
                         as_stream(stream));
}

extern "C" int dls_sign_from_counts(const int32_t *counts, int64_t P, float *sign_out,
                                    uint64_t *vote_planes, dls_stream_t stream) {
    DLS_REQUIRE(counts && (sign_out || vote_planes), DLS_EINVAL,
                "dls_sign_from_counts: null pointer");
    DLS_REQUIRE(P > 0 && P % 4 == 0 && aligned16(counts) && (!sign_out || aligned16(sign_out)),
                DLS_ELAYOUT, "dls_sign_from_counts: P=%lld must be a multiple of 4", (long long)P);
    const int64_t ntiles = (P + 255) / 256;
    hipLaunchKernelGGL(k_sign_from_counts, dim3((unsigned)((ntiles + 3) / 4)), dim3(kBlock), 0,
                       as_stream(stream), counts, P, ntiles, sign_out, vote_planes);
    return check_launch("dls_sign_from_counts");
}

extern "C" int dls_sign_sgd_direction(const float *grad, float *buf, int64_t P, float momentum,
                                      float one_minus_dampening, int32_t nesterov, int32_t first,
                                      uint64_t *planes, float *sign_out, dls_stream_t stream) {
    DLS_REQUIRE(grad && planes && (momentum == 0.f || buf), DLS_EINVAL,
                "dls_sign_sgd_direction: null pointer");
    DLS_REQUIRE(P > 0, DLS_EINVAL, "dls_sign_sgd_direction: P=%lld", (long long)P);
    DLS_REQUIRE(aligned16(grad) && (!buf || aligned16(buf)) && (!sign_out || aligned16(sign_out)),
                DLS_ELAYOUT, "dls_sign_sgd_direction: 16-byte alignment");
    const int64_t ntiles = (P + 255) / 256;
    hipLaunchKernelGGL(k_sign_sgd_direction, dim3((unsigned)((ntiles + 3) / 4)), dim3(kBlock), 0,
                       as_stream(stream), grad, buf, P, ntiles, momentum, one_minus_dampening,
                       (int)nesterov, (int)first, planes, sign_out);
    return check_launch("dls_sign_sgd_direction");
}

extern "C" int dls_sign_sgd_apply(float *param, const uint64_t *vote_planes, int64_t P,
                                  float neg_lr, float weight_decay, dls_stream_t stream) {
    DLS_REQUIRE(param && vote_planes, DLS_EINVAL, "dls_sign_sgd_apply: null pointer");
    DLS_REQUIRE(P > 0, DLS_EINVAL, "dls_sign_sgd_apply: P=%lld", (long long)P);
    const int64_t threads = (P + 3) / 4;
    hipLaunchKernelGGL(k_sign_sgd_apply, dim3((unsigned)((threads + kBlock - 1) / kBlock)),
                       dim3(kBlock), 0, as_stream(stream), param, vote_planes, P, neg_lr,
                       weight_decay);
    return check_launch("dls_sign_sgd_apply");
}

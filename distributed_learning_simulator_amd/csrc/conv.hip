// Deterministic convolutions for the utility evaluation (SURVEY.md §8 row a-3:
// FedServer.get_metric, servers/fed_server.py:26-32 — the Shapley servers'
// v(S) = top-1 accuracy of the subset model on the test set).
//
// Why our own: v(S) must be a function of S (GTG's truncation tests and the
// rankings compare utilities, and on several ranks a coalition's utility must
// not depend on which rank evaluated it).  MIOpen's fast convolutions are not
// run-to-run reproducible on this stack, and its deterministic ones are NCHW
// Winograd kernels (the Inferencer's round-4 path, ~7.4 evals/s).  These
// kernels are reproducible by construction: every output element is reduced by
// one wave in one fixed order (no split-K, no atomics, no algorithm search).
//
// Arithmetic: fp32 activations and weights, each carried as a pair of bf16
// (hi = rne(x), lo = rne(x - hi): 16 significant bits), and every product taken
// as hi*hi + hi*lo + lo*hi on v_mfma_f32_32x32x16_bf16 with fp32 accumulation
// ("bf16x3"): a relative error per product of ~2^-16 against fp32's 2^-24, at 3
// bf16 MFMAs = 3/16 of the time of the f32-input MFMA (which runs at the fp32
// vector rate, 157 TF: a ResNet-18 eval of 10k CIFAR images is 11.1 TFLOP,
// >= 70 ms on it at peak).  The logits differ from torch's fp32 forward in the
// low bits; top-1 agrees except where the top two logits are within that error
// (tests/test_gpu_conv.py).
//
// Layouts (HBM):
//   activations  "split NHWC": uint16 [B][H][W][2C], per pixel C bf16 hi then C
//                bf16 lo (4 B per element, the size of the fp32 tensor);
//   weights      uint16 [Cout][2K], per output channel K hi then K lo,
//                k = (ky * KW + kx) * C + ci (C = the input's padded channels).
// Implicit GEMM, D[co][pixel] = sum_k W[co][k] X[k][pixel]: A = weights (rows =
// output channels), B = the input pixels' channel runs under a tap (zero outside
// the image), so a lane's 16-element MFMA fragment is one 16-B piece of a
// pixel's hi (or lo) channel run.  Each wave owns a 64 x 64 (channel x pixel)
// output tile = 2 x 2 MFMA tiles; operands are staged in chunks of 32 channels
// through LDS (register staging, rows padded by 16 B: conflict-free
// ds_read_b128 fragments).  Kernels:
//   k_conv3x3_pipe16  3x3 stride-1 convolutions (the default): k_conv3x3_pipe's
//                   pipeline on v_mfma_f32_16x16x32_bf16 (4 x 4 tiles of 16 x 16
//                   per wave; -0.9 % per forward, profiles/r06_forward_mf16_ab.txt);
//   k_conv3x3_pipe  3x3 stride-1 convolutions: the block's pixels are whole
//                   output rows, so its input is ONE halo tile staged once per
//                   channel chunk and read by all 9 taps at shifted rows; every
//                   operand staged by LDS-DMA into XOR-swizzled rows and kept in
//                   flight across the barriers (a 3-slot weight ring, 1 or 2
//                   halo buffers);
//   k_conv3x3_halo  the same tiling register-staged (shapes whose halo tile the
//                   pipeline's LDS budget does not fit; none of ResNet-18's);
//   k_conv3x3s2_phase  3x3 stride-2 convolutions as four stride-1 ones over
//                   the input's row / column parity images, on the same
//                   pipeline (each input pixel staged once per channel chunk);
//   k_conv_bf16x3   anything else (1x1, sizes the tilings do not fit): every
//                   (tap, chunk) gathers its B tile;
//   k_conv_stem     the 3-channel 3x3 stem with its im2col fused (a block walks 2
//                   pixel tiles; its epilogue passes split the pixels).
// Every launch walks its XCDs' tile runs forwards or backwards — the opposite of
// the direction its input was written in (conv_walk_direction), so a layer starts
// on what the previous one wrote last; no output depends on the order.
// The epilogue goes through LDS: the raw tile is transposed to [pixel][channel]
// and each thread applies the eval batch norm with the batch-norm library's
// arithmetic (infer.hip, k_bn_act_exact: fma(w, (x - mean) * iv, b)), the
// residual add and the ReLU to 8 channels of a pixel and stores 16-B hi and lo
// pieces — the next convolution's operand — so a ResNet block is 2 (or 3)
// launches and no separate batch-norm pass.  Measured per layer and variant:
// profiles/r05_conv_probe.txt, DESIGN.md §4.
#include "dls_common.h"

#include <mutex>

#ifndef DLS_CONV_GENERIC_ONLY
#define DLS_CONV_GENERIC_ONLY 0
#endif
#ifndef DLS_CONV_PHASE  // probe knob: 0 = the generic kernel for 3x3 stride-2 shapes
#define DLS_CONV_PHASE 1
#endif
#ifndef DLS_STEM_WINDOW  // probe knob: 0 = the stem's 27 terms gathered from global memory
#define DLS_STEM_WINDOW 1
#endif
#ifndef DLS_CONV_MF16  // probe knob: 0 = the 3x3 stride-1 pipeline on 32x32x16 MFMAs (k_conv3x3_pipe)
#define DLS_CONV_MF16 1
#endif
#ifndef DLS_STEM_TILES  // probe knob: pixel tiles per block of the CIFAR stem (k_conv_stem, XT)
#define DLS_STEM_TILES 2
#endif
#ifndef DLS_CONV_SERPENTINE  // probe knob: 0 = every launch walks its tiles forward
#define DLS_CONV_SERPENTINE 1
#endif
#ifndef DLS_PIPE_NARROW  // probe knob: bit 0/1/2 = 128-channel-multiple layers 16/8/4 wide in 64-channel 4-wave blocks
#define DLS_PIPE_NARROW 1  // 16 wide: -0.9 % per forward; 8 wide: null; 4 wide: +0.6 % (profiles/r06_forward_narrow_ab.txt)
#endif
#ifndef DLS_STEM_PIXSPLIT  // probe knob: 1 = the stem's two epilogue passes split the pixels, not the channels
#define DLS_STEM_PIXSPLIT 1
#endif
#ifndef DLS_CONV_PIPE  // probe knob: 0 = no LDS-DMA pipeline (k_conv3x3_halo for every 3x3 stride-1 shape)
#define DLS_CONV_PIPE 1
#endif

namespace dls {
namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;
typedef __attribute__((ext_vector_type(2))) uint32_t u32x2;

__device__ __forceinline__ uint32_t bf16_rne(float x) {
    const uint32_t u = __float_as_uint(x);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (u >> 16) | 0x40u;  // NaN stays a (quiet) NaN
    return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}

// x = hi + lo + O(2^-17 |x|); lo = 0 for non-finite x (hi carries the inf / NaN)
__device__ __forceinline__ void split2(float x, uint32_t &hi, uint32_t &lo) {
    hi = bf16_rne(x);
    const float r = x - __uint_as_float(hi << 16);
    lo = (__float_as_uint(x) & 0x7f800000u) == 0x7f800000u ? 0u : bf16_rne(r);
}

__device__ __forceinline__ float bf16_to_f32(uint32_t h) { return __uint_as_float(h << 16); }

typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
typedef __attribute__((ext_vector_type(2))) float f32x2;

// split2 of an element pair, packed: hi2 / lo2 hold a's bf16 in the low and b's
// in the high half.  The conversions are gfx950's v_cvt_pk_bf16_f32, which is
// bf16_rne bit for bit on all 2^32 fp32 patterns, NaN payloads included
// (tools/bf16_cvt_probe.hip, profiles/r05_bf16_cvt_probe.txt): the same bits as
// two split2 calls in a fifth of the instructions.
__device__ __forceinline__ void split2x2(float a, float b, uint32_t &hi2, uint32_t &lo2) {
    hi2 = __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{a, b}, bf16x2));
    float ra = a - __uint_as_float(hi2 << 16);
    float rb = b - __uint_as_float(hi2 & 0xffff0000u);
    ra = (__float_as_uint(a) & 0x7f800000u) == 0x7f800000u ? 0.f : ra;
    rb = (__float_as_uint(b) & 0x7f800000u) == 0x7f800000u ? 0.f : rb;
    lo2 = __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{ra, rb}, bf16x2));
}

struct ConvArgs {
    const uint16_t *x;      // split NHWC input [B][H][W][2C]
    const uint16_t *w;      // split weights [Cout][2K]
    const float *consts;    // eval batch norm [mean | iv | w | b] x Cout, or null
    const uint16_t *res;    // split residual [B][Ho][Wo][2 Cout], or null
    uint16_t *y;            // split output [B][Ho][Wo][2 Cout]
    int H, W, C, Ho, Wo, Cout, KW, taps, stride, pad, K, M, relu;
    int pix_tiles, co_tiles;
    int B, TI, TR, NH;  // halo kernel: images / rows per pixel tile, halo rows
    int rev;            // 1: each XCD walks its tile run backwards (tile_of_block)
};

constexpr int kWaveTile = 64;  // a wave's output tile: 64 channels x 64 pixels
constexpr int kBK = 32;        // channels per staged chunk
constexpr int kRowB = 4 * kBK + 16;  // LDS row: kBK hi, kBK lo (bf16), 16 B pad

typedef f32x16 WaveAcc[2][2];
typedef f32x4 WaveAcc16[4][4];  // the same 64 x 64 tile as 4 x 4 tiles of 16 x 16

// One staged chunk (kBK channels) into the wave's 2 x 2 tiles: A rows from `arow`
// (this lane's row r of the wave's first 32-channel tile; the second at +32
// rows), B rows of the two 32-pixel tiles at b0 / b1 (this lane's pixel).
// Products in the fixed order lo*hi, hi*lo, hi*hi per k-step.
__device__ __forceinline__ void mfma_chunk(WaveAcc &acc, const uint8_t *arow, const uint8_t *b0,
                                           const uint8_t *b1, int h) {
    constexpr int BK = kBK, RB = kRowB;
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
        const int off = 32 * s + 16 * h;  // bytes: k = 16 s + 8 h .. + 7
        bf16x8 ah[2], al[2], bh[2], bl[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            ah[i] = *reinterpret_cast<const bf16x8 *>(arow + i * 32 * RB + off);
            al[i] = *reinterpret_cast<const bf16x8 *>(arow + i * 32 * RB + 2 * BK + off);
        }
        bh[0] = *reinterpret_cast<const bf16x8 *>(b0 + off);
        bl[0] = *reinterpret_cast<const bf16x8 *>(b0 + 2 * BK + off);
        bh[1] = *reinterpret_cast<const bf16x8 *>(b1 + off);
        bl[1] = *reinterpret_cast<const bf16x8 *>(b1 + 2 * BK + off);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
            }
    }
}

// One k-step's fragments (16 channels): A hi / lo of the wave's two channel
// tiles, B hi / lo of its two pixel tiles; mfma_frag takes mfma_chunk's products
// in mfma_chunk's order
struct Frag {
    bf16x8 ah[2], al[2], bh[2], bl[2];
};

__device__ __forceinline__ void mfma_frag(WaveAcc &acc, const Frag &f) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.al[i], f.bh[j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.ah[i], f.bl[j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.ah[i], f.bh[j], acc[i][j], 0, 0, 0);
        }
}

__device__ __forceinline__ void zero_acc(WaveAcc &acc) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
}

// Epilogue through LDS (smem >= BNP * (4 BMC / NPASS + 16) bytes, free: every
// wave past its last read of the staged operands): the raw tiles are transposed
// to [pixel][channel] fp32, then each thread takes 8 channels of a pixel — batch
// norm fma(w, (x - mean) * iv, b), + residual (hi + lo), ReLU, split — and stores
// 16-B hi and lo pieces: a block's threads write whole runs of its pixels' rows.
// Lane (r, h) of wave (wc, wp) holds pixel wp*64 + 32 j + r, channels
// wc*64 + 32 i + 8 g + 4 h + e in acc[i][j][4 g + e].  NPASS = 2 transposes one
// 32-channel tile i of every wave per pass (half the LDS; the same arithmetic
// per element): pass p's local channel lc is channel (lc / 32) * 64 + 32 p +
// lc % 32 of the block.
// The raw tile of a wave into the epilogue's [pixel][channel] fp32 image (pass p)
template <int NPASS, int EROW>
__device__ __forceinline__ void acc_to_lds(const WaveAcc &acc, uint8_t *smem, int wc, int wp, int lane, int p) {
    const int r = lane & 31, h = lane >> 5;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            if (NPASS == 2 && i != p) continue;
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int pl = wp * kWaveTile + 32 * j + r;
                const int cl = NPASS == 1 ? wc * kWaveTile + 32 * i + 8 * g + 4 * h : wc * 32 + 8 * g + 4 * h;
                *reinterpret_cast<f32x4 *>(smem + pl * EROW + cl * 4) =
                    f32x4{acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]};
            }
        }
}

// 16x16x32 tiles: lane (r = l & 15, q = l >> 4) of tile (i, j) holds channels
// 16 i + 4 q + e of pixel 16 j + r
template <int NPASS, int EROW>
__device__ __forceinline__ void acc_to_lds(const WaveAcc16 &acc, uint8_t *smem, int wc, int wp, int lane, int) {
    static_assert(NPASS == 1, "one epilogue pass");
    const int r = lane & 15, q = lane >> 4;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int pl = wp * kWaveTile + 16 * j + r;
            const int cl = wc * kWaveTile + 16 * i + 4 * q;
            *reinterpret_cast<f32x4 *>(smem + pl * EROW + cl * 4) = acc[i][j];
        }
}

// PSPLIT (NPASS = 2, one channel tile): the passes split the pixels instead —
// pass p transposes the waves whose pixels lie in its half, every channel — so
// each pass stores whole 128-B runs of a pixel's hi (or lo) channels.
template <int BMC, int BNP, int NT, int NPASS = 1, class Acc = WaveAcc, bool PSPLIT = false>
__device__ __forceinline__ void epilogue_lds(const Acc &acc, uint8_t *smem, const ConvArgs &a,
                                             int co0, int pix0, int wc, int wp, int tid) {
    static_assert(NPASS == 1 || NPASS == 2, "epilogue passes");
    static_assert(!PSPLIT || (NPASS == 2 && BMC == kWaveTile && BNP % (2 * kWaveTile) == 0), "pixel passes");
    constexpr int SLAB = PSPLIT ? BMC : BMC / NPASS;  // channels per pass
    constexpr int PPP = PSPLIT ? BNP / NPASS : BNP;   // pixels per pass
    constexpr int EROW = 4 * SLAB + 16;
    constexpr int GPP = SLAB / 8;      // 8-channel groups per pixel
    constexpr int NPC = PPP * GPP / NT;
    static_assert(NT % GPP == 0 && (PPP * GPP) % NT == 0, "epilogue shape");
    const int lane = tid & 63;
    const int lc = 8 * (tid % GPP);  // a thread's channel group is fixed per pass
#pragma unroll
    for (int p = 0; p < NPASS; ++p) {
        const int co = co0 + (NPASS == 1 || PSPLIT ? lc : (lc / 32) * kWaveTile + 32 * p + lc % 32);
        const int pp0 = pix0 + (PSPLIT ? p * PPP : 0);  // the pass's first pixel
        // the pass's residual pieces are loaded before the transpose, their
        // latency behind its LDS writes and barrier (-1 to -2 % on the residual
        // layers, profiles/r06_conv_ab.txt)
        u32x4 rpf[NPC][2];
        if (a.res) {
#pragma unroll
            for (int u = 0; u < NPC; ++u) {
                const int px = pp0 + (tid + NT * u) / GPP;
                const int64_t ob = (int64_t)(px < a.M ? px : 0) * (2 * a.Cout) + co;
                rpf[u][0] = *reinterpret_cast<const u32x4 *>(a.res + ob);
                rpf[u][1] = *reinterpret_cast<const u32x4 *>(a.res + ob + a.Cout);
            }
        }
        if (p > 0) __syncthreads();  // the previous pass's reads are done
        if constexpr (PSPLIT) {
            if (wp * kWaveTile / PPP == p)  // this wave's pixels are the pass's: rows wp*64 - p*PPP ..
                acc_to_lds<1, EROW>(acc, smem - (ptrdiff_t)p * PPP * EROW, wc, wp, lane, 0);
        } else {
            acc_to_lds<NPASS, EROW>(acc, smem, wc, wp, lane, p);
        }
        __syncthreads();
        // the 8 channels' batch-norm constants as element pairs: 8 vector loads
        f32x2 m2[4], iv2[4], wv2[4], bv2[4];
        if (a.consts) {
            const f32x4 *c4[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) c4[t] = reinterpret_cast<const f32x4 *>(a.consts + t * a.Cout + co);
#pragma unroll
            for (int hh = 0; hh < 2; ++hh) {
                const f32x4 cm = c4[0][hh], ci = c4[1][hh], cw = c4[2][hh], cb = c4[3][hh];
                m2[2 * hh] = f32x2{cm[0], cm[1]};
                m2[2 * hh + 1] = f32x2{cm[2], cm[3]};
                iv2[2 * hh] = f32x2{ci[0], ci[1]};
                iv2[2 * hh + 1] = f32x2{ci[2], ci[3]};
                wv2[2 * hh] = f32x2{cw[0], cw[1]};
                wv2[2 * hh + 1] = f32x2{cw[2], cw[3]};
                bv2[2 * hh] = f32x2{cb[0], cb[1]};
                bv2[2 * hh + 1] = f32x2{cb[2], cb[3]};
            }
        }
#pragma unroll
        for (int u = 0; u < NPC; ++u) {
            const int pl = (tid + NT * u) / GPP;
            const int px = pp0 + pl;
            if (px >= a.M) continue;
            const f32x4 v0 = *reinterpret_cast<const f32x4 *>(smem + pl * EROW + lc * 4);
            const f32x4 v1 = *reinterpret_cast<const f32x4 *>(smem + pl * EROW + lc * 4 + 16);
            f32x2 v2[4] = {f32x2{v0[0], v0[1]}, f32x2{v0[2], v0[3]}, f32x2{v1[0], v1[1]}, f32x2{v1[2], v1[3]}};
            const int64_t ob = (int64_t)px * (2 * a.Cout) + co;
            if (a.consts) {  // fma(w, (x - mean) * iv, b), element pairs on packed fp32
#pragma unroll
                for (int q = 0; q < 4; ++q) v2[q] = __builtin_elementwise_fma(wv2[q], (v2[q] - m2[q]) * iv2[q], bv2[q]);
            }
            if (a.res) {  // + (hi + lo)
                const u32x4 rh = rpf[u][0], rl = rpf[u][1];
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    v2[q] = v2[q] + (f32x2{__uint_as_float(rh[q] << 16), __uint_as_float(rh[q] & 0xffff0000u)} +
                                     f32x2{__uint_as_float(rl[q] << 16), __uint_as_float(rl[q] & 0xffff0000u)});
            }
            float v[8] = {v2[0].x, v2[0].y, v2[1].x, v2[1].y, v2[2].x, v2[2].y, v2[3].x, v2[3].y};
            if (a.relu) {  // keeps NaN, as torch; one select per element (no branches)
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] = ((v[e] > 0.f) | (v[e] != v[e])) ? v[e] : 0.f;
            }
            uint32_t hi[4], lo[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) split2x2(v[2 * q], v[2 * q + 1], hi[q], lo[q]);
            *reinterpret_cast<u32x4 *>(a.y + ob) = u32x4{hi[0], hi[1], hi[2], hi[3]};
            *reinterpret_cast<u32x4 *>(a.y + ob + a.Cout) = u32x4{lo[0], lo[1], lo[2], lo[3]};
        }
    }
}

// XCD-aware tile order: the 8 XCDs take consecutive blockIdx round-robin (block
// b on XCD b % 8); give each XCD a contiguous run of tiles (any grid size: XCD x
// holds ceil((nblk - x) / 8) blocks), (pixel tile, channel tile) pairs with the
// channel tile fastest, so blocks reading the same input pixels share an L2.
// (Channel tile slowest instead, so an XCD's blocks share weights: null,
// profiles/r06_conv_ab.txt.)  rev: each XCD walks its run from the end, so a
// layer whose input was written forwards starts on the pixels written last (still
// in the Infinity Cache); the host alternates it along the forward
// (conv_walk_direction).  The order of the tiles never changes any output's bits.
__device__ __forceinline__ void tile_of_block(int co_tiles, int &co_t, int &pix_t, int rev) {
    const int nblk = gridDim.x, bid = blockIdx.x, x = bid & 7;
    // blocks on XCDs 0..x-1: sum of ceil((nblk - j) / 8)
    const int q = nblk >> 3, rmd = nblk & 7;
    const int cnt = q + (x < rmd ? 1 : 0);  // blocks on XCD x
    const int k = rev ? cnt - 1 - (bid >> 3) : (bid >> 3);
    const int t = x * q + (x < rmd ? x : rmd) + k;
    co_t = t % co_tiles;
    pix_t = t / co_tiles;
}

// ---------------------------------------------------------------- generic
// Any stride / padding / kernel size: every chunk stages the A rows (channels x
// kBK) and the B rows (each output pixel's input pixel under the chunk's tap,
// zero outside the image) through LDS, register-staged: double-buffered (NBUF =
// 2, one barrier per chunk) or one buffer (NBUF = 1, two barriers per chunk, half
// the LDS); NPASS: the epilogue's channel passes (epilogue_lds).  (Measured and
// dropped: two register sets, each chunk's loads issued two chunks ahead —
// 196 VGPRs, bit-identical, the stride-2 and 1x1 convolutions 45-60 % slower,
// profiles/r05_conv_probe.txt r05c5.)
template <int WCO, int WPIX, int NBUF = 2, int NPASS = 1>
__global__ __launch_bounds__(64 * WCO * WPIX) void k_conv_bf16x3(ConvArgs a) {
    static_assert(NBUF == 1 || NBUF == 2, "staging buffers");
    constexpr int NT = 64 * WCO * WPIX;
    constexpr int BMC = kWaveTile * WCO;   // output channels per block
    constexpr int BNP = kWaveTile * WPIX;  // pixels per block
    constexpr int PPR = kBK / 4;           // 16-B pieces per row
    constexpr int HP = kBK / 8;            // of which hi
    constexpr int RPP = NT / PPR;          // rows per staging pass
    constexpr int NA = BMC / RPP, NB = BNP / RPP;
    constexpr int STAGE = NBUF * (BMC + BNP) * kRowB;
    constexpr int EPI = BNP * (4 * BMC / NPASS + 16);
    static_assert(NT % PPR == 0 && BMC % RPP == 0 && BNP % RPP == 0, "staging shape");
    __shared__ __attribute__((aligned(16))) uint8_t smem[STAGE > EPI ? STAGE : EPI];

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wc = wid / WPIX, wp = wid % WPIX;
    int co_t, pix_t;
    tile_of_block(a.co_tiles, co_t, pix_t, a.rev);
    const int co0 = co_t * BMC;
    const int pix0 = pix_t * BNP;

    // staging assignment: piece `part` of rows tid / PPR + RPP * u
    const int part = tid % PPR, row0 = tid / PPR;
    const int poff = part < HP ? part * 8 : kBK + (part - HP) * 8;  // element offset in a chunk
    int pbase[NB], piy[NB], pix_[NB];
#pragma unroll
    for (int u = 0; u < NB; ++u) {
        const int p = pix0 + row0 + RPP * u;
        if (p < a.M) {
            const int hw = a.Ho * a.Wo;
            const int b = p / hw, rem = p - b * hw;
            const int oy = rem / a.Wo, ox = rem - oy * a.Wo;
            pbase[u] = b * a.H * a.W;
            piy[u] = oy * a.stride - a.pad;
            pix_[u] = ox * a.stride - a.pad;
        } else {
            pbase[u] = 0;
            piy[u] = -(1 << 20);  // never inside the image: loads zero
            pix_[u] = 0;
        }
    }
    const uint16_t *wrow[NA];
#pragma unroll
    for (int u = 0; u < NA; ++u) wrow[u] = a.w + (int64_t)(co0 + row0 + RPP * u) * (2 * a.K);

    const int cchunks = a.C / kBK;
    const int nchunks = a.taps * cchunks;
    u32x4 ra[NA], rb[NB];
    auto load = [&](int c) {
        const int tap = c / cchunks, ci0 = (c - tap * cchunks) * kBK;
        const int ky = tap / a.KW, kx = tap - ky * a.KW;
        const int kc = tap * a.C + ci0;
        const int wo = part < HP ? kc + part * 8 : a.K + kc + (part - HP) * 8;
#pragma unroll
        for (int u = 0; u < NA; ++u) ra[u] = *reinterpret_cast<const u32x4 *>(wrow[u] + wo);
        const int xo = part < HP ? ci0 + part * 8 : a.C + ci0 + (part - HP) * 8;
#pragma unroll
        for (int u = 0; u < NB; ++u) {
            const int iy = piy[u] + ky, ix = pix_[u] + kx;
            if ((unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W) {
                const int64_t pe = (int64_t)(pbase[u] + iy * a.W + ix) * (2 * a.C) + xo;
                rb[u] = *reinterpret_cast<const u32x4 *>(a.x + pe);
            } else {
                rb[u] = u32x4{0u, 0u, 0u, 0u};
            }
        }
    };
    auto store = [&](int buf) {
        uint8_t *As = smem + buf * (BMC + BNP) * kRowB;
        uint8_t *Bs = As + BMC * kRowB;
#pragma unroll
        for (int u = 0; u < NA; ++u)
            *reinterpret_cast<u32x4 *>(As + (row0 + RPP * u) * kRowB + poff * 2) = ra[u];
#pragma unroll
        for (int u = 0; u < NB; ++u)
            *reinterpret_cast<u32x4 *>(Bs + (row0 + RPP * u) * kRowB + poff * 2) = rb[u];
    };

    WaveAcc acc;
    zero_acc(acc);
    const int r = lane & 31, h = lane >> 5;
    load(0);
    store(0);
    __syncthreads();
    for (int c = 0; c < nchunks; ++c) {
        const bool more = c + 1 < nchunks;
        if (more) load(c + 1);
        const uint8_t *base = smem + (NBUF == 2 ? (c & 1) : 0) * (BMC + BNP) * kRowB;
        const uint8_t *b0 = base + (BMC + wp * kWaveTile + r) * kRowB;
        mfma_chunk(acc, base + (wc * kWaveTile + r) * kRowB, b0, b0 + 32 * kRowB, h);
        if (NBUF == 1 && more) __syncthreads();  // every wave is done with the buffer
        if (more) store(NBUF == 2 ? (c + 1) & 1 : 0);
        __syncthreads();
    }
    epilogue_lds<BMC, BNP, NT, NPASS>(acc, smem, a, co0, pix0, wc, wp, tid);
}

// ------------------------------------------------------ 3x3, stride 1, pad 1
// The block's pixels are a rectangle of whole output rows (TR rows of one image,
// or TI whole images), so its input is one halo tile: TI x (TR + 2) x (W + 2)
// pixels, staged once per chunk of kBK channels and read by all 9 taps at shifted
// rows — instead of 9 gathered B tiles (8-9x less LDS writing and L2 reading).
// The weights of one (chunk, tap) are double-buffered per tap; the next chunk's
// halo loads into registers at the chunk's first tap and is written after its
// last (single-buffered halo: 2 blocks per CU).
// (Measured slower: each wave loading its A fragments straight from global memory
// into registers a tap ahead, with no A staging and no barrier per tap — 20-40 %
// slower on every shape, profiles/r05_conv_probe.txt.)
// SKEW: halo row hr at hr * kRowB + (hr / 16) * 16 bytes, so that rows 16 apart
// (which the 32-pixel MFMA tiles of 4- to 16-wide images read in one pass) fall
// in different banks: 1-3 % faster on those layers, 3 % slower on 32-wide ones
// (profiles/r05_conv_probe.txt), so the launcher skews for W <= 16.  Measured and
// dropped (same file): the weights loaded two (chunk, tap) steps ahead instead of
// one (no change); the weights of a whole kernel row (3 taps) staged at once, two
// barriers per 3 taps instead of one per tap (layer1 -3 %, the 128-512-channel
// layers +30-45 %: one block per CU); 8-wave blocks, one per CU (512 pixels x 64
// channels: layer1 +15-18 %; 256 x 128: +2-10 %); persistent blocks that load the
// next tile's first halo chunk during this tile's epilogue (layer1 +0-2 %, 512
// channels -3 %, 10-22 VGPRs spilled: a wash); a ring of three weight buffers on
// the 64-channel layers (78 KB, still two blocks per CU) so that each wave reads
// the next tap's first k-step fragments before the barrier and resumes its MFMAs
// right after it (layer1 -0.1 to -0.6 %: the barrier's restart latency is not what
// bounds it); branch-free halo staging (every lane loading, padding rows from
// pixel 0 then zeroed; stores unconditional): 2-10 % slower, the loads cost more
// than the branches (r05c6).  What does bound it (the same file,
// r05x2): with one bf16 product per k-step instead of three the layers take
// 65-85 % of their time — the staging, the fragments' LDS reads and the barriers
// barely overlap the MFMAs at two waves per SIMD.
template <int WCO, int WPIX, int NHMAX, bool SKEW = false>
__global__ __launch_bounds__(64 * WCO * WPIX, 2) void k_conv3x3_halo(ConvArgs a) {
    constexpr int BK = kBK, RB = kRowB;
    constexpr int NT = 64 * WCO * WPIX;
    constexpr int BMC = kWaveTile * WCO;
    constexpr int BNP = kWaveTile * WPIX;
    constexpr int PPR = BK / 4, HP = BK / 8, RPP = NT / PPR;
    constexpr int NA = BMC / RPP;
    constexpr int HROWS = RPP * NHMAX;  // halo rows the LDS image holds
    constexpr int HBYTES = HROWS * RB + (SKEW ? (HROWS / 16 + 1) * 16 : 0);
    constexpr int STAGE = HBYTES + 2 * BMC * RB;
    constexpr int EPI = BNP * (4 * BMC + 16);
    static_assert(NT % PPR == 0 && BMC % RPP == 0, "staging shape");
    __shared__ __attribute__((aligned(16))) uint8_t smem[STAGE > EPI ? STAGE : EPI];
    uint8_t *halo = smem;
    uint8_t *abuf = smem + HBYTES;
    auto hoff = [](int hr) { return hr * RB + (SKEW ? (hr >> 4) * 16 : 0); };

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wc = wid / WPIX, wp = wid % WPIX;
    int co_t, pt;
    tile_of_block(a.co_tiles, co_t, pt, a.rev);
    const int co0 = co_t * BMC;
    const int pix0 = pt * BNP;
    const int W = a.W, H = a.H, W2 = W + 2;
    const int hrows_img = (a.TR + 2) * W2;
    int b0, y0;
    if (a.TR == H) {
        b0 = pt * a.TI;
        y0 = 0;
    } else {
        const int tpi = H / a.TR;
        b0 = pt / tpi;
        y0 = (pt - b0 * tpi) * a.TR;
    }

    const int part = tid % PPR, row0 = tid / PPR;
    const int poff = part < HP ? part * 8 : BK + (part - HP) * 8;
    // input pixel of each halo row this thread stages: -1 zero, -2 past the tile
    int hpix[NHMAX];
#pragma unroll
    for (int u = 0; u < NHMAX; ++u) {
        const int hr = row0 + RPP * u;
        int pix = -2;
        if (hr < a.NH) {
            const int ti = hr / hrows_img, rem = hr - ti * hrows_img;
            const int ry = rem / W2, rx = rem - ry * W2;
            const int b = b0 + ti, iy = y0 - 1 + ry, ix = rx - 1;
            pix = (b < a.B && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W)
                      ? (b * H + iy) * W + ix
                      : -1;
        }
        hpix[u] = pix;
    }
    const uint16_t *wrow[NA];
#pragma unroll
    for (int u = 0; u < NA; ++u) wrow[u] = a.w + (int64_t)(co0 + row0 + RPP * u) * (2 * a.K);

    u32x4 hreg[NHMAX], areg[NA];
    auto hload = [&](int cc) {
        const int xo = part < HP ? cc * BK + part * 8 : a.C + cc * BK + (part - HP) * 8;
#pragma unroll
        for (int u = 0; u < NHMAX; ++u)
            hreg[u] = hpix[u] >= 0
                          ? *reinterpret_cast<const u32x4 *>(a.x + (int64_t)hpix[u] * (2 * a.C) + xo)
                          : u32x4{0u, 0u, 0u, 0u};
    };
    auto hstore = [&]() {
#pragma unroll
        for (int u = 0; u < NHMAX; ++u)
            if (hpix[u] != -2)
                *reinterpret_cast<u32x4 *>(halo + hoff(row0 + RPP * u) + poff * 2) = hreg[u];
    };
    auto aload = [&](int cc, int tap) {
        const int kc = tap * a.C + cc * BK;
        const int wo = part < HP ? kc + part * 8 : a.K + kc + (part - HP) * 8;
#pragma unroll
        for (int u = 0; u < NA; ++u) areg[u] = *reinterpret_cast<const u32x4 *>(wrow[u] + wo);
    };
    auto astore = [&](int buf) {
#pragma unroll
        for (int u = 0; u < NA; ++u)
            *reinterpret_cast<u32x4 *>(abuf + (buf * BMC + row0 + RPP * u) * RB + poff * 2) = areg[u];
    };

    // this lane's output pixels (wp*64 + 32 j + r) as halo rows under tap (0, 0)
    const int r = lane & 31, h = lane >> 5;
    int hb[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int pl = wp * kWaveTile + 32 * j + r;
        const int tw = a.TR * W;
        const int ti = pl / tw, rem = pl - ti * tw;
        const int oy = rem / W, ox = rem - oy * W;
        hb[j] = ti * hrows_img + oy * W2 + ox;
    }

    WaveAcc acc;
    zero_acc(acc);
    const int nc = a.C / BK;
    hload(0);
    aload(0, 0);
    hstore();
    astore(0);
    __syncthreads();
    int step = 0;
    for (int cc = 0; cc < nc; ++cc) {
#pragma unroll
        for (int tap = 0; tap < 9; ++tap, ++step) {
            const bool last = tap == 8;
            const bool nxt = !last || cc + 1 < nc;
            if (nxt) aload(last ? cc + 1 : cc, last ? 0 : tap + 1);
            // the next chunk's halo loads go out after tap 0's weight loads, so
            // that tap 0's weight store does not wait for them (vmcnt counts loads
            // in issue order); the taps unrolled, so the waits are exact counts
            // (-3 % per forward with the residual prefetch, profiles/r06_conv_ab.txt)
            if (tap == 0 && cc + 1 < nc) hload(cc + 1);
            const int ky = tap / 3, kx = tap - 3 * ky;
            const int sh = ky * W2 + kx;
            mfma_chunk(acc, abuf + ((step & 1) * BMC + wc * kWaveTile + r) * RB, halo + hoff(hb[0] + sh),
                       halo + hoff(hb[1] + sh), h);
            if (nxt) astore((step + 1) & 1);
            if (last && cc + 1 < nc) {
                __syncthreads();  // every wave is done with this chunk's halo
                hstore();
            }
            __syncthreads();
        }
    }
    epilogue_lds<BMC, BNP, NT>(acc, smem, a, co0, pix0, wc, wp, tid);
}

// ------------------------------------------- 3x3, stride 1: LDS-DMA pipeline
// The halo kernel's tiling (whole output rows, one halo tile per 32-channel
// chunk, the weights of one (chunk, tap) per step) with every operand staged by
// LDS-DMA (global_load_lds_dwordx4: no staging registers, no ds_write pass) and
// kept in flight across the barriers:
//   * weights: a ring of 3 buffers; step t's tile is issued in step t - 2;
//   * halo (NHB = 2, an 8-wave block per CU): two buffers; chunk c + 1's rows go
//     out during chunk c's taps 0..NHI-1;
//   * each step waits (counted vmcnt, raw s_barrier) only for what the NEXT step
//     reads, and each wave reads the next step's first k-step fragments before
//     the barrier, so the MFMAs resume right after it.
// The halo tile holds TR + 2 image rows of each of its TI images and no padding
// columns: a lane whose tap falls left or right of the image reads a zero row
// kept beside the buffers.  Per layer against k_conv3x3_halo
// (profiles/r06_conv_pipe_ab.txt): -9 % on 16x16 (4-wave, NHB = 1), -12 % on
// 8x8 and -14 % on 4x4 (8-wave, NHB = 2), -1 to -2 % on 32x32 (64 channels,
// 4-wave, NHB = 1).
// LDS rows are 128 B (32 hi + 32 lo bf16) with the 16-B pieces XOR-swizzled by
// (s >> 1) & 7, s = the row's position in the MFMA lane order (the weight row;
// for a halo row, the output pixel it is under tap (0, 0) — consecutive along
// the tile's pixels at every tap): every ds_read_b128 lane group of 16 lanes hits
// 16 distinct 4-bank groups.  The DMA writes each wave-instruction's 64 pieces
// lane-linearly, so the swizzle is applied to the lanes' SOURCE addresses.
// Every output element is reduced in the halo kernel's order (chunks, taps,
// k-steps, lo*hi, hi*lo, hi*hi): the same bits.
__device__ __attribute__((aligned(16))) uint32_t kZeroPiece[4];  // source of the halo's padding pieces

__device__ __forceinline__ void glds16(const uint16_t *src, uint8_t *lds_base) {
    __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void *)lds_base, 16, 0, 0);
}

constexpr int kWaitLgkm0 = 0xc07f;  // s_waitcnt lgkmcnt(0) (vmcnt, expcnt at their maxima)

template <int NW>
__device__ __forceinline__ void retire_and_barrier(bool piece_in_flight) {
    // the step's halo piece (issued after its weights) may stay in flight
    if (piece_in_flight)
        asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// NHB = 1 (one halo buffer, blocks of <= 80 KB that fit two to a CU): the next
// chunk's halo is loaded after the chunk's last tap, its latency exposed in this
// block and covered by the other block on the CU.
template <int WCO, int WPIX, int NHI, int NHB = 2, int OCC = 1>
__global__ __launch_bounds__(64 * WCO * WPIX, OCC) void k_conv3x3_pipe(ConvArgs a) {
    constexpr int NW = WCO * WPIX, NT = 64 * NW;
    constexpr int BMC = kWaveTile * WCO, BNP = kWaveTile * WPIX;
    constexpr int RB = 128;                 // LDS row: 32 hi + 32 lo bf16
    constexpr int HROWS = 8 * NW * NHI;     // halo rows per buffer (8 rows per wave-instruction)
    constexpr int HB = HROWS * RB, AB = BMC * RB;
    constexpr int NAI = BMC / (8 * NW);     // weight DMAs per wave per step
    constexpr int STAGE = NHB * HB + 3 * AB + 2 * RB;  // + the zero rows
    constexpr int EPI = BNP * (4 * BMC + 16);
    static_assert(BMC % (8 * NW) == 0 && NAI >= 1, "weight rows per wave");
    static_assert(NHB == 1 || NHI <= 7, "the halo pieces go out in taps 0..6");
    static_assert(NHB == 1 || NHB == 2, "halo buffers");
    static_assert(kBK == 32, "128-byte rows");
    __shared__ __attribute__((aligned(16))) uint8_t smem[STAGE > EPI ? STAGE : EPI];
    uint8_t *const hbuf0 = smem;
    uint8_t *const abuf0 = smem + NHB * HB;
    // what a tap reads left / right of the image: two zero rows (256-B aligned),
    // each lane reading the one of its row's parity, so that it hits the banks a
    // halo row of its position would (no conflicts with the other lanes)
    uint8_t *const zrow = abuf0 + 3 * AB;

    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int wc = wv / WPIX, wp = wv % WPIX;
    int co_t, pt;
    tile_of_block(a.co_tiles, co_t, pt, a.rev);
    const int co0 = co_t * BMC;
    const int pix0 = pt * BNP;
    const int W = a.W, H = a.H, TR = a.TR;
    const int hrows_img = (TR + 2) * W;  // TR + 2 image rows, no padding columns
    int b0, y0;
    if (TR == H) {
        b0 = pt * a.TI;
        y0 = 0;
    } else {
        const int tpi = H / TR;
        b0 = pt / tpi;
        y0 = (pt - b0 * tpi) * TR;
    }

    // DMA sources: lane l of a wave-instruction fills slot l & 7 of row l >> 3 of
    // its 8 rows with the piece (l & 7) ^ swizzle(row)
    // a halo DMA lane's source, one register per DMA: input pixel * 8 + piece, or
    // -1 for the zero piece
    const int sl = lane & 7, lr = lane >> 3;
    int hsrc[NHI];
#pragma unroll
    for (int u = 0; u < NHI; ++u) {
        const int hr = 8 * (u * NW + wv) + lr;
        int pix = -1, s = 0;
        if (hr < a.NH) {
            const int ti = hr / hrows_img, rem = hr - ti * hrows_img;
            const int ry = rem / W, rx = rem - ry * W;
            s = hr - 2 * W * ti;  // = the row's pixel under tap (1, 1): consecutive along a tile
            const int b = b0 + ti, iy = y0 - 1 + ry;
            if (b < a.B && (unsigned)iy < (unsigned)H) pix = (b * H + iy) * W + rx;
        }
        hsrc[u] = pix >= 0 ? pix * 8 + (sl ^ ((s >> 1) & 7)) : -1;
    }
    // the zero piece's address, opaque to the compiler: computed once, not
    // re-loaded from the GOT in the loop (a scalar load there would make every
    // lgkmcnt wait a full drain)
    const uint16_t *zero = reinterpret_cast<const uint16_t *>(kZeroPiece);
    asm volatile("" : "+s"(zero));
    const uint16_t *asrc[NAI];
#pragma unroll
    for (int u = 0; u < NAI; ++u) {
        const int row = 8 * (wv * NAI + u) + lr;
        const int p = sl ^ ((row >> 1) & 7);
        asrc[u] = a.w + (int64_t)(co0 + row) * (2 * a.K) + ((p & 4) ? a.K : 0) + 8 * (p & 3);
    }
    auto issue_weights = [&](int step, int slot) {  // step's weights into ring slot slot % 3
        const int cc = step / 9, tap = step - 9 * cc;
        const int kc = tap * a.C + cc * kBK;
        uint8_t *dst = abuf0 + (slot % 3) * AB;
#pragma unroll
        for (int u = 0; u < NAI; ++u) glds16(asrc[u] + kc, dst + (wv * NAI + u) * 8 * RB);
    };
    auto issue_halo = [&](int u, int cc) {
        const int v = hsrc[u], p = v & 7;
        const uint16_t *src =
            v >= 0 ? a.x + (int64_t)(v >> 3) * (2 * a.C) + ((p & 4) ? a.C : 0) + 8 * (p & 3) + cc * kBK : zero;
        glds16(src, hbuf0 + (NHB == 2 ? (cc & 1) * HB : 0) + (u * NW + wv) * 8 * RB);
    };

    // fragment addresses: lane (r, h) reads A rows wc*64 + 32 i + r and the halo
    // rows of pixels wp*64 + 32 j + r
    const int r = lane & 31, h = lane >> 5;
    const int fa = (r >> 1) & 7;
    const int arow = (wc * kWaveTile + r) * RB;
    // pixel tile 1 is tile 0 shifted by 32 pixels: W divides 32 (try_launch_pipe),
    // so it has tile 0's columns, and its halo rows sit a block-uniform dhb further
    int hb0, pl0, ox0;
    {
        pl0 = wp * kWaveTile + r;
        const int tw = TR * W;
        const int ti = pl0 / tw, rem = pl0 - ti * tw;
        const int oy = rem / W;
        ox0 = rem - oy * W;
        hb0 = ti * hrows_img + oy * W + ox0;  // its halo row under tap (0, 1)
    }
    const int dhb = TR * W >= 32 ? 32 : (32 / (TR * W)) * hrows_img;
    auto frag = [&](Frag &f, int step, int tap, int s) {
        const uint8_t *ab = abuf0 + (step % 3) * AB + arow;
        const uint8_t *hbb = hbuf0 + (NHB == 2 ? ((step / 9) & 1) * HB : 0);
        const int qh = 16 * ((2 * s + h) ^ fa), ql = 16 * ((4 + 2 * s + h) ^ fa);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            f.ah[i] = *reinterpret_cast<const bf16x8 *>(ab + i * 32 * RB + qh);
            f.al[i] = *reinterpret_cast<const bf16x8 *>(ab + i * 32 * RB + ql);
        }
        const int ky = tap / 3, kx = tap - 3 * ky;
        const int sh = ky * W + kx - 1;
        const bool in = (unsigned)(ox0 + kx - 1) < (unsigned)W;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int fb = ((pl0 + 32 * j + sh) >> 1) & 7;
            const uint8_t *row = in ? hbb + (hb0 + j * dhb + sh) * RB : zrow + ((pl0 + sh) & 1) * RB;
            f.bh[j] = *reinterpret_cast<const bf16x8 *>(row + 16 * ((2 * s + h) ^ fb));
            f.bl[j] = *reinterpret_cast<const bf16x8 *>(row + 16 * ((4 + 2 * s + h) ^ fb));
        }
    };

    WaveAcc acc;
    zero_acc(acc);
    const int nc = a.C / kBK, T = 9 * nc;
    if (tid < 2 * RB / 16) *reinterpret_cast<u32x4 *>(zrow + 16 * tid) = u32x4{0u, 0u, 0u, 0u};
#pragma unroll
    for (int u = 0; u < NHI; ++u) issue_halo(u, 0);
    issue_weights(0, 0);
    issue_weights(T > 1 ? 1 : 0, 1);
    retire_and_barrier<NW>(false);
    Frag f0, f1;
    frag(f0, 0, 0, 0);
    for (int cc = 0; cc < nc; ++cc) {
        const bool more = cc + 1 < nc;
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
            // unconditional in every step (the last steps re-load the last
            // weights into a buffer no later step reads; the fragments past the
            // last step read stale LDS), so that the compiler's lgkmcnt / vmcnt
            // counts stay exact
            const int t = 9 * cc + tap;
            const bool piece = NHB == 2 && more && tap < NHI;
            issue_weights(t + 2 < T ? t + 2 : T - 1, t + 2);
            if (piece) issue_halo(tap, cc + 1);
            // the order is pinned: each k-step's reads go out a whole k-step of
            // MFMAs ahead of their use (left alone, the compiler sinks them next
            // to their MFMAs to save registers)
            __builtin_amdgcn_s_waitcnt(kWaitLgkm0);
            frag(f1, t, tap, 1);
            __builtin_amdgcn_sched_barrier(0);
            mfma_frag(acc, f0);
            __builtin_amdgcn_sched_barrier(0);
            const bool reload = NHB == 1 && tap == 8 && more;  // the next chunk's halo is not in yet
            if (!reload) {
                __builtin_amdgcn_s_waitcnt(kWaitLgkm0);
                frag(f0, t + 1, tap == 8 ? 0 : tap + 1, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
            mfma_frag(acc, f1);
            retire_and_barrier<NW>(piece);
            if (reload) {  // every wave is past its reads of this chunk's halo
#pragma unroll
                for (int u = 0; u < NHI; ++u) issue_halo(u, cc + 1);
                retire_and_barrier<NW>(false);
                frag(f0, t + 1, 0, 0);
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // every wave is past its last fragment read
    epilogue_lds<BMC, BNP, NT>(acc, smem, a, co0, pix0, wc, wp, tid);
}

// k_conv3x3_pipe on v_mfma_f32_16x16x32_bf16: a wave's 64 x 64 tile as 4 x 4
// tiles of 16 x 16, one MFMA per (tile, product) covering the whole 32-channel
// step (the 16 A / B fragment reads per step are k_conv3x3_pipe's 16).  Under
// load the chip holds a higher clock on this shape than on 32x32x16
// (MI355X_MICROARCH.md, DVFS give-back item 7).  The 16-B pieces are swizzled
// by row & 7 (a 16-row fragment read at any row offset is conflict-free; the
// 32-row form's (row >> 1) & 7 is 2-way at odd offsets).  A step's fragments are
// read whole a step ahead (two sets in registers), the next step's during this
// step's 48 MFMAs.  Reduction order per output: chunks, taps, then per step the
// products lo*hi, hi*lo, hi*hi over the 32 channels inside the MFMA — not
// k_conv3x3_pipe's bits.
// A step's fragments in two parts: A (all four channel tiles) with pixel tiles
// 0-1, and pixel tiles 2-3 (read during the MFMAs of the first part)
struct Frag16A {
    bf16x8 ah[4], al[4], bh[2], bl[2];
};
struct Frag16B {
    bf16x8 bh[2], bl[2];
};

// the MFMAs of pixel tiles jb, jb + 1 (products lo*hi, hi*lo, hi*hi)
__device__ __forceinline__ void mfma_half16(WaveAcc16 &acc, const Frag16A &fa, const bf16x8 (&bh)[2],
                                            const bf16x8 (&bl)[2], int jb) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            f32x4 &c = acc[i][jb + j];
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa.al[i], bh[j], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa.ah[i], bl[j], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa.ah[i], bh[j], c, 0, 0, 0);
        }
}

template <int WCO, int WPIX, int NHI, int NHB = 2, int OCC = 1>
__global__ __launch_bounds__(64 * WCO * WPIX, OCC) void k_conv3x3_pipe16(ConvArgs a) {
    constexpr int NW = WCO * WPIX, NT = 64 * NW;
    constexpr int BMC = kWaveTile * WCO, BNP = kWaveTile * WPIX;
    constexpr int RB = 128;
    constexpr int HROWS = 8 * NW * NHI;
    constexpr int HB = HROWS * RB, AB = BMC * RB;
    constexpr int NAI = BMC / (8 * NW);
    constexpr int STAGE = NHB * HB + 3 * AB + 2 * RB;
    constexpr int EPI = BNP * (4 * BMC + 16);
    static_assert(BMC % (8 * NW) == 0 && NAI >= 1, "weight rows per wave");
    static_assert(NHB == 1 || NHI <= 7, "the halo pieces go out in taps 0..6");
    static_assert(NHB == 1 || NHB == 2, "halo buffers");
    static_assert(kBK == 32, "128-byte rows");
    __shared__ __attribute__((aligned(16))) uint8_t smem[STAGE > EPI ? STAGE : EPI];
    uint8_t *const hbuf0 = smem;
    uint8_t *const abuf0 = smem + NHB * HB;
    uint8_t *const zrow = abuf0 + 3 * AB;

    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int wc = wv / WPIX, wp = wv % WPIX;
    int co_t, pt;
    tile_of_block(a.co_tiles, co_t, pt, a.rev);
    const int co0 = co_t * BMC;
    const int pix0 = pt * BNP;
    const int W = a.W, H = a.H, TR = a.TR;
    const int hrows_img = (TR + 2) * W;
    int b0, y0;
    if (TR == H) {
        b0 = pt * a.TI;
        y0 = 0;
    } else {
        const int tpi = H / TR;
        b0 = pt / tpi;
        y0 = (pt - b0 * tpi) * TR;
    }

    // DMA sources as k_conv3x3_pipe's, the piece swizzled by the row's key & 7
    const int sl = lane & 7, lr = lane >> 3;
    int hsrc[NHI];
#pragma unroll
    for (int u = 0; u < NHI; ++u) {
        const int hr = 8 * (u * NW + wv) + lr;
        int pix = -1, s = 0;
        if (hr < a.NH) {
            const int ti = hr / hrows_img, rem = hr - ti * hrows_img;
            const int ry = rem / W, rx = rem - ry * W;
            s = hr - 2 * W * ti;
            const int b = b0 + ti, iy = y0 - 1 + ry;
            if (b < a.B && (unsigned)iy < (unsigned)H) pix = (b * H + iy) * W + rx;
        }
        hsrc[u] = pix >= 0 ? pix * 8 + (sl ^ (s & 7)) : -1;
    }
    const uint16_t *zero = reinterpret_cast<const uint16_t *>(kZeroPiece);
    asm volatile("" : "+s"(zero));
    const uint16_t *asrc[NAI];
#pragma unroll
    for (int u = 0; u < NAI; ++u) {
        const int row = 8 * (wv * NAI + u) + lr;
        const int p = sl ^ (row & 7);
        asrc[u] = a.w + (int64_t)(co0 + row) * (2 * a.K) + ((p & 4) ? a.K : 0) + 8 * (p & 3);
    }
    auto issue_weights = [&](int step, int slot) {
        const int cc = step / 9, tap = step - 9 * cc;
        int Cv = a.C;  // opaque per step: no per-tap source addresses hoisted out of the loop
        asm volatile("" : "+s"(Cv));
        const int kc = tap * Cv + cc * kBK;
        uint8_t *dst = abuf0 + (slot % 3) * AB;
#pragma unroll
        for (int u = 0; u < NAI; ++u) glds16(asrc[u] + kc, dst + (wv * NAI + u) * 8 * RB);
    };
    auto issue_halo = [&](int u, int cc) {
        const int v = hsrc[u], p = v & 7;
        const uint16_t *src =
            v >= 0 ? a.x + (int64_t)(v >> 3) * (2 * a.C) + ((p & 4) ? a.C : 0) + 8 * (p & 3) + cc * kBK : zero;
        glds16(src, hbuf0 + (NHB == 2 ? (cc & 1) * HB : 0) + (u * NW + wv) * 8 * RB);
    };

    // lane (r, q): A rows wc*64 + 16 i + r, pieces q (hi) and 4 + q (lo); B rows of
    // the pixels wp*64 + 16 j + r
    const int r = lane & 15, q = lane >> 4;
    const int arow = (wc * kWaveTile + r) * RB;
    const int qa = 16 * (q ^ (r & 7)), qla = 16 * ((4 + q) ^ (r & 7));  // (wc*64 + 16 i + r) & 7 = r & 7
    int hb[4], ox[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int pl = wp * kWaveTile + 16 * j + r;
        const int tw = TR * W;
        const int ti = pl / tw, rem = pl - ti * tw;
        const int oy = rem / W;
        ox[j] = rem - oy * W;
        hb[j] = ti * hrows_img + oy * W + ox[j];  // its halo row under tap (0, 1)
    }
    const int pl0 = wp * kWaveTile + r;
    // B fragments of pixel tiles jb, jb + 1 at a step's tap
    auto fragb = [&](bf16x8 (&bh)[2], bf16x8 (&bl)[2], int step, int tap, int jb) {
        const uint8_t *hbb = hbuf0 + (NHB == 2 ? ((step / 9) & 1) * HB : 0);
        const int ky = tap / 3, kx = tap - 3 * ky;
        // W made opaque per read: the rows are recomputed each step (a few adds)
        // instead of 9 taps x 4 tiles of addresses hoisted out of the chunk loop
        int Wv = W;
        asm volatile("" : "+s"(Wv));
        const int sh = ky * Wv + kx - 1;
        const int key = (pl0 + sh) & 7;  // + 16 j: the same key
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const bool in = (unsigned)(ox[jb + j] + kx - 1) < (unsigned)Wv;
            const uint8_t *row = in ? hbb + (hb[jb + j] + sh) * RB : zrow + ((pl0 + sh) & 1) * RB;
            bh[j] = *reinterpret_cast<const bf16x8 *>(row + 16 * (q ^ key));
            bl[j] = *reinterpret_cast<const bf16x8 *>(row + 16 * ((4 + q) ^ key));
        }
    };
    auto fraga = [&](Frag16A &f, int step, int tap) {
        const uint8_t *ab = abuf0 + (step % 3) * AB + arow;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            f.ah[i] = *reinterpret_cast<const bf16x8 *>(ab + i * 16 * RB + qa);
            f.al[i] = *reinterpret_cast<const bf16x8 *>(ab + i * 16 * RB + qla);
        }
        fragb(f.bh, f.bl, step, tap, 0);
    };

    WaveAcc16 acc;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int nc = a.C / kBK, T = 9 * nc;
    if (tid < 2 * RB / 16) *reinterpret_cast<u32x4 *>(zrow + 16 * tid) = u32x4{0u, 0u, 0u, 0u};
#pragma unroll
    for (int u = 0; u < NHI; ++u) issue_halo(u, 0);
    issue_weights(0, 0);
    issue_weights(T > 1 ? 1 : 0, 1);
    retire_and_barrier<NW>(false);
    Frag16A fa;
    Frag16B fb;
    fraga(fa, 0, 0);
    for (int cc = 0; cc < nc; ++cc) {
        const bool more = cc + 1 < nc;
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
            const int t = 9 * cc + tap;
            const bool piece = NHB == 2 && more && tap < NHI;
            issue_weights(t + 2 < T ? t + 2 : T - 1, t + 2);
            if (piece) issue_halo(tap, cc + 1);
            const bool reload = NHB == 1 && tap == 8 && more;  // the next chunk's halo is not in yet
            __builtin_amdgcn_s_waitcnt(kWaitLgkm0);  // A and pixel tiles 0-1 of this step
            fragb(fb.bh, fb.bl, t, tap, 2);
            __builtin_amdgcn_sched_barrier(0);
            mfma_half16(acc, fa, fa.bh, fa.bl, 0);
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_waitcnt(kWaitLgkm0);  // pixel tiles 2-3
            const Frag16A cur = fa;
            if (!reload) fraga(fa, t + 1, tap == 8 ? 0 : tap + 1);  // past the last step: stale LDS, unused
            __builtin_amdgcn_sched_barrier(0);
            mfma_half16(acc, cur, fb.bh, fb.bl, 2);
            __builtin_amdgcn_sched_barrier(0);
            retire_and_barrier<NW>(piece);
            if (reload) {  // every wave is past its reads of this chunk's halo
#pragma unroll
                for (int u = 0; u < NHI; ++u) issue_halo(u, cc + 1);
                retire_and_barrier<NW>(false);
                fraga(fa, t + 1, 0);
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // every wave is past its last fragment read
    epilogue_lds<BMC, BNP, NT, 1, WaveAcc16>(acc, smem, a, co0, pix0, wc, wp, tid);
}

// --------------------------------------------- 3x3, stride 2, pad 1: phases
// A stride-2 3x3 convolution is four stride-1 ones over the input's row / column
// parity images P_ab(q, r) = x(2q + a, 2r + b), each Ho x Wo: tap (ky, kx) reads
// P_ab with a = (ky + 1) & 1, b = (kx + 1) & 1 at (oy + dq, ox + dr), dq = -1 for
// ky = 0 (else 0), dr = -1 for kx = 0.  Phase (1,1) has taps (0,0) (0,2) (2,0)
// (2,2), (1,0) has (0,1) (2,1), (0,1) has (1,0) (1,2), (0,0) has (1,1).  Each
// phase's halo is TI x (TR + 1) x Wo rows (output tile + one row above; no
// padding columns: a tap left of the image reads a zero row), so each input pixel
// is staged once per channel chunk — the gather kernel stages 2.25 per output
// pixel per chunk, 9 B tiles.  k_conv3x3_pipe's machinery otherwise: 8-wave
// blocks, LDS-DMA into swizzled 128-B rows, a 3-slot weight ring two steps ahead,
// two halo buffers (phase g + 1's rows go out in phase g's first step); the next
// step's first fragments are read before the barrier within a phase, after it
// across phases (the next phase's halo lands by the phase's end).  Reduction
// order: chunks, phases, taps, k-steps — deterministic, not the generic
// kernel's bits.
__device__ constexpr int kPhaseTap[9] = {0, 2, 6, 8, 1, 7, 3, 5, 4};  // step -> tap (ky * 3 + kx)

template <int WCO, int WPIX, int NHI>
__global__ __launch_bounds__(64 * WCO * WPIX, 1) void k_conv3x3s2_phase(ConvArgs a) {
    constexpr int NW = WCO * WPIX, NT = 64 * NW;
    constexpr int BMC = kWaveTile * WCO, BNP = kWaveTile * WPIX;
    constexpr int RB = 128;
    constexpr int HROWS = 8 * NW * NHI;
    constexpr int HB = HROWS * RB, AB = BMC * RB;
    constexpr int NAI = BMC / (8 * NW);
    constexpr int STAGE = 2 * HB + 3 * AB + 2 * RB;
    constexpr int EPI = BNP * (4 * BMC + 16);
    static_assert(BMC % (8 * NW) == 0 && NAI >= 1, "weight rows per wave");
    static_assert(kBK == 32, "128-byte rows");
    __shared__ __attribute__((aligned(16))) uint8_t smem[STAGE > EPI ? STAGE : EPI];
    uint8_t *const hbuf0 = smem;
    uint8_t *const abuf0 = smem + 2 * HB;
    uint8_t *const zrow = abuf0 + 3 * AB;  // two zero rows, read by parity (k_conv3x3_pipe)

    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int wc = wv / WPIX, wp = wv % WPIX;
    int co_t, pt;
    tile_of_block(a.co_tiles, co_t, pt, a.rev);
    const int co0 = co_t * BMC;
    const int pix0 = pt * BNP;
    const int H = a.H, W = a.W, Ho = a.Ho, Wo = a.Wo, TR = a.TR;
    const int hrows_img = (TR + 1) * Wo;
    int b0, y0;
    if (TR == Ho) {
        b0 = pt * a.TI;
        y0 = 0;
    } else {
        const int tpi = Ho / TR;
        b0 = pt / tpi;
        y0 = (pt - b0 * tpi) * TR;
    }

    // halo DMA lane sources: the input pixel of phase (1,1) — (2q + 1, 2r + 1) —
    // or -1, and the piece; phase (a, b) reads (2q + a, 2r + b), 1 - a rows and
    // 1 - b columns back
    const int sl = lane & 7, lr = lane >> 3;
    int hpix[NHI], hpc[NHI];
#pragma unroll
    for (int u = 0; u < NHI; ++u) {
        const int hr = 8 * (u * NW + wv) + lr;
        int v = -1, s = 0;
        if (hr < a.NH) {
            const int ti = hr / hrows_img, rem = hr - ti * hrows_img;
            const int qq = rem / Wo, r = rem - qq * Wo;
            const int b = b0 + ti, q = y0 - 1 + qq;
            s = hr - ti * Wo;  // the row's pixel under dq = -1: consecutive along a tile
            if (b < a.B && q >= 0) v = (b * H + 2 * q + 1) * W + 2 * r + 1;
        }
        hpix[u] = v;
        hpc[u] = sl ^ ((s >> 1) & 7);
    }
    const uint16_t *zero = reinterpret_cast<const uint16_t *>(kZeroPiece);
    asm volatile("" : "+s"(zero));
    const uint16_t *asrc[NAI];
#pragma unroll
    for (int u = 0; u < NAI; ++u) {
        const int row = 8 * (wv * NAI + u) + lr;
        const int p = sl ^ ((row >> 1) & 7);
        asrc[u] = a.w + (int64_t)(co0 + row) * (2 * a.K) + ((p & 4) ? a.K : 0) + 8 * (p & 3);
    }
    auto issue_weights = [&](int step, int slot) {
        const int cc = step / 9, tap = kPhaseTap[step - 9 * cc];
        const int kc = tap * a.C + cc * kBK;
        uint8_t *dst = abuf0 + (slot % 3) * AB;
#pragma unroll
        for (int u = 0; u < NAI; ++u) glds16(asrc[u] + kc, dst + (wv * NAI + u) * 8 * RB);
    };
    // phase g = 4 cc + p (p: 0 = (1,1), 1 = (1,0), 2 = (0,1), 3 = (0,0)) into buffer g & 1
    auto issue_halo = [&](int g) {
        const int cc = g >> 2, p = g & 3;
        const int back = (p < 2 ? 0 : W) + ((p & 1) ? 1 : 0);  // (1 - a) rows + (1 - b) columns
#pragma unroll
        for (int u = 0; u < NHI; ++u) {
            const int v = hpix[u], pc = hpc[u];
            const uint16_t *src =
                v >= 0 ? a.x + (int64_t)(v - back) * (2 * a.C) + ((pc & 4) ? a.C : 0) + 8 * (pc & 3) + cc * kBK
                       : zero;
            glds16(src, hbuf0 + (g & 1) * HB + (u * NW + wv) * 8 * RB);
        }
    };

    const int r = lane & 31, h = lane >> 5;
    const int fa = (r >> 1) & 7;
    const int arow = (wc * kWaveTile + r) * RB;
    int hb0, pl0, ox0;
    {
        pl0 = wp * kWaveTile + r;
        const int tw = TR * Wo;
        const int ti = pl0 / tw, rem = pl0 - ti * tw;
        const int oy = rem / Wo;
        ox0 = rem - oy * Wo;
        hb0 = ti * hrows_img + oy * Wo + ox0;  // its halo row under dq = -1, dr = 0
    }
    const int dhb = TR * Wo >= 32 ? 32 : (32 / (TR * Wo)) * hrows_img;
    auto frag = [&](Frag &f, int step, int s) {
        const int cc = step / 9, k = step - 9 * cc;
        const int tap = kPhaseTap[k], g = 4 * cc + (k < 4 ? 0 : k < 6 ? 1 : k < 8 ? 2 : 3);
        const int ky = tap / 3, kx = tap - 3 * ky;
        const uint8_t *ab = abuf0 + (step % 3) * AB + arow;
        const uint8_t *hbb = hbuf0 + (g & 1) * HB;
        const int qh = 16 * ((2 * s + h) ^ fa), ql = 16 * ((4 + 2 * s + h) ^ fa);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            f.ah[i] = *reinterpret_cast<const bf16x8 *>(ab + i * 32 * RB + qh);
            f.al[i] = *reinterpret_cast<const bf16x8 *>(ab + i * 32 * RB + ql);
        }
        const int sh = (ky == 0 ? 0 : Wo) + (kx == 0 ? -1 : 0);  // (1 + dq) * Wo + dr
        const bool in = kx != 0 || ox0 > 0;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int fb = ((pl0 + 32 * j + sh) >> 1) & 7;
            const uint8_t *row = in ? hbb + (hb0 + j * dhb + sh) * RB : zrow + ((pl0 + sh) & 1) * RB;
            f.bh[j] = *reinterpret_cast<const bf16x8 *>(row + 16 * ((2 * s + h) ^ fb));
            f.bl[j] = *reinterpret_cast<const bf16x8 *>(row + 16 * ((4 + 2 * s + h) ^ fb));
        }
    };

    WaveAcc acc;
    zero_acc(acc);
    const int nc = a.C / kBK, T = 9 * nc;
    if (tid < 2 * RB / 16) *reinterpret_cast<u32x4 *>(zrow + 16 * tid) = u32x4{0u, 0u, 0u, 0u};
    issue_halo(0);
    issue_weights(0, 0);
    issue_weights(T > 1 ? 1 : 0, 1);
    retire_and_barrier<NW>(false);
    Frag f0, f1;
    frag(f0, 0, 0);
    for (int cc = 0; cc < nc; ++cc) {
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            const int t = 9 * cc + k;
            const bool first = k == 0 || k == 4 || k == 6 || k == 8;  // a phase's first step
            const bool last = k == 3 || k == 5 || k == 7 || k == 8;   // a phase's last step
            const int g = 4 * cc + (k < 4 ? 0 : k < 6 ? 1 : k < 8 ? 2 : 3);
            issue_weights(t + 2 < T ? t + 2 : T - 1, t + 2);
            // the next phase's halo into the buffer the previous phase read (every
            // wave is past its last read of it: the barrier before this phase)
            if (first && g + 1 < 4 * nc) issue_halo(g + 1);
            __builtin_amdgcn_s_waitcnt(kWaitLgkm0);
            frag(f1, t, 1);
            __builtin_amdgcn_sched_barrier(0);
            mfma_frag(acc, f0);
            __builtin_amdgcn_sched_barrier(0);
            if (!last) {
                __builtin_amdgcn_s_waitcnt(kWaitLgkm0);
                frag(f0, t + 1, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
            mfma_frag(acc, f1);
            // this step's weights retired; the next phase's halo (issued after them
            // in the phase's first step) stays in flight until the phase's last step
            if (first && !last && g + 1 < 4 * nc)
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NHI) : "memory");
            else
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            if (last) frag(f0, t + 1, 0);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // every wave is past its last fragment read
    epilogue_lds<BMC, BNP, NT>(acc, smem, a, co0, pix0, wc, wp, tid);
}

// ------------------------------------------------------------------ stem
// A first layer whose whole reduction is one chunk (KH * KW * C <= kBK: the
// 3-channel 3x3 stem of a CIFAR ResNet, 27 terms): the im2col is fused — each
// thread gathers its output pixel's inputs straight from the fp32 NCHW image
// batch (k = (ky * KW + kx) * C + ci, zero outside the image and past the 27),
// splits them and writes the pixel's B row to LDS — then one chunk of MFMAs and
// the epilogue.  Weights: dls_conv_pack_weights_im2col_f32 with Kp = kBK.
// CIN / KHW > 0: the input channels and the (square) kernel size as constants
// (the index arithmetic of the 27-term gather folds away); 0: runtime a.C / a.KW.
// LDS is what bounds its occupancy (a short block: gather, 24 MFMAs, epilogue),
// so each wave loads its A fragments straight from the weights (16 B per lane
// and fragment, L2-resident) and the epilogue transposes 32 channels at a time:
// 37 KB per block, 4 blocks per CU (the LDS-staged weights and one 64-channel
// epilogue pass: 70 KB, 2 blocks).  The same products in the same order and the
// same epilogue arithmetic: the same bits.
// XT (3 channels, 3x3, stride 1, pad 1, 32-wide images, 8 rows per tile): the
// block's input window (3 x 10 rows x 34 columns, zero outside the image) is
// staged in LDS by one 16-B load per thread and the 27 terms gathered from there,
// instead of 27 scalar loads per thread from global memory; the same values.
constexpr int kStemWinRow = 40;  // floats per window row: image column ix at ix + 4
// NTL > 1 (XT): a block walks NTL consecutive pixel tiles with its A fragments
// loaded once, the next tile's input window loaded into registers while this
// tile is gathered, multiplied and stored; the same arithmetic per tile.
template <int WPIX, int CIN = 0, int KHW = 0, bool XT = false, int NTL = 1>
__global__ __launch_bounds__(64 * WPIX) void k_conv_stem(ConvArgs a, const float *__restrict__ x) {
    constexpr int NT = 64 * WPIX, BNP = kWaveTile * WPIX;
    constexpr int STAGE = BNP * kRowB;
    constexpr int EPI = BNP * (4 * kWaveTile / 2 + 16);  // two epilogue passes
    constexpr int WIN = XT ? 3 * 10 * kStemWinRow * 4 : 0;
    static_assert(NT == BNP, "one pixel row per thread");
    static_assert(!XT || (CIN == 3 && KHW == 3 && BNP == 256), "the staged window's shape");
    static_assert(NTL == 1 || XT, "tile walks: the staged-window form");
    __shared__ __attribute__((aligned(16))) uint8_t smem[(STAGE > EPI ? STAGE : EPI) + WIN];
    uint8_t *Bs = smem;
    float *win = reinterpret_cast<float *>(smem + (STAGE > EPI ? STAGE : EPI));
    const int tid = threadIdx.x, lane = tid & 63, wp = tid >> 6;
    const int r = lane & 31, h = lane >> 5;
    int co_t, pix_t;
    tile_of_block(a.co_tiles, co_t, pix_t, a.rev);
    const int co0 = co_t * kWaveTile;
    // the window rows oy0 - 1 .. oy0 + 8 of a tile's image, 8 columns x 4 per thread
    auto load_window = [&](int p0) {
        f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
        const int b = p0 / (a.H * 32), oy0 = (p0 - b * a.H * 32) / 32;
        if (tid < 240) {
            const int ci = tid / 80, rem = tid - ci * 80, wy = rem / 8, c4 = rem - wy * 8;
            const int iy = oy0 - 1 + wy;
            if (b < a.B && (unsigned)iy < (unsigned)a.H)
                v = *reinterpret_cast<const f32x4 *>(x + (((int64_t)b * 3 + ci) * a.H + iy) * 32 + 4 * c4);
        }
        return v;
    };
    f32x4 wnext = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (XT) wnext = load_window(pix_t * NTL * BNP);
    // A fragments of both k-steps (in flight during the gather): channel tile i,
    // lane row co0 + 32 i + r, k = 16 s + 8 h .. + 7 (hi), + K (lo)
    Frag f[kBK / 16];
#pragma unroll
    for (int s = 0; s < kBK / 16; ++s)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const uint16_t *wr = a.w + (int64_t)(co0 + 32 * i + r) * (2 * a.K) + 16 * s + 8 * h;
            f[s].ah[i] = *reinterpret_cast<const bf16x8 *>(wr);
            f[s].al[i] = *reinterpret_cast<const bf16x8 *>(wr + a.K);
        }
    for (int tl = 0; tl < NTL; ++tl) {
    const int pix0 = (pix_t * NTL + tl) * BNP;
    if (pix0 >= a.M) break;  // block-uniform
    if constexpr (XT) {
        if (tl > 0) __syncthreads();  // the previous tile's epilogue is done with the LDS
        if (tid < 240) {
            const int ci = tid / 80, rem = tid - ci * 80, wy = rem / 8, c4 = rem - wy * 8;
            *reinterpret_cast<f32x4 *>(win + (ci * 10 + wy) * kStemWinRow + 4 + 4 * c4) = wnext;
        } else if (tid < 240 + 15) {  // the padding columns (image columns -1 and 32) of 30 rows
            const int q = tid - 240;
            win[(2 * q) * kStemWinRow + 3] = 0.f;
            win[(2 * q) * kStemWinRow + 36] = 0.f;
            win[(2 * q + 1) * kStemWinRow + 3] = 0.f;
            win[(2 * q + 1) * kStemWinRow + 36] = 0.f;
        }
        __syncthreads();
        if (tl + 1 < NTL && pix0 + BNP < a.M) wnext = load_window(pix0 + BNP);  // in flight until the next tile
    }
    // this thread's pixel: gather, split, one LDS row
    {
        const int p = pix0 + tid;
        uint32_t hw[kBK / 2], lw[kBK / 2];
#pragma unroll
        for (int q = 0; q < kBK / 2; ++q) hw[q] = lw[q] = 0u;
        if (p < a.M) {
            const int hwo = a.Ho * a.Wo;
            const int b = p / hwo, rem = p - b * hwo;
            const int oy = rem / a.Wo, ox = rem - oy * a.Wo;
            const int C = CIN > 0 ? CIN : a.C, KW = KHW > 0 ? KHW : a.KW;
            const int nk = CIN > 0 ? CIN * KHW * KHW : a.taps * a.C;
            auto gather = [&](int k) {
                float v = 0.f;
                if (k < nk) {
                    const int tap = k / C, ci = k - tap * C;
                    const int ky = tap / KW, kx = tap - ky * KW;
                    if constexpr (XT) {
                        v = win[(ci * 10 + (tid >> 5) + ky) * kStemWinRow + ox + kx + 3];
                    } else {
                        const int iy = oy * a.stride - a.pad + ky, ix = ox * a.stride - a.pad + kx;
                        if ((unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W)
                            v = x[(((int64_t)b * C + ci) * a.H + iy) * a.W + ix];
                    }
                }
                return v;
            };
#pragma unroll
            for (int q = 0; q < kBK / 2; ++q) split2x2(gather(2 * q), gather(2 * q + 1), hw[q], lw[q]);
        }
#pragma unroll
        for (int q = 0; q < kBK / 8; ++q) {
            *reinterpret_cast<u32x4 *>(Bs + tid * kRowB + 16 * q) =
                u32x4{hw[4 * q], hw[4 * q + 1], hw[4 * q + 2], hw[4 * q + 3]};
            *reinterpret_cast<u32x4 *>(Bs + tid * kRowB + 2 * kBK + 16 * q) =
                u32x4{lw[4 * q], lw[4 * q + 1], lw[4 * q + 2], lw[4 * q + 3]};
        }
    }
    __syncthreads();
    WaveAcc acc;
    zero_acc(acc);
    const uint8_t *b0 = Bs + (wp * kWaveTile + r) * kRowB, *b1 = b0 + 32 * kRowB;
#pragma unroll
    for (int s = 0; s < kBK / 16; ++s) {  // mfma_chunk's order: k-step, then tiles
        const int off = 32 * s + 16 * h;
        f[s].bh[0] = *reinterpret_cast<const bf16x8 *>(b0 + off);
        f[s].bl[0] = *reinterpret_cast<const bf16x8 *>(b0 + 2 * kBK + off);
        f[s].bh[1] = *reinterpret_cast<const bf16x8 *>(b1 + off);
        f[s].bl[1] = *reinterpret_cast<const bf16x8 *>(b1 + 2 * kBK + off);
        mfma_frag(acc, f[s]);
    }
    __syncthreads();  // the epilogue reuses the operands' LDS
    epilogue_lds<kWaveTile, BNP, NT, 2, WaveAcc, DLS_STEM_PIXSPLIT>(acc, smem, a, co0, pix0, 0, wp, tid);
    }
}

// fp32 NCHW image batch -> split NHWC with Cp >= C channels (zeros beyond C)
__global__ __launch_bounds__(256) void k_pack_input(const float *__restrict__ x, int64_t n, int C,
                                                   int HW, int Cp, uint16_t *__restrict__ y) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // (pixel, ci) with ci fastest
    if (i >= n) return;
    const int ci = (int)(i % Cp);
    const int64_t pix = i / Cp;
    const int64_t b = pix / HW, s = pix - b * HW;
    const float v = ci < C ? x[(b * C + ci) * HW + s] : 0.f;
    uint32_t hi, lo;
    split2(v, hi, lo);
    y[pix * 2 * Cp + ci] = (uint16_t)hi;
    y[pix * 2 * Cp + Cp + ci] = (uint16_t)lo;
}

// fp32 [Cout][Cin][KH][KW] -> split [Cout][2K]: k = (ky * KW + kx) * Cp + ci
// (per-tap channel runs padded to Cp), or with FLAT k = (ky * KW + kx) * Cin + ci
// for k < KH * KW * Cin, zero up to K (the im2col operand's order)
template <bool FLAT>
__global__ __launch_bounds__(256) void k_pack_weights(const float *__restrict__ w, int Cout, int Cin,
                                                     int KH, int KW, int K, int Cp,
                                                     uint16_t *__restrict__ y) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)Cout * K) return;
    const int co = (int)(i / K), k = (int)(i - (int64_t)co * K);
    const int cdiv = FLAT ? Cin : Cp;
    const int tap = k / cdiv, ci = k - tap * cdiv;
    const int ky = tap / KW, kx = tap - ky * KW;
    const bool live = FLAT ? k < KH * KW * Cin : ci < Cin;
    const float v = live ? w[(((int64_t)co * Cin + ci) * KH + ky) * KW + kx] : 0.f;
    uint32_t hi, lo;
    split2(v, hi, lo);
    y[(int64_t)co * 2 * K + k] = (uint16_t)hi;
    y[(int64_t)co * 2 * K + K + k] = (uint16_t)lo;
}

// im2col of an fp32 NCHW batch for a first layer with few input channels: split
// NHWC [B][Ho][Wo][2 Kp], k = (ky * KW + kx) * C + ci (zero outside the image and
// for k >= KH * KW * C); the convolution is then a 1x1 one with Kp channels
// (ResNet-18's 3-channel stem: 27 -> 32 instead of 9 taps x 32 padded channels).
__global__ __launch_bounds__(256) void k_pack_im2col(const float *__restrict__ x, int64_t n, int C, int H,
                                                    int W, int KH, int KW, int stride, int pad, int Ho,
                                                    int Wo, int Kp, uint16_t *__restrict__ y) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // (output pixel, k), k fastest
    if (i >= n) return;
    const int k = (int)(i % Kp);
    const int64_t pix = i / Kp;
    const int64_t hw = (int64_t)Ho * Wo;
    const int64_t b = pix / hw;
    const int rem = (int)(pix - b * hw);
    const int oy = rem / Wo, ox = rem - oy * Wo;
    const int tap = k / C, ci = k - tap * C;
    const int ky = tap / KW, kx = tap - ky * KW;
    const int iy = oy * stride - pad + ky, ix = ox * stride - pad + kx;
    float v = 0.f;
    if (k < KH * KW * C && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W)
        v = x[((b * C + ci) * H + iy) * W + ix];
    uint32_t hi, lo;
    split2(v, hi, lo);
    y[pix * 2 * Kp + k] = (uint16_t)hi;
    y[pix * 2 * Kp + Kp + k] = (uint16_t)lo;
}

// Global average pool + linear layer over split NHWC [B][HW][2C]: one block per
// image, every sum in one fixed order (per channel: pixels in order; per output:
// a fixed tree over the block) -> logits [B][O] fp32.
constexpr int kPoolBlock = 256;
__global__ __launch_bounds__(kPoolBlock) void k_pool_linear(const uint16_t *__restrict__ x, int HW, int C,
                                                            const float *__restrict__ wt,
                                                            const float *__restrict__ bias, int O,
                                                            float *__restrict__ out) {
    __shared__ float red[kPoolBlock];
    __shared__ float feat[2048];
    const int b = blockIdx.x, tid = threadIdx.x;
    const uint16_t *xb = x + (int64_t)b * HW * 2 * C;
    const float inv = 1.f / (float)HW;
    for (int c = tid; c < C; c += kPoolBlock) {
        float s = 0.f;
        for (int q = 0; q < HW; ++q)
            s += bf16_to_f32(xb[(int64_t)q * 2 * C + c]) + bf16_to_f32(xb[(int64_t)q * 2 * C + C + c]);
        feat[c] = s * inv;
    }
    __syncthreads();
    for (int o = 0; o < O; ++o) {
        float s = 0.f;
        for (int c = tid; c < C; c += kPoolBlock) s = __builtin_fmaf(feat[c], wt[(int64_t)o * C + c], s);
        red[tid] = s;
        __syncthreads();
        for (int k = kPoolBlock / 2; k > 0; k >>= 1) {
            if (tid < k) red[tid] += red[tid + k];
            __syncthreads();
        }
        if (tid == 0) out[(int64_t)b * O + o] = red[0] + (bias ? bias[o] : 0.f);
        __syncthreads();
    }
}

// The generic kernel's LDS form: 64-channel tiles (WCO = 1: 64 x 256 blocks)
// stage through one buffer (two barriers per chunk) and transpose their epilogue
// in two 32-channel passes, 46 instead of 92 KB per block (3 blocks per CU
// instead of 1): the 32 -> 64-channel 1x1 convolution over the stem's im2col
// 223 -> 153 us per 1000 images.  The 128-channel tiles keep double-buffered
// staging and one epilogue pass (74 KB, 2 blocks per CU): their lean form,
// 37 KB and 4 blocks per CU, made the stride-2 3x3 convolutions 2-3.5 % slower
// (profiles/r05_conv_probe.txt r05g)
template <int WCO, int WPIX>
int launch_conv(ConvArgs a, hipStream_t st) {
    constexpr int NBUF = WCO == 1 ? 1 : 2, NPASS = WCO == 1 ? 2 : 1;
    a.pix_tiles = (a.M + kWaveTile * WPIX - 1) / (kWaveTile * WPIX);
    a.co_tiles = a.Cout / (kWaveTile * WCO);
    const int64_t blocks = (int64_t)a.pix_tiles * a.co_tiles;
    if (blocks > INT32_MAX) {
        set_error("dls_conv_bn_act_split: %lld blocks", (long long)blocks);
        return DLS_EINVAL;
    }
    hipLaunchKernelGGL((k_conv_bf16x3<WCO, WPIX, NBUF, NPASS>), dim3((unsigned)blocks), dim3(64 * WCO * WPIX), 0,
                       st, a);
    return check_launch("dls_conv_bn_act_split");
}

// The halo kernel when the pixel tile can be whole output rows: returns 1 if
// launched (or the launch failed: rc set), 0 if the shape does not fit it.
template <int WCO, int WPIX, int NHMAX, bool SKEW>
int try_launch_halo(ConvArgs a, hipStream_t st, int &rc) {
    constexpr int BNP = kWaveTile * WPIX;
    constexpr int RPP = 64 * WCO * WPIX / (kBK / 4);
    const int H = a.H, W = a.W;
    if (W > BNP || BNP % W) return 0;
    const int TR = H < BNP / W ? H : BNP / W;
    int TI = 1;
    if (TR == H) {
        if (BNP % (H * W)) return 0;
        TI = BNP / (H * W);
    } else if (H % TR) {
        return 0;
    }
    const int NH = TI * (TR + 2) * (W + 2);
    if (NH > RPP * NHMAX) return 0;
    a.TI = TI;
    a.TR = TR;
    a.NH = NH;
    a.pix_tiles = (a.M + BNP - 1) / BNP;
    a.co_tiles = a.Cout / (kWaveTile * WCO);
    const int64_t blocks = (int64_t)a.pix_tiles * a.co_tiles;
    if (blocks > INT32_MAX) return 0;
    hipLaunchKernelGGL((k_conv3x3_halo<WCO, WPIX, NHMAX, SKEW>), dim3((unsigned)blocks), dim3(64 * WCO * WPIX), 0,
                       st, a);
    rc = check_launch("dls_conv_bn_act_split");
    return 1;
}

// The stride-2 phase pipeline (k_conv3x3s2_phase) when its phase halos fit NHI
// DMAs per wave
template <int WCO, int WPIX, int NHI>
int try_launch_phase(ConvArgs a, hipStream_t st, int &rc) {
    constexpr int BNP = kWaveTile * WPIX;
    const int H = a.H, W = a.W, Ho = a.Ho, Wo = a.Wo;
    if ((H | W) & 1 || 2 * Ho != H || 2 * Wo != W || 32 % Wo || a.Cout % (kWaveTile * WCO)) return 0;
    if ((int64_t)a.B * H * W >= (1ll << 30)) return 0;  // input pixel indices in 32 bits
    const int TR = Ho < BNP / Wo ? Ho : BNP / Wo;
    int TI = 1;
    if (TR == Ho) {
        if (BNP % (Ho * Wo)) return 0;
        TI = BNP / (Ho * Wo);
    } else if (Ho % TR) {
        return 0;
    }
    if (TR * Wo >= 32 ? (TR * Wo) % 64 : 32 % (TR * Wo)) return 0;
    const int NH = TI * (TR + 1) * Wo;
    if (NH > 8 * WCO * WPIX * NHI) return 0;
    a.TI = TI;
    a.TR = TR;
    a.NH = NH;
    a.pix_tiles = (a.M + BNP - 1) / BNP;
    a.co_tiles = a.Cout / (kWaveTile * WCO);
    const int64_t blocks = (int64_t)a.pix_tiles * a.co_tiles;
    if (blocks > INT32_MAX) return 0;
    hipLaunchKernelGGL((k_conv3x3s2_phase<WCO, WPIX, NHI>), dim3((unsigned)blocks), dim3(64 * WCO * WPIX), 0, st, a);
    rc = check_launch("dls_conv_bn_act_split");
    return 1;
}

// The LDS-DMA pipeline (k_conv3x3_pipe, or k_conv3x3_pipe16 with DLS_CONV_MF16)
// when the halo tile fits NHI DMAs per wave
template <int WCO, int WPIX, int NHI, int NHB = 2, int OCC = 1>
int try_launch_pipe(ConvArgs a, hipStream_t st, int &rc) {
    constexpr int BNP = kWaveTile * WPIX;
    const int H = a.H, W = a.W;
    if (32 % W) return 0;  // a wave's two 32-pixel tiles share their columns
    if ((int64_t)a.B * H * W >= (1ll << 28)) return 0;  // halo sources: input pixel * 8 + piece in 32 bits
    const int TR = H < BNP / W ? H : BNP / W;
    int TI = 1;
    if (TR == H) {
        if (BNP % (H * W)) return 0;
        TI = BNP / (H * W);
    } else if (H % TR) {
        return 0;
    }
    // pixel tile 1 = tile 0 + 32 pixels in the same image tile, or whole images on
    if (TR * W >= 32 ? (TR * W) % 64 : 32 % (TR * W)) return 0;
    const int NH = TI * (TR + 2) * W;  // halo rows without the padding columns
    if (NH > 8 * WCO * WPIX * NHI || a.Cout % (kWaveTile * WCO)) return 0;
    a.TI = TI;
    a.TR = TR;
    a.NH = NH;
    a.pix_tiles = (a.M + BNP - 1) / BNP;
    a.co_tiles = a.Cout / (kWaveTile * WCO);
    const int64_t blocks = (int64_t)a.pix_tiles * a.co_tiles;
    if (blocks > INT32_MAX) return 0;
    if (DLS_CONV_MF16)
        hipLaunchKernelGGL((k_conv3x3_pipe16<WCO, WPIX, NHI, NHB, OCC>), dim3((unsigned)blocks),
                           dim3(64 * WCO * WPIX), 0, st, a);
    else
        hipLaunchKernelGGL((k_conv3x3_pipe<WCO, WPIX, NHI, NHB, OCC>), dim3((unsigned)blocks),
                           dim3(64 * WCO * WPIX), 0, st, a);
    rc = check_launch("dls_conv_bn_act_split");
    return 1;
}

// The walk direction of a launch: the opposite of the one its input was
// written in (a launch records its output's), forwards for an input no recent
// launch wrote.  Performance only: no output depends on it.
struct WalkMemo {
    std::mutex m;
    const void *ptr[16] = {};
    int dir[16] = {};
    int next = 0;
};
WalkMemo g_walk;

int conv_walk_direction(const void *x) {
    if (!DLS_CONV_SERPENTINE) return 0;
    std::lock_guard<std::mutex> g(g_walk.m);
    for (int i = 0; i < 16; ++i)
        if (g_walk.ptr[i] == x) return !g_walk.dir[i];
    return 0;
}

void conv_record_walk(const void *y, int dir) {
    if (!DLS_CONV_SERPENTINE) return;
    std::lock_guard<std::mutex> g(g_walk.m);
    for (int i = 0; i < 16; ++i)
        if (g_walk.ptr[i] == y) {
            g_walk.dir[i] = dir;
            return;
        }
    g_walk.ptr[g_walk.next] = y;
    g_walk.dir[g_walk.next] = dir;
    g_walk.next = (g_walk.next + 1) & 15;
}

}  // namespace
}  // namespace dls

using namespace dls;

extern "C" {

int dls_conv_pack_input_f32(const float *x, int64_t B, int32_t C, int32_t H, int32_t W, int32_t Cp,
                            uint16_t *out, dls_stream_t stream) {
    DLS_REQUIRE(x && out, DLS_EINVAL, "dls_conv_pack_input_f32: null pointer");
    DLS_REQUIRE(B >= 0 && C > 0 && H > 0 && W > 0 && Cp >= C && Cp % 32 == 0, DLS_EINVAL,
                "dls_conv_pack_input_f32: B=%lld C=%d H=%d W=%d Cp=%d (Cp >= C, a multiple of 32)",
                (long long)B, C, H, W, Cp);
    const int64_t n = B * H * W * (int64_t)Cp;
    if (n == 0) return DLS_OK;
    hipLaunchKernelGGL(k_pack_input, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream),
                       x, n, (int)C, (int)(H * W), (int)Cp, out);
    return check_launch("dls_conv_pack_input_f32");
}

int dls_conv_pack_weights_f32(const float *w, int32_t Cout, int32_t Cin, int32_t KH, int32_t KW,
                              int32_t Cp, uint16_t *out, dls_stream_t stream) {
    DLS_REQUIRE(w && out, DLS_EINVAL, "dls_conv_pack_weights_f32: null pointer");
    DLS_REQUIRE(Cout > 0 && Cin > 0 && KH > 0 && KW > 0 && Cp >= Cin && Cp % 32 == 0 &&
                    (int64_t)KH * KW * Cp <= (1 << 24),
                DLS_EINVAL, "dls_conv_pack_weights_f32: Cout=%d Cin=%d KH=%d KW=%d Cp=%d", Cout, Cin,
                KH, KW, Cp);
    const int K = KH * KW * Cp;
    const int64_t n = (int64_t)Cout * K;
    hipLaunchKernelGGL(k_pack_weights<false>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       as_stream(stream), w, (int)Cout, (int)Cin, (int)KH, (int)KW, K, (int)Cp, out);
    return check_launch("dls_conv_pack_weights_f32");
}

int dls_conv_pack_weights_im2col_f32(const float *w, int32_t Cout, int32_t Cin, int32_t KH, int32_t KW,
                                     int32_t Kp, uint16_t *out, dls_stream_t stream) {
    DLS_REQUIRE(w && out, DLS_EINVAL, "dls_conv_pack_weights_im2col_f32: null pointer");
    DLS_REQUIRE(Cout > 0 && Cin > 0 && KH > 0 && KW > 0 && Kp >= KH * KW * Cin && Kp % 32 == 0 &&
                    Kp <= (1 << 24),
                DLS_EINVAL, "dls_conv_pack_weights_im2col_f32: Cout=%d Cin=%d KH=%d KW=%d Kp=%d", Cout,
                Cin, KH, KW, Kp);
    const int64_t n = (int64_t)Cout * Kp;
    hipLaunchKernelGGL(k_pack_weights<true>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       as_stream(stream), w, (int)Cout, (int)Cin, (int)KH, (int)KW, (int)Kp, (int)Kp, out);
    return check_launch("dls_conv_pack_weights_im2col_f32");
}

int dls_conv_pack_im2col_f32(const float *x, int64_t B, int32_t C, int32_t H, int32_t W, int32_t KH,
                             int32_t KW, int32_t stride, int32_t pad, int32_t Kp, uint16_t *out,
                             dls_stream_t stream) {
    DLS_REQUIRE(x && out, DLS_EINVAL, "dls_conv_pack_im2col_f32: null pointer");
    DLS_REQUIRE(B >= 0 && C > 0 && H > 0 && W > 0 && KH > 0 && KW > 0 && stride > 0 && pad >= 0 &&
                    H + 2 * pad >= KH && W + 2 * pad >= KW && Kp >= KH * KW * C && Kp % 32 == 0 &&
                    Kp <= (1 << 24),
                DLS_EINVAL, "dls_conv_pack_im2col_f32: B=%lld C=%d H=%d W=%d KH=%d KW=%d Kp=%d",
                (long long)B, C, H, W, KH, KW, Kp);
    const int Ho = (H + 2 * pad - KH) / stride + 1, Wo = (W + 2 * pad - KW) / stride + 1;
    const int64_t n = B * Ho * Wo * (int64_t)Kp;
    if (n == 0) return DLS_OK;
    hipLaunchKernelGGL(k_pack_im2col, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream),
                       x, n, (int)C, (int)H, (int)W, (int)KH, (int)KW, (int)stride, (int)pad, Ho, Wo,
                       (int)Kp, out);
    return check_launch("dls_conv_pack_im2col_f32");
}

int dls_conv_bn_act_split(const uint16_t *x, int64_t B, int32_t H, int32_t W, int32_t C,
                          const uint16_t *w, int32_t Cout, int32_t KH, int32_t KW, int32_t stride,
                          int32_t pad, const float *consts, const uint16_t *residual, int32_t relu,
                          uint16_t *y, dls_stream_t stream) {
    DLS_REQUIRE(x && w && y, DLS_EINVAL, "dls_conv_bn_act_split: null pointer");
    DLS_REQUIRE(B >= 0 && H > 0 && W > 0 && C >= 32 && C % 32 == 0 && Cout >= 64 && Cout % 64 == 0 &&
                    KH > 0 && KW > 0 && stride > 0 && pad >= 0 && H + 2 * pad >= KH &&
                    W + 2 * pad >= KW && (int64_t)KH * KW * C <= (1 << 24),
                DLS_EINVAL,
                "dls_conv_bn_act_split: B=%lld H=%d W=%d C=%d Cout=%d KH=%d KW=%d stride=%d pad=%d "
                "(C a multiple of 32, Cout of 64)",
                (long long)B, H, W, C, Cout, KH, KW, stride, pad);
    DLS_REQUIRE(aligned16(x) && aligned16(w) && aligned16(y) && (!consts || aligned16(consts)) &&
                    (!residual || aligned16(residual)),
                DLS_ELAYOUT, "dls_conv_bn_act_split: 16-byte alignment");
    const int Ho = (H + 2 * pad - KH) / stride + 1, Wo = (W + 2 * pad - KW) / stride + 1;
    const int64_t M = B * Ho * Wo;
    if (M == 0) return DLS_OK;
    // pixel indices are 32-bit inside the kernel; element offsets 64-bit
    DLS_REQUIRE(M <= INT32_MAX / 2 && B * H * W <= INT32_MAX / 2, DLS_EINVAL,
                "dls_conv_bn_act_split: %lld output pixels", (long long)M);
    ConvArgs a{x, w, consts, residual, y, (int)H, (int)W, (int)C, Ho, Wo, (int)Cout, (int)KW,
               (int)(KH * KW), (int)stride, (int)pad, (int)(KH * KW * C), (int)M, relu ? 1 : 0, 0, 0,
               (int)B, 0, 0, 0};
    a.rev = conv_walk_direction(x);
    conv_record_walk(y, a.rev);
    hipStream_t st = as_stream(stream);
    const bool wide = Cout % 128 == 0;
    // The kernel choice is a function of the shape alone (never of the process's
    // environment): a coalition's utility must be the same bits on every rank.
    // DLS_CONV_GENERIC_ONLY=1 (compile-time probe knob, tools/build_variants.py):
    // the generic kernel for every shape.
    if (!DLS_CONV_GENERIC_ONLY && KH == 3 && KW == 3 && stride == 1 && pad == 1) {
        int rc = DLS_OK;
        // the LDS-DMA pipelines (profiles/r06_conv_pipe_ab.txt): 128-channel
        // multiples 16 wide in 64-channel 4-wave blocks of one whole 16x16 image
        // (no halo rows re-read, half the weight bytes per MFMA), else in
        // 128-channel 4-wave one-halo-buffer blocks two per CU on images at least
        // 16 wide, else in 8-wave double-buffered ones (8x8, 4x4); 64 channels in
        // 4-wave one-halo-buffer blocks (32x32)
        const bool narrow = (W == 16 && (DLS_PIPE_NARROW & 1)) || (W == 8 && (DLS_PIPE_NARROW & 2)) ||
                            (W == 4 && (DLS_PIPE_NARROW & 4));
        if (DLS_CONV_PIPE && narrow &&
            (try_launch_pipe<1, 4, 10, 1, 2>(a, st, rc) || try_launch_pipe<1, 4, 12, 1, 2>(a, st, rc)))
            return rc;
        if (DLS_CONV_PIPE && wide &&
            ((W >= 16 && try_launch_pipe<2, 2, 5, 1, 2>(a, st, rc)) || try_launch_pipe<2, 4, 5>(a, st, rc) ||
             try_launch_pipe<2, 4, 6>(a, st, rc)))
            return rc;
        if (DLS_CONV_PIPE && !wide && try_launch_pipe<1, 4, 10, 1, 2>(a, st, rc)) return rc;
        const bool skew = W <= 16;
        const int hit = wide ? (skew ? try_launch_halo<2, 2, 9, true>(a, st, rc)
                                     : try_launch_halo<2, 2, 9, false>(a, st, rc))
                             : (skew ? try_launch_halo<1, 4, 11, true>(a, st, rc)
                                     : try_launch_halo<1, 4, 11, false>(a, st, rc));
        if (hit) return rc;
    }
    if (DLS_CONV_PHASE && !DLS_CONV_GENERIC_ONLY && KH == 3 && KW == 3 && stride == 2 && pad == 1 && wide) {
        int rc = DLS_OK;
        if (try_launch_phase<2, 4, 5>(a, st, rc)) return rc;
    }
    return wide ? launch_conv<2, 2>(a, st) : launch_conv<1, 4>(a, st);
}

int dls_conv_stem_bn_act_f32(const float *x, int64_t B, int32_t C, int32_t H, int32_t W, const uint16_t *w,
                             int32_t Cout, int32_t KH, int32_t KW, int32_t stride, int32_t pad,
                             const float *consts, int32_t relu, uint16_t *y, dls_stream_t stream) {
    DLS_REQUIRE(x && w && y, DLS_EINVAL, "dls_conv_stem_bn_act_f32: null pointer");
    DLS_REQUIRE(B >= 0 && C > 0 && H > 0 && W > 0 && KH > 0 && KW > 0 && KH * KW * C <= kBK &&
                    Cout >= 64 && Cout % 64 == 0 && stride > 0 && pad >= 0 && H + 2 * pad >= KH &&
                    W + 2 * pad >= KW,
                DLS_EINVAL,
                "dls_conv_stem_bn_act_f32: B=%lld C=%d H=%d W=%d Cout=%d KH=%d KW=%d (KH*KW*C <= %d, "
                "Cout a multiple of 64)",
                (long long)B, C, H, W, Cout, KH, KW, kBK);
    DLS_REQUIRE(aligned16(w) && aligned16(y) && (!consts || aligned16(consts)), DLS_ELAYOUT,
                "dls_conv_stem_bn_act_f32: 16-byte alignment");
    const int Ho = (H + 2 * pad - KH) / stride + 1, Wo = (W + 2 * pad - KW) / stride + 1;
    const int64_t M = B * Ho * Wo;
    if (M == 0) return DLS_OK;
    DLS_REQUIRE(M <= INT32_MAX / 2, DLS_EINVAL, "dls_conv_stem_bn_act_f32: %lld output pixels",
                (long long)M);
    constexpr int WPIX = 4;
    ConvArgs a{nullptr, w, consts, nullptr, y, (int)H, (int)W, (int)C, Ho, Wo, (int)Cout, (int)KW,
               (int)(KH * KW), (int)stride, (int)pad, kBK, (int)M, relu ? 1 : 0, 0, 0, (int)B, 0, 0, 0};
    conv_record_walk(y, 0);  // the stem walks forwards; the next layer backwards
    a.pix_tiles = (int)((M + kWaveTile * WPIX - 1) / (kWaveTile * WPIX));
    a.co_tiles = Cout / kWaveTile;
    const int64_t blocks = (int64_t)a.pix_tiles * a.co_tiles;
    DLS_REQUIRE(blocks <= INT32_MAX, DLS_EINVAL, "dls_conv_stem_bn_act_f32: %lld blocks", (long long)blocks);
    if (DLS_STEM_WINDOW && C == 3 && KH == 3 && KW == 3 && stride == 1 && pad == 1 && W == 32 && H % 8 == 0) {
        // the CIFAR ResNet stem, window staged in LDS, DLS_STEM_TILES pixel tiles per block
        constexpr int NTL = DLS_STEM_TILES;
        const int64_t walks = (int64_t)((a.pix_tiles + NTL - 1) / NTL) * a.co_tiles;
        hipLaunchKernelGGL((k_conv_stem<WPIX, 3, 3, true, NTL>), dim3((unsigned)walks), dim3(64 * WPIX), 0,
                           as_stream(stream), a, x);
    }
    else if (C == 3 && KH == 3 && KW == 3)
        hipLaunchKernelGGL((k_conv_stem<WPIX, 3, 3>), dim3((unsigned)blocks), dim3(64 * WPIX), 0,
                           as_stream(stream), a, x);
    else
        hipLaunchKernelGGL(k_conv_stem<WPIX>, dim3((unsigned)blocks), dim3(64 * WPIX), 0, as_stream(stream), a, x);
    return check_launch("dls_conv_stem_bn_act_f32");
}

int dls_pool_linear_split(const uint16_t *x, int64_t B, int32_t HW, int32_t C, const float *weight,
                          const float *bias, int32_t O, float *out, dls_stream_t stream) {
    DLS_REQUIRE(x && weight && out, DLS_EINVAL, "dls_pool_linear_split: null pointer");
    DLS_REQUIRE(B >= 0 && HW > 0 && C > 0 && C <= 2048 && O > 0, DLS_EINVAL,
                "dls_pool_linear_split: B=%lld HW=%d C=%d O=%d (C <= 2048)", (long long)B, HW, C, O);
    if (B == 0) return DLS_OK;
    hipLaunchKernelGGL(k_pool_linear, dim3((unsigned)B), dim3(kPoolBlock), 0, as_stream(stream), x,
                       (int)HW, (int)C, weight, bias, (int)O, out);
    return check_launch("dls_pool_linear_split");
}

}  // extern "C"

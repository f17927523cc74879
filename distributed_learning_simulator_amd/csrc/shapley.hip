// Shapley subset aggregation as an fp32 MFMA contraction, for gfx950.
//
// The Shapley servers build one subset model per evaluated coalition
// (servers/GTG_shapley_value_server.py:56, multiround_shapley_value_server.py:37),
// each a weighted mean of |S| client rows.  A batch of S coalitions is the dense
// product  out[S, P] = C[S, K] . U[K, P]  with c_si = n_i / N_S (0 if i not in S).
//
// Tiling (v_mfma_f32_32x32x2_f32, exact f32 in/out, 64 cycles/SIMD):
//   - a wave owns all S rows (MT x 32, MT <= 2) x 128 parameters, as 4 N-tiles
//     whose columns interleave by 4: N-tile n column j = parameter p0 + 4j + n.
//     So each k-step needs ONE 16-byte load per lane (U[row k][p0+4j .. +3]),
//     the 4 components feed the 4 N-tiles, and the accumulators come out with 4
//     consecutive parameters per lane -> 16-byte, fully coalesced stores;
//   - C is staged once per block into LDS transposed (Ct[k][i]), so each A
//     fragment is one conflict-free ds_read_b32;
//   - persistent grid, waves walk 128-parameter column tiles.
// Roofline: U is read once per S-chunk (K*P*4 B) and S*P*4 B written; 2*S*K*P
// flop.  For K = 50 the arithmetic intensity 2SK/(4(S+K)) stays below the
// fp32-MFMA ridge (157.3 TF / 8 TB/s = 19.7 flop/B) for every S, so it is
// HBM-bound and the MFMAs just keep the VALU free.
#include "dls_common.h"

namespace dls {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;
#ifndef DLS_GEMM_NT
#define DLS_GEMM_NT 4  // N-tiles (32 columns each) per wave: 16-byte (4) or 8-byte (2) loads
#endif
constexpr int kNT = DLS_GEMM_NT;
constexpr int kTileP = 32 * kNT;
typedef float f32xnt __attribute__((ext_vector_type(kNT)));
constexpr int kMaxK = 256;

template <int MT, bool BETA, int kDepth>
__global__ __launch_bounds__(kBlock) void k_subset_gemm(const float *__restrict__ C, int64_t ldc, int S, int K,
                                                        const float *__restrict__ U, int64_t ldu,
                                                        const int32_t *__restrict__ rows, int64_t P,
                                                        float *__restrict__ out, int64_t ldo,
                                                        int64_t ntiles) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int Kp = ((K + 1) / 2 + kDepth - 1) / kDepth * kDepth * 2;  // whole pipeline rounds
    float *Ct = smem;                                        // [Kp][32*MT]
    int32_t *srow = reinterpret_cast<int32_t *>(smem + Kp * 32 * MT);  // [Kp]
    for (int idx = threadIdx.x; idx < Kp * 32 * MT; idx += kBlock) {
        const int k = idx / (32 * MT), i = idx % (32 * MT);
        Ct[idx] = (k < K && i < S) ? C[(int64_t)i * ldc + k] : 0.f;
    }
    for (int k = threadIdx.x; k < Kp + 2 * kDepth; k += kBlock) srow[k] = k < K ? rows[k] : -1;
    __syncthreads();

    const int lane = __lane_id();
    const int h = lane >> 5, col = lane & 31;
    const int wave = threadIdx.x >> 6;
    const int64_t stride = (int64_t)gridDim.x * kWaves;
    int64_t tile = (int64_t)blockIdx.x * kWaves + wave;
    if (tile >= ntiles) return;
    const int nsteps = Kp / 2;  // multiple of kDepth

    // One flattened (tile, k-step) stream: the U loads of the next 4 k-steps are
    // in flight while the MFMAs of the current one run, and across a tile seam
    // they already fetch the next tile, so the epilogue stores overlap them.
    auto loadB = [&](int64_t t, int s) -> f32xnt {
        const int64_t pp = t * kTileP + kNT * col;
        const int32_t r = srow[2 * s + h];
        f32xnt b = f32xnt(0.f);
        if (r >= 0 && t < ntiles && pp + kNT <= P)
            b = __builtin_nontemporal_load(reinterpret_cast<const f32xnt *>(U + (int64_t)r * ldu + pp));
        return b;
    };
    f32xnt b[kDepth];
#pragma unroll
    for (int i = 0; i < kDepth; ++i) b[i] = loadB(tile, i);
    for (; tile < ntiles; tile += stride) {
        const int64_t p = tile * kTileP + kNT * col;  // this lane's kNT parameters
        const bool inb = p + kNT <= P;
        const int64_t next = tile + stride;
        f32x16 acc[MT][kNT];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
            for (int n = 0; n < kNT; ++n) {
                if (BETA && inb) {
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int row = 32 * mt + (r & 3) + 8 * (r >> 2) + 4 * h;
                        acc[mt][n][r] = row < S ? out[(int64_t)row * ldo + p + n] : 0.f;
                    }
                } else {
                    acc[mt][n] = f32x16{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f,
                                        0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
                }
            }
        }
        auto mma = [&](int s, const f32xnt &b) {
            const int k = 2 * s + h;
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) {
                const float a = Ct[k * 32 * MT + 32 * mt + col];
#pragma unroll
                for (int n = 0; n < kNT; ++n)
                    acc[mt][n] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b[n], acc[mt][n], 0, 0, 0);
            }
        };
        for (int s = 0; s < nsteps; s += kDepth) {
            const bool seam = s + kDepth >= nsteps;
            const int64_t lt = seam ? next : tile;
            const int ls = seam ? s + kDepth - nsteps : s + kDepth;
#pragma unroll
            for (int i = 0; i < kDepth; ++i) {
                mma(s + i, b[i]);
                b[i] = loadB(lt, ls + i);
            }
        }
        if (inb) {
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int row = 32 * mt + (r & 3) + 8 * (r >> 2) + 4 * h;
                    if (row < S) {
                        f32xnt v;
#pragma unroll
                        for (int n = 0; n < kNT; ++n) v[n] = acc[mt][n][r];
                        // non-temporal: the subset models stream out past the caches
                        // (measured 4 % faster with the U reads in flight)
                        __builtin_nontemporal_store(
                            v, reinterpret_cast<f32xnt *>(out + (int64_t)row * ldo + p));
                    }
                }
            }
        }
    }
}

template <int MT, bool BETA, int kDepth>
unsigned grid_blocks(int64_t ntiles, size_t lds) {
    // exactly the resident blocks (persistent): every wave gets ntiles/(blocks*4) tiles
    const int64_t cap =
        resident_blocks(reinterpret_cast<const void *>(k_subset_gemm<MT, BETA, kDepth>), kBlock, lds);
    const int64_t want = (ntiles + kWaves - 1) / kWaves;
    return (unsigned)(want < cap ? want : cap);
}

}  // namespace
}  // namespace dls

using namespace dls;

extern "C" int dls_subset_gemm_f32(const float *C, int32_t S, int32_t K, const float *U,
                                   int64_t ldu, const int32_t *rows, int64_t P, float *out,
                                   int64_t ldo, dls_stream_t stream) {
    DLS_REQUIRE(C && U && rows && out, DLS_EINVAL, "dls_subset_gemm_f32: null pointer");
    DLS_REQUIRE(S > 0 && K > 0 && P > 0, DLS_EINVAL, "dls_subset_gemm_f32: S=%d K=%d P=%lld", S, K,
                (long long)P);
    DLS_REQUIRE(P % 4 == 0 && ldu % 4 == 0 && ldo % 4 == 0 && aligned16(U) && aligned16(out),
                DLS_ELAYOUT, "dls_subset_gemm_f32: P, ldu, ldo multiples of 4; 16-byte alignment");
    hipStream_t st = as_stream(stream);
    const int64_t ntiles = (P + kTileP - 1) / kTileP;
    // S in chunks of 64 subsets (two 32-row MFMA tiles), K in chunks of 256 clients
    for (int s0 = 0; s0 < S; s0 += 64) {
        const int Sc = S - s0 < 64 ? S - s0 : 64;
        for (int k0 = 0; k0 < K; k0 += kMaxK) {
            const int Kc = K - k0 < kMaxK ? K - k0 : kMaxK;
            // pipeline depth (k-steps in flight) 4 or 5: whichever pads K less
            // (K = 50 -> 25 k-steps = 5 rounds of 5, no padded MFMAs)
            const int steps = (Kc + 1) / 2;
            const int depth = ((steps + 4) / 5 * 5 - steps) < ((steps + 3) / 4 * 4 - steps) ? 5 : 4;
            const int Kp = (steps + depth - 1) / depth * depth * 2;
            const int MT = Sc > 32 ? 2 : 1;
            const size_t lds =
                (size_t)Kp * 32 * MT * sizeof(float) + (size_t)(Kp + 2 * depth) * sizeof(int32_t);
            // C chunk: rows s0.., columns k0.. of the row-major [S, K] matrix (ld K)
            const float *Cc = C + (int64_t)s0 * K + k0;
            const int beta = k0 > 0;
            float *oc = out + (int64_t)s0 * ldo;
#define DLS_GEMM_LAUNCH(MT_, B_, D_)                                                            \
    hipLaunchKernelGGL((k_subset_gemm<MT_, B_, D_>), dim3(grid_blocks<MT_, B_, D_>(ntiles, lds)), \
                       dim3(kBlock), lds, st, Cc, (int64_t)K, Sc, Kc, U, ldu, rows + k0, P, oc,    \
                       ldo, ntiles)
#define DLS_GEMM_MT_BETA(D_)                    \
    if (MT == 2 && beta) DLS_GEMM_LAUNCH(2, true, D_);   \
    else if (MT == 2) DLS_GEMM_LAUNCH(2, false, D_);     \
    else if (beta) DLS_GEMM_LAUNCH(1, true, D_);         \
    else DLS_GEMM_LAUNCH(1, false, D_);
            if (depth == 5) {
                DLS_GEMM_MT_BETA(5)
            } else {
                DLS_GEMM_MT_BETA(4)
            }
#undef DLS_GEMM_MT_BETA
#undef DLS_GEMM_LAUNCH
            int rc = check_launch("dls_subset_gemm_f32");
            if (rc) return rc;
        }
    }
    return DLS_OK;
}

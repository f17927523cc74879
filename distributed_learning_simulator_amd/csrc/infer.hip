// Utility-evaluation inference helpers for gfx950 (SURVEY.md §8 row a-3:
// FedServer.get_metric, servers/fed_server.py:26-32, the Shapley servers'
// v(S) = accuracy of the subset model on the test set).
//
// Eval-mode batch norm over NHWC (channels_last) activations, fused with the
// residual add and the ReLU that follow it in a ResNet block:
//     y = act(fl(fl(x * alpha_c) + beta_c) [+ r])
// with ATen's CPU inference constants alpha_c = fl(invstd_c * w_c),
// beta_c = fl(b_c - fl(mean_c * alpha_c)), invstd_c = fl(1 / fl(sqrt(fl(var_c + eps)))).
// One HBM pass (8 B per element, 12 with the residual) instead of MIOpen's
// batch-norm kernel followed by separate add and clamp kernels (three passes;
// the batch-norm kernel alone ran at ~1.4 TB/s, profiles/r02a_kernel_stats_all.csv).
// HBM-bound: algorithmic bytes per launch = rows * C * (8 or 12).
#include "dls_common.h"

namespace dls {
namespace {

constexpr int kBnBlock = 256;
constexpr int kBnUnroll = 4;  // float4s per thread in flight

__global__ __launch_bounds__(kBnBlock) void k_bn_fold(const float *__restrict__ w,
                                                      const float *__restrict__ b,
                                                      const float *__restrict__ mean,
                                                      const float *__restrict__ var, float eps,
                                                      int C, float *__restrict__ alpha,
                                                      float *__restrict__ beta) {
    const int c = blockIdx.x * kBnBlock + threadIdx.x;
    if (c >= C) return;
    const float invstd = 1.f / sqrtf(var[c] + eps);  // -ffp-contract=off: each op rounds once
    const float a = w ? invstd * w[c] : invstd;
    alpha[c] = a;
    beta[c] = (b ? b[c] : 0.f) - mean[c] * a;
}

// FIXED: C/4 divides the grid's thread count, so a thread's channel group never
// changes and its (alpha, beta) stay in registers.
// y may alias x (the in-place call of the fused forward) or r: no __restrict__ on
// them; every element is read before its own store and by the same thread.
template <bool FIXED, bool RES, bool RELU>
__global__ __launch_bounds__(kBnBlock) void k_bn_act(const f32x4 *x, int64_t n4, int C4,
                                                     const f32x4 *__restrict__ alpha,
                                                     const f32x4 *__restrict__ beta,
                                                     const f32x4 *r, f32x4 *y) {
    const int64_t stride = (int64_t)gridDim.x * kBnBlock;
    int64_t i = (int64_t)blockIdx.x * kBnBlock + threadIdx.x;
    f32x4 a = {}, bb = {};
    if (FIXED) {
        const int cg = (int)(i % C4);
        a = alpha[cg];
        bb = beta[cg];
    }
    auto one = [&](f32x4 v, f32x4 rv, int64_t k) {
        f32x4 av = a, bv = bb;
        if (!FIXED) {
            const int cg = (int)(k % C4);
            av = alpha[cg];
            bv = beta[cg];
        }
        f32x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            float t = v[e] * av[e];
            t = t + bv[e];
            if (RES) t = t + rv[e];
            if (RELU) t = t > 0.f ? t : (t == t ? 0.f : t);  // relu keeps NaN, as torch
            o[e] = t;
        }
        return o;
    };
    for (; i + (kBnUnroll - 1) * stride < n4; i += kBnUnroll * stride) {
        f32x4 v[kBnUnroll], rv[kBnUnroll];
#pragma unroll
        for (int u = 0; u < kBnUnroll; ++u) {
            v[u] = __builtin_nontemporal_load(x + i + u * stride);
            if (RES) rv[u] = __builtin_nontemporal_load(r + i + u * stride);
        }
#pragma unroll
        for (int u = 0; u < kBnUnroll; ++u)
            y[i + u * stride] = one(v[u], RES ? rv[u] : f32x4{}, i + u * stride);
    }
    for (; i < n4; i += stride) {
        const f32x4 v = x[i];
        y[i] = one(v, RES ? r[i] : f32x4{}, i);
    }
}

// The same pass with the per-channel arithmetic of the GPU library the reference
// model's own eval forward runs on this stack (torch's eval BatchNorm2d goes to
// MIOpen's MIOpenBatchNormFwdInferSpatialEst: inhat = (x - mean) * invVariance,
// out = mad(scale, inhat, bias), invVariance = rsqrt(|var + eps|) per channel):
//     y = act(fma(w_c, fl(fl(x - mean_c) * iv_c), b_c) [+ r])
// consts = [mean | iv | w | b], C floats each (k_bn_fold_exact), iv by v_rsq_f32
// and the multiply-add fused, as that kernel compiles here: bit-identical to the
// module's forward (tests/test_gpu_infer.py; the correctly rounded 1/sqrt, or an
// unfused multiply-add, differ on 10-60 % of the elements), so the fused ResNet
// forward is the same function as model(x), one HBM pass per batch norm (+ the
// residual add and ReLU after it) instead of three.
__global__ __launch_bounds__(kBnBlock) void k_bn_fold_exact(const float *__restrict__ w,
                                                            const float *__restrict__ b,
                                                            const float *__restrict__ mean,
                                                            const float *__restrict__ var,
                                                            float eps, int C,
                                                            float *__restrict__ consts) {
    const int c = blockIdx.x * kBnBlock + threadIdx.x;
    if (c >= C) return;
    consts[c] = mean[c];
    consts[C + c] = __builtin_amdgcn_rsqf(fabsf(var[c] + eps));  // v_rsq_f32
    consts[2 * C + c] = w ? w[c] : 1.f;
    consts[3 * C + c] = b ? b[c] : 0.f;
}

template <bool FIXED, bool RES, bool RELU>
__global__ __launch_bounds__(kBnBlock) void k_bn_act_exact(const f32x4 *x, int64_t n4, int C4,
                                                           const f32x4 *__restrict__ consts,
                                                           const f32x4 *r, f32x4 *y) {
    const int64_t stride = (int64_t)gridDim.x * kBnBlock;
    int64_t i = (int64_t)blockIdx.x * kBnBlock + threadIdx.x;
    f32x4 m = {}, iv = {}, wv = {}, bv = {};
    auto consts_of = [&](int cg) {
        m = consts[cg];
        iv = consts[C4 + cg];
        wv = consts[2 * C4 + cg];
        bv = consts[3 * C4 + cg];
    };
    if (FIXED) consts_of((int)(i % C4));
    auto one = [&](f32x4 v, f32x4 rv, int64_t k) {
        if (!FIXED) consts_of((int)(k % C4));
        f32x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float h = (v[e] - m[e]) * iv[e];
            float t = __builtin_fmaf(wv[e], h, bv[e]);
            if (RES) t = t + rv[e];
            if (RELU) t = t > 0.f ? t : (t == t ? 0.f : t);  // relu keeps NaN, as torch
            o[e] = t;
        }
        return o;
    };
    for (; i + (kBnUnroll - 1) * stride < n4; i += kBnUnroll * stride) {
        f32x4 v[kBnUnroll], rv[kBnUnroll];
#pragma unroll
        for (int u = 0; u < kBnUnroll; ++u) {
            v[u] = __builtin_nontemporal_load(x + i + u * stride);
            if (RES) rv[u] = __builtin_nontemporal_load(r + i + u * stride);
        }
#pragma unroll
        for (int u = 0; u < kBnUnroll; ++u)
            y[i + u * stride] = one(v[u], RES ? rv[u] : f32x4{}, i + u * stride);
    }
    for (; i < n4; i += stride) {
        const f32x4 v = x[i];
        y[i] = one(v, RES ? r[i] : f32x4{}, i);
    }
}

// The same pass over NCHW (contiguous) activations: a float4 holds 4 spatial
// positions of one (image, channel) plane (HW % 4 == 0), whose channel is
// (k / HW4) % C; shifts and masks when HW4 and C are powers of two.  MIOpen's
// deterministic convolutions exist for NCHW only (its NHWC ones fall back to a
// naive kernel, ~100x slower: profiles/r04q_eval_det.txt), so the Inferencer's
// reproducible path runs NCHW.
template <bool POW2, bool RES, bool RELU>
__global__ __launch_bounds__(kBnBlock) void k_bn_act_exact_nchw(const f32x4 *x, int64_t n4, int C,
                                                                int HW4, int sh, int cm,
                                                                const float *__restrict__ consts,
                                                                const f32x4 *r, f32x4 *y) {
    const int64_t stride = (int64_t)gridDim.x * kBnBlock;
    int64_t i = (int64_t)blockIdx.x * kBnBlock + threadIdx.x;
    auto one = [&](f32x4 v, f32x4 rv, int64_t k) {
        const int c = POW2 ? (int)((k >> sh) & cm) : (int)((k / HW4) % C);
        const float m = consts[c], iv = consts[C + c], wv = consts[2 * C + c],
                    bv = consts[3 * C + c];
        f32x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float h = (v[e] - m) * iv;
            float t = __builtin_fmaf(wv, h, bv);
            if (RES) t = t + rv[e];
            if (RELU) t = t > 0.f ? t : (t == t ? 0.f : t);  // relu keeps NaN, as torch
            o[e] = t;
        }
        return o;
    };
    for (; i + (kBnUnroll - 1) * stride < n4; i += kBnUnroll * stride) {
        f32x4 v[kBnUnroll], rv[kBnUnroll];
#pragma unroll
        for (int u = 0; u < kBnUnroll; ++u) {
            v[u] = __builtin_nontemporal_load(x + i + u * stride);
            if (RES) rv[u] = __builtin_nontemporal_load(r + i + u * stride);
        }
#pragma unroll
        for (int u = 0; u < kBnUnroll; ++u)
            y[i + u * stride] = one(v[u], RES ? rv[u] : f32x4{}, i + u * stride);
    }
    for (; i < n4; i += stride) {
        const f32x4 v = x[i];
        y[i] = one(v, RES ? r[i] : f32x4{}, i);
    }
}

// Planes whose size is not a multiple of 4 (e.g. a 7x7 layer3 plane of a 28x28
// input: ResNet-18's adaptive pooling takes any input size): one element per
// lane, the same arithmetic.
template <bool RES, bool RELU>
__global__ __launch_bounds__(kBnBlock) void k_bn_act_exact_nchw1(const float *x, int64_t n, int C,
                                                                 int64_t HW,
                                                                 const float *__restrict__ consts,
                                                                 const float *r, float *y) {
    const int64_t stride = (int64_t)gridDim.x * kBnBlock;
    for (int64_t i = (int64_t)blockIdx.x * kBnBlock + threadIdx.x; i < n; i += stride) {
        const int c = (int)((i / HW) % C);
        const float h = (x[i] - consts[c]) * consts[C + c];
        float t = __builtin_fmaf(consts[2 * C + c], h, consts[3 * C + c]);
        if (RES) t = t + r[i];
        if (RELU) t = t > 0.f ? t : (t == t ? 0.f : t);
        y[i] = t;
    }
}

}  // namespace
}  // namespace dls

using namespace dls;

extern "C" int dls_bn_act_exact_nchw_f32(const float *x, int64_t N, int32_t C, int64_t HW,
                                         const float *consts, const float *residual, int32_t relu,
                                         float *y, dls_stream_t stream) {
    DLS_REQUIRE(x && consts && y, DLS_EINVAL, "dls_bn_act_exact_nchw_f32: null pointer");
    DLS_REQUIRE(N > 0 && C > 0 && HW > 0 && HW / 4 < (1 << 30), DLS_EINVAL,
                "dls_bn_act_exact_nchw_f32: N=%lld C=%d HW=%lld", (long long)N, C, (long long)HW);
    if (HW % 4 != 0 || !aligned16(x) || !aligned16(y) || (residual && !aligned16(residual))) {
        const int64_t n = N * C * HW;
        int64_t blocks = (n + kBnBlock - 1) / kBnBlock;
        if (blocks > 65536) blocks = 65536;
        hipStream_t st1 = as_stream(stream);
        const bool res1 = residual != nullptr;
#define DLS_BN1(R_, A_)                                                                        \
    hipLaunchKernelGGL((k_bn_act_exact_nchw1<R_, A_>), dim3((unsigned)blocks), dim3(kBnBlock), 0, \
                       st1, x, n, (int)C, HW, consts, residual, y)
        if (res1) {
            if (relu) DLS_BN1(true, true); else DLS_BN1(true, false);
        } else {
            if (relu) DLS_BN1(false, true); else DLS_BN1(false, false);
        }
#undef DLS_BN1
        return check_launch("dls_bn_act_exact_nchw_f32");
    }
    const int64_t n4 = N * C * (HW / 4);
    const int HW4 = (int)(HW / 4);
    int64_t blocks = (n4 + (int64_t)kBnBlock * kBnUnroll - 1) / ((int64_t)kBnBlock * kBnUnroll);
    const int64_t cap = (int64_t)resident_blocks(reinterpret_cast<const void *>(
                                                     k_bn_act_exact_nchw<true, false, true>),
                                                 kBnBlock, 0) * 4;
    if (blocks > cap) blocks = cap;
    if (blocks < 1) blocks = 1;
    const bool pow2 = (HW4 & (HW4 - 1)) == 0 && (C & (C - 1)) == 0;
    int sh = 0;
    while ((1 << sh) < HW4) ++sh;
    const f32x4 *xv = reinterpret_cast<const f32x4 *>(x);
    const f32x4 *rv = reinterpret_cast<const f32x4 *>(residual);
    f32x4 *yv = reinterpret_cast<f32x4 *>(y);
    hipStream_t st = as_stream(stream);
    const dim3 grid((unsigned)blocks), block(kBnBlock);
    const bool res = residual != nullptr;
#define DLS_BNC(P_, R_, A_)                                                                    \
    hipLaunchKernelGGL((k_bn_act_exact_nchw<P_, R_, A_>), grid, block, 0, st, xv, n4, (int)C, \
                       HW4, sh, (int)C - 1, consts, rv, yv)
    if (pow2) {
        if (res) {
            if (relu) DLS_BNC(true, true, true); else DLS_BNC(true, true, false);
        } else {
            if (relu) DLS_BNC(true, false, true); else DLS_BNC(true, false, false);
        }
    } else {
        if (res) {
            if (relu) DLS_BNC(false, true, true); else DLS_BNC(false, true, false);
        } else {
            if (relu) DLS_BNC(false, false, true); else DLS_BNC(false, false, false);
        }
    }
#undef DLS_BNC
    return check_launch("dls_bn_act_exact_nchw_f32");
}

extern "C" int dls_bn_fold_exact_f32(const float *weight, const float *bias, const float *mean,
                                     const float *var, float eps, int32_t C, float *consts,
                                     dls_stream_t stream) {
    DLS_REQUIRE(mean && var && consts, DLS_EINVAL, "dls_bn_fold_exact_f32: null pointer");
    DLS_REQUIRE(C > 0, DLS_EINVAL, "dls_bn_fold_exact_f32: C=%d", C);
    hipLaunchKernelGGL(k_bn_fold_exact, dim3((unsigned)((C + kBnBlock - 1) / kBnBlock)),
                       dim3(kBnBlock), 0, as_stream(stream), weight, bias, mean, var, eps, (int)C,
                       consts);
    return check_launch("dls_bn_fold_exact_f32");
}

extern "C" int dls_bn_act_exact_nhwc_f32(const float *x, int64_t rows, int32_t C,
                                         const float *consts, const float *residual, int32_t relu,
                                         float *y, dls_stream_t stream) {
    DLS_REQUIRE(x && consts && y, DLS_EINVAL, "dls_bn_act_exact_nhwc_f32: null pointer");
    DLS_REQUIRE(rows > 0 && C > 0 && C % 4 == 0, DLS_EINVAL,
                "dls_bn_act_exact_nhwc_f32: rows=%lld C=%d (C a multiple of 4)", (long long)rows, C);
    DLS_REQUIRE(aligned16(x) && aligned16(y) && aligned16(consts) &&
                    (!residual || aligned16(residual)),
                DLS_ELAYOUT, "dls_bn_act_exact_nhwc_f32: 16-byte alignment");
    const int64_t n4 = rows * (C / 4);
    const int C4 = C / 4;
    int64_t blocks = (n4 + (int64_t)kBnBlock * kBnUnroll - 1) / ((int64_t)kBnBlock * kBnUnroll);
    const int64_t cap = (int64_t)resident_blocks(reinterpret_cast<const void *>(
                                                     k_bn_act_exact<true, false, true>),
                                                 kBnBlock, 0) * 4;
    if (blocks > cap) blocks = cap;
    if (blocks < 1) blocks = 1;
    const bool fixed = ((int64_t)kBnBlock * blocks) % C4 == 0;
    const f32x4 *xv = reinterpret_cast<const f32x4 *>(x);
    const f32x4 *cv = reinterpret_cast<const f32x4 *>(consts);
    const f32x4 *rv = reinterpret_cast<const f32x4 *>(residual);
    f32x4 *yv = reinterpret_cast<f32x4 *>(y);
    hipStream_t st = as_stream(stream);
    const dim3 grid((unsigned)blocks), block(kBnBlock);
    const bool res = residual != nullptr;
#define DLS_BNX(F_, R_, A_) \
    hipLaunchKernelGGL((k_bn_act_exact<F_, R_, A_>), grid, block, 0, st, xv, n4, C4, cv, rv, yv)
    if (fixed) {
        if (res) {
            if (relu) DLS_BNX(true, true, true); else DLS_BNX(true, true, false);
        } else {
            if (relu) DLS_BNX(true, false, true); else DLS_BNX(true, false, false);
        }
    } else {
        if (res) {
            if (relu) DLS_BNX(false, true, true); else DLS_BNX(false, true, false);
        } else {
            if (relu) DLS_BNX(false, false, true); else DLS_BNX(false, false, false);
        }
    }
#undef DLS_BNX
    return check_launch("dls_bn_act_exact_nhwc_f32");
}

extern "C" int dls_bn_fold_f32(const float *weight, const float *bias, const float *mean,
                               const float *var, float eps, int32_t C, float *alpha, float *beta,
                               dls_stream_t stream) {
    DLS_REQUIRE(mean && var && alpha && beta, DLS_EINVAL, "dls_bn_fold_f32: null pointer");
    DLS_REQUIRE(C > 0, DLS_EINVAL, "dls_bn_fold_f32: C=%d", C);
    hipLaunchKernelGGL(k_bn_fold, dim3((unsigned)((C + kBnBlock - 1) / kBnBlock)), dim3(kBnBlock),
                       0, as_stream(stream), weight, bias, mean, var, eps, (int)C, alpha, beta);
    return check_launch("dls_bn_fold_f32");
}

extern "C" int dls_bn_act_nhwc_f32(const float *x, int64_t rows, int32_t C, const float *alpha,
                                   const float *beta, const float *residual, int32_t relu,
                                   float *y, dls_stream_t stream) {
    DLS_REQUIRE(x && alpha && beta && y, DLS_EINVAL, "dls_bn_act_nhwc_f32: null pointer");
    DLS_REQUIRE(rows > 0 && C > 0 && C % 4 == 0, DLS_EINVAL,
                "dls_bn_act_nhwc_f32: rows=%lld C=%d (C a multiple of 4)", (long long)rows, C);
    DLS_REQUIRE(aligned16(x) && aligned16(y) && aligned16(alpha) && aligned16(beta) &&
                    (!residual || aligned16(residual)),
                DLS_ELAYOUT, "dls_bn_act_nhwc_f32: 16-byte alignment");
    const int64_t n4 = rows * (C / 4);
    const int C4 = C / 4;
    // a few resident generations of blocks, each thread kBnUnroll float4s deep
    int64_t blocks = (n4 + (int64_t)kBnBlock * kBnUnroll - 1) / ((int64_t)kBnBlock * kBnUnroll);
    const int64_t cap = (int64_t)resident_blocks(reinterpret_cast<const void *>(
                                                     k_bn_act<true, false, true>),
                                                 kBnBlock, 0) * 4;
    if (blocks > cap) blocks = cap;
    if (blocks < 1) blocks = 1;
    const bool fixed = ((int64_t)kBnBlock * blocks) % C4 == 0;
    const f32x4 *xv = reinterpret_cast<const f32x4 *>(x);
    const f32x4 *av = reinterpret_cast<const f32x4 *>(alpha);
    const f32x4 *bv = reinterpret_cast<const f32x4 *>(beta);
    const f32x4 *rv = reinterpret_cast<const f32x4 *>(residual);
    f32x4 *yv = reinterpret_cast<f32x4 *>(y);
    hipStream_t st = as_stream(stream);
    const dim3 grid((unsigned)blocks), block(kBnBlock);
#define DLS_BN(F_, R_, A_) \
    hipLaunchKernelGGL((k_bn_act<F_, R_, A_>), grid, block, 0, st, xv, n4, C4, av, bv, rv, yv)
    const bool res = residual != nullptr;
    if (fixed) {
        if (res) {
            if (relu) DLS_BN(true, true, true); else DLS_BN(true, true, false);
        } else {
            if (relu) DLS_BN(true, false, true); else DLS_BN(true, false, false);
        }
    } else {
        if (res) {
            if (relu) DLS_BN(false, true, true); else DLS_BN(false, true, false);
        } else {
            if (relu) DLS_BN(false, false, true); else DLS_BN(false, false, false);
        }
    }
#undef DLS_BN
    return check_launch("dls_bn_act_nhwc_f32");
}

/*
 * dls_hip.h — C-ABI of libdls_hip.so, the MI355X (gfx950) implementation of the
 * server-side aggregation hot path of chen-zichen/distributed_learning_simulator.
 *
 * Every entry point replaces one reference hook (file:line in the reference
 * repository) and is called from the Python host layer
 * (distributed_learning_simulator_amd/_native.py, via ctypes).
 *
 * Contract:
 *   - plain pointers and sizes; every array argument is DEVICE memory owned by
 *     the caller (allocated by torch); nothing is retained after return;
 *   - `stream` is a hipStream_t passed as void*; every launch is asynchronous on
 *     it; no entry point synchronises, allocates or frees (graph-capturable);
 *   - return 0 on success, a negative DLS_E* code for a bad argument, or a
 *     positive hipError_t; dls_last_error() then describes it (thread-local);
 *   - all entry points are re-entrant; nothing throws across the ABI.
 *
 * Flattened parameter layout ("flat rows"): a client's parameter dict is one row
 * of a client-major matrix, tensors concatenated in dict (named_parameters)
 * order, each tensor starting at a multiple of 64 elements; `ld*` is the row
 * stride in elements.
 */
#ifndef DLS_HIP_H
#define DLS_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DLS_ABI_VERSION 2

#define DLS_OK 0
#define DLS_EINVAL (-1)     /* bad size / null pointer / unsupported mode */
#define DLS_ELAYOUT (-2)    /* misaligned pointer or leading dimension */

/* FedAvg modes */
#define DLS_FEDAVG_EXACT 0  /* reference op order: acc (+)= fl(fl(x*n_i)/N) in client order; bit-exact */
#define DLS_FEDAVG_FMA 1    /* acc = fma(x, w_i, acc) with w_i = fl(n_i/N); normwise ~1e-7 */

/* Sign planes: parameters are grouped by 64; group g is two uint64 words,
 * word 2g = "positive" plane, word 2g+1 = "negative" plane, bit j of either
 * is parameter 64*g + j.  NaN sets both bits; parameters past P are 0.
 * A client row holds DLS_SIGN_WORDS(P) words (padded to whole 256-param
 * tiles, 8 words per tile). */
#define DLS_SIGN_TILE 256
#define DLS_SIGN_WORDS(P) ((((P) + 255) / 256) * 8)
/* Vote counts: #pos - #neg, plus DLS_SIGN_NAN_MARK if any counted client sent
 * NaN for that parameter; a count >= DLS_SIGN_NAN_MARK/2 decodes as "poisoned"
 * (vote 0), which survives an int32 sum over up to 127 ranks. */
#define DLS_SIGN_NAN_MARK (1 << 24)

typedef void *dls_stream_t;

const char *dls_last_error(void);
int dls_abi_version(void);
/* First 16 hex digits of the SHA-256 of the library's sources and headers
 * (the csrc .hip sources, csrc/dls_common.h, csrc/quant_common.h, include/dls_hip.h, concatenated in build
 * order), fixed at build time: ties a loaded library to its source tree. */
const char *dls_source_hash(void);
int dls_device_count(void);
/* 1 if the dequant kernels divide by `divisor` (= fl32(N), fed_server.py:60)
 * with the two-constant method q = fma(a, yh, RN(a*yl)) — proven correctly
 * rounded for this divisor by an exhaustive host-side mantissa check, cached —
 * and 0 if they use the 3-op Markstein correction.  Host only; no GPU needed. */
int dls_two_constant_division(float divisor);

/* ------------------------------------------------------------------ FedAvg
 * Replaces FedServer.get_subset_model (servers/fed_server.py:44-66) for a
 * non-empty subset.
 *   U      fp32 [*, ldu]    client rows (flat parameter layout)
 *   rows   int32 [K]        row of U for each client, in the reference's
 *                           iteration order (dict key order / subset tuple)
 *   weight fp32 [K]         fl32(n_i): the Python int sample counts as torch
 *                           converts them (fed_server.py:59)
 *   total  fl32(sum n_i)    (fed_server.py:51-53,60)
 *   out    fp32 [P]         out = first term, then += (fed_server.py:62-65)
 * P, ldu multiples of 4; U and out 16-byte aligned. */
int dls_fedavg_f32(const float *U, int64_t ldu, const int32_t *rows, const float *weight,
                   int32_t K, float total, int64_t P, int32_t mode, float *out,
                   dls_stream_t stream);

/* Batched subset aggregation in reference order: S subsets at once.
 * Subset s lists sub_rows[sub_off[s] .. sub_off[s+1]) with matching
 * sub_weight[], divisor sub_total[s]; result row s of out [S, ldo].
 * Replaces the get_subset_model calls of the Shapley servers
 * (servers/GTG_shapley_value_server.py:56, multiround_shapley_value_server.py:37). */
int dls_subset_fedavg_f32(const float *U, int64_t ldu, const int32_t *sub_off,
                          const int32_t *sub_rows, const float *sub_weight,
                          const float *sub_total, int32_t S, int64_t P, float *out,
                          int64_t ldo, dls_stream_t stream);

/* The same batch, reading each client row ONCE (the Shapley servers' default
 * path: servers/GTG_shapley_value_server.py:56 and
 * servers/multiround_shapley_value_server.py:37 call get_subset_model,
 * servers/fed_server.py:44-66, once per coalition; a batch's coalitions share
 * their clients).
 *   urows   int32 [Ku]   row of U of each client of the batch's union
 *   uweight fp32  [Ku]   fl32(n_j)
 *   member  uint64 [Ku]  bit s set iff client j belongs to coalition s
 *   sub_total fp32 [S]   fl32(N_s) of coalition s, a HOST array (the library
 *                        derives each coalition's division constants on the
 *                        host, cf. dls_two_constant_division); S <= DLS_SUBSET_UNION_MAX
 * Row s of out [S, ldo] is coalition s's weighted mean, its members summed in
 * union order: bit-exact with the reference when every coalition lists its
 * clients in the union's order (the caller orders the union so — sorted
 * worker-id tuples, as the Shapley servers pass them, always are).  A coalition
 * without members leaves its row undefined. */
#define DLS_SUBSET_UNION_MAX 64
int dls_subset_fedavg_union_f32(const float *U, int64_t ldu, const int32_t *urows,
                                const float *uweight, const uint64_t *member, int32_t Ku,
                                const float *sub_total, int32_t S, int64_t P, float *out,
                                int64_t ldo, dls_stream_t stream);

/* Subset aggregation as a dense fp32 MFMA contraction: out[S, P] = C[S, K] · U[rows, P]
 * (C row-major [S, K], c_si = n_i / N_S; rows[K] selects the K client rows of U).
 * fp32 in / fp32 accumulate (v_mfma_f32_32x32x2_f32): an fma chain in client
 * order, normwise ~1e-7 from the exact weighted mean. */
int dls_subset_gemm_f32(const float *C, int32_t S, int32_t K, const float *U, int64_t ldu,
                        const int32_t *rows, int64_t P, float *out, int64_t ldo,
                        dls_stream_t stream);

/* -------------------------------------------------------------- sign vote
 * Producer side of workers/sign_sgd_worker.py:44 (torch.sign) + the 16x smaller
 * wire format: pack fp32 vectors X [K, ldx] into planes [K, ldp] (ldp >=
 * DLS_SIGN_WORDS(P)).  Values other than -1, 0, +1, NaN are counted into
 * *nonternary (device int32, accumulated; caller zeroes it) when it is
 * non-null, because the vote of such inputs would differ from the reference's
 * fp32 sum. */
int dls_sign_pack_f32(const float *X, int64_t ldx, int32_t K, int64_t P, uint64_t *planes,
                      int64_t ldp, int32_t *nonternary, dls_stream_t stream);

/* SignSGDServer.__worker (servers/sign_sgd_server.py:12-21): counts[p] =
 * sum over the K client rows of (+1 pos, -1 neg, +NAN_MARK nan).  `rows` may be
 * NULL (rows 0..K-1).  counts may be all-reduced (int32 sum) across ranks. */
int dls_sign_vote_count(const uint64_t *planes, int64_t ldp, const int32_t *rows, int32_t K,
                        int64_t P, int32_t *counts, dls_stream_t stream);

/* counts -> torch.sign(sum) as fp32 {-1, +0, +1} (NaN-poisoned -> 0, as CPU
 * torch.sign(nan)), and optionally the vote packed in the plane format. */
int dls_sign_from_counts(const int32_t *counts, int64_t P, float *sign_out,
                         uint64_t *vote_planes, dls_stream_t stream);

/* Fused single-device vote: planes -> any of fp32 signs, int32 counts and the
 * vote packed in the plane format (DLS_SIGN_WORDS(P) words, NaN-poisoned and
 * tied parameters 0); NULL outputs are skipped, at least one must be given. */
int dls_sign_vote(const uint64_t *planes, int64_t ldp, const int32_t *rows, int32_t K, int64_t P,
                  int32_t *counts, float *sign_out, uint64_t *vote_planes, dls_stream_t stream);

/* Worker step, workers/sign_sgd_worker.py:32-44 fused: momentum / dampening /
 * nesterov on grad (buf updated in place; first=1 clones), torch.sign, pack to
 * planes, optional fp32 sign copy.  a = fl32(1 - dampening).  Writes exactly
 * 2*ceil(P/64) plane words, so one tensor can fill its slice of a shared row
 * (tensors start at multiples of 64 parameters). */
int dls_sign_sgd_direction(const float *grad, float *buf, int64_t P, float momentum,
                           float one_minus_dampening, int32_t nesterov, int32_t first,
                           uint64_t *planes, float *sign_out, dls_stream_t stream);

/* workers/sign_sgd_worker.py:48-57: p = fma(vote + wd*p, -lr, p) with the vote
 * read from packed planes (NaN-poisoned or tied -> 0). */
int dls_sign_sgd_apply(float *param, const uint64_t *vote_planes, int64_t P, float neg_lr,
                       float weight_decay, dls_stream_t stream);

/* ----------------------------------------------------------------- quant
 * Wave tile of the flattened parameter space for the fused dequant-FedAvg
 * kernels.  A tile lies inside one tensor; host code builds the table once per
 * layout, with the "fast" tiles first: int tiles (kind 1/2) whose real
 * elements all lie in channel chan0, grouped by 1 KiB slice count. */
typedef struct dls_qtile {
    int64_t dst;     /* first output element (flat layout offset, multiple of 16) */
    int64_t src;     /* first element within a client row of Q (kind 1/2) or F (kind 0) */
    int32_t len;     /* elements: <= 4096 for the grouped tiles, <= 1024 for the rest;
                        lanes cover 16-element chunks (lane l, KiB slice g: element
                        1024 g + 16 l) up to the next multiple of 64 (the rows are
                        padded to 64) and write 0 past len, so the output's row
                        padding is always zero */
    int32_t kind;    /* 0 = fp32 tensor, 1 = int8 per-channel, 2 = uint8 per-channel */
    int32_t chan0;   /* channel (index into the client's scale/zp row) of element 0 */
    int32_t row_len; /* elements per output channel */
    int32_t row_pos; /* position of element 0 inside its channel row */
    int32_t chan_end; /* one past the tensor's last channel (clamps padded tails) */
} dls_qtile;

/* FedQuantServer._process_client_parameter (servers/fed_quant_server.py:25-33)
 * fused into FedServer.get_subset_model (servers/fed_server.py:44-66):
 *   out[e] (+)= fl(fl(fl(fl(q - zp[c]) * scale[c]) * n_i) / N)  (int tensors)
 *   out[e] (+)= fl(fl(x * n_i) / N)                              (fp32 tensors)
 * bit-exact in client order.  Q int8/uint8 [*, ldq], F fp32 [*, ldf],
 * sz fp32 pairs (fl32(scale), zero_point): client row r, channel c at pair
 * r * sz_row + c * sz_chan (the store keeps them channel-major: sz_row = 1).
 * nfast: host array of DLS_QTILE_GROUPS counts; the table starts with
 * nfast[0..3] one-channel int tiles of 4, 3, 2, 1 KiB slices (every real
 * element in channel chan0), then nfast[4..7] multi-channel int tiles of 4, 3,
 * 2, 1 KiB slices (channel rows a multiple of 16 elements: no lane's 16-element
 * chunk straddles two channels; a tile spanning more than 4 channels takes the
 * per-client path), then nfast[8] fp32 tiles of <= 256 elements,
 * nfast[9] int tiles of <= 256 elements of tensors with channel rows of >= 4
 * elements (a lane's 4 elements span at most two channels); the remaining tiles
 * (len <= 1024) are int tiles of any shape (see dls_qtile). */
#define DLS_QTILE_GROUPS 10
int dls_dequant_fedavg(const dls_qtile *tiles, int32_t ntiles, const int32_t *nfast, const void *Q,
                       int64_t ldq, const float *F, int64_t ldf, const float *sz, int64_t sz_row,
                       int64_t sz_chan, const int32_t *rows, const float *weight, int32_t K,
                       float total, float *out, dls_stream_t stream);
/* The same with a mode (DLS_FEDAVG_EXACT: dls_dequant_fedavg, bit-exact;
 * DLS_FEDAVG_FMA: the int tiles of groups 0-7 accumulate out = fma(q - zp, c,
 * out) with one constant per (client, channel) c = fl(fl(scale * n_i) / N)
 * (q - zp exact) — a conversion and two packed ops per element pair instead of
 * the exact mode's six, a different rounding of each term: within the
 * north-star's 1e-6 FedAvg tolerance (normwise), not bit-exact; groups 8-9 and
 * the general tiles run their exact kernels.  Groups 0-7 run on one kernel in
 * launch pieces of one wave per SIMD, so the one-channel / lane split does not
 * matter here: the store's FMA table lane-tiles every int tensor whose channel
 * rows are a multiple of 16 elements, long rows included). */
int dls_dequant_fedavg_mode(const dls_qtile *tiles, int32_t ntiles, const int32_t *nfast,
                            const void *Q, int64_t ldq, const float *F, int64_t ldf,
                            const float *sz, int64_t sz_row, int64_t sz_chan, const int32_t *rows,
                            const float *weight, int32_t K, float total, int32_t mode, float *out,
                            dls_stream_t stream);

/* Per-segment min / max of x over [seg_off[s], seg_off[s+1]) (torch.aminmax);
 * seg_off is device int64 [nseg+1] with seg_off[nseg] == total.  NaNs are
 * ignored (fminf/fmaxf). */
int dls_segment_minmax_f32(const float *x, const int64_t *seg_off, int32_t nseg, float *mins,
                           float *maxs, int64_t total, dls_stream_t stream);

/* MinMaxObserver-style qparams on device (torch.ao _calculate_qparams, fp32):
 *   affine:    scale = max((max(hi,0) - min(lo,0)) / (qmax - qmin), eps),
 *              zp = clamp(qmin - rne(min(lo,0) / scale), qmin, qmax);
 *   symmetric: scale = max(max(-min(lo,0), max(hi,0)) / ((qmax - qmin) / 2), eps),
 *              zp = 0 (signed range) or (qmin + qmax + 1) / 2 (unsigned). */
int dls_qparams_minmax(const float *mins, const float *maxs, int32_t nseg, int32_t qmin,
                       int32_t qmax, int32_t symmetric, float *scale, int32_t *zp,
                       dls_stream_t stream);

/* Affine quantize per segment (torch quantize_per_tensor / _per_channel):
 * q = clamp(rne(x * fl(1/scale)) + zp, qmin, qmax) stored as one byte (int8 for
 * qmin < 0, else uint8); stochastic=1 replaces rne by floor(v + u),
 * u = counter-based uniform(seed, element) (parity unpinned).  deq (optional)
 * = fl(fl(q - zp) * scale), the client-side dequant formula. */
int dls_quantize_affine(const float *x, const int64_t *seg_off, int32_t nseg, const float *scale,
                        const int32_t *zp, int32_t qmin, int32_t qmax, void *q, float *deq,
                        int32_t stochastic, uint64_t seed, int64_t total, dls_stream_t stream);

/* ------------------------------------------------------- utility evaluation
 * Eval-mode batch norm for the Shapley servers' utility inference
 * (servers/fed_server.py:26-32 get_metric -> tester.inference()).
 * dls_bn_fold_f32: per channel alpha = fl(invstd * w), beta = fl(b - fl(mean * alpha)),
 * invstd = fl(1 / fl(sqrt(fl(var + eps)))) (ATen's CPU inference constants);
 * weight / bias may be null (affine=False: w = 1, b = 0).
 * dls_bn_act_nhwc_f32: y = fl(fl(x * alpha_c) + beta_c), then + residual (if
 * not null) and ReLU (if relu) over a channels_last [rows = N*H*W, C] fp32
 * tensor in one pass; C a multiple of 4, 16-byte aligned pointers; y may
 * alias x. */
int dls_bn_fold_f32(const float *weight, const float *bias, const float *mean, const float *var,
                    float eps, int32_t C, float *alpha, float *beta, dls_stream_t stream);
int dls_bn_act_nhwc_f32(const float *x, int64_t rows, int32_t C, const float *alpha,
                        const float *beta, const float *residual, int32_t relu, float *y,
                        dls_stream_t stream);
/* The same pass with the GPU library's eval batch-norm arithmetic (the reference
 * model's own eval forward on this stack runs MIOpen's
 * MIOpenBatchNormFwdInferSpatialEst): y = fma(w_c, fl(fl(x - mean_c) * iv_c), b_c),
 * iv_c = v_rsq_f32(|var_c + eps|), then + residual and ReLU as above: bit-identical
 * to torch's eval BatchNorm2d here.  dls_bn_fold_exact_f32 writes
 * consts = [mean | iv | w | b] (4*C floats, 16-byte aligned). */
int dls_bn_fold_exact_f32(const float *weight, const float *bias, const float *mean,
                          const float *var, float eps, int32_t C, float *consts,
                          dls_stream_t stream);
int dls_bn_act_exact_nhwc_f32(const float *x, int64_t rows, int32_t C, const float *consts,
                              const float *residual, int32_t relu, float *y, dls_stream_t stream);
/* The same exact pass over an NCHW (contiguous) [N, C, H, W] fp32 tensor, HW =
 * H*W (MIOpen's deterministic convolutions are NCHW ones: the reproducible
 * utility evaluation runs in that layout): float4 planes when HW is a multiple
 * of 4 and the pointers 16-byte aligned, one element per lane otherwise (any
 * input size: ResNet-18's adaptive pooling takes 28x28, whose layer3 planes are
 * 7x7).  y may alias x. */
int dls_bn_act_exact_nchw_f32(const float *x, int64_t N, int32_t C, int64_t HW,
                              const float *consts, const float *residual, int32_t relu, float *y,
                              dls_stream_t stream);

/* Deterministic convolutions of the utility evaluation (replace the tester's
 * torch / MIOpen conv2d in the model forward behind servers/fed_server.py:26-32;
 * csrc/conv.hip).  Every output is reduced in one fixed order by one wave: the
 * same inputs give the same bits in any process.  fp32 values are carried as
 * bf16 pairs (hi = rne(x), lo = rne(x - hi)), products as hi*hi + hi*lo + lo*hi
 * with fp32 accumulation.
 * "split NHWC" activation: uint16 [B][H][W][2C] (per pixel C hi, then C lo).
 * split weights: uint16 [Cout][2K] (K hi, then K lo), k = (ky*KW + kx)*Cp + ci.
 * dls_conv_pack_input_f32: NCHW fp32 [B][C][H][W] -> split NHWC with Cp channels
 * (Cp >= C, a multiple of 32; zeros beyond C).
 * dls_conv_pack_weights_f32: fp32 [Cout][Cin][KH][KW] -> split weights, Cp as above.
 * dls_conv_pack_im2col_f32 / dls_conv_pack_weights_im2col_f32: a first layer with
 * few input channels as a 1x1 convolution over its im2col: split NHWC
 * [B][Ho][Wo][2 Kp] / split weights [Cout][2 Kp], k = (ky*KW + kx)*C + ci, zero
 * for k >= KH*KW*C (Kp a multiple of 32).
 * dls_conv_bn_act_split: y = act(bn(conv(x, w)) [+ residual]) in split NHWC;
 * bn = the exact eval batch norm above (consts = [mean | iv | w | b], or null:
 * none); residual split NHWC of y's shape or null; relu 0/1.  C a multiple of
 * 32, Cout of 64; 16-byte aligned pointers; y must not alias x or residual.
 * dls_conv_stem_bn_act_f32: the same for a first layer whose reduction is one chunk
 * (KH*KW*C <= 32: a 3-channel 3x3 stem), straight from the fp32 NCHW image batch
 * (the im2col fused), w from dls_conv_pack_weights_im2col_f32 (Kp = 32).
 * dls_pool_linear_split: logits[b][o] = sum_c mean_pixels(x[b])[c] * weight[o][c]
 * + bias[o] over a split NHWC [B][HW][2C] activation (C <= 2048; bias may be
 * null), every sum in a fixed order. */
int dls_conv_pack_input_f32(const float *x, int64_t B, int32_t C, int32_t H, int32_t W, int32_t Cp,
                            uint16_t *out, dls_stream_t stream);
int dls_conv_pack_weights_f32(const float *w, int32_t Cout, int32_t Cin, int32_t KH, int32_t KW,
                              int32_t Cp, uint16_t *out, dls_stream_t stream);
int dls_conv_pack_im2col_f32(const float *x, int64_t B, int32_t C, int32_t H, int32_t W, int32_t KH,
                             int32_t KW, int32_t stride, int32_t pad, int32_t Kp, uint16_t *out,
                             dls_stream_t stream);
int dls_conv_pack_weights_im2col_f32(const float *w, int32_t Cout, int32_t Cin, int32_t KH, int32_t KW,
                                     int32_t Kp, uint16_t *out, dls_stream_t stream);
int dls_conv_bn_act_split(const uint16_t *x, int64_t B, int32_t H, int32_t W, int32_t C,
                          const uint16_t *w, int32_t Cout, int32_t KH, int32_t KW, int32_t stride,
                          int32_t pad, const float *consts, const uint16_t *residual, int32_t relu,
                          uint16_t *y, dls_stream_t stream);
int dls_conv_stem_bn_act_f32(const float *x, int64_t B, int32_t C, int32_t H, int32_t W, const uint16_t *w,
                             int32_t Cout, int32_t KH, int32_t KW, int32_t stride, int32_t pad,
                             const float *consts, int32_t relu, uint16_t *y, dls_stream_t stream);
int dls_pool_linear_split(const uint16_t *x, int64_t B, int32_t HW, int32_t C, const float *weight,
                          const float *bias, int32_t O, float *out, dls_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* DLS_HIP_H */

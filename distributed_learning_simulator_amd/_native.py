"""ctypes binding of libdls_hip.so (the C-ABI declared in include/dls_hip.h).

Every wrapper takes torch tensors that already live on the current HIP device,
passes raw pointers and the current stream to the library, and raises
``RuntimeError`` (with ``dls_last_error()``) on a non-zero status.  There is no
CPU or PyTorch fallback: if the library cannot be loaded, or a tensor is not on
the GPU, the call fails loudly.
"""
import ctypes
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DLS_HIP_LIB", os.path.join(_HERE, "libdls_hip.so"))

FEDAVG_EXACT = 0
FEDAVG_FMA = 1
SIGN_NAN_MARK = 1 << 24
QTILE_GROUPS = 10  # DLS_QTILE_GROUPS
SUBSET_UNION_MAX = 64  # DLS_SUBSET_UNION_MAX: coalitions per dls_subset_fedavg_union_f32 call


def sign_words(P):
    """uint64 words per client row of sign planes (DLS_SIGN_WORDS)."""
    return ((P + 255) // 256) * 8


def sign_row_pitch(P):
    """The row pitch (uint64 words) of a store of sign-plane rows: sign_words(P)
    rounded up to 128 bytes, so that every row starts on a cache line and the
    vote's 128-byte-aligned wave ranges never share a line (dls_sign_vote)."""
    return (sign_words(P) + 15) // 16 * 16


class QTile(ctypes.Structure):
    """struct dls_qtile (include/dls_hip.h)."""

    _fields_ = [
        ("dst", ctypes.c_int64),
        ("src", ctypes.c_int64),
        ("len", ctypes.c_int32),
        ("kind", ctypes.c_int32),
        ("chan0", ctypes.c_int32),
        ("row_len", ctypes.c_int32),
        ("row_pos", ctypes.c_int32),
        ("chan_end", ctypes.c_int32),
    ]


_i32, _i64, _f32, _p, _u64 = (ctypes.c_int32, ctypes.c_int64, ctypes.c_float, ctypes.c_void_p,
                              ctypes.c_uint64)

# name -> argtypes (restype int unless noted); mirrors include/dls_hip.h
SIGNATURES = {
    "dls_last_error": ([], ctypes.c_char_p),
    "dls_abi_version": ([], _i32),
    "dls_source_hash": ([], ctypes.c_char_p),
    "dls_device_count": ([], _i32),
    "dls_two_constant_division": ([_f32], _i32),
    "dls_fedavg_f32": ([_p, _i64, _p, _p, _i32, _f32, _i64, _i32, _p, _p], _i32),
    "dls_subset_fedavg_f32": ([_p, _i64, _p, _p, _p, _p, _i32, _i64, _p, _i64, _p], _i32),
    "dls_subset_fedavg_union_f32": ([_p, _i64, _p, _p, _p, _i32, _p, _i32, _i64, _p, _i64, _p],
                                    _i32),
    "dls_subset_gemm_f32": ([_p, _i32, _i32, _p, _i64, _p, _i64, _p, _i64, _p], _i32),
    "dls_sign_pack_f32": ([_p, _i64, _i32, _i64, _p, _i64, _p, _p], _i32),
    "dls_sign_vote_count": ([_p, _i64, _p, _i32, _i64, _p, _p], _i32),
    "dls_sign_from_counts": ([_p, _i64, _p, _p, _p], _i32),
    "dls_sign_vote": ([_p, _i64, _p, _i32, _i64, _p, _p, _p, _p], _i32),
    "dls_sign_sgd_direction": ([_p, _p, _i64, _f32, _f32, _i32, _i32, _p, _p, _p], _i32),
    "dls_sign_sgd_apply": ([_p, _p, _i64, _f32, _f32, _p], _i32),
    "dls_dequant_fedavg": ([_p, _i32, _p, _p, _i64, _p, _i64, _p, _i64, _i64, _p, _p, _i32, _f32,
                            _p, _p],
                           _i32),
    "dls_dequant_fedavg_mode": ([_p, _i32, _p, _p, _i64, _p, _i64, _p, _i64, _i64, _p, _p, _i32,
                                 _f32, _i32, _p, _p], _i32),
    "dls_segment_minmax_f32": ([_p, _p, _i32, _p, _p, _i64, _p], _i32),
    "dls_qparams_minmax": ([_p, _p, _i32, _i32, _i32, _i32, _p, _p, _p], _i32),
    "dls_quantize_affine": ([_p, _p, _i32, _p, _p, _i32, _i32, _p, _p, _i32, _u64, _i64, _p],
                            _i32),
    "dls_bn_fold_f32": ([_p, _p, _p, _p, _f32, _i32, _p, _p, _p], _i32),
    "dls_bn_act_nhwc_f32": ([_p, _i64, _i32, _p, _p, _p, _i32, _p, _p], _i32),
    "dls_bn_fold_exact_f32": ([_p, _p, _p, _p, _f32, _i32, _p, _p], _i32),
    "dls_bn_act_exact_nhwc_f32": ([_p, _i64, _i32, _p, _p, _i32, _p, _p], _i32),
    "dls_bn_act_exact_nchw_f32": ([_p, _i64, _i32, _i64, _p, _p, _i32, _p, _p], _i32),
    "dls_conv_pack_input_f32": ([_p, _i64, _i32, _i32, _i32, _i32, _p, _p], _i32),
    "dls_conv_pack_weights_f32": ([_p, _i32, _i32, _i32, _i32, _i32, _p, _p], _i32),
    "dls_conv_pack_im2col_f32": ([_p, _i64, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _p, _p],
                                 _i32),
    "dls_conv_pack_weights_im2col_f32": ([_p, _i32, _i32, _i32, _i32, _i32, _p, _p], _i32),
    "dls_conv_bn_act_split": ([_p, _i64, _i32, _i32, _i32, _p, _i32, _i32, _i32, _i32, _i32, _p, _p,
                               _i32, _p, _p], _i32),
    "dls_conv_stem_bn_act_f32": ([_p, _i64, _i32, _i32, _i32, _p, _i32, _i32, _i32, _i32, _i32, _p,
                                  _i32, _p, _p], _i32),
    "dls_pool_linear_split": ([_p, _i64, _i32, _i32, _p, _p, _i32, _p, _p], _i32),
}

_lib = None
_lock = threading.Lock()


def lib():
    """Load libdls_hip.so once (raises if it was not built)."""
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                if not os.path.exists(LIB_PATH):
                    raise RuntimeError(
                        f"libdls_hip.so not found at {LIB_PATH}; build it with "
                        "`make -C distributed_learning_simulator_amd/csrc` (no CPU fallback)")
                L = ctypes.CDLL(LIB_PATH)
                for name, (args, res) in SIGNATURES.items():
                    f = getattr(L, name)
                    f.argtypes = args
                    f.restype = res
                _lib = L
    return _lib


def _check(rc, name):
    if rc != 0:
        msg = lib().dls_last_error().decode(errors="replace")
        raise RuntimeError(f"{name} failed (status {rc}): {msg}")


def _ptr(t):
    if t is None:
        return None
    if not t.is_cuda:
        raise RuntimeError("libdls_hip: tensor is not on the GPU (no CPU fallback)")
    return ctypes.c_void_p(t.data_ptr())


def _stream(stream=None, like=None):
    """The given stream, else the current stream of `like`'s device (worker threads
    may run with another current device than the tensors they launch on)."""
    if stream is None:
        dev = like.device if like is not None and like.is_cuda else None
        stream = torch.cuda.current_stream(dev)
    return ctypes.c_void_p(stream.cuda_stream)


CSRC_HASHED = ["dls_runtime.hip", "fedavg.hip", "sign.hip", "quant.hip", "quant_fma.hip", "shapley.hip",
               "infer.hip", "conv.hip", "dls_common.h", "quant_common.h", os.path.join("..", "..", "include", "dls_hip.h")]


def source_hash():
    """SHA-256 prefix of the library sources in this tree (the Makefile's
    dls_source_hash recipe); compare with lib().dls_source_hash()."""
    import hashlib
    h = hashlib.sha256()
    for f in CSRC_HASHED:
        with open(os.path.join(_HERE, "csrc", f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def two_constant_division(divisor):
    """1 if the dequant kernels divide by fl32(divisor) with the two-constant method
    (proven correctly rounded for it by the library's exhaustive host check)."""
    return int(lib().dls_two_constant_division(float(divisor)))


def require_gpu():
    if not torch.cuda.is_available():
        raise RuntimeError("distributed_learning_simulator_amd needs a ROCm GPU (no CPU fallback)")
    lib()


# ---------------------------------------------------------------------- FedAvg
def fedavg(U, rows, weight, total, P, out, mode=FEDAVG_EXACT, stream=None):
    """servers/fed_server.py:44-66 over rows of U (see dls_fedavg_f32)."""
    assert U.dtype == torch.float32 and out.dtype == torch.float32
    assert rows.dtype == torch.int32 and weight.dtype == torch.float32
    _check(lib().dls_fedavg_f32(_ptr(U), U.stride(0), _ptr(rows), _ptr(weight), rows.numel(),
                                float(total), P, mode, _ptr(out), _stream(stream, U)),
           "dls_fedavg_f32")
    return out


def subset_fedavg(U, sub_off, sub_rows, sub_weight, sub_total, P, out, stream=None):
    S = sub_off.numel() - 1
    _check(lib().dls_subset_fedavg_f32(_ptr(U), U.stride(0), _ptr(sub_off), _ptr(sub_rows),
                                       _ptr(sub_weight), _ptr(sub_total), S, P, _ptr(out),
                                       out.stride(0), _stream(stream, U)), "dls_subset_fedavg_f32")
    return out


def subset_fedavg_union(U, urows, uweight, member, sub_total, P, out, stream=None):
    """S <= SUBSET_UNION_MAX coalitions over one client union, each client row read
    once (dls_subset_fedavg_union_f32); member: int64 [Ku] bit masks (device);
    sub_total: the S divisors fl32(N_s) (host: a sequence of numbers)."""
    assert urows.dtype == torch.int32 and uweight.dtype == torch.float32
    assert member.dtype == torch.int64
    tot = [float(x) for x in sub_total]
    S = len(tot)
    _check(lib().dls_subset_fedavg_union_f32(_ptr(U), U.stride(0), _ptr(urows), _ptr(uweight),
                                             _ptr(member), urows.numel(), (ctypes.c_float * S)(*tot),
                                             S, P, _ptr(out), out.stride(0), _stream(stream, U)),
           "dls_subset_fedavg_union_f32")
    return out


def subset_gemm(C, U, rows, P, out, stream=None):
    S, K = C.shape
    assert C.is_contiguous() and C.dtype == torch.float32
    _check(lib().dls_subset_gemm_f32(_ptr(C), S, K, _ptr(U), U.stride(0), _ptr(rows), P, _ptr(out),
                                     out.stride(0), _stream(stream, U)), "dls_subset_gemm_f32")
    return out


# ------------------------------------------------------------------------ sign
def sign_pack(X, P, planes, nonternary=None, stream=None):
    K = X.shape[0]
    _check(lib().dls_sign_pack_f32(_ptr(X), X.stride(0), K, P, _ptr(planes), planes.stride(0),
                                   _ptr(nonternary), _stream(stream, X)), "dls_sign_pack_f32")
    return planes


def sign_vote_count(planes, rows, K, P, counts, stream=None):
    _check(lib().dls_sign_vote_count(_ptr(planes), planes.stride(0), _ptr(rows), K, P,
                                     _ptr(counts), _stream(stream, planes)), "dls_sign_vote_count")
    return counts


def sign_from_counts(counts, P, sign_out=None, vote_planes=None, stream=None):
    _check(lib().dls_sign_from_counts(_ptr(counts), P, _ptr(sign_out), _ptr(vote_planes),
                                      _stream(stream, counts)), "dls_sign_from_counts")


def sign_vote(planes, rows, K, P, sign_out, counts=None, vote_planes=None, stream=None):
    """Fused vote (dls_sign_vote): any of fp32 signs, int32 counts, packed vote."""
    _check(lib().dls_sign_vote(_ptr(planes), planes.stride(0), _ptr(rows), K, P, _ptr(counts),
                               _ptr(sign_out), _ptr(vote_planes), _stream(stream, planes)),
           "dls_sign_vote")
    return sign_out


def sign_sgd_direction(grad, buf, momentum, one_minus_dampening, nesterov, first, planes,
                       sign_out=None, stream=None):
    P = grad.numel()
    _check(lib().dls_sign_sgd_direction(_ptr(grad), _ptr(buf), P, float(momentum),
                                        float(one_minus_dampening), int(bool(nesterov)),
                                        int(bool(first)), _ptr(planes), _ptr(sign_out),
                                        _stream(stream, grad)), "dls_sign_sgd_direction")


def sign_sgd_apply(param, vote_planes, neg_lr, weight_decay, stream=None):
    _check(lib().dls_sign_sgd_apply(_ptr(param), _ptr(vote_planes), param.numel(), float(neg_lr),
                                    float(weight_decay), _stream(stream, param)), "dls_sign_sgd_apply")


# ----------------------------------------------------------------------- quant
def dequant_fedavg(tiles, ntiles, nfast, Q, F, sz, rows, weight, total, out, sz_strides=None,
                   mode=FEDAVG_EXACT, stream=None):
    """nfast: the QTILE_GROUPS counts of grouped tiles at the head of the table
    (quant_store.QuantLayout.tiles()); sz: (scale, zero point) pairs;
    sz_strides = (row, channel) strides in pairs (default: a channel-major
    [C+1, capacity, 2] tensor)."""
    assert len(nfast) == QTILE_GROUPS
    nf = (ctypes.c_int32 * QTILE_GROUPS)(*[int(x) for x in nfast])
    if sz_strides is None:
        sz_strides = (sz.stride(1) // 2, sz.stride(0) // 2)
    _check(lib().dls_dequant_fedavg_mode(_ptr(tiles), ntiles, nf, _ptr(Q),
                                         Q.stride(0) if Q is not None else 0,
                                         _ptr(F), F.stride(0) if F is not None else 0, _ptr(sz),
                                         int(sz_strides[0]), int(sz_strides[1]), _ptr(rows),
                                         _ptr(weight), rows.numel(), float(total), int(mode),
                                         _ptr(out), _stream(stream, out)), "dls_dequant_fedavg")
    return out


def segment_minmax(x, seg_off, total, mins, maxs, stream=None):
    _check(lib().dls_segment_minmax_f32(_ptr(x), _ptr(seg_off), seg_off.numel() - 1, _ptr(mins),
                                        _ptr(maxs), total, _stream(stream, x)),
           "dls_segment_minmax_f32")


def qparams_minmax(mins, maxs, scale, zp, qmin=0, qmax=255, symmetric=False, stream=None):
    _check(lib().dls_qparams_minmax(_ptr(mins), _ptr(maxs), mins.numel(), qmin, qmax,
                                    int(bool(symmetric)), _ptr(scale), _ptr(zp),
                                    _stream(stream, mins)), "dls_qparams_minmax")


def quantize(x, seg_off, total, scale, zp, q, deq=None, qmin=0, qmax=255, stochastic=False,
             seed=0, stream=None):
    _check(lib().dls_quantize_affine(_ptr(x), _ptr(seg_off), seg_off.numel() - 1, _ptr(scale),
                                     _ptr(zp), qmin, qmax, _ptr(q), _ptr(deq),
                                     int(bool(stochastic)),
                                     ctypes.c_uint64(seed & 0xFFFFFFFFFFFFFFFF), total,
                                     _stream(stream, x)), "dls_quantize_affine")


def quantize_u8(x, seg_off, total, scale, zp, q, deq=None, stochastic=False, seed=0,
                stream=None):
    quantize(x, seg_off, total, scale, zp, q, deq, 0, 255, stochastic, seed, stream)


# ----------------------------------------------------------- utility evaluation
def bn_fold(bn, alpha, beta, stream=None):
    """Eval-mode constants of a BatchNorm module (dls_bn_fold_f32) into alpha, beta [C]."""
    _check(lib().dls_bn_fold_f32(_ptr(bn.weight), _ptr(bn.bias), _ptr(bn.running_mean),
                                 _ptr(bn.running_var), float(bn.eps), bn.num_features,
                                 _ptr(alpha), _ptr(beta), _stream(stream, alpha)),
           "dls_bn_fold_f32")


def bn_act_nhwc(x, alpha, beta, residual=None, relu=True, out=None, inplace=False, stream=None):
    """y = act(x * alpha + beta [+ residual]) over a channels_last [N, C, H, W] fp32
    activation in one pass (dls_bn_act_nhwc_f32); returns y (channels_last;
    x itself when inplace)."""
    N, C, H, W = x.shape
    cl = torch.channels_last
    if not x.is_contiguous(memory_format=cl) or (
            residual is not None and not residual.is_contiguous(memory_format=cl)):
        raise RuntimeError("bn_act_nhwc: activations must be channels_last contiguous")
    if out is None:
        out = x if inplace else torch.empty_like(x, memory_format=cl)
    _check(lib().dls_bn_act_nhwc_f32(_ptr(x), N * H * W, C, _ptr(alpha), _ptr(beta),
                                     _ptr(residual), int(bool(relu)), _ptr(out),
                                     _stream(stream, x)), "dls_bn_act_nhwc_f32")
    return out


def bn_fold_exact(bn, consts, stream=None):
    """The GPU library's eval batch-norm constants of a BatchNorm module into
    consts [4*C] = [mean | iv | w | b] (dls_bn_fold_exact_f32)."""
    _check(lib().dls_bn_fold_exact_f32(_ptr(bn.weight), _ptr(bn.bias), _ptr(bn.running_mean),
                                       _ptr(bn.running_var), float(bn.eps), bn.num_features,
                                       _ptr(consts), _stream(stream, consts)),
           "dls_bn_fold_exact_f32")


def bn_act_exact_nhwc(x, consts, residual=None, relu=True, out=None, inplace=False, stream=None):
    """y = act(fma(w, (x - mean) * iv, b) [+ residual]) over a channels_last
    [N, C, H, W] fp32 activation in one pass (dls_bn_act_exact_nhwc_f32)."""
    N, C, H, W = x.shape
    cl = torch.channels_last
    if not x.is_contiguous(memory_format=cl) or (
            residual is not None and not residual.is_contiguous(memory_format=cl)):
        raise RuntimeError("bn_act_exact_nhwc: activations must be channels_last contiguous")
    if out is None:
        out = x if inplace else torch.empty_like(x, memory_format=cl)
    _check(lib().dls_bn_act_exact_nhwc_f32(_ptr(x), N * H * W, C, _ptr(consts), _ptr(residual),
                                           int(bool(relu)), _ptr(out),
                                           _stream(stream, x)), "dls_bn_act_exact_nhwc_f32")
    return out


def bn_act_exact_nchw(x, consts, residual=None, relu=True, out=None, inplace=False, stream=None):
    """bn_act_exact_nhwc over an NCHW-contiguous [N, C, H, W] fp32 activation
    (dls_bn_act_exact_nchw_f32: float4 planes when H*W is a multiple of 4, one
    element per lane otherwise)."""
    N, C, H, W = x.shape
    if not x.is_contiguous() or (residual is not None and not residual.is_contiguous()):
        raise RuntimeError("bn_act_exact_nchw: activations must be NCHW contiguous")
    if out is None:
        out = x if inplace else torch.empty_like(x, memory_format=torch.contiguous_format)
    _check(lib().dls_bn_act_exact_nchw_f32(_ptr(x), N, C, H * W, _ptr(consts), _ptr(residual),
                                           int(bool(relu)), _ptr(out),
                                           _stream(stream, x)), "dls_bn_act_exact_nchw_f32")
    return out


def bn_act_exact(x, consts, residual=None, relu=True, out=None, inplace=False, stream=None):
    """The exact eval batch-norm pass in the activation's own layout: channels_last
    (NHWC) or contiguous (NCHW)."""
    if x.is_contiguous(memory_format=torch.channels_last) and not x.is_contiguous():
        return bn_act_exact_nhwc(x, consts, residual, relu, out, inplace, stream)
    return bn_act_exact_nchw(x, consts, residual, relu, out, inplace, stream)


# ------------------------------------------------ deterministic convolutions
# "split" tensors (csrc/conv.hip): an fp32 value as a bf16 pair (hi, lo), stored
# as int16 — activations [B, H, W, 2C] (per pixel C hi then C lo), weights
# [Cout, 2K] (K hi then K lo, k = (ky*KW + kx)*Cp + ci).

def _check_same_device(fn, x, **others):
    for name, t in others.items():
        if t is not None and t.device != x.device:
            raise RuntimeError(f"{fn}: {name} is on {t.device}, the input on {x.device}")


def _check_consts(fn, consts, cout, device):
    """Eval batch-norm constants [mean | iv | w | b] x Cout: the kernels read them as
    16-byte vectors at consts + t * Cout + co."""
    if consts is None:
        return
    if (consts.dtype != torch.float32 or consts.numel() != 4 * cout or not consts.is_contiguous()
            or consts.device != device):
        raise RuntimeError(f"{fn}: consts must be a contiguous fp32 tensor of 4 * Cout = {4 * cout} "
                           f"elements on {device}")


def _overlaps(a, b):
    """True if the storage ranges of a and b intersect."""
    a0 = a.data_ptr()
    b0 = b.data_ptr()
    return a0 < b0 + b.numel() * b.element_size() and b0 < a0 + a.numel() * a.element_size()


def split_channels(c):
    """The padded channel count of a split tensor: a multiple of 32."""
    return (int(c) + 31) // 32 * 32


def conv_pack_input(x, stream=None):
    """NCHW fp32 [B, C, H, W] -> split NHWC [B, H, W, 2 Cp] (zeros beyond C)."""
    if x.dtype != torch.float32 or x.dim() != 4 or not x.is_contiguous():
        raise RuntimeError("conv_pack_input: x must be a contiguous NCHW fp32 tensor")
    B, C, H, W = x.shape
    cp = split_channels(C)
    out = torch.empty((B, H, W, 2 * cp), dtype=torch.int16, device=x.device)
    _check(lib().dls_conv_pack_input_f32(_ptr(x), B, C, H, W, cp, _ptr(out), _stream(stream, x)),
           "dls_conv_pack_input_f32")
    return out


def conv_pack_weights(w, stream=None):
    """fp32 [Cout, Cin, KH, KW] -> split weights [Cout, 2K] with K = KH*KW*Cp."""
    w = w.detach()
    if w.dtype != torch.float32 or w.dim() != 4 or not w.is_contiguous():
        raise RuntimeError("conv_pack_weights: w must be a contiguous fp32 [Cout, Cin, KH, KW]")
    co, ci, kh, kw = w.shape
    cp = split_channels(ci)
    out = torch.empty((co, 2 * kh * kw * cp), dtype=torch.int16, device=w.device)
    _check(lib().dls_conv_pack_weights_f32(_ptr(w), co, ci, kh, kw, cp, _ptr(out),
                                           _stream(stream, w)), "dls_conv_pack_weights_f32")
    return out


def conv_pack_im2col(x, ksize, stride, pad, stream=None):
    """NCHW fp32 [B, C, H, W] -> the split NHWC im2col [B, Ho, Wo, 2 Kp] of a
    (KH, KW) convolution, Kp = KH*KW*C rounded up to 32: the operand of a 1x1
    conv_bn_act with conv_pack_weights_im2col weights (few-channel first layers)."""
    if x.dtype != torch.float32 or x.dim() != 4 or not x.is_contiguous():
        raise RuntimeError("conv_pack_im2col: x must be a contiguous NCHW fp32 tensor")
    B, C, H, W = x.shape
    kh, kw = ksize
    kp = split_channels(kh * kw * C)
    ho, wo = (H + 2 * pad - kh) // stride + 1, (W + 2 * pad - kw) // stride + 1
    out = torch.empty((B, ho, wo, 2 * kp), dtype=torch.int16, device=x.device)
    _check(lib().dls_conv_pack_im2col_f32(_ptr(x), B, C, H, W, kh, kw, stride, pad, kp, _ptr(out),
                                          _stream(stream, x)), "dls_conv_pack_im2col_f32")
    return out


def conv_pack_weights_im2col(w, stream=None):
    """fp32 [Cout, Cin, KH, KW] -> split weights [Cout, 2 Kp] in conv_pack_im2col's k order."""
    w = w.detach()
    if w.dtype != torch.float32 or w.dim() != 4 or not w.is_contiguous():
        raise RuntimeError("conv_pack_weights_im2col: w must be a contiguous fp32 [Cout, Cin, KH, KW]")
    co, ci, kh, kw = w.shape
    kp = split_channels(kh * kw * ci)
    out = torch.empty((co, 2 * kp), dtype=torch.int16, device=w.device)
    _check(lib().dls_conv_pack_weights_im2col_f32(_ptr(w), co, ci, kh, kw, kp, _ptr(out),
                                                  _stream(stream, w)), "dls_conv_pack_weights_im2col_f32")
    return out


def conv_bn_act(x, w, ksize, stride, pad, consts=None, residual=None, relu=True, out=None,
                stream=None):
    """y = act(bn(conv(x)) [+ residual]) over split NHWC activations
    (dls_conv_bn_act_split); w from conv_pack_weights, ksize = (KH, KW)."""
    B, H, W, c2 = x.shape
    kh, kw = ksize
    cout = w.shape[0]
    ho, wo = (H + 2 * pad - kh) // stride + 1, (W + 2 * pad - kw) // stride + 1
    if x.dtype != torch.int16 or w.dtype != torch.int16 or not (x.is_contiguous() and w.is_contiguous()):
        raise RuntimeError("conv_bn_act: split int16 contiguous operands expected")
    if w.shape[1] != kh * kw * c2:
        raise RuntimeError(f"conv_bn_act: weights {tuple(w.shape)} do not match input channels {c2 // 2}")
    _check_same_device("conv_bn_act", x, w=w)
    _check_consts("conv_bn_act", consts, cout, x.device)
    oshape = (B, ho, wo, 2 * cout)
    if residual is not None:
        if (tuple(residual.shape) != oshape or residual.dtype != torch.int16
                or not residual.is_contiguous()):
            raise RuntimeError("conv_bn_act: residual must be a contiguous split NHWC int16 tensor "
                               "of the output's shape")
        _check_same_device("conv_bn_act", x, residual=residual)
    if out is None:
        out = torch.empty(oshape, dtype=torch.int16, device=x.device)
    else:
        if tuple(out.shape) != oshape or out.dtype != torch.int16 or not out.is_contiguous():
            raise RuntimeError(f"conv_bn_act: out must be a contiguous int16 tensor of shape {oshape}")
        _check_same_device("conv_bn_act", x, out=out)
        for name, t in (("x", x), ("residual", residual)):
            if t is not None and _overlaps(out, t):
                raise RuntimeError(f"conv_bn_act: out must not alias {name}")
    _check(lib().dls_conv_bn_act_split(_ptr(x), B, H, W, c2 // 2, _ptr(w), cout, kh, kw, stride,
                                       pad, _ptr(consts), _ptr(residual), int(bool(relu)),
                                       _ptr(out), _stream(stream, x)), "dls_conv_bn_act_split")
    return out


def conv_stem_bn_act(x, w, ksize, stride, pad, consts=None, relu=True, stream=None):
    """A few-channel first layer straight from the NCHW fp32 batch x (the im2col
    fused; KH*KW*C <= 32): y = act(bn(conv(x))) split NHWC
    (dls_conv_stem_bn_act_f32); w from conv_pack_weights_im2col."""
    if x.dtype != torch.float32 or x.dim() != 4 or not x.is_contiguous():
        raise RuntimeError("conv_stem_bn_act: x must be a contiguous NCHW fp32 tensor")
    B, C, H, W = x.shape
    kh, kw = ksize
    cout = w.shape[0]
    if w.dtype != torch.int16 or w.shape[1] != 2 * 32 or not w.is_contiguous():
        raise RuntimeError("conv_stem_bn_act: w must be conv_pack_weights_im2col output with Kp = 32")
    _check_same_device("conv_stem_bn_act", x, w=w)
    _check_consts("conv_stem_bn_act", consts, cout, x.device)
    ho, wo = (H + 2 * pad - kh) // stride + 1, (W + 2 * pad - kw) // stride + 1
    out = torch.empty((B, ho, wo, 2 * cout), dtype=torch.int16, device=x.device)
    _check(lib().dls_conv_stem_bn_act_f32(_ptr(x), B, C, H, W, _ptr(w), cout, kh, kw, stride, pad,
                                          _ptr(consts), int(bool(relu)), _ptr(out),
                                          _stream(stream, x)), "dls_conv_stem_bn_act_f32")
    return out


def pool_linear(x, weight, bias=None, stream=None):
    """Global average pool + linear layer over a split NHWC activation -> fp32
    logits [B, O] (dls_pool_linear_split)."""
    B, H, W, c2 = x.shape
    if x.dtype != torch.int16 or not x.is_contiguous():
        raise RuntimeError("pool_linear: x must be a contiguous split NHWC int16 tensor")
    if (weight.dim() != 2 or weight.shape[1] != c2 // 2 or weight.dtype != torch.float32
            or not weight.is_contiguous()):
        raise RuntimeError("pool_linear: weight must be a contiguous [O, C] fp32 tensor")
    O = weight.shape[0]
    if bias is not None and (tuple(bias.shape) != (O,) or bias.dtype != torch.float32
                             or not bias.is_contiguous()):
        raise RuntimeError("pool_linear: bias must be a contiguous [O] fp32 tensor")
    _check_same_device("pool_linear", x, weight=weight, bias=bias)
    out = torch.empty((B, O), dtype=torch.float32, device=x.device)
    _check(lib().dls_pool_linear_split(_ptr(x), B, H * W, c2 // 2, _ptr(weight.detach()),
                                       _ptr(None if bias is None else bias.detach()), O, _ptr(out),
                                       _stream(stream, x)), "dls_pool_linear_split")
    return out


def split_to_f32(x):
    """hi + lo of a split NHWC tensor as fp32 NCHW (test / debugging helper)."""
    c = x.shape[-1] // 2
    u = x.to(torch.int32) & 0xFFFF
    f = (u << 16).view(torch.float32)
    return (f[..., :c] + f[..., c:]).permute(0, 3, 1, 2).contiguous()

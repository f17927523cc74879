"""signSGD majority vote and worker step — CPU restatement (TEST INFRASTRUCTURE).

Reference server: ``SignSGDServer.__worker``, servers/sign_sgd_server.py:12-21

    total = [sum(i) for i in zip(*sign_gradients)]      # :16  Python sum: 0 + s_0 + s_1 ...
    total[idx] = torch.sign(grad)                       # :17-18

Inputs are sign tensors (values -1, 0, +1), so the fp32 sums are exact integers
and the result is sign(count_pos - count_neg) in any order.  A NaN input
poisons the sum, and CPU ``torch.sign(nan)`` is 0.  Zero sums come out as +0.0
(``0 + x`` never yields -0.0).

Reference worker: ``SignSGDWorker.__get_gredient``, workers/sign_sgd_worker.py:19-58
(momentum / dampening / nesterov transform, ``torch.sign``, then the update
``p += -lr * (vote + wd * p)``).  torch's ``add(x, alpha=a)`` is one fused
multiply-add ``fma(x, fl32(a), self)`` on the CPU (checked against the golden
vectors).

Wire format of the packed planes (the HIP kernels' layout, include/dls_hip.h,
restated here so tests can check the packing bit-for-bit): parameters are
grouped by 64; group ``g`` is two uint64 words ``[pos_g, neg_g]`` and bit ``j``
of either is parameter ``64*g + j``; rows are padded to whole tiles of 256
parameters.  pos = (x > 0), neg = (x < 0); NaN sets both bits.
"""
import numpy as np

TILE = 256
NAN_MARK = 1 << 24  # added to a vote count per NaN-poisoned client


def pack_planes(x):
    """fp32 [P] -> uint64 [ceil(P/256) * 8] in the wire layout above."""
    x = np.asarray(x, dtype=np.float32)
    P = x.shape[0]
    T = (P + TILE - 1) // TILE
    xp = np.zeros(T * TILE, np.float32)
    xp[:P] = x
    nan = np.isnan(xp)
    pos = ((xp > 0) | nan).reshape(-1, 64).astype(np.uint64)
    neg = ((xp < 0) | nan).reshape(-1, 64).astype(np.uint64)
    weights = (np.uint64(1) << np.arange(64, dtype=np.uint64))
    out = np.zeros((pos.shape[0], 2), np.uint64)
    out[:, 0] = (pos * weights).sum(1, dtype=np.uint64)
    out[:, 1] = (neg * weights).sum(1, dtype=np.uint64)
    return out.reshape(-1)


def unpack_planes(planes, P):
    """uint64 planes -> fp32 {-1, 0, +1, nan} [P] (inverse of pack_planes)."""
    w = np.asarray(planes, np.uint64).reshape(-1, 2)
    sh = np.arange(64, dtype=np.uint64)
    pos = ((w[:, 0:1] >> sh) & np.uint64(1)).reshape(-1).astype(bool)
    neg = ((w[:, 1:2] >> sh) & np.uint64(1)).reshape(-1).astype(bool)
    out = pos.astype(np.float32) - neg.astype(np.float32)
    out[pos & neg] = np.nan
    return out[:P]


def vote_counts(S):
    """int32 counts = #pos - #neg (+ NAN_MARK if any client sent a NaN)."""
    S = np.asarray(S, dtype=np.float32)
    nan = np.isnan(S)
    pos = (S > 0).sum(0)
    neg = (S < 0).sum(0)
    return (pos - neg + NAN_MARK * nan.any(0)).astype(np.int32)


def vote_from_counts(c):
    c = np.asarray(c, dtype=np.int64)
    v = np.sign(c).astype(np.float32)
    v[c >= NAN_MARK // 2] = 0.0
    return v + np.float32(0.0)  # canonical +0.0


def majority_vote(S):
    """Restates servers/sign_sgd_server.py:16-18 over K stacked sign vectors."""
    S = np.asarray(S, dtype=np.float32)
    total = np.zeros(S.shape[1], np.float32) + S[0]
    for k in range(1, S.shape[0]):
        total = total + S[k]
    with np.errstate(invalid="ignore"):
        out = np.sign(total).astype(np.float32)
    out[np.isnan(total)] = 0.0
    return out + np.float32(0.0)


def worker_direction(g, buf, first, momentum, dampening, nesterov):
    """workers/sign_sgd_worker.py:32-42 -> (d_p, new_buf)  (C: oracle/c/oracle.c)."""
    from . import _c
    return _c.sign_direction(g, buf, first, momentum, dampening, nesterov)


def worker_sign(d):
    """workers/sign_sgd_worker.py:44 (torch.sign on CPU: nan -> 0)."""
    d = np.asarray(d, np.float32)
    s = np.sign(d).astype(np.float32)
    s[np.isnan(d)] = 0.0
    return s + np.float32(0.0)


def worker_apply(p, vote, lr, weight_decay):
    """workers/sign_sgd_worker.py:48-57: d = vote (+ wd*p); p += -lr * d."""
    from . import _c
    return _c.sign_apply(p, vote, lr, weight_decay)


def sign_vote_torch_cpu(sign_gradients):
    """The reference's own torch op sequence on the CPU (servers/sign_sgd_server.py:16-18):
    per tensor a Python ``sum`` over the clients' fp32 sign tensors, then ``torch.sign``.
    ``sign_gradients``: list (one per client) of lists of fp32 CPU tensors.  Timed by
    bench.py's CPU baseline; not used as a parity reference (majority_vote is)."""
    import torch
    total = [sum(i) for i in zip(*sign_gradients)]
    return [torch.sign(g) for g in total]

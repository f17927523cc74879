"""CPU test doubles for the HIP entry points — TEST INFRASTRUCTURE ONLY.

The product path has no CPU fallback (``_native`` raises without a GPU).  To
test the host logic (stores, round protocol, Shapley scheduling, sharding and
collectives over ``gloo``) on a CPU-only machine, ``install(monkeypatch)``
swaps the ``_native`` kernel wrappers for numpy restatements with the same
arithmetic (the oracle's semantics).  GPU tests never use this module.
"""
import numpy as np
import torch

from distributed_learning_simulator_amd import _native
from oracle import sign as osign


def _f32(t):
    return t.detach().cpu().numpy()


def fedavg(U, rows, weight, total, P, out, mode=0, stream=None):
    Un = _f32(U)
    rows = _f32(rows).astype(np.int64)
    w = _f32(weight).astype(np.float32)
    N = np.float32(total)
    acc = None
    for r, wk in zip(rows, w):
        x = Un[r, :P]
        t = (x * wk) / N if mode == 0 else x * (wk / N)
        acc = t if acc is None else (acc + t if mode == 0 else acc + t)
    out[:P].copy_(torch.from_numpy(acc.astype(np.float32)))
    return out


def subset_fedavg(U, sub_off, sub_rows, sub_weight, sub_total, P, out, stream=None):
    off = _f32(sub_off).astype(np.int64)
    rows = _f32(sub_rows)
    w = _f32(sub_weight)
    tot = _f32(sub_total)
    for s in range(len(off) - 1):
        fedavg(U, torch.from_numpy(rows[off[s]:off[s + 1]].copy()),
               torch.from_numpy(w[off[s]:off[s + 1]].copy()), float(tot[s]), P, out[s])
    return out


def subset_fedavg_union(U, urows, uweight, member, sub_total, P, out, stream=None):
    rows = _f32(urows).astype(np.int64)
    w = _f32(uweight)
    m = _f32(member).view(np.uint64)
    tot = np.asarray([float(x) for x in sub_total], np.float32)
    for s in range(tot.size):
        sel = [j for j in range(rows.size) if (int(m[j]) >> s) & 1]
        fedavg(U, torch.from_numpy(rows[sel].astype(np.int32)),
               torch.from_numpy(w[sel].copy()), float(tot[s]), P, out[s])
    return out


def subset_gemm(C, U, rows, P, out, stream=None):
    Cn = _f32(C).astype(np.float64)
    Un = _f32(U)[_f32(rows).astype(np.int64), :P].astype(np.float64)
    out[:, :P].copy_(torch.from_numpy((Cn @ Un).astype(np.float32)))
    return out


def sign_pack(X, P, planes, nonternary=None, stream=None):
    Xn = _f32(X)
    for k in range(Xn.shape[0]):
        row = osign.pack_planes(Xn[k, :P])
        planes[k, : row.size].copy_(torch.from_numpy(row.view(np.int64)))
    if nonternary is not None:
        v = Xn[:, :P]
        bad = ~(np.isin(v, [-1.0, 0.0, 1.0]) | np.isnan(v))
        nonternary += int(bad.sum())
    return planes


def sign_vote_count(planes, rows, K, P, counts, stream=None):
    w = _f32(planes).view(np.uint64)
    idx = range(K) if rows is None else _f32(rows).astype(np.int64)
    S = np.stack([osign.unpack_planes(w[r], P) for r in idx])
    counts.copy_(torch.from_numpy(osign.vote_counts(S)))
    return counts


def sign_from_counts(counts, P, sign_out=None, vote_planes=None, stream=None):
    v = osign.vote_from_counts(_f32(counts)[:P])
    if sign_out is not None:
        sign_out[:P].copy_(torch.from_numpy(v))
    if vote_planes is not None:
        row = osign.pack_planes(v)
        vote_planes[: row.size].copy_(torch.from_numpy(row.view(np.int64)))


def sign_vote(planes, rows, K, P, sign_out, counts=None, vote_planes=None, stream=None):
    c = torch.empty(P, dtype=torch.int32)
    sign_vote_count(planes, rows, K, P, c)
    if counts is not None:
        counts.copy_(c)
    sign_from_counts(c, P, sign_out, vote_planes)
    return sign_out


def dequant_fedavg(tiles, ntiles, nfast, Q, F, sz, rows, weight, total, out, sz_strides=None,
                   mode=0, stream=None):
    """dls_dequant_fedavg_mode driven by the tile table (so column sub-tables are
    honoured): per tile, the reference formula fl(fl(fl(fl(q - zp) * s) * n) / N)
    (fp32: fl(fl(x * n) / N)) summed in client order; FMA mode sums the same terms
    (numpy has no fused multiply-add; what the host tests check is the table and
    chunk plumbing, not the FMA rounding)."""
    from distributed_learning_simulator_amd.quant_store import QTILE_DTYPE
    t = _f32(tiles).view(QTILE_DTYPE)[:ntiles]
    Qn = _f32(Q) if Q is not None else None
    Fn = _f32(F) if F is not None else None
    szn = _f32(sz)
    if sz_strides is None:  # channel-major [C+1, capacity, 2]
        sz_row, sz_chan = sz.stride(1) // 2, sz.stride(0) // 2
    else:
        sz_row, sz_chan = sz_strides
    pairs = szn.reshape(-1, 2)
    rows = _f32(rows).astype(np.int64)
    w = _f32(weight).astype(np.float32)
    N = np.float32(total)
    for tt in t:  # only the tiles' elements are written (the rest of out may be on the wire)
        dst, src, ln, kind = int(tt["dst"]), int(tt["src"]), int(tt["len"]), int(tt["kind"])
        lenpad = -(-ln // 64) * 64
        acc = None
        for r, wk in zip(rows, w):
            if kind == 0:
                x = Fn[r, src:src + ln].astype(np.float32)
            else:
                q = Qn[r, src:src + ln]
                q = q.view(np.int8) if kind == 1 else q
                e = np.arange(ln)
                ch = np.minimum(int(tt["chan0"]) + (int(tt["row_pos"]) + e) // int(tt["row_len"]),
                                int(tt["chan_end"]) - 1)
                pr = pairs[r * sz_row + ch * sz_chan]
                x = ((q.astype(np.float32) - pr[:, 1]) * pr[:, 0]).astype(np.float32)
            term = (x * wk).astype(np.float32) / N
            acc = term if acc is None else (acc + term).astype(np.float32)
        o = np.zeros(lenpad, np.float32)
        o[:ln] = acc
        out[dst:dst + lenpad].copy_(torch.from_numpy(o))
    return out


def segment_minmax(x, seg_off, total, mins, maxs, stream=None):
    xn = _f32(x)
    off = _f32(seg_off).astype(np.int64)
    for s_ in range(off.size - 1):
        seg = xn[off[s_]:off[s_ + 1]]
        mins[s_] = float(np.nanmin(seg)) if seg.size else float("inf")
        maxs[s_] = float(np.nanmax(seg)) if seg.size else float("-inf")


def qparams_minmax(mins, maxs, scale, zp, qmin=0, qmax=255, symmetric=False, stream=None):
    from oracle import quant as oq
    assert not symmetric
    for i in range(mins.numel()):
        s_, z = oq.minmax_qparams(float(mins[i]), float(maxs[i]), qmin, qmax)
        scale[i] = float(s_)
        zp[i] = int(z)


def quantize_u8(x, seg_off, total, scale, zp, q, deq=None, stochastic=False, seed=0, stream=None):
    from oracle import quant as oq
    assert not stochastic
    xn = _f32(x)
    off = _f32(seg_off).astype(np.int64)
    qn = np.empty(xn.size, np.uint8)
    dn = np.empty(xn.size, np.float32)
    sc, zz = _f32(scale), _f32(zp)
    for s_ in range(off.size - 1):
        a, b = off[s_], off[s_ + 1]
        qs = oq.quantize_affine(xn[a:b], sc[s_], int(zz[s_]))
        qn[a:b] = qs
        dn[a:b] = oq.dequant_affine(qs, sc[s_], int(zz[s_]))
    q.copy_(torch.from_numpy(qn))
    if deq is not None:
        deq.copy_(torch.from_numpy(dn))


_DOUBLES = ("fedavg", "subset_fedavg", "subset_fedavg_union", "subset_gemm", "sign_pack",
            "sign_vote_count", "sign_from_counts", "sign_vote", "dequant_fedavg",
            "segment_minmax", "qparams_minmax", "quantize_u8")


def install(monkeypatch):
    monkeypatch.setattr(_native, "require_gpu", lambda: None)
    for name in _DOUBLES:
        monkeypatch.setattr(_native, name, globals()[name])


def install_global():
    """Same as install() for spawned processes (no pytest monkeypatch there)."""
    _native.require_gpu = lambda: None
    for name in _DOUBLES:
        setattr(_native, name, globals()[name])

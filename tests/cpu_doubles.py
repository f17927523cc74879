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


def install(monkeypatch):
    monkeypatch.setattr(_native, "require_gpu", lambda: None)
    for name in ("fedavg", "subset_fedavg", "subset_fedavg_union", "subset_gemm", "sign_pack",
                 "sign_vote_count", "sign_from_counts", "sign_vote"):
        monkeypatch.setattr(_native, name, globals()[name])


def install_global():
    """Same as install() for spawned processes (no pytest monkeypatch there)."""
    _native.require_gpu = lambda: None
    for name in ("fedavg", "subset_fedavg", "subset_fedavg_union", "subset_gemm", "sign_pack",
                 "sign_vote_count", "sign_from_counts", "sign_vote"):
        setattr(_native, name, globals()[name])

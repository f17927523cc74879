"""Device-resident client-update stores and the aggregation calls on them.

HBM layout:

* ``ClientUpdateStore.U``  fp32 [capacity, P]: one row per client, the flat
  parameter layout of ``layout.ParameterLayout`` (tensors in dict order, each
  64-element aligned).  A FedAvg round is one ``dls_fedavg_f32`` launch over K
  rows: K*P*4 bytes read once, P*4 written.
* ``ClientParameters`` keeps the reference's ``self.parameters`` mapping
  (servers/fed_server.py:15,69-73,87) — ``{worker_id: (n_i, dict)}`` in arrival
  order — but the dict values are views of the client's row in ``U``, so the
  reference hooks and user code still see per-tensor dicts.
"""
import heapq
import threading

import torch

from . import _native
from .layout import ParameterLayout


def _i32(xs, device):
    return torch.tensor(list(xs), dtype=torch.int32).to(device, non_blocking=True)


def _f32(xs, device):
    return torch.tensor(list(xs), dtype=torch.float32).to(device, non_blocking=True)


def union_order(subsets):
    """One client order that lists every subset's clients in that subset's own
    order (a topological merge of the subsets), or None if there is none (two
    subsets order a pair of clients differently, or a subset repeats a client).
    Ties go to the client seen first, so sorted subsets give the sorted union."""
    first, succ, indeg = {}, {}, {}
    for sub in subsets:
        if len(set(sub)) != len(sub):
            return None
        for c in sub:
            if c not in first:
                first[c] = len(first)
                succ[c] = set()
                indeg[c] = 0
        for a, b in zip(sub, sub[1:]):
            if b not in succ[a]:
                succ[a].add(b)
                indeg[b] += 1
    ready = [(first[c], c) for c in first if indeg[c] == 0]
    heapq.heapify(ready)
    order = []
    while ready:
        _, c = heapq.heappop(ready)
        order.append(c)
        for b in succ[c]:
            indeg[b] -= 1
            if indeg[b] == 0:
                heapq.heappush(ready, (first[b], b))
    return order if len(order) == len(first) else None


def union_batch(subsets, n_of_row, device):
    """Tables of dls_subset_fedavg_union_f32 for <= 64 subsets (row lists) over one
    union order: (urows int32, uweight fp32, member int64 masks) on the device and
    the divisors as a host list, or None when no common order exists."""
    order = union_order(subsets)
    if order is None:
        return None
    pos = {r: j for j, r in enumerate(order)}
    member = [0] * len(order)
    for s, sub in enumerate(subsets):
        for r in sub:
            member[pos[r]] |= 1 << s
    member = [m - (1 << 64) if m >= 1 << 63 else m for m in member]  # as int64
    totals = [float(sum(int(n_of_row[r]) for r in sub)) for sub in subsets]
    return (_i32(order, device), _f32([int(n_of_row[r]) for r in order], device),
            torch.tensor(member, dtype=torch.int64).to(device, non_blocking=True), totals)


class ClientUpdateStore:
    """``acquire_range = (lo, hi)``: this process's own clients take rows [lo, hi)
    only (a fixed block; the sharded Shapley servers all-gather every rank's block
    into the rest of ``U`` in place); rows outside it may be lent to other
    ranks' clients and are never put on the free list."""

    def __init__(self, layout: ParameterLayout, device, capacity=1, acquire_range=None):
        self.layout = layout
        self.device = torch.device(device)
        self.U = torch.zeros((max(1, capacity), layout.P), dtype=torch.float32, device=self.device)
        self._range = acquire_range
        lo, hi = acquire_range if acquire_range is not None else (0, self.U.shape[0])
        self._free = list(range(lo, hi))[::-1]
        self._lock = threading.Lock()

    @property
    def capacity(self):
        return self.U.shape[0]

    def acquire(self):
        with self._lock:
            if not self._free:
                if self._range is not None:
                    raise RuntimeError(f"all {self._range[1] - self._range[0]} rows of this "
                                       "rank's block are in use")
                old = self.U
                new_cap = max(2 * old.shape[0], 1)
                self.U = torch.zeros((new_cap, self.layout.P), dtype=torch.float32,
                                     device=self.device)
                self.U[: old.shape[0]].copy_(old)
                self._free = list(range(old.shape[0], new_cap))[::-1]
            return self._free.pop()

    def release(self, row):
        with self._lock:
            if self._range is None or self._range[0] <= row < self._range[1]:
                self._free.append(row)

    def write(self, row, parameter_dict):
        self.layout.copy_into(parameter_dict, self.U[row])

    def accepts(self, parameter_dict):
        return self.layout.matches(parameter_dict)

    def row(self, row):
        return self.U[row]

    def views(self, row):
        return self.layout.views(self.U[row])

    # ------------------------------------------------------------ aggregation
    def fedavg(self, rows, ns, mode=_native.FEDAVG_EXACT, out=None, total=None, cols=None):
        """Weighted mean of rows in the given order (servers/fed_server.py:44-66).

        ``total`` (default: sum of ``ns``) is the divisor N; a shard of a sharded
        round passes the global N and gets its partial sum.  ``cols = (c0, c1)``
        (multiples of 4) reduces only flat elements [c0, c1) into ``out`` (of that
        length); rows / ns may then be device int32 / fp32 tensors, reused across
        column ranges."""
        c0, c1 = cols if cols is not None else (0, self.layout.P)
        if out is None:
            out = torch.empty(c1 - c0, dtype=torch.float32, device=self.device)
        if total is None:
            total = sum(int(n) for n in ns)
        r = rows if torch.is_tensor(rows) else _i32(rows, self.device)
        w = ns if torch.is_tensor(ns) else _f32([int(n) for n in ns], self.device)
        _native.fedavg(self.U[:, c0:], r, w, float(total), c1 - c0, out, mode=mode)
        return out

    def subset_models(self, subsets, n_of_row, method="exact", out=None):
        """S subset models at once.  subsets: list of row lists (non-empty, in order)."""
        S = len(subsets)
        P = self.layout.P
        if out is None:
            out = torch.empty((S, P), dtype=torch.float32, device=self.device)
        if method == "exact" and all(subsets):
            # each client row read once per batch of <= 64 coalitions (the union
            # kernel), when one client order suits every coalition (always for the
            # Shapley servers' sorted tuples); else one coalition per grid row
            tables = [union_batch(subsets[c0:c0 + _native.SUBSET_UNION_MAX], n_of_row, self.device)
                      for c0 in range(0, S, _native.SUBSET_UNION_MAX)]
            if all(t is not None for t in tables):
                for i, t in enumerate(tables):
                    c0 = i * _native.SUBSET_UNION_MAX
                    _native.subset_fedavg_union(self.U, *t, P, out[c0:c0 + len(t[3])])
                return out
        if method == "exact":
            off, flat_rows, flat_w, totals = [0], [], [], []
            for sub in subsets:
                flat_rows.extend(sub)
                ws = [int(n_of_row[r]) for r in sub]
                flat_w.extend(ws)
                totals.append(float(sum(ws)))
                off.append(len(flat_rows))
            _native.subset_fedavg(self.U, _i32(off, self.device), _i32(flat_rows, self.device),
                                  _f32(flat_w, self.device), _f32(totals, self.device), P, out)
        elif method == "gemm":
            rows = sorted({r for sub in subsets for r in sub})
            col = {r: j for j, r in enumerate(rows)}
            C = torch.zeros((S, len(rows)), dtype=torch.float64)
            for s, sub in enumerate(subsets):
                tot = float(sum(int(n_of_row[r]) for r in sub))
                for r in sub:
                    C[s, col[r]] = int(n_of_row[r]) / tot
            _native.subset_gemm(C.float().to(self.device), self.U, _i32(rows, self.device), P, out)
        else:
            raise ValueError(f"unknown subset method {method!r}")
        return out


class SlicedClientUpdateStore:
    """Client rows stored slice-major for the bit-exact sharded FedAvg exchange
    (distributed.ShardedFedServer, exchange="alltoall"): the flat row is cut into
    ``world`` slices of L elements (distributed.slice_bounds) and ``B`` is fp32
    [world, capacity, L], so slice d of every client this rank holds is ONE
    contiguous block B[d] — the all-to-all sends straight from the store, one
    block per peer, with no per-client operation and no staging copy.  A
    client's dict is written tensor by tensor into its slices (a tensor that
    straddles a slice boundary is written in pieces); ``views`` returns views of
    the tensors that lie in one slice and copies of the (at most world - 1)
    straddling ones."""

    def __init__(self, layout: ParameterLayout, device, capacity, world, L):
        self.layout = layout
        self.device = torch.device(device)
        self.world, self.L = world, L
        self.B = torch.zeros((world, max(1, capacity), L), dtype=torch.float32, device=self.device)
        self._free = list(range(self.B.shape[1]))[::-1]
        self._lock = threading.Lock()

    @property
    def capacity(self):
        return self.B.shape[1]

    def acquire(self):
        with self._lock:
            if not self._free:
                old = self.B
                cap = 2 * old.shape[1]
                self.B = torch.zeros((self.world, cap, self.L), dtype=torch.float32,
                                     device=self.device)
                self.B[:, : old.shape[1]].copy_(old)
                self._free = list(range(old.shape[1], cap))[::-1]
            return self._free.pop()

    def release(self, row):
        with self._lock:
            self._free.append(row)

    def accepts(self, parameter_dict):
        return self.layout.matches(parameter_dict)

    def _pieces(self, o, m):
        """(slice, start in slice, start in tensor, length) of flat range [o, o+m)."""
        L, out, e = self.L, [], o
        while e < o + m:
            s, a = divmod(e, L)
            n = min(o + m - e, L - a)
            out.append((s, a, e - o, n))
            e += n
        return out

    def write(self, row, parameter_dict):
        dst, src = [], []
        for name, m, o in zip(self.layout.names, self.layout.numels, self.layout.offsets):
            t = parameter_dict[name].detach().reshape(-1)
            t = t if t.dtype == torch.float32 else t.float()
            for s, a, b, n in self._pieces(o, m):
                dst.append(self.B[s, row, a:a + n])
                src.append(t[b:b + n])
        torch._foreach_copy_(dst, src, non_blocking=True)

    def views(self, row):
        out = {}
        for name, shape, m, o in zip(self.layout.names, self.layout.shapes, self.layout.numels,
                                     self.layout.offsets):
            parts = [self.B[s, row, a:a + n] for s, a, _, n in self._pieces(o, m)]
            out[name] = (parts[0] if len(parts) == 1 else torch.cat(parts)).view(shape)
        return out

    def row(self, row):
        """The client's flat row (a copy: its slices are not contiguous)."""
        return self.B[:, row, :].reshape(-1)[: self.layout.P]


class ClientParameters(dict):
    """``self.parameters`` of the reference FedServer, backed by a ClientUpdateStore.

    ``params[worker_id] = (n, parameter_dict)`` copies the dict into the
    worker's row; ``params[worker_id]`` returns ``(n, dict of row views)``.
    """

    def __init__(self, store_factory):
        """store_factory(first_payload) -> store with acquire/release/write/views/accepts."""
        super().__init__()
        self._store_factory = store_factory
        self.store = None
        self._rows = {}

    def _ensure_store(self, parameter_dict):
        if self.store is None:
            self.store = self._store_factory(parameter_dict)
        elif not self.store.accepts(parameter_dict):
            raise ValueError("client parameter dict does not match the model layout")

    def __setitem__(self, worker_id, value):
        n, parameter_dict = value
        self._ensure_store(parameter_dict)
        row = self._rows.get(worker_id)
        if row is None:
            row = self.store.acquire()
            self._rows[worker_id] = row
        self.store.write(row, parameter_dict)
        super().__setitem__(worker_id, int(n))

    def __getitem__(self, worker_id):
        n = super().__getitem__(worker_id)
        return n, self.store.views(self._rows[worker_id])

    def __delitem__(self, worker_id):
        super().__delitem__(worker_id)
        self.store.release(self._rows.pop(worker_id))

    def items(self):
        return [(k, self[k]) for k in self.keys()]

    def values(self):
        return [self[k] for k in self.keys()]

    def pop(self, worker_id, *default):
        if worker_id not in self and default:
            return default[0]
        v = self[worker_id]
        del self[worker_id]
        return v

    def clear(self):
        for k in list(self.keys()):
            del self[k]

    def row_of(self, worker_id):
        return self._rows[worker_id]

    def adopt(self, entries):
        """Re-register the clients as [(worker_id, n, row)] in that order, for rows
        the store already holds (the sharded Shapley gather lands every rank's
        clients in place): no copy; rows this process did not acquire are never
        released to its free list (ClientUpdateStore.acquire_range)."""
        rows = {w: r for w, _, r in entries}
        for w in list(self.keys()):
            if self._rows[w] != rows.get(w):
                self.store.release(self._rows[w])
        dict.clear(self)
        self._rows = {}
        for w, n, r in entries:
            self._rows[w] = r
            dict.__setitem__(self, w, int(n))

    def n_of(self, worker_id):
        return dict.__getitem__(self, worker_id)

    def n_of_row(self):
        return {r: dict.__getitem__(self, w) for w, r in self._rows.items()}

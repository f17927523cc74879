"""Multi-GPU servers: clients sharded over the GPUs of one node, RCCL exchange.

The reference is one process with one server device (servers/server.py:6-35;
workers are threads, simulator.py:60-69).  On an MI355X node the hot path
runs one process per GPU (``torch.distributed`` with the ``nccl`` backend,
which is RCCL over xGMI on ROCm).  Each rank owns the updates of its own
clients (``clients_per_round`` = local clients; ``worker_number`` stays the
global K), aggregates them locally with the same HIP kernels, and one
collective combines the ranks:

* FedAvg / fed_quant: every rank computes its partial sum with the GLOBAL N
  (an int64 all-reduce of the local sample counts), then an fp32 SUM
  all-reduce of the P-element partial, pipelined in chunks so the RCCL
  transfer of chunk c overlaps the reduction of chunk c+1.  Reference-order
  within a shard, cross-rank sums in RCCL order: normwise ~1e-7 vs the exact
  mean (north-star tolerance 1e-6), not bit-exact.
  ``ShardedFedServer(exchange="alltoall")`` is the bit-exact alternative:
  parameter slices per rank, the client rows stored slice-major so that ONE
  ``all_to_all_single`` moves every client's slice to its owner straight from
  the store, the reference-order kernel over all clients on each slice, one
  all-gather.
* sign vote: int32 vote counts per rank, SUM all-reduce, then sign on every
  rank — bit-exact for any number of ranks.

Client-to-rank placement mirrors the reference's ``worker_id % ngpu``
(simulator.py:68).
"""
import time

import torch
import torch.distributed as dist

from . import _native
from .servers.fed_quant_server import FedQuantServer
from .servers.fed_server import FedServer
from .servers.sign_sgd_server import SignSGDServer, SignVoteResult
from .task_queue import RepeatedResult


def rank_of_worker(worker_id, world_size):
    """simulator.py:68 places worker i on device i % ngpu."""
    return worker_id % world_size


def local_workers(worker_number, rank, world_size):
    return [w for w in range(worker_number) if rank_of_worker(w, world_size) == rank]


def _world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


def global_sample_count(local_ns, device, group=None):
    t = torch.tensor([sum(int(n) for n in local_ns)], dtype=torch.int64, device=device)
    if _world()[0] > 1:
        dist.all_reduce(t, group=group)
    return int(t.item())


def chunk_bounds(P, chunks):
    """Element bounds of ``chunks`` pieces of a P-element vector, multiples of 256,
    sizes decreasing linearly (weights chunks, chunks-1, ..., 1): only the last
    piece's all-reduce runs after the last reduction kernel, so it is the small one."""
    tot = chunks * (chunks + 1) // 2
    acc, bounds = 0, [0]
    for c in range(chunks - 1):
        acc += chunks - c
        bounds.append(min(P, P * acc // tot // 256 * 256))
    bounds.append(P)
    return bounds


def allreduce_chunked(flat, chunks=3, group=None, produce=None):
    """SUM all-reduce of a flat fp32 vector in ``chunks`` pieces (chunk_bounds).

    ``produce(c0, c1)`` (optional) fills flat[c0:c1] first; chunk c's all-reduce
    is issued asynchronously before chunk c+1 is produced, so RCCL over xGMI
    overlaps the next chunk's reduction kernel."""
    P = flat.numel()
    bounds = chunk_bounds(P, chunks)
    handles = []
    for c in range(chunks):
        c0, c1 = bounds[c], bounds[c + 1]
        if c1 <= c0:
            continue
        if produce is not None:
            produce(c0, c1)
        if _world()[0] > 1:
            handles.append(dist.all_reduce(flat[c0:c1], async_op=True, group=group))
    for h in handles:
        h.wait()
    return flat


class _ShardedMixin:
    def _init_shard(self, worker_number, group, chunks):
        # before FedServer.__init__, which publishes the initial broadcast to
        # clients_per_round consumers
        self.group = group
        self.chunks = chunks
        world, rank = _world()
        self.world_size, self.rank = world, rank
        self.local_worker_ids = local_workers(worker_number, rank, world)

    @property
    def clients_per_round(self):
        return len(self.local_worker_ids)


def slice_bounds(P, world):
    """Parameter slices of a P-element row (P a multiple of 64) for ``world`` ranks:
    contiguous, equal lengths L (a multiple of 64; the last slices are short or
    empty when P is not a multiple of L), so the slice means all-gather straight
    into one [world * L] output."""
    L = -(-P // (64 * world)) * 64
    return [min(P, r * L) for r in range(world)] + [P]


class ShardedFedServer(_ShardedMixin, FedServer):
    """FedServer whose round is spread over all ranks (one process per GPU).

    ``exchange="allreduce"`` (default): each rank reduces its own clients with the
    global N, then a chunked fp32 SUM all-reduce — one P-element exchange,
    normwise ~1e-7 of the exact mean.  ``exchange="alltoall"``: bit-exact for any
    number of ranks: every rank owns a parameter slice; the store
    is slice-major, so ONE ``all_to_all_single`` sends slice d of every row of the
    rank's store to rank d straight from the store (no staging copy); each rank
    runs the reference-order kernel over ALL K clients on its slice, and an
    all-gather assembles the mean — bits identical to one FedServer that saw the
    clients in the same order.  Its traffic is the whole store: every call moves
    capacity x P fp32 per rank (its released and unused rows and its own slice
    included), whatever the subset size — against one P-vector for the
    all-reduce.

    ``order`` (alltoall only) is the client order of the sum: ``"arrival"`` (the
    reference's: ``self.parameters.keys()`` in insertion order,
    servers/fed_server.py:69-73,81) merges the ranks' arrivals by the
    node-wide monotonic clock at which each update reached its rank's queue
    thread (ties by worker id) — the reference's order, and like the
    reference's it depends on thread timing, so two runs can give different
    bits; the clock is only comparable within one node, so when the ranks span
    several hosts the server falls back to ``"worker_id"`` (with a warning).
    ``"worker_id"`` sorts by id: the same bits on every run."""

    def __init__(self, group=None, chunks=3, exchange="allreduce", order="arrival", **kwargs):
        if exchange not in ("allreduce", "alltoall"):
            raise ValueError(f"exchange must be 'allreduce' or 'alltoall', not {exchange!r}")
        if order not in ("arrival", "worker_id"):
            raise ValueError(f"order must be 'arrival' or 'worker_id', not {order!r}")
        self.exchange = exchange
        self.order = order
        self._arrival = {}
        self._clock = time.monotonic_ns  # system-wide on Linux: comparable across ranks
        self._init_shard(kwargs["worker_number"], group, chunks)
        if exchange == "alltoall" and order == "arrival" and self.world_size > 1:
            import socket
            hosts = [None] * self.world_size
            dist.all_gather_object(hosts, socket.gethostname(), group=group)
            if len(set(hosts)) > 1:
                import logging
                logging.getLogger("distributed_learning_simulator_amd").warning(
                    "order='arrival' needs one node's monotonic clock; ranks span %d hosts, "
                    "summing in worker-id order", len(set(hosts)))
                self.order = "worker_id"
        super().__init__(**kwargs)

    def _make_store(self, parameter_dict):
        if self.exchange != "alltoall":
            return super()._make_store(parameter_dict)
        from .aggregation import SlicedClientUpdateStore
        from .layout import ParameterLayout
        layout = ParameterLayout.from_dict(parameter_dict)
        bounds = slice_bounds(layout.P, self.world_size)
        return SlicedClientUpdateStore(layout, self.device, self.store_capacity, self.world_size,
                                       bounds[1] - bounds[0])

    def _process_worker_data(self, data, __):
        wid = data[0]
        if wid not in self._arrival:  # a re-sent update keeps its first place, like a dict key
            self._arrival[wid] = self._clock()
        result = super()._process_worker_data(data, __)
        if result is not None:  # the round is over: its clients' updates were cleared
            self._arrival.clear()
        return result

    def _global_order(self, ids):
        """[(worker_id, n, home rank, row in home's store)] of every rank's clients
        in summation order, and every rank's store capacity."""
        dev, world = self.device, self.world_size
        kmax = max(1, -(-self.worker_number // world))  # >= any rank's local clients
        cap = self.parameters.store.capacity
        meta = [[int(wid), self.parameters.n_of(wid), self._arrival.get(wid, 0),
                 self.parameters.row_of(wid), cap] for wid in ids]
        meta += [[-1, 0, 0, 0, cap]] * (kmax - len(meta))
        meta = torch.tensor(meta, dtype=torch.int64).to(dev)  # one host -> device copy
        metas = torch.empty((world * kmax, 5), dtype=torch.int64, device=dev)
        dist.all_gather_into_tensor(metas, meta, group=self.group)
        metas = metas.tolist()
        caps = [metas[r * kmax][4] for r in range(world)]
        entries = [(t, wid, n, i // kmax, row) for i, (wid, n, t, row, _) in enumerate(metas)
                   if wid >= 0]
        if self.order == "worker_id":
            entries.sort(key=lambda e: e[1])
        else:
            entries.sort(key=lambda e: (e[0], e[1]))
        return [(wid, n, home, row) for _, wid, n, home, row in entries], caps

    def _bitexact_mean(self, ids):
        """exchange="alltoall": the mean of every rank's clients, bit-exact.

        The store is slice-major (SlicedClientUpdateStore: B [world, capacity, L]),
        so ONE all_to_all_single sends block B[d] — slice d of every client this
        rank holds — to rank d, straight from the store, and lands every rank's
        block for my slice in ``recv`` [sum of capacities, L]; the kernel then
        walks those rows in the summation order (row indices, no gather)."""
        store = self.parameters.store
        P, dev, world, me = store.layout.P, self.device, self.world_size, self.rank
        order, caps = self._global_order(ids)
        L = store.L
        mine = slice_bounds(P, world)[me + 1] - slice_bounds(P, world)[me]
        base = [0]
        for c in caps:
            base.append(base[-1] + c)
        recv = torch.empty((base[-1], L), dtype=torch.float32, device=dev)
        send = store.B.view(-1)
        in_splits = [store.capacity * L] * world
        out_splits = [c * L for c in caps]
        if dist.get_backend(self.group) == "gloo" and recv.is_cuda:  # gloo: host tensors
            rh = torch.empty(recv.shape, dtype=torch.float32)
            dist.all_to_all_single(rh.view(-1), send.cpu(), out_splits, in_splits, group=self.group)
            recv.copy_(rh)
        else:
            dist.all_to_all_single(recv.view(-1), send, out_splits, in_splits, group=self.group)
        total = sum(n for _, n, _, _ in order)
        part = torch.zeros(L, dtype=torch.float32, device=dev)
        if mine > 0:  # a rank whose slice is empty (P < 64 * world) only joins the gather
            from .aggregation import _f32, _i32
            from .servers.fed_server import _MODES
            rows = _i32([base[home] + row for _, _, home, row in order], dev)
            _native.fedavg(recv, rows, _f32([n for _, n, _, _ in order], dev), float(total), mine,
                           part, mode=_MODES[self.aggregation_mode])
        out = torch.empty(world * L, dtype=torch.float32, device=dev)
        if dist.get_backend(self.group) == "gloo" and part.is_cuda:
            oh = torch.empty(world * L, dtype=torch.float32)
            dist.all_gather_into_tensor(oh, part.cpu(), group=self.group)
            out.copy_(oh)
        else:
            dist.all_gather_into_tensor(out, part, group=self.group)
        return out[:P]

    def get_subset_model(self, client_subset):
        if not client_subset:
            return self.prev_model
        if self.exchange == "alltoall":
            ids = [i for i in client_subset if i in self.parameters]
            return self.parameters.store.layout.views(self._bitexact_mean(ids))
        ids = [i for i in client_subset if i in self.parameters]
        ns = [self.parameters.n_of(i) for i in ids]
        total = global_sample_count(ns, self.device, self.group)
        store = self.parameters.store
        rows = [self.parameters.row_of(i) for i in ids]
        out = torch.zeros(store.layout.P, dtype=torch.float32, device=self.device)
        produce = None
        if rows:
            from .aggregation import _f32, _i32
            from .servers.fed_server import _MODES
            r, w = _i32(rows, self.device), _f32(ns, self.device)
            mode = _MODES[self.aggregation_mode]

            def produce(c0, c1):  # reduce chunk c while chunk c-1 is on the wire
                store.fedavg(r, w, mode=mode, total=total, out=out[c0:c1], cols=(c0, c1))
        allreduce_chunked(out, self.chunks, self.group, produce=produce)
        return store.layout.views(out)


class ShardedFedQuantServer(_ShardedMixin, FedQuantServer):
    """FedQuantServer over all ranks: each rank dequantizes and averages its own
    clients with the global N, column chunk by column chunk (the store's tile
    sub-tables, ``QuantizedClientStore.fedavg(cols=...)``), and chunk c's SUM
    all-reduce is on the wire while chunk c+1 is reduced — the same pipeline as
    ShardedFedServer's, in the server's ``aggregation_mode``."""

    def __init__(self, group=None, chunks=3, **kwargs):
        self._init_shard(kwargs["worker_number"], group, chunks)
        super().__init__(**kwargs)

    def get_subset_model(self, client_subset):
        if not client_subset:
            return self.prev_model
        ids = [i for i in client_subset if i in self.parameters]
        ns = [self.parameters.n_of(i) for i in ids]
        total = global_sample_count(ns, self.device, self.group)
        store = self.parameters.store
        out = torch.zeros(store.layout.P, dtype=torch.float32, device=self.device)
        produce = None
        if ids:
            from .aggregation import _f32, _i32
            from .servers.fed_server import _MODES
            r = _i32([self.parameters.row_of(i) for i in ids], self.device)
            w = _f32(ns, self.device)
            mode = _MODES[self.aggregation_mode]

            def produce(c0, c1):  # reduce chunk c while chunk c-1 is on the wire
                store.fedavg(r, w, out=out, total=total, mode=mode, cols=(c0, c1))
        allreduce_chunked(out, self.chunks, self.group, produce=produce)
        return store.layout.views(out)


class ShardedSignSGDServer(SignSGDServer):
    """Vote over clients on all ranks: local int32 counts, SUM all-reduce, sign."""

    def __init__(self, group=None, **kwargs):
        super().__init__(**kwargs)
        self.group = group
        world, rank = _world()
        self.local_worker_ids = local_workers(self.worker_number, rank, world)

    def _process_worker_data(self, sign_gradient, __=None):
        slot = len(self.sign_gradients)
        if self._planes is not None and slot >= self._planes.shape[0]:
            raise RuntimeError("more sign gradients than local workers")
        self._store_client(slot, sign_gradient)
        self.sign_gradients.append(slot)
        if len(self.sign_gradients) != len(self.local_worker_ids):
            return None
        bad = int(self._bad.item())
        if bad:
            self._bad.zero_()
            self.sign_gradients = []
            raise ValueError(f"sign gradients hold {bad} values outside {{-1, 0, +1}}")
        P = self._layout.P
        counts = torch.empty(P, dtype=torch.int32, device=self.device)
        self._count(len(self.sign_gradients), P, counts)
        if _world()[0] > 1:
            dist.all_reduce(counts, group=self.group)
        sign_out = torch.empty(P, dtype=torch.float32, device=self.device)
        vote_planes = torch.empty(_native.sign_words(P), dtype=torch.int64, device=self.device)
        self._from_counts(counts, P, sign_out, vote_planes)
        result = SignVoteResult(self._layout.views(sign_out).values())
        result.vote_planes = vote_planes
        result.counts = counts
        self.sign_gradients = []
        return RepeatedResult(data=result, num=len(self.local_worker_ids))

    def _count(self, K, P, counts):
        _native.sign_vote_count(self._planes, None, K, P, counts)

    def _from_counts(self, counts, P, sign_out, vote_planes):
        _native.sign_from_counts(counts, P, sign_out, vote_planes)

    def _ensure(self, shapes):
        first = self._layout is None
        super()._ensure(shapes)
        if first and self._planes.shape[0] != len(self.local_worker_ids):
            self._planes = self._planes[: max(1, len(self.local_worker_ids))].contiguous()


class _ShardedShapleyMixin(_ShardedMixin):
    """Shapley servers on several ranks: each rank receives its own
    clients' updates into its own block of rows of the store (rows
    [rank * kmax, (rank + 1) * kmax) of U [world * kmax, P]), one in-place
    ``all_gather_into_tensor`` per round fills every other block (RCCL over
    xGMI, no staging copy), the arrived rows are registered without a copy, and
    the coalitions of every evaluation batch are dealt round-robin over the
    ranks (``ShapleyValueServer.evaluate_subsets``)."""

    @property
    def _kmax(self):
        return max(1, -(-self.worker_number // self.world_size))

    def _make_store(self, parameter_dict):
        from .aggregation import ClientUpdateStore
        from .layout import ParameterLayout
        k = self._kmax
        return ClientUpdateStore(ParameterLayout.from_dict(parameter_dict), self.device,
                                 capacity=self.world_size * k,
                                 acquire_range=(self.rank * k, (self.rank + 1) * k))

    def _gather_clients(self):
        store = self.parameters.store
        k, me, world = self._kmax, self.rank, self.world_size
        local = list(self.parameters.keys())
        # (worker id, n, row) of the local clients, built on the host, one copy
        meta = [[int(w), self.parameters.n_of(w), self.parameters.row_of(w)] for w in local]
        meta += [[-1, 0, 0]] * (k - len(meta))
        meta = torch.tensor(meta, dtype=torch.int64).to(self.device)
        metas = torch.empty((world * k, 3), dtype=torch.int64, device=self.device)
        dist.all_gather_into_tensor(metas, meta, group=self.group)
        U = store.U[: world * k]
        mine = store.U[me * k:(me + 1) * k]
        if dist.get_backend(self.group) == "gloo":  # gloo: host tensors, no in-place aliasing
            uh = torch.empty(U.shape, dtype=torch.float32)
            dist.all_gather_into_tensor(uh, mine.cpu().clone(), group=self.group)
            U.copy_(uh)
        else:  # in place: rank r's block is its input (RCCL's in-place all-gather)
            dist.all_gather_into_tensor(U, mine, group=self.group)
        # every rank now holds all K clients, registered in worker-id order
        entries = sorted((w, n, row) for w, n, row in metas.tolist() if w >= 0)
        self.parameters.adopt(entries)

    def _before_aggregate(self):
        self._gather_clients()

def _sharded_shapley(cls):
    class Sharded(_ShardedShapleyMixin, cls):
        def __init__(self, group=None, **kwargs):
            self._init_shard(kwargs["worker_number"], group, 1)
            super().__init__(**kwargs)

    Sharded.__name__ = "Sharded" + cls.__name__
    Sharded.__qualname__ = Sharded.__name__
    return Sharded


from .servers.GTG_shapley_value_server import GTGShapleyValueServer  # noqa: E402
from .servers.multiround_shapley_value_server import MultiRoundShapleyValueServer  # noqa: E402

ShardedGTGShapleyValueServer = _sharded_shapley(GTGShapleyValueServer)
ShardedMultiRoundShapleyValueServer = _sharded_shapley(MultiRoundShapleyValueServer)


def get_sharded_server(algorithm, **kwargs):
    """factory.get_server for one process per GPU (torch.distributed initialised)."""
    table = {"fed": ShardedFedServer, "fed_quant": ShardedFedQuantServer,
             "sign_SGD": ShardedSignSGDServer, "GTG_shapley_value": ShardedGTGShapleyValueServer,
             "multiround_shapley_value": ShardedMultiRoundShapleyValueServer}
    if algorithm not in table:
        raise RuntimeError("unknown algorithm:" + algorithm)
    return table[algorithm](**kwargs)

"""Shapley-value server base (reference: servers/shapley_value_server.py:9-14).

Adds, on top of the reference's ``powerset``, the batched coalition evaluator
both Shapley servers use: a batch of S coalitions becomes S subset models in
one kernel launch (``dls_subset_fedavg_f32``, bit-exact reference order — the
default, because accuracy utilities are discontinuous — or the fp32 MFMA
contraction ``dls_subset_gemm_f32`` with ``subset_method="gemm"``), then each
model is scored with ``get_metric`` (servers/fed_server.py:26-32).  Under
``torch.distributed`` with several ranks the coalitions are dealt round-robin
over the ranks and the utilities are summed with one all-reduce (each rank
fills only its own entries), so every rank ends with the full table.
"""
import inspect
from itertools import chain, combinations

import torch
import torch.distributed as dist

from ..model_util import ModelUtil
from .fed_server import FedServer


class ShapleyValueServer(FedServer):
    def __init__(self, subset_method="exact", subset_batch=None, eval_streams=1, **kwargs):
        super().__init__(**kwargs)
        self.subset_method = subset_method
        self.subset_batch = subset_batch
        # queued utility forwards in flight at once, one HIP stream each (1: all
        # on the current stream); the utilities are the same bits either way.
        # Two or three in flight measured no faster (31.58 vs 31.66 evals/s, each
        # layer's grid fills the chip, profiles/r06_stream_eval_probe.txt)
        self.eval_streams = eval_streams
        self._streams = None
        self.evaluated_subsets = []  # coalitions evaluated this round, in evaluation order

    def powerset(self, iterable):
        "powerset([1,2,3]) --> () (1,) (2,) (3,) (1,2) (1,3) (2,3) (1,2,3)"
        s = list(iterable)
        return chain.from_iterable(combinations(s, r) for r in range(len(s) + 1))

    def _batch_size(self):
        if self.subset_batch:
            return self.subset_batch
        P = self.parameters.store.layout.P
        return max(1, min(64, (2 << 30) // (4 * P)))  # <= 2 GiB of subset models

    def _eval_stream_list(self):
        """The streams the queued forwards rotate over, or None (one stream)."""
        dev = getattr(self.tester, "device", None) or self.device
        dev = torch.device(dev) if dev is not None else None
        if (self.eval_streams is None or self.eval_streams < 2 or dev is None
                or dev.type != "cuda"
                or "stream" not in inspect.signature(self.tester.correct_async).parameters):
            return None
        if self._streams is None or len(self._streams) != self.eval_streams:
            self._streams = [torch.cuda.Stream(dev) for _ in range(self.eval_streams)]
        return self._streams

    def evaluate_subsets(self, subsets):
        """Utilities of coalitions (tuples of worker ids) -> list of floats, in order."""
        subsets = [tuple(s) for s in subsets]
        world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        rank = dist.get_rank() if world > 1 else 0
        mine = [i for i in range(len(subsets)) if i % world == rank]
        values = [0.0] * len(subsets)
        store = self.parameters.store
        bs = self._batch_size()
        # the default accuracy metric on a tester that can count without a host
        # synchronisation: the batch's evaluations are queued back to back and
        # their counts read once (int(count) / n: the same floats as get_metric)
        # (not when a subclass or the instance replaces get_metric)
        queued = (getattr(self.get_metric, "__func__", None) is FedServer.get_metric
                  and self.tester is not None and hasattr(self.tester, "correct_async"))
        streams = self._eval_stream_list() if queued else None
        for b0 in range(0, len(mine), bs):
            idx = mine[b0:b0 + bs]
            nonempty = [i for i in idx if subsets[i]]
            out = None
            if nonempty:
                rows = [[self.parameters.row_of(w) for w in subsets[i]] for i in nonempty]
                out = store.subset_models(rows, self.parameters.n_of_row(), method=self.subset_method)
            pos = {i: k for k, i in enumerate(nonempty)}
            pending = []
            for i in idx:
                model = store.layout.views(out[pos[i]]) if subsets[i] else self.prev_model
                if queued:
                    ModelUtil(self.tester.model).load_parameter_dict(model)
                    if streams:
                        c = self.tester.correct_async(stream=streams[len(pending) % len(streams)])
                    else:
                        c = self.tester.correct_async()
                    pending.append((i, c))
                else:
                    values[i] = float(self.get_metric(model))
                self.evaluated_subsets.append(subsets[i])
            if pending:
                if streams:
                    cur = torch.cuda.current_stream(streams[0].device)
                    for st in streams:
                        cur.wait_stream(st)
                n = self.tester.dataset[0].shape[0]
                counts = torch.stack([c for _, c in pending]).tolist()  # one synchronisation
                for (i, _), c in zip(pending, counts):
                    values[i] = int(c) / n
                # the tester's state as get_metric leaves it: its accuracy metric holds
                # the last evaluated coalition's (the queued path counts top-1 only;
                # loss_metric keeps the last full inference()'s value)
                self.tester.accuracy_metric.value = values[pending[-1][0]]
        if world > 1:
            t = torch.tensor(values, dtype=torch.float64, device=self.device)
            dist.all_reduce(t)
            values = t.tolist()
        return values

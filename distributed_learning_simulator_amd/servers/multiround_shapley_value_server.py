"""Multi-round exact Shapley server (reference: servers/multiround_shapley_value_server.py:9-61).

Every coalition of the power set (2^N, D7: N <= ~16) is evaluated — here as
batched subset-model launches plus utility evaluations fanned out over ranks
(``ShapleyValueServer.evaluate_subsets``) instead of 2^N sequential
``get_subset_model`` + ``get_metric`` calls — and
SV_i = sum_{S containing i} (v(S) - v(S\\{i})) / (C(N-1, |S|-1) * N)  (:42-55),
accumulated in the reference's dict order.  The ``metric_<round>`` pickle side
effect (:56-57) is kept (``metric_dir``; None disables it).

D5: the reference reads ``round_trunc_threshold`` from kwargs that
``Server.__init__`` then rejects, so round truncation is unreachable there; it
is accepted here as a keyword (default None = the reference's behaviour).
"""
import logging
import math
import os
import pickle

import torch.distributed as dist

from .shapley_value_server import ShapleyValueServer

log = logging.getLogger("distributed_learning_simulator_amd")


class MultiRoundShapleyValueServer(ShapleyValueServer):
    def __init__(self, round_trunc_threshold=None, metric_dir=".", **kwargs):
        super().__init__(**kwargs)
        self.shapley_values = dict()
        self.round_trunc_threshold = round_trunc_threshold
        self.metric_dir = metric_dir

    def _process_aggregated_parameter(self, aggregated_parameter: dict):
        N = self.worker_number
        self.evaluated_subsets = []
        metrics = dict()
        if self.round_trunc_threshold is not None:
            last_round_metric = self.get_metric(self.prev_model)
            this_round_metric = self.get_metric(aggregated_parameter)
            metrics[()] = last_round_metric
            metrics[tuple(sorted(range(N)))] = this_round_metric
            log.info("this_round_metric %s last_round_metric %s round_trunc_threshold %s",
                     this_round_metric, last_round_metric, self.round_trunc_threshold)
            if abs(this_round_metric - last_round_metric) <= self.round_trunc_threshold:
                self.shapley_values[self.round] = {i: 0 for i in range(N)}
                return aggregated_parameter
        todo, seen = [], set(metrics)
        for subset in self.powerset(range(N)):
            key = tuple(sorted(subset))
            if key not in seen:
                seen.add(key)
                todo.append(key)
        for key, value in zip(todo, self.evaluate_subsets(todo)):
            metrics[key] = value
            log.info("round %s key %s metric %s", self.round, key, value)
        round_shapley_values = dict()
        for subset, metric in metrics.items():
            if not subset:
                continue
            for client_id in subset:
                marginal_contribution = (
                    metric - metrics[tuple(sorted(i for i in subset if i != client_id))])
                if client_id not in round_shapley_values:
                    round_shapley_values[client_id] = 0
                round_shapley_values[client_id] += marginal_contribution / (
                    (math.comb(N - 1, len(subset) - 1)) * N)
        rank0 = not (dist.is_available() and dist.is_initialized()) or dist.get_rank() == 0
        if self.metric_dir is not None and rank0:
            with open(os.path.join(self.metric_dir, "metric_" + str(self.round)), "wb") as f:
                pickle.dump(metrics, f)
        self.shapley_values[self.round] = round_shapley_values
        log.error("shapley_values %s", self.shapley_values)
        return aggregated_parameter

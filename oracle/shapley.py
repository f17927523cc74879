"""Shapley-value servers — CPU restatement (TEST INFRASTRUCTURE, see oracle/__init__.py).

Pure-Python restatements, for small N, of

* ``ShapleyValueServer.powerset``                         servers/shapley_value_server.py:11-14
* ``MultiRoundShapleyValueServer._process_aggregated_parameter``
                                                          servers/multiround_shapley_value_server.py:15-61
* ``GTGShapleyValueServer._process_aggregated_parameter`` + ``not_convergent``
                                                          servers/GTG_shapley_value_server.py:20-100

``subset_model(subset)`` and ``metric(model)`` are callables supplied by the
caller (the reference's ``get_subset_model`` / ``get_metric``).  The GTG loop
consumes the global ``np.random`` stream exactly as the reference does: one
``np.random.permutation`` per worker per while-pass (:42-49), and reproduces
the reference's aliasing of ``marginal_contribution`` in
``contribution_records`` (:64-65: the same list object appended N times).
"""
import math
from itertools import chain, combinations

import numpy as np


def powerset(iterable):
    s = list(iterable)
    return chain.from_iterable(combinations(s, r) for r in range(len(s) + 1))


def multiround_shapley(N, subset_model, metric):
    """Returns (shapley dict, metrics dict in evaluation order)."""
    metrics = {}
    for subset in powerset(range(N)):  # :34-40
        key = tuple(sorted(subset))
        if key not in metrics:
            metrics[key] = metric(subset_model(subset))
    sv = {}
    for subset, m in metrics.items():  # :42-55
        if not subset:
            continue
        for cid in subset:
            mc = m - metrics[tuple(sorted(i for i in subset if i != cid))]
            if cid not in sv:
                sv[cid] = 0
            sv[cid] += mc / (math.comb(N - 1, len(subset) - 1) * N)
    return sv, metrics


def gtg_not_convergent(index, records, converge_min, last_k=10, criteria=0.05):
    """servers/GTG_shapley_value_server.py:79-100."""
    if index <= converge_min:
        return True
    all_vals = (np.cumsum(records, 0) / np.reshape(np.arange(1, len(records) + 1), (-1, 1)))[-last_k:]
    errors = np.mean(np.abs(all_vals[-last_k:] - all_vals[-1:]) / (np.abs(all_vals[-1:]) + 1e-12), -1)
    return bool(np.max(errors) > criteria)


def gtg_shapley(N, prev_model, agg_model, subset_model, metric, eps=0.001,
                round_trunc_threshold=0.01):
    """Returns (shapley dict, list of subsets evaluated in order)."""
    last = metric(prev_model)  # :21
    this = metric(agg_model)  # :22
    if abs(last - this) <= round_trunc_threshold:  # :29-31
        return {i: 0 for i in range(N)}, []
    converge_min = max(30, N)
    metrics, evaluated = {}, []
    index = 0
    records = []
    while gtg_not_convergent(index, records, converge_min):  # :36
        for worker_id in range(N):  # :37
            index += 1
            v = [0 for _ in range(N + 1)]
            v[0] = last
            mc = [0 for _ in range(N)]
            perm = np.concatenate((np.array([worker_id]), np.random.permutation(
                [i for i in range(N) if i != worker_id]))).astype(int)
            for j in range(1, N + 1):
                subset = tuple(sorted(perm[:j].tolist()))
                if abs(this - v[j - 1]) >= eps:  # :54
                    if subset not in metrics:
                        evaluated.append(subset)
                        metrics[subset] = metric(subset_model(subset))
                    v[j] = metrics[subset]
                else:
                    v[j] = v[j - 1]
                mc[perm[j - 1]] = v[j] - v[j - 1]
                records.append(mc)  # D6: same object, N times per permutation
    sv = np.sum(records, 0) / len(records)  # :68
    return {k: s for k, s in enumerate(sv)}, evaluated

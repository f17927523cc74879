"""FedAvg weighted mean — CPU restatement (TEST INFRASTRUCTURE, see oracle/__init__.py).

Reference: ``FedServer.get_subset_model``, servers/fed_server.py:44-66.

    total = sum(n_i for i in subset)                        # :51-53  (Python int)
    for i in subset:                                        # :54     (iteration order)
        for k in params_i:                                  # :56
            tmp = p.to(dev) * n_i / total                   # :57-61  fl32(fl32(p*n)/N)
            avg[k] = tmp  if first else  avg[k] + tmp       # :62-65

The Python ints are converted to fp32 by torch's scalar path (so ``n_i`` above
2**24 is rounded); every operation is a single IEEE fp32 rounding.
"""
import numpy as np


def fedavg_reference_order(U, n, order):
    """Bit-exact restatement over a client-major matrix.

    U: float32 [K, P] (row = one client's flattened parameter dict)
    n: sample counts (Python ints), indexed by row
    order: the rows in the reference's iteration order (``self.parameters`` key
    order, or the Shapley subset tuple).
    """
    order = [int(i) for i in order]
    total = np.float32(sum(int(n[i]) for i in order))
    acc = None
    for i in order:
        tmp = (U[i] * np.float32(int(n[i]))) / total
        acc = tmp if acc is None else acc + tmp
    return acc


def fedavg_torch_cpu(tensors, n, order):
    """The reference's own torch op sequence on the CPU (servers/fed_server.py:52-65).

    ``tensors``: list of per-client dicts {name: fp32 CPU tensor}.  This is what
    ``bench.py`` times as the CPU baseline: the same torch ops, the same order.
    """
    total = 0
    for i in order:
        total += int(n[i])
    avg = {}
    for i in order:
        for k, p in tensors[i].items():
            tmp = p * int(n[i]) / total
            if k not in avg:
                avg[k] = tmp
            else:
                avg[k] += tmp
    return avg


def fedavg_weighted(U, n, order):
    """Exact (fp64) weighted mean, for normwise-tolerance checks of reordered sums."""
    order = [int(i) for i in order]
    w = np.array([int(n[i]) for i in order], dtype=np.float64)
    return (w[:, None] * U[order].astype(np.float64)).sum(0) / w.sum()

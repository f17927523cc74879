"""Loaders for the golden fixtures written by make_golden.py (data only)."""
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def load(name):
    return np.load(os.path.join(HERE, name), allow_pickle=False)


def meta(npz):
    return json.loads(str(npz["meta"]))


def shapley_cases():
    with open(os.path.join(HERE, "shapley.json")) as f:
        return json.load(f)


def layout_size(layout):
    return sum(int(np.prod(s)) for _, s in layout)


def split(flat, layout):
    out, off = {}, 0
    for name, shape in layout:
        m = int(np.prod(shape))
        out[name] = np.asarray(flat[off:off + m]).reshape(shape)
        off += m
    return out


def shapley_large_cases():
    """GTG N=50 / multiround N=12 (shapley_large.npz) in the shapley_cases() form;
    'evaluated' as sorted tuples decoded from the stored bit masks."""
    z = load("shapley_large.npz")
    cases = []
    for m in meta(z):
        t = m["tag"]
        K = m["K"]
        case = dict(m)
        case.update(U=z[f"{t}_U"], n=[int(x) for x in z[f"{t}_n"]], prev=z[f"{t}_prev"],
                    target=z[f"{t}_target"],
                    sv={str(i): float(v) for i, v in enumerate(z[f"{t}_sv"])},
                    evaluated=[tuple(i for i in range(K) if (int(b) >> i) & 1)
                               for b in z[f"{t}_evaluated"]],
                    metric_pickle=(z[f"{t}_metric_pickle"].tobytes()
                                   if f"{t}_metric_pickle" in z.files else None))
        cases.append(case)
    return cases

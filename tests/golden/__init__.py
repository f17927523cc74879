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

"""Flat parameter layout: how a parameter dict maps onto one row of HBM.

The reference passes client updates around as ``dict[str, Tensor]`` in
``named_parameters`` order (workers/fed_worker.py:30-35) and aggregates them
tensor by tensor (servers/fed_server.py:56-65).  Here every dict becomes one
row of a client-major fp32 matrix so that a whole FL round is ONE streaming
kernel: tensors are concatenated in dict order, each starting at a multiple of
64 elements (256 B) so every tensor view and every kernel tile is 16-byte
aligned.  The padding between tensors is zero and never exposed.
"""
import math

import torch

ALIGN = 64  # elements


def _round_up(x, a):
    return (x + a - 1) // a * a


class ParameterLayout:
    def __init__(self, items):
        """items: iterable of (name, shape)."""
        self.names = []
        self.shapes = []
        self.numels = []
        self.offsets = []
        off = 0
        for name, shape in items:
            shape = tuple(int(s) for s in shape)
            n = int(math.prod(shape)) if shape else 1
            self.names.append(name)
            self.shapes.append(shape)
            self.numels.append(n)
            self.offsets.append(off)
            off += _round_up(max(n, 1), ALIGN)
        self.P = max(off, ALIGN)  # padded row length (multiple of 64)
        self.numel = sum(self.numels)
        self._index = {n: i for i, n in enumerate(self.names)}

    @classmethod
    def from_dict(cls, d):
        return cls((k, tuple(v.shape)) for k, v in d.items())

    def __len__(self):
        return len(self.names)

    def __eq__(self, other):
        return isinstance(other, ParameterLayout) and self.names == other.names and \
            self.shapes == other.shapes

    def matches(self, d):
        if list(d.keys()) != self.names:
            return False
        return all(tuple(v.shape) == s for v, s in zip(d.values(), self.shapes))

    def segments(self):
        """int64 [T+1] boundaries of the *unpadded* tensors in a compact concat."""
        return [0] + list(itertools_accumulate(self.numels))

    def views(self, flat):
        """dict name -> view of a flat row (shares storage)."""
        return {n: flat[o:o + m].view(s)
                for n, s, m, o in zip(self.names, self.shapes, self.numels, self.offsets)}

    def copy_into(self, d, row):
        """Copy a parameter dict into a flat row (one multi-tensor copy)."""
        dst = [row[o:o + m].view(s)
               for s, m, o in zip(self.shapes, self.numels, self.offsets)]
        src = [d[n].detach() for n in self.names]
        src = [t if t.dtype == torch.float32 else t.float() for t in src]
        torch._foreach_copy_(dst, src, non_blocking=True)

    def flatten(self, d, device=None, dtype=torch.float32):
        dev = device if device is not None else next(iter(d.values())).device
        row = torch.zeros(self.P, dtype=dtype, device=dev)
        self.copy_into(d, row)
        return row

    def offset_of(self, name):
        return self.offsets[self._index[name]]


def itertools_accumulate(xs):
    s = 0
    for x in xs:
        s += x
        yield s

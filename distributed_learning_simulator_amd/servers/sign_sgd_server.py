"""signSGD majority-vote server (reference: servers/sign_sgd_server.py:7-21).

The reference sums K lists of fp32 sign tensors with Python ``sum`` and takes
``torch.sign`` (:16-18) — 4 bytes per parameter per client on the wire and K x
(#tensors) torch ops.  Here each client's signs become 2-bit planes in HBM
(``dls_sign_pack_f32``, or sent already packed by the device-side
``SignSGDWorker``) and one ``dls_sign_vote`` launch produces the vote,
bit-exact (integer counts; ties and zeros -> 0; NaN-poisoned -> 0 like CPU
``torch.sign(nan)``).

D1: the reference defines ``__worker`` (name-mangled, never reached by the
queue, so its workers block forever).  This server wires the vote to
``_process_worker_data``, the evident intent, and keeps
``_SignSGDServer__worker`` as an alias.
"""
import torch

from .. import _native
from ..layout import ParameterLayout
from ..task_queue import RepeatedResult
from .server import Server


class PackedSigns:
    """A client's signs already packed on device: planes uint64-as-int64 [W]."""

    def __init__(self, planes, shapes):
        self.planes = planes
        self.shapes = [tuple(s) for s in shapes]


class SignVoteResult(list):
    """The broadcast list of fp32 sign tensors, plus the packed vote for device workers."""

    vote_planes = None
    counts = None


class SignSGDServer(Server):
    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        _native.require_gpu()
        self.sign_gradients: list = []
        self._layout = None
        self._planes = None  # int64 [K, sign_row_pitch(P)] (uint64 words)
        self._X = None  # fp32 staging row for list inputs
        self._bad = None

    def _ensure(self, shapes):
        if self._layout is None:
            self._layout = ParameterLayout((str(i), s) for i, s in enumerate(shapes))
            P = self._layout.P
            # rows of sign_words(P) words at a 128-byte pitch (sign_row_pitch)
            self._planes = torch.zeros((self.worker_number, _native.sign_row_pitch(P)),
                                       dtype=torch.int64, device=self.device)
            self._X = torch.zeros((1, P), dtype=torch.float32, device=self.device)
            self._bad = torch.zeros(1, dtype=torch.int32, device=self.device)
        elif [tuple(s) for s in shapes] != self._layout.shapes:
            raise ValueError("sign gradient shapes differ between clients")

    def _store_client(self, slot, sign_gradient):
        if isinstance(sign_gradient, PackedSigns):
            self._ensure(sign_gradient.shapes)
            self._planes[slot, :sign_gradient.planes.numel()].copy_(sign_gradient.planes,
                                                                   non_blocking=True)
            return
        shapes = [tuple(t.shape) for t in sign_gradient]
        self._ensure(shapes)
        d = {str(i): t for i, t in enumerate(sign_gradient)}
        self._layout.copy_into(d, self._X[0])
        _native.sign_pack(self._X, self._layout.P, self._planes[slot:slot + 1], self._bad)

    def _process_worker_data(self, sign_gradient, __=None):
        """servers/sign_sgd_server.py:12-21, wired to the queue (D1)."""
        slot = len(self.sign_gradients)
        self._store_client(slot, sign_gradient)
        self.sign_gradients.append(slot)
        if len(self.sign_gradients) != self.worker_number:
            return None
        bad = int(self._bad.item())
        if bad:
            self._bad.zero_()
            self.sign_gradients = []
            raise ValueError(f"sign gradients hold {bad} values outside {{-1, 0, +1}}; the "
                             "reference's fp32 sum would not be a majority vote")
        P = self._layout.P
        sign_out = torch.empty(P, dtype=torch.float32, device=self.device)
        vote_planes = torch.empty(_native.sign_words(P), dtype=torch.int64, device=self.device)
        # one launch: fp32 signs for the reference's broadcast list and the packed
        # vote for device-side workers (no int32 counts on a single device)
        _native.sign_vote(self._planes, None, self.worker_number, P, sign_out,
                          vote_planes=vote_planes)
        result = SignVoteResult(self._layout.views(sign_out).values())
        result.vote_planes = vote_planes
        self.sign_gradients = []
        return RepeatedResult(data=result, num=self.worker_number)

    _SignSGDServer__worker = _process_worker_data

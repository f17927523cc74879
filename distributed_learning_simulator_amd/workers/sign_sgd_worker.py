"""signSGD worker (reference: workers/sign_sgd_worker.py:10-58), device-side.

The reference replaces ``optimizer.step()`` with a per-parameter Python loop:
momentum / dampening / nesterov (:32-42), ``torch.sign(d_p).cpu()`` (:44: a
4-byte-per-parameter device-to-host copy), send, receive the vote, then
``p -= lr * (vote + wd * p)`` (:48-57).  Here one fused kernel per parameter
tensor (``dls_sign_sgd_direction``) updates the momentum buffer in the
optimizer state, takes the sign and packs it straight into the tensor's slice
of one 2-bit plane row that stays on the GPU; the vote comes back packed and
``dls_sign_sgd_apply`` applies it in place.  Arithmetic is bit-identical to the
reference's torch ops (golden vectors, tests/test_gpu_sign.py).
"""
import torch
from torch.optim.sgd import SGD

from .. import _native
from ..layout import ParameterLayout
from ..servers.sign_sgd_server import PackedSigns, SignVoteResult
from ..trainer import ModelExecutorCallbackPoint
from .worker import Worker


class SignSGDWorker(Worker):
    def __init__(self, **kwargs):
        kwargs.pop("round")
        super().__init__(**kwargs)
        assert isinstance(self.trainer.get_optimizer(), SGD)
        self.trainer.add_named_callback(ModelExecutorCallbackPoint.OPTIMIZER_STEP, "sign",
                                        self.__get_gredient)

    def train(self, device):
        # The reference worker inherits the base no-op train() (workers/worker.py:21-23)
        # on top of D1; here it trains (``--epoch`` epochs, every step voted).
        self.trainer.set_device(device)
        self.trainer.train()

    @torch.no_grad()
    def __get_gredient(self, optimizer, **kwargs):
        params, hyper = [], []
        for group in optimizer.param_groups:
            for p in group["params"]:
                if p.grad is None:
                    continue
                params.append(p)
                hyper.append(group)
        layout = ParameterLayout((str(i), tuple(p.shape)) for i, p in enumerate(params))
        planes = torch.zeros(_native.sign_words(layout.P), dtype=torch.int64,
                             device=params[0].device)
        for i, (p, group) in enumerate(zip(params, hyper)):
            momentum = group["momentum"]
            state = optimizer.state[p]
            first = momentum != 0 and "momentum_buffer" not in state
            if momentum != 0 and first:
                state["momentum_buffer"] = torch.empty_like(p)
            buf = state.get("momentum_buffer") if momentum != 0 else None
            off = layout.offsets[i] // 64 * 2
            _native.sign_sgd_direction(p.grad.contiguous(), buf, momentum,
                                       1 - group["dampening"], group["nesterov"], first,
                                       planes[off:])
        self.worker_data_queue.add_task(PackedSigns(planes, layout.shapes))
        result = self.worker_data_queue.get_result()
        if not isinstance(result, SignVoteResult) or result.vote_planes is None:
            raise RuntimeError("SignSGDWorker expects the packed vote of SignSGDServer")
        vote = result.vote_planes.to(params[0].device)
        for i, (p, group) in enumerate(zip(params, hyper)):
            off = layout.offsets[i] // 64 * 2
            _native.sign_sgd_apply(p.data, vote[off:], -group["lr"], group["weight_decay"])

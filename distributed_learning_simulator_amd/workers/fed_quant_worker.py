"""Quantized FedAvg worker (reference: workers/fed_quant_worker.py:15-69).

The reference trains with the absent library's QAT, sends
``qat.get_quantized_parameters()`` to a ``self.server`` attribute that does not
exist (D2, so it never runs), logs the pickle-size compression ratio (``model_util.get_data_serialization_size``) and loads
the server's answer.  This worker keeps the evident protocol on the task
queue: after each ``trainer.train()`` it quantizes every weight tensor (dim >= 2)
per output channel, symmetric int8 — torch's default QAT weight scheme
(``per_channel_symmetric``, qint8) — on the GPU with the library's
segment min/max + qparams + quantize kernels, sends
``(worker_id, n, {name: (int8 weight, scale[C], zero_point[C]) | fp32})``
and loads the dequantized aggregate the ``FedQuantServer`` broadcasts.
"""
import logging

import torch

from .. import _native
from ..model_util import ModelUtil, get_data_serialization_size
from ..trainer import ModelExecutorCallbackPoint
from .fed_worker import dataset_size
from .worker import Worker

log = logging.getLogger("distributed_learning_simulator_amd")


@torch.no_grad()
def quantize_per_channel_symmetric(w):
    """int8 per-output-channel symmetric quantization on device -> (q, scale, zp)."""
    C = w.shape[0]
    flat = w.detach().reshape(-1).contiguous().float()
    row = flat.numel() // C
    dev = flat.device
    seg = torch.arange(0, C + 1, dtype=torch.int64, device=dev) * row
    mins = torch.empty(C, dtype=torch.float32, device=dev)
    maxs = torch.empty(C, dtype=torch.float32, device=dev)
    _native.segment_minmax(flat, seg, flat.numel(), mins, maxs)
    scale = torch.empty(C, dtype=torch.float32, device=dev)
    zp = torch.empty(C, dtype=torch.int32, device=dev)
    _native.qparams_minmax(mins, maxs, scale, zp, -128, 127, symmetric=True)
    q = torch.empty(flat.numel(), dtype=torch.int8, device=dev)
    _native.quantize(flat, seg, flat.numel(), scale, zp, q, qmin=-128, qmax=127)
    return q.reshape(w.shape), scale, zp


class FedQuantWorker(Worker):
    def __init__(self, **kwargs):
        worker_round = kwargs.pop("round")
        super().__init__(**kwargs)
        self.round = worker_round
        self.trainer.add_named_callback(ModelExecutorCallbackPoint.AFTER_EXECUTE, "quantization",
                                        self.__send_parameters)
        # serialized sizes, as the reference (workers/fed_quant_worker.py:28-30,43)
        self.parameter_size = get_data_serialization_size(
            ModelUtil(self.trainer.model).get_parameter_dict())
        self.quantized_parameter_size = None

    def train(self, device):
        self.trainer.set_device(device)
        parameter_dict = self.worker_data_queue.get_result()
        ModelUtil(self.trainer.model).load_parameter_dict(parameter_dict)
        for _ in range(self.round):
            self.trainer.train()

    def quantized_parameters(self):
        payload = {}
        for name, p in self.trainer.model.named_parameters():
            payload[name] = quantize_per_channel_symmetric(p) if p.dim() >= 2 else p.detach().clone()
        return payload

    def __send_parameters(self, **kwargs):
        trainer = kwargs["model_executor"]
        payload = self.quantized_parameters()
        if self.quantized_parameter_size is None:
            self.quantized_parameter_size = get_data_serialization_size(payload)
        log.warning("parameter_size is %s, quantized_parameter_size is %s, compression ratio is %s",
                    self.parameter_size, self.quantized_parameter_size,
                    float(self.quantized_parameter_size) / float(self.parameter_size))
        self.worker_data_queue.add_task((self.worker_id, dataset_size(trainer.dataset), payload))
        parameter_dict = self.worker_data_queue.get_result()
        ModelUtil(trainer.model).load_parameter_dict(parameter_dict)

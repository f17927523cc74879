"""Minimal stand-ins for the two libraries the reference imports but does not ship.

TEST INFRASTRUCTURE ONLY — used by ``make_golden.py`` in the build container to
import the reference's ``servers/*.py`` / ``workers/*.py`` (read as-is from
/root/reference) and record golden vectors.  Nothing here runs on the GPU box.

The reference depends on ``cyy_naive_lib`` and ``cyy_naive_pytorch_lib``
(absent, no pinned version).  Each stub reproduces only the
behaviour the reference's call sites rely on:

* ``RepeatedResult(data, num)``          servers/fed_server.py:20-24,88-91
* ``ThreadTaskQueue(worker_fun)``        servers/server.py:15-17
* ``get_logger()``                       every server module
* ``get_device()``                       servers/fed_server.py:50 (CPU here)
* ``ModelUtil.get/load_parameter_dict``  servers/fed_server.py:17,27
* ``ModelExecutorCallbackPoint``         workers/*.py (enum names only)
* ``stochastic_quantization`` etc.       servers/fed_quant_server.py:2-6 (unused
  by the golden vectors: the stochastic re-quantization is parity-unpinned)
"""
import enum
import logging
import sys
import types

import torch


class RepeatedResult:
    def __init__(self, data, num):
        self.data = data
        self.num = num


class ThreadTaskQueue:
    """Synchronous stand-in: ``add_task`` calls ``worker_fun(task, None)``."""

    def __init__(self, worker_fun, **_):
        self.worker_fun = worker_fun
        self.results = []

    def put_result(self, result):
        self.results.append(result)

    def add_task(self, task):
        res = self.worker_fun(task, None)
        if res is not None:
            self.results.append(res)

    def get_result(self):
        res = self.results[-1]
        return res.data if isinstance(res, RepeatedResult) else res

    def stop(self):
        pass


class ModelUtil:
    def __init__(self, model):
        self.model = model

    def get_parameter_dict(self, detach=True):
        return {k: v.detach().clone() for k, v in self.model.named_parameters()}

    def load_parameter_dict(self, parameter_dict):
        with torch.no_grad():
            for k, v in self.model.named_parameters():
                v.copy_(parameter_dict[k])


class ModelExecutorCallbackPoint(enum.Enum):
    AFTER_EXECUTE = enum.auto()
    OPTIMIZER_STEP = enum.auto()


def _mod(name, **attrs):
    m = types.ModuleType(name)
    for k, v in attrs.items():
        setattr(m, k, v)
    sys.modules[name] = m
    return m


def install():
    log = logging.getLogger("ref")
    _mod("cyy_naive_lib")
    _mod("cyy_naive_lib.log", get_logger=lambda: log, set_file_handler=lambda *_: None)
    _mod("cyy_naive_lib.data_structure")
    _mod("cyy_naive_lib.data_structure.task_queue", RepeatedResult=RepeatedResult)
    _mod("cyy_naive_lib.data_structure.thread_task_queue", ThreadTaskQueue=ThreadTaskQueue)
    _mod("cyy_naive_pytorch_lib")
    _mod("cyy_naive_pytorch_lib.data_structure")
    _mod(
        "cyy_naive_pytorch_lib.data_structure.torch_process_task_queue",
        TorchProcessTaskQueue=ThreadTaskQueue,
    )
    _mod("cyy_naive_pytorch_lib.device", get_device=lambda: torch.device("cpu"),
         get_cpu_device=lambda: torch.device("cpu"))
    _mod("cyy_naive_pytorch_lib.model_util", ModelUtil=ModelUtil)
    _mod("cyy_naive_pytorch_lib.model_executor",
         ModelExecutorCallbackPoint=ModelExecutorCallbackPoint)
    _mod("cyy_naive_pytorch_lib.trainer", Trainer=object)
    _mod("cyy_naive_pytorch_lib.algorithm")
    _mod("cyy_naive_pytorch_lib.algorithm.quantization")
    _mod("cyy_naive_pytorch_lib.algorithm.quantization.scheme",
         stochastic_quantization=lambda level: (None, None))
    _mod("cyy_naive_pytorch_lib.tensor", concat_dict_values=None,
         get_data_serialization_size=None, load_dict_values=None)

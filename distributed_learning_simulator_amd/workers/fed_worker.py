"""FedAvg worker (reference: workers/fed_worker.py:8-39).

Same protocol: load the server's initial model, train ``round`` times, and
after each ``trainer.train()`` (AFTER_EXECUTE callback) send
``(worker_id, len(dataset), parameter_dict)`` and load the aggregate.  The
parameter dict stays on the worker's GPU (the reference's server then copies it
with ``.to(device)``, servers/fed_server.py:58); here the server's store copies
it device-to-device into the client's HBM row.
"""
import logging

from ..model_util import ModelUtil
from ..trainer import ModelExecutorCallbackPoint
from .worker import Worker

log = logging.getLogger("distributed_learning_simulator_amd")


def dataset_size(dataset):
    """len(trainer.dataset) (workers/fed_worker.py:34); (X, y) tuples count samples."""
    if isinstance(dataset, (tuple, list)) and len(dataset) == 2 and hasattr(dataset[0], "shape"):
        return int(dataset[0].shape[0])
    return len(dataset)


class FedWorker(Worker):
    def __init__(self, **kwargs):
        worker_round = kwargs.pop("round")
        super().__init__(**kwargs)
        self.round = worker_round
        self.trainer.add_named_callback(ModelExecutorCallbackPoint.AFTER_EXECUTE,
                                        "send_parameter", self.__send_parameters)

    def train(self, device):
        self.trainer.set_device(device)
        parameter_dict = self.worker_data_queue.get_result()
        ModelUtil(self.trainer.model).load_parameter_dict(parameter_dict)
        log.info("end load initial parameter_dict")
        for _ in range(self.round):
            self.trainer.train()

    def __send_parameters(self, **kwargs):
        trainer = kwargs["model_executor"]
        parameter_dict = ModelUtil(trainer.model).get_parameter_dict(detach=True)
        log.info("add_parameter_dict")
        self.worker_data_queue.add_task((self.worker_id, dataset_size(trainer.dataset), parameter_dict))
        log.info("end add_parameter_dict")
        parameter_dict = self.worker_data_queue.get_result()
        ModelUtil(trainer.model).load_parameter_dict(parameter_dict)
        log.info("end load_parameter_dict")

"""Server base: owns the task queue (reference: servers/server.py:6-35)."""
from ..model_util import get_device
from ..task_queue import SynchronousTaskQueue, ThreadTaskQueue


class Server:
    def __init__(self, tester, worker_number, multi_process: bool = False, device=None,
                 synchronous: bool = False):
        """Same arguments as the reference (servers/server.py:7).

        ``multi_process`` selected ``TorchProcessTaskQueue`` in the reference; here
        cross-process exchange is RCCL (``distributed.py``), so both values use the
        in-process queue.  ``device`` (default: current GPU) and ``synchronous``
        (run hooks on the caller's thread) are additions.
        """
        self.__tester = tester
        self.__worker_num = worker_number
        self.device = device if device is not None else get_device()
        queue_cls = SynchronousTaskQueue if synchronous else ThreadTaskQueue
        self.__worker_data_queue = queue_cls(worker_fun=self._process_worker_data,
                                             device=self.device)

    @property
    def tester(self):
        return self.__tester

    @property
    def worker_number(self):
        return self.__worker_num

    @property
    def worker_data_queue(self):
        return self.__worker_data_queue

    def stop(self):
        self.worker_data_queue.stop()

    def _process_worker_data(self, *args, **kwargs):
        pass

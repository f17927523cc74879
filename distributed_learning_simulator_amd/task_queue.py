"""In-process task queue — the reference's "communication backend".

The reference's servers own a ``ThreadTaskQueue(worker_fun=...)`` from the
absent ``cyy_naive_lib`` (servers/server.py:15-17): workers ``add_task`` their
payload (workers/fed_worker.py:33-35), a queue thread runs the server's
``_process_worker_data(task, extra)`` and every non-None return is published
with ``put_result``; workers block in ``get_result`` (workers/fed_worker.py:37).
A ``RepeatedResult(data, num)`` (servers/fed_server.py:88-91) is handed to
``num`` consumers before it is retired.  This module restates that contract.
"""
import collections
import threading

import torch


class RepeatedResult:
    """A result handed to ``num`` distinct consumers (servers/fed_server.py:88-91)."""

    def __init__(self, data, num):
        self.data = data
        self.num = num
        self.consumers = set()


_STOP = object()
_consumer = threading.local()  # a fresh token per thread (thread idents are reused)
_consumer_ids = iter(range(1 << 62))
_consumer_lock = threading.Lock()


def _thread_token():
    tok = getattr(_consumer, "token", None)
    if tok is None:
        with _consumer_lock:
            tok = _consumer.token = ("thread", next(_consumer_ids))
    return tok


class ThreadTaskQueue:
    def __init__(self, worker_fun, device=None):
        self._worker_fun = worker_fun
        self._device = device
        self._tasks = collections.deque()
        self._results = collections.deque()
        self._cv = threading.Condition()
        self._error = None
        self._thread = threading.Thread(target=self._loop, name="dls-server-queue", daemon=True)
        self._thread.start()

    def _loop(self):
        if self._device is not None and self._device.type == "cuda":
            torch.cuda.set_device(self._device)
        while True:
            with self._cv:
                while not self._tasks:
                    self._cv.wait()
                task = self._tasks.popleft()
            if task is _STOP:
                return
            try:
                res = self._worker_fun(task, None)
            except BaseException as e:  # surfaced to every get_result caller
                with self._cv:
                    self._error = e
                    self._cv.notify_all()
                continue
            if res is not None:
                self.put_result(res)

    def add_task(self, task):
        with self._cv:
            self._tasks.append(task)
            self._cv.notify_all()

    def put_result(self, result):
        with self._cv:
            self._results.append(result)
            self._cv.notify_all()

    def get_result(self, timeout=None, consumer=None):
        """Next result this consumer (default: the calling thread) has not taken yet.

        A fast worker that asks for round r+1 while slower workers still hold
        round r's broadcast must not take round r's copy twice, so a
        RepeatedResult is served once per consumer and retired after ``num``."""
        key = _thread_token() if consumer is None else consumer

        def pick():
            for i, r in enumerate(self._results):
                if isinstance(r, RepeatedResult):
                    if key not in r.consumers:
                        return i
                else:
                    return i
            return None

        with self._cv:
            ok = self._cv.wait_for(lambda: pick() is not None or self._error is not None, timeout)
            if self._error is not None:
                raise RuntimeError("server queue task failed") from self._error
            if not ok:
                raise TimeoutError("ThreadTaskQueue.get_result timed out")
            i = pick()
            r = self._results[i]
            if isinstance(r, RepeatedResult):
                r.consumers.add(key)
                if len(r.consumers) >= r.num:
                    del self._results[i]
                return r.data
            del self._results[i]
            return r

    def stop(self):
        self.add_task(_STOP)
        self._thread.join()


class SynchronousTaskQueue(ThreadTaskQueue):
    """Runs ``worker_fun`` on the caller's thread (deterministic tests, SPMD ranks)."""

    def __init__(self, worker_fun, device=None):
        self._worker_fun = worker_fun
        self._results = collections.deque()
        self._cv = threading.Condition()
        self._error = None

    def add_task(self, task):
        res = self._worker_fun(task, None)
        if res is not None:
            self.put_result(res)

    def stop(self):
        pass

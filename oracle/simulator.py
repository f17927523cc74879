"""Config 1 on the CPU — the reference's FedAvg simulator loop restated (TEST
INFRASTRUCTURE, see oracle/__init__.py: only bench.py's ``cpu_baseline`` leg
times it).

Reference flow, FedAvg with K workers for R rounds (simulator.py:33-72):

* IID split of the training set over the K workers (simulator.py:48-50);
* every worker starts from the server's initial broadcast, the tester's model
  (servers/fed_server.py:16-24, workers/fed_worker.py:22-23), and per round runs
  ``trainer.train()`` — ``epoch`` epochs of SGD on its shard
  (workers/fed_worker.py:25-26) — then sends ``(worker_id, len(dataset),
  parameter_dict)`` (workers/fed_worker.py:28-35);
* the server, once all K are in, averages them with ``get_subset_model``'s torch
  op sequence in arrival order (servers/fed_server.py:44-66, 81: restated by
  ``oracle.fedavg.fedavg_torch_cpu``), deep-copies the result, measures the test
  accuracy of the shared tester (servers/fed_server.py:84-86) and broadcasts it;
  every worker loads it (workers/fed_worker.py:37-39).

The reference's workers are threads that train concurrently and arrive in
whatever order; here they train one after the other on the host cores (torch's
intra-op threads) and arrive in worker-id order, the same work per round.  The
models and synthetic data are the ones the GPU simulator uses
(distributed_learning_simulator_amd.models): the reference's come from an
absent library.
"""
import copy
import time

import torch

from .fedavg import fedavg_torch_cpu


def _train_epochs(model, X, y, epochs, batch_size, lr, gen):
    opt = torch.optim.SGD(model.parameters(), lr=lr)
    model.train()
    for _ in range(epochs):
        perm = torch.randperm(X.shape[0], generator=gen)
        for i in range(0, X.shape[0], batch_size):
            idx = perm[i:i + batch_size]
            opt.zero_grad(set_to_none=True)
            torch.nn.functional.cross_entropy(model(X[idx]), y[idx]).backward()
            opt.step()


@torch.no_grad()
def _accuracy(model, X, y, batch_size=1024):
    model.eval()
    correct = 0
    for i in range(0, X.shape[0], batch_size):
        correct += int((model(X[i:i + batch_size]).argmax(1) == y[i:i + batch_size]).sum())
    return correct / X.shape[0]


def run_fedavg_cpu(model_cls, train, test, worker_number, rounds, epoch=1, batch_size=64,
                   learning_rate=0.01, seed=0, max_seconds=None):
    """Runs up to ``rounds`` FedAvg rounds on the CPU; returns the per-round wall
    times (s) and test accuracies.  ``max_seconds`` bounds the sample: no new
    round starts once that much time has passed (at least one round runs)."""
    X, y = train
    Xt, yt = test
    torch.manual_seed(seed)
    tester = model_cls()
    global_model = {k: v.detach().clone() for k, v in tester.named_parameters()}
    perm = torch.randperm(X.shape[0], generator=torch.Generator().manual_seed(seed))
    shards = torch.chunk(perm, worker_number)
    workers = [model_cls() for _ in range(worker_number)]
    gens = [torch.Generator().manual_seed(seed + w) for w in range(worker_number)]
    times, accs = [], []
    t_start = time.perf_counter()
    for _ in range(rounds):
        t0 = time.perf_counter()
        sent, ns = [], []
        for w, model in enumerate(workers):
            with torch.no_grad():
                for k, p in model.named_parameters():
                    p.copy_(global_model[k])
            idx = shards[w]
            _train_epochs(model, X[idx], y[idx], epoch, batch_size, learning_rate, gens[w])
            sent.append({k: p.detach().clone() for k, p in model.named_parameters()})
            ns.append(int(idx.numel()))
        avg = fedavg_torch_cpu(sent, ns, list(range(worker_number)))
        global_model = copy.deepcopy(avg)
        with torch.no_grad():
            for k, p in tester.named_parameters():
                p.copy_(global_model[k])
        accs.append(_accuracy(tester, Xt, yt))
        times.append(time.perf_counter() - t0)
        if max_seconds is not None and time.perf_counter() - t_start >= max_seconds:
            break
    return times, accs

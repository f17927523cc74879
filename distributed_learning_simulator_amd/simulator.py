"""Simulator entry point (reference: simulator.py:18-72, config.py:6-25, simulator.sh).

    python -m distributed_learning_simulator_amd.simulator --dataset_name MNIST \\
        --model_name LeNet5 --distributed_algorithm fed --worker_number 10 --round 5 \\
        --epoch 1 --learning_rate 0.01 --log_level INFO [--aggregation_mode fma]

Same flags and flow as the reference: IID split of the training set over the
workers (:48-50), a tester on the test split (:51), ``factory.get_server``
(:52-57), one thread per worker placed on GPU ``worker_id % ngpu`` (:59-69),
per-run log file ``log/<algo>/<dataset>/<model>/<date>.log`` (:38-46).
Datasets are synthetic of the named shape (no network: MNIST-shaped 1x32x32 /
CIFAR-shaped 3x32x32, 10 classes, learnable class templates + noise).
"""
import argparse
import datetime
import logging
import os
import threading

import torch

from .factory import get_server, get_worker
from .models import MODELS, synthetic_classification
from .trainer import Inferencer, Trainer

DATASETS = {"MNIST": (1, 32, 32), "CIFAR10": (3, 32, 32)}


def get_config(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--distributed_algorithm", type=str, required=True)
    ap.add_argument("--worker_number", type=int, required=True)
    ap.add_argument("--round", type=int, required=True)
    ap.add_argument("--dataset_name", type=str, default="MNIST")
    ap.add_argument("--model_name", type=str, default="LeNet5")
    ap.add_argument("--epoch", type=int, default=1)
    ap.add_argument("--learning_rate", type=float, default=0.01)
    ap.add_argument("--optimizer_name", type=str, default="SGD")
    ap.add_argument("--momentum", type=float, default=0.0)
    ap.add_argument("--weight_decay", type=float, default=0.0)
    ap.add_argument("--batch_size", type=int, default=64)
    ap.add_argument("--log_level", type=str, default="INFO")
    ap.add_argument("--train_size", type=int, default=10000)
    ap.add_argument("--test_size", type=int, default=2000)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--log_dir", type=str, default="log")
    # the FedAvg arithmetic of the fed / fed_quant / Shapley servers: "exact" (the
    # reference's op order, bit for bit) or "fma" (one fused multiply-add per
    # element and client, within the north star's normwise 1e-6 FedAvg tolerance;
    # the fed_quant path that meets the 80 % HBM bar)
    ap.add_argument("--aggregation_mode", type=str, default="exact", choices=("exact", "fma"))
    # the tester's convolutions (trainer.Inferencer): "dls", the library's
    # deterministic bf16x3 ones (a coalition's utility the same bits in every
    # process), or "miopen", torch's fp32 forward with MIOpen's deterministic
    # algorithms (the reference tester's arithmetic, ~4x slower)
    ap.add_argument("--tester_conv", type=str, default="dls", choices=("dls", "miopen"))
    return ap.parse_args(argv)


def server_kwargs(config):
    """The keyword arguments run() passes to factory.get_server beside tester /
    worker_number / multi_process: the aggregation mode for the FedAvg-based
    servers (sign_SGD votes; it has no FedAvg)."""
    if config.distributed_algorithm == "sign_SGD":
        return {}
    return {"aggregation_mode": config.aggregation_mode}


def get_cuda_devices():
    return [torch.device("cuda", i) for i in range(torch.cuda.device_count())]


def run(config, devices=None, sharded=None):
    """simulator.py:33-72.  ``devices``: the GPUs the worker threads use (default all
    visible); ``sharded``: get_server's (default: sharded servers when
    torch.distributed is initialised with more than one rank) — a caller that runs
    a one-process simulation inside a multi-rank job passes False."""
    log = logging.getLogger("distributed_learning_simulator_amd")
    log.setLevel(config.log_level)
    if config.log_dir:
        path = os.path.join(config.log_dir, config.distributed_algorithm, config.dataset_name,
                            config.model_name,
                            "{date:%Y-%m-%d_%H:%M:%S}.log".format(date=datetime.datetime.now()))
        os.makedirs(os.path.dirname(path), exist_ok=True)
        log.addHandler(logging.FileHandler(path))
    shape = DATASETS[config.dataset_name]
    X, y = synthetic_classification(config.train_size, shape, seed=config.seed)
    Xt, yt = synthetic_classification(config.test_size, shape, seed=config.seed + 1)
    torch.manual_seed(config.seed)
    model_cls = MODELS[config.model_name]
    devices = list(devices) if devices else get_cuda_devices()
    server_device = devices[0]
    tester = Inferencer(model_cls().to(server_device), (Xt, yt), device=server_device,
                        conv=getattr(config, "tester_conv", "dls"))
    server = get_server(config.distributed_algorithm, sharded=sharded, tester=tester,
                        worker_number=config.worker_number, multi_process=False,
                        **server_kwargs(config))
    # IID split (simulator.py:48-50)
    perm = torch.randperm(X.shape[0], generator=torch.Generator().manual_seed(config.seed))
    shards = torch.chunk(perm, config.worker_number)
    errors = []

    def create_worker_and_train(worker_id, device):
        try:
            torch.cuda.set_device(device)
            idx = shards[worker_id]
            trainer = Trainer(model_cls(), (X[idx], y[idx]), (Xt, yt), epoch=config.epoch,
                              batch_size=config.batch_size, learning_rate=config.learning_rate,
                              momentum=config.momentum, weight_decay=config.weight_decay,
                              optimizer_name=config.optimizer_name, device=device,
                              seed=config.seed + worker_id)
            worker = get_worker(config.distributed_algorithm, trainer=trainer,
                                worker_data_queue=server.worker_data_queue, round=config.round,
                                worker_id=worker_id)
            worker.train(device=device)
        except BaseException as e:  # surfaced after join
            errors.append(e)
            raise

    threads = [threading.Thread(target=create_worker_and_train,
                                args=(i, devices[i % len(devices)]), daemon=True)
               for i in range(config.worker_number)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    server.stop()
    if errors:
        raise RuntimeError("worker failed") from errors[0]
    return server


def main(argv=None):
    logging.basicConfig(format="%(asctime)s %(levelname)s %(message)s")
    config = get_config(argv)
    server = run(config)
    acc = None
    if hasattr(server, "prev_model") and server.tester is not None and server.prev_model:
        acc = server.get_metric(server.prev_model)
    print(f"finished {config.distributed_algorithm}: rounds={getattr(server, 'round', None)} "
          f"test_accuracy={acc}")
    return server


if __name__ == "__main__":
    main()

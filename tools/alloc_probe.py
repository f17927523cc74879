#!/usr/bin/env python3
"""Probe: FedAvg (K=100 ResNet-18) time on client rows from torch's allocator vs
hipExtMallocWithFlags(default / contiguous), several allocations each."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from distributed_learning_simulator_amd.layout import ParameterLayout  # noqa: E402
from distributed_learning_simulator_amd.model_shapes import resnet18_cifar  # noqa: E402
from tools.timing_probe import time_fedavg  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")


class Raw:
    def __init__(self, ptr, shape):
        self.__cuda_array_interface__ = {"shape": shape, "typestr": "<f4",
                                         "data": (ptr, False), "version": 2}


def hip_alloc(nbytes, flags):
    p = ctypes.c_void_p()
    rc = hip.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(nbytes), ctypes.c_uint(flags))
    assert rc == 0, rc
    return p.value


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    P = ParameterLayout(resnet18_cifar()).P
    K = 100
    g = torch.Generator(device=dev).manual_seed(1)
    n = torch.randint(100, 1000, (K,), generator=g, device=dev).tolist()
    rows = torch.arange(K, dtype=torch.int32, device=dev)
    w = torch.tensor(n, dtype=torch.float32, device=dev)
    out = torch.empty(P, device=dev)
    tot = float(sum(n))
    for label in os.environ.get("PROBE_ORDER", "contig,default,torch").split(","):
        res, keep = [], []
        for i in range(5):
            if label == "torch":
                buf = torch.empty((K, P), device=dev)
            else:
                ptr = hip_alloc(K * P * 4, 0x4 if label == "contig" else 0x0)
                buf = torch.as_tensor(Raw(ptr, (K, P)), device=dev)
            buf.normal_(generator=g).mul_(0.05)
            res.append(round(time_fedavg(buf, rows, w, tot, P, out), 1))
            keep.append(buf)
        print(f"{label:8s} (us): {res}", flush=True)


if __name__ == "__main__":
    main()

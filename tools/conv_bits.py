#!/usr/bin/env python3
"""ResNet-18 logits of the library's convolutions (models.ResNet18.forward_split) on
seeded weights and 4,096 seeded CIFAR-shaped images, saved to / compared with a
file: run once per library build (DLS_HIP_LIB=...) to check that two builds give
the same bits.

    DLS_HIP_LIB=tools/_variants/libdls_old.so python tools/conv_bits.py save gpurun_out/x/ref.pt
    DLS_HIP_LIB=tools/_variants/libdls_new.so python tools/conv_bits.py check gpurun_out/x/ref.pt
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def logits():
    from distributed_learning_simulator_amd.models import ResNet18, synthetic_classification
    dev = torch.device("cuda", 0)
    torch.manual_seed(11)
    model = ResNet18().to(dev).eval()
    g = torch.Generator().manual_seed(12)
    with torch.no_grad():
        for m in model.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.running_mean.copy_(torch.randn(m.num_features, generator=g) * 0.1)
                m.running_var.copy_(torch.rand(m.num_features, generator=g) + 0.5)
                m.weight.copy_(torch.rand(m.num_features, generator=g) + 0.5)
                m.bias.copy_(torch.randn(m.num_features, generator=g) * 0.1)
        X, _ = synthetic_classification(4096, (3, 32, 32), seed=13)
        X = X.to(dev)
        X[0, 0, 0, :4] = torch.tensor([float("nan"), float("inf"), -float("inf"), 1e-40])  # non-finite inputs
        return model.forward_split(X, model.pack_split()).cpu()


def main(mode, path):
    y = logits()
    if mode == "save":
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        torch.save(y, path)
        print("saved", path, tuple(y.shape))
        return 0
    ref = torch.load(path, weights_only=True)
    same = torch.equal(y.view(torch.int32), ref.view(torch.int32))
    print("logits bit-identical to", path, ":", same)
    return 0 if same else 1


if __name__ == "__main__":
    sys.exit(main(sys.argv[1], sys.argv[2]))

#!/usr/bin/env python3
"""Where does ResNet-18's fused eval forward first differ from the module's?"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from distributed_learning_simulator_amd import _native  # noqa: E402
from distributed_learning_simulator_amd.models import ResNet18, synthetic_classification  # noqa: E402

dev = torch.device("cuda", 0)


def same(a, b):
    return torch.equal(a.contiguous().view(torch.int32), b.contiguous().view(torch.int32))


def main():
    torch.manual_seed(0)
    model = ResNet18().to(dev)
    g = torch.Generator().manual_seed(1)
    with torch.no_grad():
        for m in model.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.running_mean.copy_(torch.randn(m.num_features, generator=g) * 0.1)
                m.running_var.copy_(torch.rand(m.num_features, generator=g) + 0.5)
                m.weight.copy_(torch.rand(m.num_features, generator=g) + 0.5)
                m.bias.copy_(torch.randn(m.num_features, generator=g) * 0.1)
    X, _ = synthetic_classification(600, (3, 32, 32), seed=3)
    model.eval().to(memory_format=torch.channels_last)
    xb = X.to(dev).contiguous(memory_format=torch.channels_last)
    fold = model.fold_bn()
    with torch.no_grad():
        r1 = model(xb)
        r2 = model(xb)
        f1 = model.forward_fused(xb, fold)
        f2 = model.forward_fused(xb, fold)
        print("module twice identical", same(r1, r2), "fused twice identical", same(f1, f2),
              "fused vs module", same(f1, r1), flush=True)
        c = model.conv1(xb)
        a = F.relu(model.bn1(c))
        b = _native.bn_act_exact_nhwc(c, fold[id(model.bn1)], relu=True)
        print("stem conv out contiguous(cl)", c.is_contiguous(memory_format=torch.channels_last),
              "stem bn+relu identical", same(a, b), flush=True)
        out_m, out_f = a, b
        for li, layer in enumerate((model.layer1, model.layer2, model.layer3, model.layer4)):
            for bi, blk in enumerate(layer):
                om = blk(out_m)
                of = blk.forward_fused(out_m.clone(memory_format=torch.channels_last), fold)
                c1 = blk.conv1(out_m)
                c1b = blk.conv1(out_m.clone(memory_format=torch.channels_last))
                h_m = F.relu(blk.bn1(c1))
                h_f = _native.bn_act_exact_nhwc(c1, fold[id(blk.bn1)], relu=True)
                c2m = blk.conv2(h_m)
                c2f = blk.conv2(h_f)
                print(f"layer{li + 1}.{bi}: block identical {same(om, of)}; conv1 repeat {same(c1, c1b)}; "
                      f"bn1+relu {same(h_m, h_f)}; conv2 on those {same(c2m, c2f)}; "
                      f"h_m cl {h_m.is_contiguous(memory_format=torch.channels_last)} "
                      f"h_f cl {h_f.is_contiguous(memory_format=torch.channels_last)} "
                      f"strides {h_m.stride()} {h_f.stride()}", flush=True)
                out_m = om


if __name__ == "__main__":
    main()

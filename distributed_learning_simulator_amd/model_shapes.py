"""Parameter shape tables of the models the BASELINE configs name.

The reference builds its models inside the absent ``cyy_naive_pytorch_lib``;
these are the standard architectures' ``named_parameters`` shapes (conv
weights, batch-norm affine parameters, linear layers), used to lay out
synthetic client updates of the right size and tensor mix:

* ResNet-18, CIFAR-10 head (3x3 stem, no max-pool): 11,173,962 parameters, 62 tensors
* VGG-16, ImageNet head: 138,357,544 parameters, 32 tensors
* LeNet-5 (MNIST): 61,706 parameters, 10 tensors
"""
import math


def resnet18_cifar(num_classes=10):
    shapes = [("conv1.weight", (64, 3, 3, 3)), ("bn1.weight", (64,)), ("bn1.bias", (64,))]
    cin = 64
    for li, cout in enumerate([64, 128, 256, 512], start=1):
        for b in range(2):
            stride = 2 if (li > 1 and b == 0) else 1
            pre = f"layer{li}.{b}"
            shapes += [(f"{pre}.conv1.weight", (cout, cin, 3, 3)), (f"{pre}.bn1.weight", (cout,)),
                       (f"{pre}.bn1.bias", (cout,)), (f"{pre}.conv2.weight", (cout, cout, 3, 3)),
                       (f"{pre}.bn2.weight", (cout,)), (f"{pre}.bn2.bias", (cout,))]
            if stride != 1 or cin != cout:
                shapes += [(f"{pre}.shortcut.0.weight", (cout, cin, 1, 1)),
                           (f"{pre}.shortcut.1.weight", (cout,)),
                           (f"{pre}.shortcut.1.bias", (cout,))]
            cin = cout
    shapes += [("linear.weight", (num_classes, 512)), ("linear.bias", (num_classes,))]
    return shapes


def vgg16(num_classes=1000):
    cfg = [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"]
    shapes, cin, i = [], 3, 0
    for v in cfg:
        if v == "M":
            i += 1
            continue
        shapes += [(f"features.{i}.weight", (v, cin, 3, 3)), (f"features.{i}.bias", (v,))]
        cin = v
        i += 2
    shapes += [("classifier.0.weight", (4096, 512 * 7 * 7)), ("classifier.0.bias", (4096,)),
               ("classifier.3.weight", (4096, 4096)), ("classifier.3.bias", (4096,)),
               ("classifier.6.weight", (num_classes, 4096)), ("classifier.6.bias", (num_classes,))]
    return shapes


def lenet5(num_classes=10):
    return [("conv1.weight", (6, 1, 5, 5)), ("conv1.bias", (6,)),
            ("conv2.weight", (16, 6, 5, 5)), ("conv2.bias", (16,)),
            ("fc1.weight", (120, 400)), ("fc1.bias", (120,)),
            ("fc2.weight", (84, 120)), ("fc2.bias", (84,)),
            ("fc3.weight", (num_classes, 84)), ("fc3.bias", (num_classes,))]


def numel(shapes):
    return sum(math.prod(s) for _, s in shapes)


SHAPES = {"resnet18": resnet18_cifar, "vgg16": vgg16, "lenet5": lenet5}

"""Model definitions for the BASELINE configs (random init; no checkpoints).

Parameter names and shapes match ``model_shapes`` (LeNet-5 61,706 params,
ResNet-18/CIFAR-10 11,173,962 params).  The reference builds its models in the
absent ``cyy_naive_pytorch_lib``; these standard definitions stand in.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F


class LeNet5(nn.Module):
    def __init__(self, num_classes=10):
        super().__init__()
        self.conv1 = nn.Conv2d(1, 6, 5)
        self.conv2 = nn.Conv2d(6, 16, 5)
        self.fc1 = nn.Linear(400, 120)
        self.fc2 = nn.Linear(120, 84)
        self.fc3 = nn.Linear(84, num_classes)

    def forward(self, x):  # x: [B, 1, 32, 32]
        x = F.max_pool2d(F.relu(self.conv1(x)), 2)
        x = F.max_pool2d(F.relu(self.conv2(x)), 2)
        x = x.flatten(1)
        return self.fc3(F.relu(self.fc2(F.relu(self.fc1(x)))))


class _Block(nn.Module):
    def __init__(self, cin, cout, stride):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, cout, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(cout)
        self.conv2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(cout)
        self.shortcut = nn.Sequential()
        if stride != 1 or cin != cout:
            self.shortcut = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False),
                                          nn.BatchNorm2d(cout))

    def forward(self, x):
        out = F.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        return F.relu(out + self.shortcut(x))

    def forward_fused(self, x, fold):
        """Eval-mode forward: each batch norm (with the ReLU / residual add after it)
        is one dls_bn_act_exact_{nhwc,nchw}_f32 pass (the activation's layout), in
        place on the convolution's output; the same ops and roundings as forward()
        on the GPU, so the same bits."""
        from . import _native
        out = _native.bn_act_exact(self.conv1(x), fold[id(self.bn1)], relu=True, inplace=True)
        out = self.conv2(out)
        if len(self.shortcut):
            sc = _native.bn_act_exact(self.shortcut[0](x), fold[id(self.shortcut[1])],
                                           relu=False, inplace=True)
        else:
            sc = x
        return _native.bn_act_exact(out, fold[id(self.bn2)], residual=sc, relu=True,
                                         inplace=True)


class ResNet18(nn.Module):
    """CIFAR-10 ResNet-18 (3x3 stem, no max-pool)."""

    def __init__(self, num_classes=10):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, 3, 1, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        layers, cin = [], 64
        for li, cout in enumerate([64, 128, 256, 512]):
            blocks = []
            for b in range(2):
                stride = 2 if (li > 0 and b == 0) else 1
                blocks.append(_Block(cin, cout, stride))
                cin = cout
            layers.append(nn.Sequential(*blocks))
        self.layer1, self.layer2, self.layer3, self.layer4 = layers
        self.linear = nn.Linear(512, num_classes)

    def forward(self, x):
        out = F.relu(self.bn1(self.conv1(x)))
        out = self.layer4(self.layer3(self.layer2(self.layer1(out))))
        out = F.adaptive_avg_pool2d(out, 1).flatten(1)
        return self.linear(out)

    @torch.no_grad()
    def fold_bn(self):
        """{id(bn): consts [4*C] = [mean | iv | w | b]} of every batch norm for
        forward_fused (eval mode, running statistics; recomputed per evaluation
        since the weights change; dls_bn_fold_exact_f32)."""
        from . import _native
        fold = {}
        for m in self.modules():
            if isinstance(m, nn.BatchNorm2d):
                c = torch.empty(4 * m.num_features, device=m.running_mean.device)
                _native.bn_fold_exact(m, c)
                fold[id(m)] = c
        return fold

    @torch.no_grad()
    def pack_split(self):
        """The operands of forward_split: {id(conv): split weights}, {id(bn):
        exact eval batch-norm consts} and {id(linear): (weight, bias) copies}
        (recomputed per evaluation: the weights change with the coalition).  The
        forward reads nothing else of the module, so the module may be overwritten
        once this returns while the forward is still queued on another stream."""
        from . import _native
        pk = {}
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                if m.bias is not None or m.groups != 1 or m.dilation != (1, 1):
                    raise RuntimeError("forward_split: plain bias-free convolutions only")
                # the 3-channel stem as a 1x1 convolution over its im2col (27 -> 32
                # channels instead of 9 taps x 32 padded ones)
                pack = (_native.conv_pack_weights_im2col if m is self.conv1
                        else _native.conv_pack_weights)
                pk[id(m)] = pack(m.weight.contiguous())
            elif isinstance(m, nn.BatchNorm2d):
                c = torch.empty(4 * m.num_features, device=m.running_mean.device)
                _native.bn_fold_exact(m, c)
                pk[id(m)] = c
            elif isinstance(m, nn.Linear):
                pk[id(m)] = (m.weight.detach().contiguous().clone(),
                             None if m.bias is None else m.bias.detach().contiguous().clone())
        return pk

    def split_activation_bytes(self, H, W):
        """Device bytes one image holds at the peak of forward_split at H x W inputs:
        the fp32 input plus four split activations (4 B per element: a block's
        input, h, shortcut and output) at the largest (pixels x channels) of any
        layer; Inferencer.split_batch sizes the forward batch with it."""
        ho = (H + 2 * self.conv1.padding[0] - self.conv1.kernel_size[0]) // self.conv1.stride[0] + 1
        wo = (W + 2 * self.conv1.padding[1] - self.conv1.kernel_size[1]) // self.conv1.stride[1] + 1
        peak = ho * wo * self.conv1.out_channels
        for layer in (self.layer1, self.layer2, self.layer3, self.layer4):
            for blk in layer:
                s = blk.conv1.stride[0]
                ho, wo = (ho - 1) // s + 1, (wo - 1) // s + 1
                peak = max(peak, ho * wo * blk.conv1.out_channels)
        return 4 * self.conv1.in_channels * H * W + 4 * 4 * peak

    def forward_split(self, x, pk):
        """forward() for the utility evaluation on the GPU with the library's
        deterministic convolutions (csrc/conv.hip): every conv + eval batch norm
        (+ residual add) + ReLU one launch over split NHWC activations, then the
        pooled linear layer; the same bits for the same model and input in any
        process.  x: NCHW fp32 [B, 3, H, W]; pk = pack_split()."""
        from . import _native

        def cba(inp, conv, bn, residual=None, relu=True):
            return _native.conv_bn_act(inp, pk[id(conv)], conv.kernel_size, conv.stride[0],
                                       conv.padding[0], pk[id(bn)], residual, relu)

        c1 = self.conv1
        if c1.kernel_size[0] * c1.kernel_size[1] * c1.in_channels <= 32:  # the im2col fused
            out = _native.conv_stem_bn_act(x.contiguous(), pk[id(c1)], c1.kernel_size, c1.stride[0],
                                           c1.padding[0], pk[id(self.bn1)], True)
        else:
            xs = _native.conv_pack_im2col(x.contiguous(), c1.kernel_size, c1.stride[0], c1.padding[0])
            out = _native.conv_bn_act(xs, pk[id(c1)], (1, 1), 1, 0, pk[id(self.bn1)], None, True)
        for layer in (self.layer1, self.layer2, self.layer3, self.layer4):
            for blk in layer:
                h = cba(out, blk.conv1, blk.bn1)
                sc = cba(out, blk.shortcut[0], blk.shortcut[1], relu=False) if len(blk.shortcut) else out
                out = cba(h, blk.conv2, blk.bn2, residual=sc)
        lw, lb = pk[id(self.linear)]
        return _native.pool_linear(out, lw, lb)

    def forward_fused(self, x, fold):
        """forward() for utility evaluation on the GPU: NHWC or NCHW activations,
        MIOpen convolutions, every batch norm + ReLU (+ residual add) fused into one
        hand-written pass (dls_bn_act_exact_nhwc_f32 / _nchw_f32) with the
        batch-norm library's own arithmetic: the logits are bit-identical to
        forward()'s (tests/test_gpu_infer.py)."""
        from . import _native
        out = _native.bn_act_exact(self.conv1(x), fold[id(self.bn1)], relu=True, inplace=True)
        for layer in (self.layer1, self.layer2, self.layer3, self.layer4):
            for blk in layer:
                out = blk.forward_fused(out, fold)
        out = F.adaptive_avg_pool2d(out, 1).flatten(1)
        return self.linear(out)


def split_conv_macs(model, H, W):
    """(issued, model) multiply-accumulates per image of ResNet18.forward_split at
    H x W inputs: issued counts the padded operands the MFMAs run on (input
    channels rounded up to 32; the stem's im2col 27 -> 32), model the convolutions'
    own (+ the linear layer, as both)."""
    shapes = {}
    hooks = [m.register_forward_hook(lambda m, i, o: shapes.__setitem__(id(m), o.shape))
             for m in model.modules() if isinstance(m, nn.Conv2d)]
    try:
        with torch.no_grad():
            p = next(model.parameters())
            model.eval()(torch.zeros(1, model.conv1.in_channels, H, W, device=p.device))
    finally:
        for h in hooks:
            h.remove()
    issued = useful = model.linear.in_features * model.linear.out_features
    for m in model.modules():
        if isinstance(m, nn.Conv2d):
            _, co, ho, wo = shapes[id(m)]
            k = m.kernel_size[0] * m.kernel_size[1]
            useful += ho * wo * co * k * m.in_channels
            if m is model.conv1:
                issued += ho * wo * co * ((k * m.in_channels + 31) // 32 * 32)
            else:
                issued += ho * wo * co * k * ((m.in_channels + 31) // 32 * 32)
    return issued, useful


MODELS = {"LeNet5": LeNet5, "ResNet18": ResNet18}


def synthetic_classification(n, shape, num_classes=10, seed=0, noise=0.7):
    """Learnable synthetic data of the named shape: class templates + Gaussian noise
    (there is no network access for MNIST / CIFAR-10)."""
    g = torch.Generator().manual_seed(seed)
    templates = torch.randn((num_classes,) + tuple(shape), generator=torch.Generator().manual_seed(1234))
    y = torch.randint(0, num_classes, (n,), generator=g)
    X = templates[y] + noise * torch.randn((n,) + tuple(shape), generator=g)
    return X.float(), y

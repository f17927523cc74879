import sys; sys.path.insert(0, '/root/repo')
import torch, numpy as np
from distributed_learning_simulator_amd.models import ResNet18, synthetic_classification
from distributed_learning_simulator_amd.trainer import Inferencer
dev = torch.device('cuda')
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
X, y = synthetic_classification(600, (3, 32, 32), seed=3)
model.eval().to(memory_format=torch.channels_last)
xb = X.to(dev).contiguous(memory_format=torch.channels_last)
def pred(tag):
    with torch.no_grad():
        o = torch.cat([model(xb[i:i + 256]) for i in range(0, 600, 256)])
        full = model(xb)
    print(tag, 'nan batches', int(torch.isnan(o).any(1).sum()), 'nan full', int(torch.isnan(full).any(1).sum()),
          'acc', float((o.argmax(1).cpu() == y).float().mean()), 'xb nan', bool(torch.isnan(xb).any()), flush=True)
pred('start')
with torch.no_grad():
    got = model.forward_fused(xb, model.fold_bn())
pred('after forward_fused')
inf = Inferencer(model, (X, y), batch_size=256, device=dev, fused_eval=True)
print('fused acc', inf.inference()[1])
pred('after fused inferencer')
plain = Inferencer(model, (X, y), batch_size=256, device=dev)
print('plain acc', plain.inference()[1])
pred('after plain inferencer')

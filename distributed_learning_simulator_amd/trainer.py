"""Minimal trainer / inferencer with the callback surface the reference uses.

The reference drives local training through the absent
``cyy_naive_pytorch_lib`` Trainer: ``trainer.train()`` runs ``--epoch``
epochs, fires ``ModelExecutorCallbackPoint.OPTIMIZER_STEP`` callbacks in place
of ``optimizer.step()`` when registered (workers/sign_sgd_worker.py:15-17) and
``AFTER_EXECUTE`` callbacks with ``model_executor=trainer`` at the end
(workers/fed_worker.py:13-17,28-39).  The server's tester exposes
``inference()``, ``accuracy_metric.get_accuracy(1)`` and
``loss_metric.get_loss(1)`` (servers/fed_server.py:26-32).  Local training is
outside the hot path; this is the plumbing config 1 needs.
"""
import enum

import torch


class ModelExecutorCallbackPoint(enum.Enum):
    BEFORE_EXECUTE = enum.auto()
    OPTIMIZER_STEP = enum.auto()
    AFTER_EXECUTE = enum.auto()


class MachineLearningPhase(enum.Enum):
    Training = enum.auto()
    Test = enum.auto()


class _Accuracy:
    def __init__(self):
        self.value = None

    def get_accuracy(self, _epoch=1):
        return self.value


class _Loss:
    def __init__(self):
        self.value = None

    def get_loss(self, _epoch=1):
        return self.value


class Inferencer:
    """The tester (ref servers/fed_server.py:26-32): top-1 accuracy / mean loss of
    ``model`` over ``dataset``.

    Models that have a ``forward_fused`` eval path (models.ResNet18) run it on the
    GPU (``fused_eval``, default on): every batch norm + ReLU (+ residual add) as
    one hand-written NHWC pass (dls_bn_act_exact_nhwc_f32) with the batch-norm
    library's own arithmetic, ~1.8x faster utility evaluations whose logits are
    bit-identical to the module's forward (tests/test_gpu_infer.py), so Shapley
    utilities are those of the plain PyTorch-ROCm model either way.
    ``fused_eval=False`` runs the module's forward."""

    def __init__(self, model, dataset, batch_size=1024, device=None, fused_eval=True):
        self.model = model
        self.fused_eval = fused_eval
        self.dataset = dataset
        self.batch_size = batch_size
        self.device = device or next(model.parameters()).device
        self.accuracy_metric = _Accuracy()
        self.loss_metric = _Loss()

    def set_device(self, device):
        self.device = torch.device(device)
        self.model.to(self.device)

    @torch.no_grad()
    def inference(self):
        X, y = self.dataset
        self.model.eval()
        if X.dim() == 4 and torch.device(self.device).type == "cuda":
            # NHWC convolutions: measured 8-18 % faster than NCHW for this model family
            # on MI355X (tools/eval_probe.py); results are the same up to fp32 reassociation
            self.model.to(memory_format=torch.channels_last)
        # a model with a fused eval forward (models.ResNet18): every batch norm + ReLU
        # (+ residual add) is one hand-written NHWC pass instead of three kernels
        fused = (getattr(self.model, "forward_fused", None)
                 if self.fused_eval and X.dim() == 4 and torch.device(self.device).type == "cuda"
                 else None)
        fold = self.model.fold_bn() if fused is not None else None
        correct = torch.zeros((), dtype=torch.int64, device=self.device)
        loss_sum = torch.zeros((), dtype=torch.float64, device=self.device)
        for i in range(0, X.shape[0], self.batch_size):
            xb = X[i:i + self.batch_size].to(self.device, non_blocking=True)
            yb = y[i:i + self.batch_size].to(self.device, non_blocking=True)
            if xb.dim() == 4 and xb.is_cuda:
                xb = xb.contiguous(memory_format=torch.channels_last)
            out = fused(xb, fold) if fused is not None else self.model(xb)
            loss_sum += torch.nn.functional.cross_entropy(out, yb, reduction="sum").double()
            correct += (out.argmax(1) == yb).sum()
        n = X.shape[0]
        # one host synchronisation per evaluation instead of two per batch
        self.accuracy_metric.value = int(correct) / n
        self.loss_metric.value = torch.tensor(float(loss_sum) / n)
        return self.loss_metric.value, self.accuracy_metric.value, None


class Trainer:
    def __init__(self, model, dataset, test_dataset=None, epoch=1, batch_size=64,
                 learning_rate=0.01, momentum=0.0, weight_decay=0.0, optimizer_name="SGD",
                 device=None, seed=0):
        self.model = model
        self.dataset = dataset
        self.test_dataset = test_dataset
        self.epoch = epoch
        self.batch_size = batch_size
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self._callbacks = {p: {} for p in ModelExecutorCallbackPoint}
        if optimizer_name == "SGD":
            self._optimizer = torch.optim.SGD(model.parameters(), lr=learning_rate,
                                              momentum=momentum, weight_decay=weight_decay)
        elif optimizer_name == "Adam":
            self._optimizer = torch.optim.Adam(model.parameters(), lr=learning_rate,
                                               weight_decay=weight_decay)
        else:
            raise ValueError(f"unknown optimizer {optimizer_name}")
        self._gen = torch.Generator().manual_seed(seed)

    def __len__(self):
        return self.dataset[0].shape[0]

    def set_device(self, device):
        self.device = torch.device(device)
        self.model.to(self.device)

    def get_optimizer(self):
        return self._optimizer

    def add_named_callback(self, point, name, fn):
        self._callbacks[point][name] = fn

    def get_inferencer(self, phase=MachineLearningPhase.Test, copy_model=False):
        model = self.model
        if copy_model:
            import copy
            model = copy.deepcopy(model)
        return Inferencer(model, self.test_dataset, device=self.device)

    def train(self):
        X, y = self.dataset
        opt = self._optimizer
        self.model.to(self.device)
        for cb in self._callbacks[ModelExecutorCallbackPoint.BEFORE_EXECUTE].values():
            cb(model_executor=self)
        for _ in range(self.epoch):
            self.model.train()
            perm = torch.randperm(X.shape[0], generator=self._gen)
            for i in range(0, X.shape[0], self.batch_size):
                idx = perm[i:i + self.batch_size]
                xb = X[idx].to(self.device, non_blocking=True)
                yb = y[idx].to(self.device, non_blocking=True)
                opt.zero_grad(set_to_none=True)
                loss = torch.nn.functional.cross_entropy(self.model(xb), yb)
                loss.backward()
                steps = self._callbacks[ModelExecutorCallbackPoint.OPTIMIZER_STEP]
                if steps:
                    for cb in steps.values():
                        cb(opt, device=self.device, model_executor=self)
                else:
                    opt.step()
        for cb in self._callbacks[ModelExecutorCallbackPoint.AFTER_EXECUTE].values():
            cb(model_executor=self)

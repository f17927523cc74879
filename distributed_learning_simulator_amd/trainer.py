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
import contextlib
import enum
import threading

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


_flags_lock = threading.Lock()
_flags_depth = 0
_flags_saved = None


@contextlib.contextmanager
def _deterministic_convs():
    """torch.backends.cudnn.deterministic = True, benchmark = False (MIOpen: only
    deterministic convolution solutions) while any inference runs; the previous
    values come back when the last one ends (nested / concurrent testers share
    one save)."""
    global _flags_depth, _flags_saved
    cudnn = torch.backends.cudnn
    with _flags_lock:
        if _flags_depth == 0:
            _flags_saved = (cudnn.deterministic, cudnn.benchmark)
            cudnn.deterministic, cudnn.benchmark = True, False
        _flags_depth += 1
    try:
        yield
    finally:
        with _flags_lock:
            _flags_depth -= 1
            if _flags_depth == 0:
                cudnn.deterministic, cudnn.benchmark = _flags_saved


class Inferencer:
    """The tester (ref servers/fed_server.py:26-32): top-1 accuracy / mean loss of
    ``model`` over ``dataset``.

    The utility of a coalition must be a function of the coalition: GTG's
    truncation tests (servers/GTG_shapley_value_server.py:29,54) and the client
    ranking compare utilities, and on several GPUs a coalition's utility must not
    depend on which rank evaluated it.

    Models with a ``forward_split`` eval path (models.ResNet18) run it on the GPU
    (``conv="dls"``, the default, with ``fused_eval``): the library's own
    convolutions (csrc/conv.hip), each fused with its eval batch norm, residual
    add and ReLU, reduced in one fixed order — the same bits for the same model
    and input in any process, with no algorithm search and no process-wide
    switches.  Their products are bf16x3 (fp32 values as bf16 pairs): the logits
    differ from the module's fp32 forward in the low bits, top-1 only at near-ties
    (tests/test_gpu_conv.py).

    ``conv="miopen"`` runs torch / MIOpen convolutions instead.  MIOpen's default
    algorithms are not run-to-run reproducible on this stack (the 512-channel
    layers of ResNet-18 gave different bits for the same input), so that path
    runs with ``torch.backends.cudnn.deterministic = True, benchmark = False``
    (``deterministic``, default on) for the duration of ``inference()`` /
    ``logits()``: torch's process-wide switches, restored after it.  MIOpen's
    deterministic solutions are NCHW ones (on channels_last it falls back to a
    naive kernel, ~19 s per 10k CIFAR images, profiles/r04q_eval_det.txt), so that
    path keeps activations NCHW; ``deterministic=False`` runs channels_last.
    There, models with a ``forward_fused`` eval path run every batch norm + ReLU
    (+ residual add) as one hand-written pass (dls_bn_act_exact_*_f32) with
    MIOpen's own batch-norm arithmetic: logits bit-identical to the module's
    forward, checked once per Inferencer on its first batch norm (if the bits
    differ it runs the module's forward).  ``fused_eval=False`` always runs the
    module's forward."""

    SPLIT_MIN_BATCH = 10000  # images per forward_split call when they fit SPLIT_MEM_FRACTION
    SPLIT_MEM_FRACTION = 0.25  # of the device's free memory for one forward's activations

    def __init__(self, model, dataset, batch_size=1024, device=None, fused_eval=True,
                 deterministic=True, conv="dls", cache_dataset=True):
        if conv not in ("dls", "miopen"):
            raise ValueError(f"Inferencer: conv must be 'dls' or 'miopen', not {conv!r}")
        self.model = model
        self.fused_eval = fused_eval
        self.deterministic = deterministic
        self.conv = conv
        self.dataset = dataset
        self.batch_size = batch_size
        self.device = device or next(model.parameters()).device
        # cache_dataset: a host-resident test set is copied to the device once and
        # kept there (a CIFAR-10 test set is 123 MB of HBM), instead of a pageable
        # host-to-device copy per evaluation; False keeps it on the host, pinned
        # once, and copies it asynchronously per evaluation
        self.cache_dataset = cache_dataset
        self._data_cache = None  # (X, y, X._version, y._version, device, Xc, yc)
        self.accuracy_metric = _Accuracy()
        self.loss_metric = _Loss()
        self._fused_checked = None  # None: not yet checked; else (layout, the check's verdict)

    def _resident_dataset(self):
        """(X, y) where the forward reads it: the dataset itself when it is already on
        the device (or the tester runs on the CPU); else the device copy
        (cache_dataset) or a pinned host copy, made on first use and remade only when
        the dataset object or its contents (tensor version counters) change."""
        X, y = self.dataset
        dev = torch.device(self.device)
        if dev.type != "cuda" or (X.device == dev and y.device == dev):
            return X, y
        c = self._data_cache
        if (c is not None and c[0] is X and c[1] is y and c[2] == X._version
                and c[3] == y._version and c[4] == dev):
            return c[5], c[6]
        self._data_cache = None  # drop the stale copy before making the new one
        if self.cache_dataset:
            Xc = X.to(dev).contiguous()
            yc = y.to(dev)
        else:
            Xc = X.contiguous().pin_memory() if X.device.type == "cpu" else X
            yc = y.contiguous().pin_memory() if y.device.type == "cpu" else y
        self._data_cache = (X, y, X._version, y._version, dev, Xc, yc)
        return Xc, yc

    def split_batch(self, n):
        """Images per forward_split call for an n-image test set: at least
        SPLIT_MIN_BATCH (one 10k-image forward is the fastest form) when that many
        images' activations fit SPLIT_MEM_FRACTION of the device's free memory,
        else as many as fit (the tester's batch_size is no lower bound: every
        image's logits are the same bits in any batch, tests/test_gpu_conv.py)."""
        per_image = self.model.split_activation_bytes(*self.dataset[0].shape[2:])
        dev = torch.device(self.device)
        free, _ = torch.cuda.mem_get_info(dev)
        # blocks the caching allocator holds but does not use are free to this forward
        free += torch.cuda.memory_reserved(dev) - torch.cuda.memory_allocated(dev)
        return split_forward_batch(n, self.batch_size, self.SPLIT_MIN_BATCH, per_image,
                                   self.SPLIT_MEM_FRACTION * free)

    def set_device(self, device):
        self.device = torch.device(device)
        self.model.to(self.device)

    def _split_forward(self):
        """model.forward_split when this Inferencer runs the library's convolutions."""
        if not (self.fused_eval and self.conv == "dls" and self.dataset[0].dim() == 4
                and torch.device(self.device).type == "cuda"):
            return None
        return getattr(self.model, "forward_split", None)

    def _flags(self):
        if (not self.deterministic or torch.device(self.device).type != "cuda"
                or self._split_forward() is not None):
            return contextlib.nullcontext()
        return _deterministic_convs()

    def _memory_format(self):
        """The activation layout of the GPU forward: NCHW with deterministic
        convolutions (MIOpen has no fast deterministic NHWC ones), else NHWC."""
        return torch.contiguous_format if self.deterministic else torch.channels_last

    def _fused_matches_module(self):
        """One eval batch norm of the model through the fused pass vs ``bn(x)`` on a
        small activation in the forward's layout: True when the bits agree."""
        from . import _native
        bn = next((m for m in self.model.modules() if isinstance(m, torch.nn.BatchNorm2d)), None)
        if bn is None:
            return True
        g = torch.Generator().manual_seed(0)
        consts = torch.empty(4 * bn.num_features, device=self.device)
        _native.bn_fold_exact(bn, consts)
        for hw in (6, 7):  # float4 planes, and planes of an odd size (the per-element path)
            x = (torch.randn(2, bn.num_features, hw, hw, generator=g) * 3).to(self.device)
            x = x.contiguous(memory_format=self._memory_format())
            y = _native.bn_act_exact(x, consts, relu=False)
            if not torch.equal(y.view(torch.int32), bn(x).view(torch.int32)):
                return False
        return True

    def _fused_forward(self, X):
        if not (self.fused_eval and X.dim() == 4 and torch.device(self.device).type == "cuda"):
            return None
        fused = getattr(self.model, "forward_fused", None)
        if fused is None:
            return None
        fmt = self._memory_format()
        if self._fused_checked is None or self._fused_checked[0] != fmt:
            self._fused_checked = (fmt, self._fused_matches_module())
            if not self._fused_checked[1]:
                import logging
                logging.getLogger("distributed_learning_simulator_amd").warning(
                    "fused eval batch norm differs from the module's on this stack; "
                    "running the module's forward")
        return fused if self._fused_checked[1] else None

    def _batches(self):
        """Logits of every batch, in order (the model in eval mode)."""
        X, y = self._resident_dataset()
        self.model.eval()
        split = self._split_forward()
        if split is not None:
            # the library's convolutions give every image the same bits whatever
            # batch it runs in (tests/test_gpu_conv.py), so the forward takes up to
            # SPLIT_MIN_BATCH images at a time when their activations fit the memory
            # budget: a 10k-image evaluation in one forward runs 3 % faster than in
            # 2,048-image ones and 4 % faster than in 1,000-image ones
            # (profiles/r05_conv_probe.txt r05bs3)
            yield from self._split_batches(X, y, split, self.model.pack_split())
            return
        fmt = self._memory_format()
        if X.dim() == 4 and torch.device(self.device).type == "cuda":
            # NHWC convolutions: measured 8-18 % faster than NCHW for this model family
            # on MI355X with MIOpen's default algorithms (tools/eval_probe.py); the
            # deterministic ones are NCHW (tools/eval_det_probe.py)
            self.model.to(memory_format=fmt)
        # a model with a fused eval forward (models.ResNet18): every batch norm + ReLU
        # (+ residual add) is one hand-written NHWC pass instead of three kernels
        fused = self._fused_forward(X)
        fold = self.model.fold_bn() if fused is not None else None
        for i in range(0, X.shape[0], self.batch_size):
            xb = X[i:i + self.batch_size].to(self.device, non_blocking=True)
            yb = y[i:i + self.batch_size].to(self.device, non_blocking=True)
            if xb.dim() == 4 and xb.is_cuda:
                xb = xb.contiguous(memory_format=fmt)
            yield (fused(xb, fold) if fused is not None else self.model(xb)), yb

    def _split_batches(self, X, y, split, pk):
        bs = self.split_batch(X.shape[0])
        for i in range(0, X.shape[0], bs):
            xb = X[i:i + bs].to(self.device, torch.float32, non_blocking=True)
            yb = y[i:i + bs].to(self.device, non_blocking=True)
            yield split(xb.contiguous(), pk), yb

    @torch.no_grad()
    def logits(self):
        """The logits ``inference()`` scores, concatenated over the dataset."""
        with self._flags():
            return torch.cat([out for out, _ in self._batches()])

    @torch.no_grad()
    def correct_async(self, stream=None):
        """The top-1 correct count over the dataset as a device int64 tensor, with
        no host synchronisation: ``inference()``'s accuracy is ``int(count) / n``.
        The Shapley servers queue a batch of coalitions' evaluations this way and
        read all counts with one synchronisation.

        ``stream``: run the forward there (the library's convolutions only; else
        it runs on the current stream).  The model's operands are packed on the
        current stream first (ResNet18.pack_split copies everything the forward
        reads), so the caller may load the next model as soon as this returns
        and queue that model's forward on another stream: two forwards in flight
        fill each other's layer ramps and memory phases.  The count is ready on
        ``stream``; make the current stream wait for it before reading it.  The
        same bits on any stream (every kernel's arithmetic is fixed by the
        shape)."""
        split = self._split_forward() if stream is not None else None
        if split is not None:
            cur = torch.cuda.current_stream(self.device)
            X, y = self._resident_dataset()
            self.model.eval()
            pk = self.model.pack_split()
            stream.wait_stream(cur)
            for t in (X, y):
                if t.is_cuda:
                    t.record_stream(stream)
            with torch.cuda.stream(stream):
                correct = torch.zeros((), dtype=torch.int64, device=self.device)
                for out, yb in self._split_batches(X, y, split, pk):
                    correct += (out.argmax(1) == yb).sum()
            for t in pk.values():  # freed by the host now, read by `stream` later
                for u in (t if isinstance(t, tuple) else (t,)):
                    if u is not None:
                        u.record_stream(stream)
            return correct
        with self._flags():
            correct = torch.zeros((), dtype=torch.int64, device=self.device)
            for out, yb in self._batches():
                correct += (out.argmax(1) == yb).sum()
        return correct

    @torch.no_grad()
    def inference(self):
        with self._flags():
            correct = torch.zeros((), dtype=torch.int64, device=self.device)
            loss_sum = torch.zeros((), dtype=torch.float64, device=self.device)
            for out, yb in self._batches():
                loss_sum += torch.nn.functional.cross_entropy(out, yb, reduction="sum").double()
                correct += (out.argmax(1) == yb).sum()
            n = self.dataset[0].shape[0]
            # one host synchronisation per evaluation instead of two per batch
            self.accuracy_metric.value = int(correct) / n
            self.loss_metric.value = torch.tensor(float(loss_sum) / n)
        return self.loss_metric.value, self.accuracy_metric.value, None


def split_forward_batch(n, batch_size, min_batch, per_image_bytes, budget_bytes):
    """The forward batch of Inferencer.split_batch: max(batch_size, min_batch)
    images (never more than n) when their activations fit the budget, else as many
    as fit (at least one)."""
    want = max(1, min(n, max(batch_size, min_batch)))
    fit = int(budget_bytes // max(1, per_image_bytes))
    return max(1, min(want, fit))


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

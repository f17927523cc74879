"""Generate the golden vectors that pin ``oracle/`` and the HIP kernels.

Runs ONLY in the build container, where the reference is mounted read-only at
/root/reference.  It imports the reference's own ``servers/*.py`` and
``workers/*.py`` (with ``_ref_stubs`` standing in for the two absent ``cyy_*``
libraries), drives them on seeded synthetic inputs, and writes
small ``.npz`` fixtures next to this file.  The fixtures are data (inputs and the
reference's outputs); no reference source is copied.

The reference's shipped ``__pycache__/*.pyc`` bytecode is never loaded:
``sys.pycache_prefix`` points the import system at an empty private directory.

    python tests/golden/make_golden.py            # rewrites tests/golden/*.npz
"""
import contextlib
import copy
import json
import math
import os
import sys
import tempfile

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"

sys.dont_write_bytecode = True
sys.pycache_prefix = tempfile.mkdtemp(prefix="dls_ref_pyc_")
sys.path.insert(0, HERE)
import _ref_stubs  # noqa: E402

_ref_stubs.install()
sys.path.insert(0, REF)

from servers.fed_quant_server import FedQuantServer  # noqa: E402
from servers.fed_server import FedServer  # noqa: E402
from servers.GTG_shapley_value_server import GTGShapleyValueServer  # noqa: E402
from servers.multiround_shapley_value_server import MultiRoundShapleyValueServer  # noqa: E402
from servers.sign_sgd_server import SignSGDServer  # noqa: E402
from workers.sign_sgd_worker import SignSGDWorker  # noqa: E402

# A small ResNet-like parameter layout with ragged tensor sizes (odd lengths,
# a 1-element tensor, a 27-element conv row) in named_parameters order.
LAYOUT_SMALL = [
    ("conv1.weight", (8, 3, 3, 3)),
    ("bn1.weight", (8,)),
    ("bn1.bias", (8,)),
    ("layer1.0.conv1.weight", (8, 8, 3, 3)),
    ("layer1.0.odd", (7,)),
    ("fc.weight", (10, 72)),
    ("fc.bias", (10,)),
    ("scale", (1,)),
]
# ~1e5 parameters, still quick for the CPU oracle.
LAYOUT_MED = [
    ("conv1.weight", (32, 3, 3, 3)),
    ("bn1.weight", (32,)),
    ("bn1.bias", (32,)),
    ("layer1.0.conv1.weight", (32, 32, 3, 3)),
    ("layer1.0.conv2.weight", (32, 32, 3, 3)),
    ("layer2.0.conv1.weight", (64, 32, 3, 3)),
    ("layer2.0.shortcut.weight", (64, 32, 1, 1)),
    ("fc.weight", (10, 1025)),
    ("fc.bias", (10,)),
]


class ParamModel(torch.nn.Module):
    def __init__(self, layout, gen):
        super().__init__()
        self._names = []
        for name, shape in layout:
            p = torch.nn.Parameter(torch.randn(*shape, generator=gen) * 0.05)
            self.register_parameter(name.replace(".", "__"), p)
            self._names.append(name)

    def named_parameters(self, *args, **kwargs):  # keep dotted names
        for name in self._names:
            yield name, getattr(self, name.replace(".", "__"))


class _Acc:
    def get_accuracy(self, _k):
        return 0.0


class Tester:
    def __init__(self, model):
        self.model = model
        self.accuracy_metric = _Acc()

    def inference(self):
        pass


def psize(layout):
    return sum(int(np.prod(s)) for _, s in layout)


def flat(d, layout):
    return np.concatenate([d[k].detach().reshape(-1).numpy() for k, _ in layout])


def unflat(v, layout):
    out, off = {}, 0
    for k, s in layout:
        n = int(np.prod(s))
        out[k] = torch.from_numpy(np.ascontiguousarray(v[off:off + n])).reshape(s)
        off += n
    return out


def synth_updates(gen, layout, K):
    """SURVEY.md §8d synthetic client updates: base + sigma_i * N(0,1)."""
    P = psize(layout)
    base = torch.randn(P, generator=gen) * 0.05
    lo, hi = math.log(1e-3), math.log(5e-2)
    sig = torch.exp(lo + (hi - lo) * torch.rand(K, generator=gen))
    U = base[None, :] + sig[:, None] * torch.randn(K, P, generator=gen)
    n = torch.randint(100, 1001, (K,), generator=gen)
    return U.float().numpy(), [int(x) for x in n]


def make_fed_server(layout, gen, K, cls=FedServer):
    model = ParamModel(layout, gen)
    return cls(tester=Tester(model), worker_number=K, multi_process=False)


# --------------------------------------------------------------------------- FedAvg
def gen_fedavg():
    out = {}
    cases = []
    for ci, (layout, K, special) in enumerate([
        (LAYOUT_SMALL, 7, False),
        (LAYOUT_MED, 16, False),
        (LAYOUT_SMALL, 5, True),
    ]):
        gen = torch.Generator().manual_seed(20250127 + ci)
        U, n = synth_updates(gen, layout, K)
        if special:
            # denormals, huge values, signed zeros, inf/nan, and a sample count
            # above 2**24 (pins the fp32 conversion of the Python int).
            U[0, :6] = [1e-40, -3e-39, 3.0e38, -0.0, 0.0, 1e-45]
            U[1, :6] = [2e-38, 1e-39, 1e38, 0.0, -0.0, -1e-45]
            U[2, 6:9] = [np.inf, -np.inf, np.nan]
            U[3, 9] = np.nan
            n = [33554435, 7, 1000, 1, 123457]
        server = make_fed_server(layout, gen, K)
        order = [int(i) for i in torch.randperm(K, generator=gen)]  # arrival order
        agg = None
        for wid in order:
            res = server._process_worker_data((wid, n[wid], unflat(U[wid], layout)), None)
            if res is not None:
                agg = res
        full = flat(agg.data, layout)
        # subsets as the Shapley servers pass them (sorted tuples) + one unsorted
        for wid in order:
            server.parameters[wid] = (n[wid], unflat(U[wid], layout))
        subsets = [(0,), (1, 3), tuple(range(0, K, 2)), tuple(sorted(order[: K // 2 + 1])),
                   (K - 1, 0, 2), tuple(range(K))]
        sub_out = [flat(server.get_subset_model(s), layout) for s in subsets]
        empty = flat(server.get_subset_model(()), layout)
        key = f"c{ci}"
        out[f"{key}_U"] = U
        out[f"{key}_n"] = np.array(n, dtype=np.int64)
        out[f"{key}_order"] = np.array(order, dtype=np.int64)
        out[f"{key}_full"] = full
        out[f"{key}_prev"] = empty
        for si, (s, o) in enumerate(zip(subsets, sub_out)):
            out[f"{key}_sub{si}_ids"] = np.array(s, dtype=np.int64)
            out[f"{key}_sub{si}_out"] = o
        cases.append({"key": key, "layout": layout, "K": K, "nsub": len(subsets)})
    out["meta"] = np.array(json.dumps(cases))
    np.savez_compressed(os.path.join(HERE, "fedavg.npz"), **out)


# --------------------------------------------------------------------- sign vote
def gen_sign_vote():
    out, cases = {}, []
    for ci, (layout, K, with_nan) in enumerate([(LAYOUT_SMALL, 6, False), (LAYOUT_MED, 9, False),
                                                (LAYOUT_SMALL, 4, True)]):
        gen = torch.Generator().manual_seed(20250127 + 10 + ci)
        P = psize(layout)
        g = torch.randn(K, P, generator=gen)
        g[torch.rand(K, P, generator=gen) < 0.01] = 0.0
        # correlated columns so that ties and strong majorities both occur
        g[:, : P // 4] = g[:, : P // 4].abs() * torch.sign(torch.randn(1, P // 4, generator=gen))
        S = torch.sign(g).float()
        if with_nan:
            S[1, 3] = float("nan")
            S[2, 11] = float("nan")
        server = SignSGDServer(tester=None, worker_number=K, multi_process=False)
        res = None
        for k in range(K):
            lst = list(unflat(S[k].numpy(), layout).values())
            res = server._SignSGDServer__worker(lst)  # D1: never wired by the queue
        vote = np.concatenate([t.reshape(-1).numpy() for t in res.data])
        out[f"c{ci}_signs"] = S.numpy()
        out[f"c{ci}_vote"] = vote
        cases.append({"key": f"c{ci}", "layout": layout, "K": K})
    out["meta"] = np.array(json.dumps(cases))
    np.savez_compressed(os.path.join(HERE, "sign_vote.npz"), **out)


# --------------------------------------------------------------------- sign worker
class _Queue:
    def __init__(self):
        self.sent = []
        self.reply = None

    def add_task(self, task):
        self.sent.append([t.clone() for t in task])

    def get_result(self):
        return self.reply


class _Trainer:
    def __init__(self, opt):
        self.opt = opt

    def get_optimizer(self):
        return self.opt

    def add_named_callback(self, *a, **k):
        pass


def gen_sign_worker():
    out, cases = {}, []
    configs = [
        dict(momentum=0.9, dampening=0.0, nesterov=False, weight_decay=0.0, lr=0.01),
        dict(momentum=0.9, dampening=0.0, nesterov=True, weight_decay=1e-4, lr=0.05),
        dict(momentum=0.5, dampening=0.1, nesterov=False, weight_decay=5e-4, lr=0.1),
        dict(momentum=0.0, dampening=0.0, nesterov=False, weight_decay=1e-3, lr=0.01),
    ]
    steps = 3
    for ci, cfg in enumerate(configs):
        gen = torch.Generator().manual_seed(20250127 + 20 + ci)
        model = ParamModel(LAYOUT_SMALL, gen)
        params = [p for _, p in model.named_parameters()]
        opt = torch.optim.SGD(params, **cfg)
        q = _Queue()
        worker = SignSGDWorker(worker_id=0, trainer=_Trainer(opt), worker_data_queue=q, round=1)
        key = f"c{ci}"
        out[f"{key}_p0"] = flat(dict(model.named_parameters()), LAYOUT_SMALL)
        for s in range(steps):
            for i, p in enumerate(params):
                # the 'scale' tensor has no gradient on step 1 (grad None -> skipped)
                if i == len(params) - 1 and s == 1:
                    p.grad = None
                else:
                    p.grad = torch.randn(p.shape, generator=gen) * 0.1
                    p.grad[torch.rand(p.shape, generator=gen) < 0.02] = 0.0
            has_grad = [p.grad is not None for p in params]
            grads = [p.grad.clone() if p.grad is not None else torch.zeros_like(p) for p in params]
            vote = [torch.sign(torch.randn(p.shape, generator=gen)) for p, h in zip(params, has_grad) if h]
            q.reply = vote
            worker._SignSGDWorker__get_gredient(opt, device=torch.device("cpu"))
            sent = q.sent[-1]
            out[f"{key}_s{s}_grad"] = np.concatenate([g.reshape(-1).numpy() for g in grads])
            out[f"{key}_s{s}_hasgrad"] = np.array(has_grad)
            full_vote, full_sent, vi = [], [], 0
            for p, h in zip(params, has_grad):
                if h:
                    full_vote.append(vote[vi].reshape(-1))
                    full_sent.append(sent[vi].reshape(-1))
                    vi += 1
                else:
                    full_vote.append(torch.zeros(p.numel()))
                    full_sent.append(torch.zeros(p.numel()))
            out[f"{key}_s{s}_vote"] = torch.cat(full_vote).numpy()
            out[f"{key}_s{s}_sent"] = torch.cat(full_sent).numpy()
            out[f"{key}_s{s}_param"] = flat(dict(model.named_parameters()), LAYOUT_SMALL)
            bufs = []
            for p in params:
                st = opt.state.get(p, {})
                b = st.get("momentum_buffer")
                bufs.append((b if b is not None else torch.zeros_like(p)).reshape(-1))
            out[f"{key}_s{s}_buf"] = torch.cat(bufs).numpy()
        cases.append({"key": key, "cfg": cfg, "steps": steps, "layout": LAYOUT_SMALL})
    out["meta"] = np.array(json.dumps(cases))
    np.savez_compressed(os.path.join(HERE, "sign_worker.npz"), **out)


# ------------------------------------------------------------------ fed_quant
def gen_dequant():
    out, cases = {}, []
    layout = LAYOUT_MED
    K = 5
    gen = torch.Generator().manual_seed(20250127 + 30)
    U, n = synth_updates(gen, layout, K)
    server = make_fed_server(layout, gen, K, cls=FedQuantServer)
    qnames = [k for k, s in layout if len(s) >= 2]
    for i in range(K):
        d = unflat(U[i], layout)
        payload = {}
        for k, s in layout:
            t = d[k]
            if k in qnames:
                C = s[0]
                if k == "layer1.0.conv2.weight":  # asymmetric quint8, nonzero zero points
                    lo = t.reshape(C, -1).min(1).values
                    hi = t.reshape(C, -1).max(1).values
                    sc = ((hi - lo) / 255.0).double()
                    zp = torch.clamp(torch.round(-lo.double() / sc), 0, 255).long()
                    qt = torch.quantize_per_channel(t, sc, zp, 0, torch.quint8)
                else:  # symmetric qint8 (torch QAT default for weights)
                    sc = (t.reshape(C, -1).abs().max(1).values / 127.0).double()
                    zp = torch.zeros(C, dtype=torch.long)
                    qt = torch.quantize_per_channel(t, sc, zp, 0, torch.qint8)
                payload[k] = (qt.int_repr(), qt.q_per_channel_scales(), qt.q_per_channel_zero_points())
                out[f"q{i}_{k}_int"] = qt.int_repr().numpy()
                out[f"q{i}_{k}_scale"] = qt.q_per_channel_scales().numpy()
                out[f"q{i}_{k}_zp"] = qt.q_per_channel_zero_points().numpy()
            else:
                payload[k] = t.clone()
                out[f"q{i}_{k}_f32"] = t.numpy()
        proc = server._process_client_parameter(payload)
        out[f"deq{i}"] = flat(proc, layout)
        server.parameters[i] = (n[i], proc)
    out["agg"] = flat(server.get_subset_model(server.parameters.keys()), layout)
    out["n"] = np.array(n, dtype=np.int64)
    cases.append({"layout": layout, "K": K, "qnames": qnames})
    out["meta"] = np.array(json.dumps(cases))
    np.savez_compressed(os.path.join(HERE, "dequant.npz"), **out)


def gen_quantize():
    """torch's deterministic affine quantize: pins q = clamp(rne(x*(1/s)) + zp)."""
    gen = torch.Generator().manual_seed(20250127 + 31)
    out = {}
    x = torch.randn(20000, generator=gen) * 0.3
    x[:5] = torch.tensor([0.0, -0.0, 1e-30, 5.0, -5.0])
    lo, hi = float(x.min()), float(x.max())
    s = (hi - lo) / 255.0
    zp = int(min(255, max(0, round(-lo / s))))
    q = torch.quantize_per_tensor(x, s, zp, torch.quint8)
    out.update(pt_x=x.numpy(), pt_scale=np.float64(s), pt_zp=np.int64(zp), pt_q=q.int_repr().numpy(),
               pt_deq=q.dequantize().numpy())
    # exact ties at .5 to pin round-half-even
    xt = torch.arange(-64, 64, dtype=torch.float32) * 0.5 * 0.0625
    qt = torch.quantize_per_tensor(xt, 0.0625, 10, torch.quint8)
    out.update(tie_x=xt.numpy(), tie_q=qt.int_repr().numpy())
    w = torch.randn(12, 5, 3, generator=gen)
    sc = (w.reshape(12, -1).abs().max(1).values / 127.0).double()
    qc = torch.quantize_per_channel(w, sc, torch.zeros(12, dtype=torch.long), 0, torch.qint8)
    out.update(pc_x=w.numpy(), pc_scale=sc.numpy(), pc_q=qc.int_repr().numpy())
    np.savez_compressed(os.path.join(HERE, "quantize.npz"), **out)


# ------------------------------------------------------------------- Shapley
def shapley_utility_factory(layout, target, scale):
    """Deterministic continuous utility standing in for tester.inference()."""
    def util(model, metric_type="acc"):
        v = flat(model, layout).astype(np.float64)
        d = v - target
        return float(1.0 / (1.0 + float(np.dot(d, d)) / scale))
    return util


def shapley_clients(gen, layout, K):
    P = psize(layout)
    prev = (torch.randn(P, generator=gen) * 0.05).numpy().astype(np.float32)
    target = (torch.randn(P, generator=gen) * 0.05).numpy().astype(np.float64)
    alphas = np.linspace(0.9, -0.2, K)  # client quality: helpful ... harmful
    U = np.empty((K, P), np.float32)
    for i in range(K):
        noise = (torch.randn(P, generator=gen) * 0.01 * (1 + i)).numpy()
        U[i] = (prev + alphas[i] * (target - prev) + noise).astype(np.float32)
    n = [int(x) for x in torch.randint(100, 1001, (K,), generator=gen)]
    scale = float(np.dot(target - prev, target - prev))
    return prev, target, U, n, scale


def run_shapley(cls, layout, K, seed, tag):
    gen = torch.Generator().manual_seed(20250127 + 40 + K)
    prev, target, U, n, scale = shapley_clients(gen, layout, K)
    model = ParamModel(layout, gen)
    with torch.no_grad():
        for (k, p), t in zip(model.named_parameters(), unflat(prev, layout).values()):
            p.copy_(t)
    server = cls(tester=Tester(model), worker_number=K, multi_process=False)
    util = shapley_utility_factory(layout, target, scale)
    server.get_metric = util
    evaluated = []
    orig = server.get_subset_model

    def spy(subset):
        evaluated.append([int(i) for i in subset])
        return orig(subset)

    server.get_subset_model = spy
    np.random.seed(seed)
    metric_pickle = None
    with tempfile.TemporaryDirectory() as td, contextlib.chdir(td) if hasattr(contextlib, "chdir") else _cd(td):
        for i in range(K):
            server._process_worker_data((i, n[i], unflat(U[i], layout)), None)
        if os.path.exists("metric_1"):  # multiround's side effect (:56-57), byte for byte
            with open("metric_1", "rb") as f:
                metric_pickle = f.read()
    sv = server.shapley_values[1]
    assert any(float(v) != 0.0 for v in sv.values()), "round truncated: choose other clients"
    return {
        "tag": tag, "K": K, "seed": seed, "U": U.tolist(), "n": n, "prev": prev.tolist(),
        "target": target.tolist(), "scale": scale, "layout": layout,
        "sv": {str(k): float(v) for k, v in sv.items()},
        "evaluated": evaluated[1:],  # [0] is the round's full aggregation
        "metric_pickle_hex": metric_pickle.hex() if metric_pickle is not None else None,
    }


@contextlib.contextmanager
def _cd(path):
    old = os.getcwd()
    os.chdir(path)
    try:
        yield
    finally:
        os.chdir(old)


SHAPLEY_LAYOUT = [("w", (6, 5)), ("b", (6,)), ("v", (11,))]


def gen_shapley():
    layout = SHAPLEY_LAYOUT
    cases = []
    for K in (3, 4, 6):
        cases.append(run_shapley(MultiRoundShapleyValueServer, layout, K, 0, f"multiround_{K}"))
    for K, seed in ((3, 0), (4, 1), (5, 2), (6, 3)):
        cases.append(run_shapley(GTGShapleyValueServer, layout, K, seed, f"gtg_{K}_{seed}"))
    with open(os.path.join(HERE, "shapley.json"), "w") as f:
        json.dump(cases, f)


def gen_shapley_large():
    """BASELINE config 5 at its stated client count: GTG at N = 50 (~4.5k
    coalitions) and multiround at N = 12 (all 4,096), on the small layout with
    the deterministic utility.  Stored compactly: coalitions as uint64 bit masks
    in evaluation order, the multiround metric_1 pickle as raw bytes."""
    out, cases = {}, []
    for cls, K, seed, tag in ((GTGShapleyValueServer, 50, 4, "gtg_50_4"),
                              (MultiRoundShapleyValueServer, 12, 0, "multiround_12")):
        c = run_shapley(cls, SHAPLEY_LAYOUT, K, seed, tag)
        out[f"{tag}_U"] = np.array(c["U"], np.float32)
        out[f"{tag}_n"] = np.array(c["n"], np.int64)
        out[f"{tag}_prev"] = np.array(c["prev"], np.float32)
        out[f"{tag}_target"] = np.array(c["target"], np.float64)
        out[f"{tag}_sv"] = np.array([c["sv"][str(i)] for i in range(K)], np.float64)
        out[f"{tag}_evaluated"] = np.array(
            [sum(1 << i for i in s) for s in c["evaluated"]], np.uint64)
        if c["metric_pickle_hex"] is not None:
            out[f"{tag}_metric_pickle"] = np.frombuffer(bytes.fromhex(c["metric_pickle_hex"]),
                                                        np.uint8)
        cases.append({"tag": tag, "K": K, "seed": seed, "scale": c["scale"],
                      "layout": SHAPLEY_LAYOUT, "n_evaluated": len(c["evaluated"])})
    out["meta"] = np.array(json.dumps(cases))
    np.savez_compressed(os.path.join(HERE, "shapley_large.npz"), **out)


if __name__ == "__main__":
    torch.set_num_threads(1)
    gen_fedavg()
    gen_sign_vote()
    gen_sign_worker()
    gen_dequant()
    gen_quantize()
    gen_shapley()
    gen_shapley_large()
    for f in sorted(os.listdir(HERE)):
        if f.endswith((".npz", ".json")):
            print(f, os.path.getsize(os.path.join(HERE, f)))

"""GPU parity: GTG / multiround Shapley servers vs the reference's golden values."""
import numpy as np
import pytest
import torch

from tests import golden as G

pytestmark = pytest.mark.gpu


class _Model(torch.nn.Module):
    def __init__(self, layout, flat):
        super().__init__()
        off = 0
        self._names = []
        for name, shape in layout:
            m = int(np.prod(shape))
            p = torch.nn.Parameter(torch.tensor(flat[off:off + m], dtype=torch.float32).reshape(shape))
            self.register_parameter(name, p)
            self._names.append(name)
            off += m


class _Tester:
    def __init__(self, model):
        self.model = model


def _setup(case, cls, **kw):
    layout = [(nm, tuple(s)) for nm, s in case["layout"]]
    K = case["K"]
    U = np.array(case["U"], np.float32)
    target = np.array(case["target"], np.float64)
    server = cls(tester=_Tester(_Model(layout, np.array(case["prev"], np.float32))),
                 worker_number=K, synchronous=True, **kw)

    def util(model, metric_type="acc"):
        v = np.concatenate([model[nm].detach().reshape(-1).cpu().double().numpy()
                            for nm, _ in layout])
        d = v - target
        return float(1.0 / (1.0 + float(np.dot(d, d)) / case["scale"]))

    server.get_metric = util
    return server, layout, U


def _run_round(server, case, layout, U):
    K = case["K"]
    for i in range(K):
        d = {nm: torch.from_numpy(v.copy()) for nm, v in G.split(U[i], layout).items()}
        server.worker_data_queue.add_task((i, int(case["n"][i]), d))
    for w in range(2 * K):  # initial broadcast + this round's broadcast
        server.worker_data_queue.get_result(consumer=w % K)
    return server.shapley_values[1]


@pytest.mark.parametrize("tag", [c["tag"] for c in G.shapley_cases()])
def test_shapley_servers_golden(tag, tmp_path):
    from distributed_learning_simulator_amd.servers.GTG_shapley_value_server import \
        GTGShapleyValueServer
    from distributed_learning_simulator_amd.servers.multiround_shapley_value_server import \
        MultiRoundShapleyValueServer
    case = next(c for c in G.shapley_cases() if c["tag"] == tag)
    if tag.startswith("gtg"):
        server, layout, U = _setup(case, GTGShapleyValueServer)
    else:
        server, layout, U = _setup(case, MultiRoundShapleyValueServer, metric_dir=str(tmp_path))
    np.random.seed(case["seed"])
    sv = _run_round(server, case, layout, U)
    for k, v in case["sv"].items():
        assert abs(float(sv[int(k)]) - v) <= 1e-12, (tag, k)
    got = {tuple(s) for s in server.evaluated_subsets}
    assert got == {tuple(s) for s in case["evaluated"]}
    if tag.startswith("multiround"):
        assert (tmp_path / "metric_1").exists()


def test_shapley_gemm_method_tolerance(tmp_path):
    """MFMA subset models: Shapley values within 1e-5 and the same client ranking."""
    from distributed_learning_simulator_amd.servers.multiround_shapley_value_server import \
        MultiRoundShapleyValueServer
    case = next(c for c in G.shapley_cases() if c["tag"] == "multiround_6")
    server, layout, U = _setup(case, MultiRoundShapleyValueServer, metric_dir=str(tmp_path),
                               subset_method="gemm")
    sv = _run_round(server, case, layout, U)
    ref = {int(k): v for k, v in case["sv"].items()}
    for k, v in ref.items():
        assert abs(float(sv[k]) - v) <= 1e-5
    assert sorted(ref, key=ref.get) == sorted(sv, key=lambda k: float(sv[k]))

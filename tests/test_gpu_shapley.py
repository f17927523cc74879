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
    U = np.asarray(case["U"], np.float32)
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
    if tag.startswith("multiround"):  # the metric_<round> pickle, byte for byte
        assert (tmp_path / "metric_1").read_bytes() == bytes.fromhex(case["metric_pickle_hex"])


@pytest.mark.parametrize("tag", ["gtg_50_4", "multiround_12"])
def test_shapley_servers_golden_config5_scale(tag, tmp_path):
    """BASELINE config 5 client count: GTG over 50 clients (4,434 coalitions, ~90
    batched union launches) and multiround over 12 (all 4,096): Shapley values
    within 1e-12 of the reference's, the identical evaluated-coalition set, and
    multiround's metric_1 pickle byte-identical to the one the reference wrote."""
    from distributed_learning_simulator_amd.servers.GTG_shapley_value_server import \
        GTGShapleyValueServer
    from distributed_learning_simulator_amd.servers.multiround_shapley_value_server import \
        MultiRoundShapleyValueServer
    case = next(c for c in G.shapley_large_cases() if c["tag"] == tag)
    if tag.startswith("gtg"):
        server, layout, U = _setup(case, GTGShapleyValueServer)
    else:
        server, layout, U = _setup(case, MultiRoundShapleyValueServer, metric_dir=str(tmp_path))
    np.random.seed(case["seed"])
    sv = _run_round(server, case, layout, U)
    for k, v in case["sv"].items():
        assert abs(float(sv[int(k)]) - v) <= 1e-12, (tag, k)
    assert len(server.evaluated_subsets) == case["n_evaluated"]
    assert {tuple(s) for s in server.evaluated_subsets} == set(case["evaluated"])
    if case["metric_pickle"] is not None:
        assert (tmp_path / "metric_1").read_bytes() == case["metric_pickle"]


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


@pytest.mark.parametrize("tag", ["gtg_50_4", "multiround_12"])
def test_shapley_gemm_method_config5_scale(tag, tmp_path):
    """north_star: the subset aggregation as the MFMA GEMM (subset_method="gemm",
    ref servers/GTG_shapley_value_server.py:56-57,
    servers/multiround_shapley_value_server.py:37-38) at config 5's client count:
    Shapley values within 1e-5 of the reference's and the identical client
    ranking (the goldens' smallest SV gap is 1.0e-4 at N=50, 4.0e-4 at N=12)."""
    from distributed_learning_simulator_amd.servers.GTG_shapley_value_server import \
        GTGShapleyValueServer
    from distributed_learning_simulator_amd.servers.multiround_shapley_value_server import \
        MultiRoundShapleyValueServer
    case = next(c for c in G.shapley_large_cases() if c["tag"] == tag)
    if tag.startswith("gtg"):
        server, layout, U = _setup(case, GTGShapleyValueServer, subset_method="gemm")
    else:
        server, layout, U = _setup(case, MultiRoundShapleyValueServer, metric_dir=str(tmp_path),
                                   subset_method="gemm")
    np.random.seed(case["seed"])
    sv = _run_round(server, case, layout, U)
    ref = {int(k): v for k, v in case["sv"].items()}
    for k, v in ref.items():
        assert abs(float(sv[k]) - v) <= 1e-5, (tag, k)
    assert sorted(ref, key=ref.get) == sorted(sv, key=lambda k: float(sv[k]))

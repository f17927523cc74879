"""GPU end-to-end: the drop-in plugin surface driven by the simulator (config 1 plumbing)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(tmp_path, *args):
    from distributed_learning_simulator_amd import simulator
    cfg = simulator.get_config(list(args) + ["--log_dir", str(tmp_path / "log")])
    return simulator.run(cfg)


def test_config1_fedavg_lenet5_10_workers_5_rounds(tmp_path):
    server = _run(tmp_path, "--distributed_algorithm", "fed", "--worker_number", "10", "--round",
                  "5", "--dataset_name", "MNIST", "--model_name", "LeNet5", "--epoch", "1",
                  "--learning_rate", "0.05", "--train_size", "6000", "--test_size", "1000")
    assert server.round == 5
    acc = server.get_metric(server.prev_model)
    assert acc > 0.25, acc  # learnable synthetic MNIST-shaped data (chance: 0.1)
    assert list((tmp_path / "log" / "fed" / "MNIST" / "LeNet5").iterdir())


def test_sign_sgd_simulation(tmp_path):
    server = _run(tmp_path, "--distributed_algorithm", "sign_SGD", "--worker_number", "4",
                  "--round", "1", "--epoch", "1", "--learning_rate", "0.001",
                  "--momentum", "0.9", "--train_size", "2048", "--test_size", "512")
    model = server.tester.model
    assert all(torch.isfinite(p).all() for p in model.parameters())


def test_fed_quant_simulation(tmp_path):
    server = _run(tmp_path, "--distributed_algorithm", "fed_quant", "--worker_number", "3",
                  "--round", "2", "--epoch", "1", "--learning_rate", "0.05",
                  "--train_size", "3000", "--test_size", "500")
    assert server.round == 2
    q, scale, zp = server.quantized_parameter
    # the reference's granularity: one quantizer over the concatenated aggregate
    # (servers/fed_quant_server.py:39): one (scale, zero point), every element once
    assert q.dtype == torch.uint8 and scale.numel() == 1 and zp.numel() == 1
    assert q.numel() == sum(v.numel() for v in server.prev_model.values())


@pytest.mark.parametrize("algo", ["GTG_shapley_value", "multiround_shapley_value"])
def test_shapley_simulation(tmp_path, algo, monkeypatch):
    monkeypatch.chdir(tmp_path)
    server = _run(tmp_path, "--distributed_algorithm", algo, "--worker_number", "3", "--round",
                  "1", "--epoch", "1", "--learning_rate", "0.05", "--train_size", "1500",
                  "--test_size", "500")
    assert len(server.shapley_values[1]) == 3

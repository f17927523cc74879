"""Plugin factory (reference: factory.py:14-35) — same algorithm names and errors."""
from .servers.fed_quant_server import FedQuantServer
from .servers.fed_server import FedServer
from .servers.GTG_shapley_value_server import GTGShapleyValueServer
from .servers.multiround_shapley_value_server import MultiRoundShapleyValueServer
from .servers.server import Server
from .servers.sign_sgd_server import SignSGDServer
from .workers.fed_quant_worker import FedQuantWorker
from .workers.fed_worker import FedWorker
from .workers.sign_sgd_worker import SignSGDWorker
from .workers.worker import Worker


def get_server(algorithm, sharded=None, **kwargs) -> Server:
    """factory.py:14-25.  ``sharded`` (default: torch.distributed initialised with
    more than one rank) returns the one-process-per-GPU servers of distributed.py."""
    if sharded is None:
        import torch.distributed as dist
        sharded = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
    if sharded:
        from .distributed import get_sharded_server
        return get_sharded_server(algorithm, **kwargs)
    if algorithm == "sign_SGD":
        return SignSGDServer(**kwargs)
    if algorithm == "fed_quant":
        return FedQuantServer(**kwargs)
    if algorithm == "fed":
        return FedServer(**kwargs)
    if algorithm == "multiround_shapley_value":
        return MultiRoundShapleyValueServer(**kwargs)
    if algorithm == "GTG_shapley_value":
        return GTGShapleyValueServer(**kwargs)
    raise RuntimeError("unknown algorithm:" + algorithm)


def get_worker(algorithm, **kwargs) -> Worker:
    if algorithm == "sign_SGD":
        return SignSGDWorker(**kwargs)
    if algorithm == "fed_quant":
        return FedQuantWorker(**kwargs)
    if algorithm in ("fed", "multiround_shapley_value", "GTG_shapley_value"):
        return FedWorker(**kwargs)
    raise RuntimeError("unknown algorithm:" + algorithm)

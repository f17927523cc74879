"""Parameter-dict helpers (the subset of the absent ``ModelUtil`` the reference uses).

Call sites: servers/fed_server.py:17 (``get_parameter_dict``), :27
(``load_parameter_dict``), workers/fed_worker.py:23,30,38.
"""
import torch


def get_device():
    """Server device (the reference's ``cyy_naive_pytorch_lib.device.get_device``)."""
    if torch.cuda.is_available():
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


class ModelUtil:
    def __init__(self, model):
        self.model = model

    def get_parameter_dict(self, detach=True):
        return {k: (v.detach().clone() if detach else v) for k, v in self.model.named_parameters()}

    @torch.no_grad()
    def load_parameter_dict(self, parameter_dict):
        params = dict(self.model.named_parameters())
        dst = [params[k] for k in parameter_dict]
        src = [v.to(params[k].device, params[k].dtype) for k, v in parameter_dict.items()]
        torch._foreach_copy_(dst, src)


_SERIALIZATION_SIZES = {}


def _structure(data):
    """Hashable (container, shape, dtype) skeleton of a nested payload."""
    if isinstance(data, torch.Tensor):
        return ("T", tuple(data.shape), str(data.dtype))
    if isinstance(data, dict):
        return ("D",) + tuple((k, _structure(v)) for k, v in data.items())
    if isinstance(data, (tuple, list)):
        return (type(data).__name__,) + tuple(_structure(v) for v in data)
    return ("O", repr(data))


def _empty_like_cpu(data):
    if isinstance(data, torch.Tensor):
        return torch.empty(tuple(data.shape), dtype=data.dtype)
    if isinstance(data, dict):
        return {k: _empty_like_cpu(v) for k, v in data.items()}
    if isinstance(data, (tuple, list)):
        return type(data)(_empty_like_cpu(v) for v in data)
    return data


def get_data_serialization_size(data) -> int:
    """Pickled size in bytes of a parameter dict / quantized payload.

    Restates ``cyy_naive_pytorch_lib.tensor.get_data_serialization_size`` (absent
    library; ``len(pickle.dumps(data))``), called at ref
    servers/fed_quant_server.py:41-42 and workers/fed_quant_worker.py:28-30,43
    for the compression-ratio log line.  Tensors are measured as CPU tensors.  The
    byte count depends only on the structure, shapes and dtypes (torch pickles raw
    storage bytes), so it is computed once per structure on empty CPU tensors
    and cached, and the device data is never copied to the host.
    """
    import pickle

    key = _structure(data)
    size = _SERIALIZATION_SIZES.get(key)
    if size is None:
        size = len(pickle.dumps(_empty_like_cpu(data)))
        _SERIALIZATION_SIZES[key] = size
    return size

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

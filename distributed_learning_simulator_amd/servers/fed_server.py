"""FedAvg server (reference: servers/fed_server.py:11-91).

Same hooks, same round protocol, same return objects; ``get_subset_model`` is
one ``dls_fedavg_f32`` launch over the clients' HBM rows instead of a Python
loop of K x (#tensors) torch ops, bit-exact with the reference's op order.
"""
import copy
import logging

from .. import _native
from ..aggregation import ClientParameters, ClientUpdateStore
from ..layout import ParameterLayout
from ..model_util import ModelUtil
from ..task_queue import RepeatedResult
from .server import Server

log = logging.getLogger("distributed_learning_simulator_amd")

_MODES = {"exact": _native.FEDAVG_EXACT, "fma": _native.FEDAVG_FMA}


class FedServer(Server):
    def __init__(self, aggregation_mode="exact", **kwargs):
        if aggregation_mode not in _MODES:
            raise ValueError(f"aggregation_mode must be one of {sorted(_MODES)}, not {aggregation_mode!r}")
        super().__init__(**kwargs)
        _native.require_gpu()
        self.round = 0
        self.aggregation_mode = aggregation_mode
        self.parameters: ClientParameters = ClientParameters(self._make_store)
        self.__prev_model = copy.deepcopy(
            ModelUtil(self.tester.model).get_parameter_dict()) if self.tester is not None else {}
        self.worker_data_queue.put_result(
            RepeatedResult(data=self.prev_model, num=self.clients_per_round))

    @property
    def clients_per_round(self):
        """Clients whose updates this process receives per round (all of them here;
        the sharded servers in ``distributed.py`` override it)."""
        return self.worker_number

    @property
    def store_capacity(self):
        """Client rows this process holds per round: its own clients (the sharded
        servers receive only their local ones; the sharded Shapley servers
        override this, they all-gather every client)."""
        return self.clients_per_round

    def _make_store(self, parameter_dict):
        return ClientUpdateStore(ParameterLayout.from_dict(parameter_dict), self.device,
                                 capacity=self.store_capacity)

    def get_metric(self, model, metric_type="acc"):
        """servers/fed_server.py:26-32 — load, run the tester, top-1 accuracy or loss."""
        if self.tester is None:
            return None
        ModelUtil(self.tester.model).load_parameter_dict(model)
        self.tester.inference()
        if metric_type == "acc":
            return self.tester.accuracy_metric.get_accuracy(1)
        return self.tester.loss_metric.get_loss(1).data.item()

    @property
    def prev_model(self):
        return self.__prev_model

    def _set_prev_model(self, model):
        self.__prev_model = model

    def _process_client_parameter(self, client_parameter: dict):
        return client_parameter

    def _before_aggregate(self):
        """Hook when this process has all its clients of the round (sharded servers)."""

    def _process_aggregated_parameter(self, aggregated_parameter: dict):
        return aggregated_parameter

    def get_subset_model(self, client_subset):
        """servers/fed_server.py:44-66 (empty subset -> previous model)."""
        if not client_subset:
            return self.__prev_model
        ids = list(client_subset)
        store = self.parameters.store
        flat = self._aggregate(store, [self.parameters.row_of(i) for i in ids],
                               [self.parameters.n_of(i) for i in ids])
        return store.layout.views(flat)

    def _aggregate(self, store, rows, ns, total=None):
        return store.fedavg(rows, ns, mode=_MODES[self.aggregation_mode], total=total)

    def _process_worker_data(self, data, __):
        worker_id, training_dataset_size, parameter_dict = data
        self.parameters[worker_id] = (
            training_dataset_size,
            self._process_client_parameter(parameter_dict),
        )
        if len(self.parameters) != self.clients_per_round:
            log.debug("%s %s,skip", len(self.parameters), self.clients_per_round)
            return None
        self._before_aggregate()
        self.round += 1
        log.info("begin aggregating")
        avg_parameter = self.get_subset_model(self.parameters.keys())
        data = self._process_aggregated_parameter(avg_parameter)
        self.__prev_model = copy.deepcopy(data)
        acc = self.get_metric(self.prev_model)
        log.info("end aggregating, test accuracy is %s", acc)
        self.parameters.clear()
        # one copy per client that feeds this process (its local clients when sharded)
        return RepeatedResult(data=data, num=self.clients_per_round)

"""MI355X-native server-side aggregation for distributed_learning_simulator.

A drop-in for the reference's Server/Worker plugin surface (``factory.get_server``
/ ``get_worker``; algorithms ``fed``, ``sign_SGD``, ``fed_quant``,
``GTG_shapley_value``, ``multiround_shapley_value``) whose hot hooks run as
hand-written HIP kernels for gfx950 through the C-ABI in ``include/dls_hip.h``
(``libdls_hip.so``, loaded by ``_native``).  There is no CPU fallback: the
aggregation hooks raise if the HIP library or the GPU is missing.
"""

__version__ = "0.1.0"

"""CPU oracle for the server-side aggregation hot path — TEST INFRASTRUCTURE.

This package is a restatement, on the CPU, of the reference algorithms that the
HIP kernels in ``distributed_learning_simulator_amd/csrc`` replace.  Every
function cites the reference ``file:line`` it follows (paths relative to the
reference repository chen-zichen/distributed_learning_simulator).

Who may use it: only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` — always as the *checker* or the timed CPU
baseline, never as the product path.  The product package never imports it.

Pinning: the restatement is checked bit-for-bit (FedAvg, sign vote, sign-SGD
worker, per-channel dequant, affine quantize) and to 1e-12 (Shapley, fp64)
against golden vectors recorded from the reference itself
(``tests/golden/make_golden.py`` imports the reference's ``servers/*.py`` and
``workers/*.py`` with stand-ins for its two absent dependencies).  The
stochastic 256-level re-quantization (``servers/fed_quant_server.py:35-51``)
lives in an absent library and is **parity unpinned**.
"""

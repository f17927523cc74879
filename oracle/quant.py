"""fed_quant arithmetic — CPU restatement (TEST INFRASTRUCTURE, see oracle/__init__.py).

* Per-channel dequant: ``FedQuantServer._process_client_parameter``,
  servers/fed_quant_server.py:25-33 — ``(v - zp[c]) * scale[c]`` with torch
  casting the 0-dim float64 scale / int64 zero point to fp32 first, i.e.
  ``fl32(fl32(q - zp) * fl32(scale))`` (C: oracle/c/oracle.c).
* Dequant + FedAvg: the dequantized dict then goes through
  ``FedServer.get_subset_model`` (servers/fed_server.py:44-66).
* Deterministic affine quantize (this build's contract for the re-quantization
  at servers/fed_quant_server.py:35-39, whose stochastic original lives in an
  absent library — parity unpinned): torch's ``quantize_per_tensor`` /
  ``quantize_per_channel`` formula ``q = clamp(rne(x * fl32(1/fl32(s))) + zp)``
  with MinMaxObserver qparams, pinned by tests/golden/quantize.npz.
"""
import numpy as np

from . import _c
from .fedavg import fedavg_reference_order

EPS = np.float32(np.finfo(np.float32).eps)


def dequant_channel(q, scale, zp):
    """servers/fed_quant_server.py:28-32 for one (int weight, scale, zp) tuple."""
    return _c.dequant_rows(q, scale, zp)


def dequant_fedavg(clients, n, order, layout):
    """clients[i] = {name: fp32 array | (int array, scale f64 [C], zp i64 [C])}."""
    rows = []
    for c in clients:
        parts = []
        for name, shape in layout:
            v = c[name]
            if isinstance(v, tuple):
                parts.append(dequant_channel(*v).reshape(-1))
            else:
                parts.append(np.asarray(v, np.float32).reshape(-1))
        rows.append(np.concatenate(parts))
    return fedavg_reference_order(np.stack(rows), n, order)


def quantize_affine(x, scale, zp, qmin=0, qmax=255):
    """torch quantize_val: q = clamp(zp + nearbyint(x * (1.0f / (float)scale)))."""
    x = np.asarray(x, np.float32)
    inv = np.float32(1.0) / np.float32(scale)
    r = np.rint(x * inv).astype(np.int64)  # round half to even, like nearbyint
    return np.clip(r + int(zp), qmin, qmax)


def quantize_per_channel(x, scales, zps, qmin=-128, qmax=127):
    x = np.asarray(x, np.float32)
    out = np.empty(x.shape, np.int64)
    for c in range(x.shape[0]):
        out[c] = quantize_affine(x[c], scales[c], zps[c], qmin, qmax)
    return out


def minmax_qparams(lo, hi, qmin=0, qmax=255):
    """torch MinMaxObserver (per_tensor_affine) qparams, all in fp32."""
    lo = np.minimum(np.float32(lo), np.float32(0))
    hi = np.maximum(np.float32(hi), np.float32(0))
    scale = (hi - lo) / np.float32(qmax - qmin)
    scale = np.maximum(scale, EPS)
    zp = qmin - int(np.rint(lo / scale))
    return np.float32(scale), int(np.clip(zp, qmin, qmax))


def dequant_affine(q, scale, zp):
    """fl32(fl32(q - zp) * fl32(scale)) — the same formula as the client dequant."""
    return (np.asarray(q, np.int64) - int(zp)).astype(np.float32) * np.float32(scale)


def requantize_tensors(flat, layout):
    """This build's deterministic re-quantization of the aggregate, per named tensor.

    Returns (q uint8 [P], scales f32 [T], zps i32 [T], dequantized f32 [P])."""
    flat = np.asarray(flat, np.float32)
    q = np.empty(flat.shape, np.uint8)
    deq = np.empty_like(flat)
    scales, zps = [], []
    off = 0
    for _, shape in layout:
        m = int(np.prod(shape))
        seg = flat[off:off + m]
        s, z = minmax_qparams(seg.min(), seg.max())
        qs = quantize_affine(seg, s, z)
        q[off:off + m] = qs
        deq[off:off + m] = dequant_affine(qs, s, z)
        scales.append(s)
        zps.append(z)
        off += m
    return q, np.array(scales, np.float32), np.array(zps, np.int32), deq


def requantize_model(flat_concat):
    """The re-quantization at the reference's granularity: ONE quantizer over the
    concatenated aggregate (``quant(concat_dict_values(aggregated_parameter))``,
    servers/fed_quant_server.py:39), deterministic MinMax affine 8-bit.

    Returns (q uint8 [n], scale f32, zp int, dequantized f32 [n])."""
    x = np.asarray(flat_concat, np.float32)
    s, z = minmax_qparams(np.nanmin(x), np.nanmax(x))
    q = quantize_affine(x, s, z)
    return q.astype(np.uint8), s, z, dequant_affine(q, s, z)


def dequant_torch_cpu(client_parameter):
    """The reference's own torch op sequence on the CPU
    (servers/fed_quant_server.py:25-33): ``weight.float()`` then a Python loop over
    the output channels ``weight[c] = (v - zero_point[c]) * scale[c]``.  Timed by
    bench.py's CPU baseline (dequant_channel is the parity reference)."""
    out = {}
    for k, v in client_parameter.items():
        if isinstance(v, tuple):
            weight, scale, zero_point = v
            weight = weight.float()
            for idx, row in enumerate(weight):
                weight[idx] = (row - zero_point[idx]) * scale[idx]
            out[k] = weight
        else:
            out[k] = v
    return out

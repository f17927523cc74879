"""Device store of quantized client payloads for the fed_quant server.

Reference payload (servers/fed_quant_server.py:25-33, produced by the QAT
worker, workers/fed_quant_worker.py:40): ``{name: (int weight [C, ...],
scale [C], zero_point [C]) | fp32 tensor}``.  The reference materialises every
client's fp32 dequantized tensors; here the int payloads stay int in HBM and
one fused kernel (``dls_dequant_fedavg``) dequantizes and averages them.

HBM layout per client row:
  Q  uint8 [capacity, ldq]   int tensors' raw bytes (int8 or uint8); every tensor and
                             the row pitch ldq on 256-B boundaries, so a wavefront's
                             1 KiB load per client covers exactly 8 cache lines
  F  fp32  [capacity, ldf]   fp32 tensors (biases ...), 64-element aligned
  sz fp32  [C+1, capacity, 2] (fl32(scale), zero_point) per output channel,
                             channel-major: a wave's per-channel table load for 64
                             clients reads 512 consecutive bytes
and a tile table (``dls_qtile``) built once per layout: wave tiles inside one
tensor, which also carry the channel bookkeeping; the tiles whose elements all
lie in one output channel (<= 4096 elements) come first, grouped by 1 KiB slice
count (``nfast``), and run on the streamlined kernels, the rest (<= 1024
elements) on the general one.
"""
import numpy as np
import torch

from . import _native
from .layout import ALIGN, ParameterLayout, _round_up

TILE = 1024  # one wavefront slice: 64 lanes x 16 elements
FAST_TILE = 4096  # one-channel tiles: up to 4 slices per wavefront
# multi-channel tiles (channel rows a multiple of 16): "adaptive" = per tensor the
# tile width (4, 3, 2 or 1 KiB, or 1-4 whole channel rows, at most 4096 elements)
# that needs the fewest tiles while every tile spans at most 4 channel rows (the
# FMA lane kernel's staged table; a tile over more rows is walked once per 4), or
# a fixed width in elements.  The store keeps one table per mode: the
# exact kernel is bound by its instruction count at the clock the chip holds
#  and runs fastest on 1 KiB tiles (4 waves per SIMD); the FMA mode
# is bound by the stream and runs fastest on the adaptive ones (same-box A/B,
# 1000 x ResNet-18: exact 2.01 vs 2.21 ms, FMA 1.96 vs 1.88 ms).
LANE_TILE = 1024  # the exact mode's (and QuantLayout.tiles()' default)
LANE_TILE_FMA = "adaptive"
LANE_TILE_MAX = 4096  # the adaptive widths' bound (elements)
FMA_ONE_CHANNEL = False  # the FMA table's long-row tensors: one-channel tiles (True) or lane tiles
F32_TILE = 256  # fp32 tensors: 64 lanes x 4 elements
SMALL_TILE = 256  # small int tiles: 64 lanes x 4 elements
FAST_WASTE = 16  # one-channel tiles need their rows' idle lanes <= row / FAST_WASTE (0: none)
QALIGN = 256  # bytes: Q tensor starts and row pitch (a 64-B pitch split lines)

QTILE_DTYPE = np.dtype([("dst", "<i8"), ("src", "<i8"), ("len", "<i4"), ("kind", "<i4"),
                        ("chan0", "<i4"), ("row_len", "<i4"), ("row_pos", "<i4"),
                        ("chan_end", "<i4")])
assert QTILE_DTYPE.itemsize == 40


def _int_repr(w):
    if w.is_quantized:
        w = w.int_repr()
    if w.dtype not in (torch.int8, torch.uint8):
        raise TypeError(f"quantized weight must be int8/uint8, got {w.dtype}")
    return w


def is_quantized_entry(v):
    return isinstance(v, tuple) and len(v) == 3


def _adaptive_lane_tile(rl, n):
    """The FMA mode's lane-tile width for an n-element tensor of rl-element channel
    rows (rl a multiple of 16): of 4096 / 3072 / 2048 / 1024 elements and 1-4 whole
    rows (<= 4096), the one with the fewest tiles whose every tile spans <= 4 rows
    (tiles start at multiples of the width from the tensor start); ties go to the
    wider.  Whole rows always qualify, so every such tensor gets lane tiles: on
    ResNet-18 the 3x3 convs take 4 KiB / 3,456 / 2,304-element tiles and the 1x1
    shortcuts 1-4 rows, 2,986 waves in all (one generation of the FMA lane kernel
    at 3 waves per SIMD)."""
    def fits(t):
        return all((e % rl + min(t, n - e) - 1) // rl + 1 <= 4 for e in range(0, n, t))
    best = None
    cap = LANE_TILE_MAX
    for t in sorted({x for x in (8192, 6144, 4096, 3072, 2048, 1024) if x <= cap} |
                    {k * rl for k in (1, 2, 3, 4) if k * rl <= cap}, reverse=True):
        if t % 16 == 0 and fits(t) and (best is None or -(-n // t) < -(-n // best)):
            best = t
    return best


class QuantLayout:
    """Per-tensor kinds and offsets for one payload structure."""

    def __init__(self, payload):
        items = []
        self.kinds, self.src, self.chan_base, self.channels, self.row_len = [], [], [], [], []
        q_off = f_off = c_off = 0
        for name, v in payload.items():
            if is_quantized_entry(v):
                w = _int_repr(v[0])
                shape = tuple(w.shape)
                kind = 1 if w.dtype == torch.int8 else 2
                C = shape[0] if shape else 1
                n = int(np.prod(shape)) if shape else 1
                self.kinds.append(kind)
                self.src.append(q_off)
                self.chan_base.append(c_off)
                self.channels.append(C)
                self.row_len.append(max(1, n // C))
                q_off += _round_up(max(n, 1), QALIGN)
                c_off += C
            else:
                shape = tuple(v.shape)
                n = int(np.prod(shape)) if shape else 1
                self.kinds.append(0)
                self.src.append(f_off)
                self.chan_base.append(0)
                self.channels.append(0)
                self.row_len.append(1)
                f_off += _round_up(max(n, 1), ALIGN)
            items.append((name, shape))
        self.layout = ParameterLayout(items)
        self.ldq = max(q_off, QALIGN)
        self.ldf = max(f_off, ALIGN)
        self.C = c_off
        self.names = self.layout.names

    def matches(self, payload):
        if list(payload.keys()) != self.names:
            return False
        for v, kind, shape in zip(payload.values(), self.kinds, self.layout.shapes):
            if (kind > 0) != is_quantized_entry(v):
                return False
            t = v[0] if kind else v
            if tuple(t.shape) != shape:
                return False
        return True

    def tiles(self, lane_tile=None, one_channel=True):
        """(table, nfast): wave tiles; nfast = counts of the 10 grouped kinds at the
        head of the table (dls_hip.h DLS_QTILE_GROUPS), then the general tiles.
        ``lane_tile``: the multi-channel tiles' width (default LANE_TILE).

        * one-channel tiles (groups 0-3: 4, 3, 2, 1 KiB slices): int tensors whose
          channel rows are long (>= 1024, multiple of 64) and fill 1 KiB slices
          well get channel-aligned tiles of up to FAST_TILE elements (a wave
          streams up to 4 KiB of every client row with one (scale, zp) per client);
        * lane-channel tiles (groups 4-7: 4, 3, 2, 1 KiB slices): the other int
          tensors whose channel rows are a multiple of 16 elements (no lane's
          16-element chunk straddles two channels: 3x3 convs, fc layers) are cut
          into LANE_TILE-element tiles from their start, each lane in its own
          channel (adaptive: the width with the fewest tiles of <= 4 channel rows,
          _adaptive_lane_tile);
        * fp32 tiles (group 8, <= F32_TILE elements): the fp32 tensors;
        * small int tiles (group 9, <= SMALL_TILE elements): the other int tensors
          with rows of at least 4 elements (a lane's 4 span <= 2 channels), except
          their 1 KiB pieces that lie inside one channel (one-channel group 3);
        * general tiles (<= TILE elements): int tensors with rows shorter than 4.

        ``one_channel=False`` (the FMA mode's table, FMA_ONE_CHANNEL): long-row
        tensors are lane-tiled too — contiguous tiles across the row boundaries
        (a 4096-element tile over a 25,088-element fc row spans <= 2 channels), so
        no row leaves a part-filled tail tile (VGG-16's fc1: 4,096 half-empty
        512-element tiles otherwise)."""
        rows, lane_rows, f32_rows, small_rows = [], [], [], []
        for i, kind in enumerate(self.kinds):
            n = self.layout.numels[i]
            rl = self.row_len[i]
            off, src, cb = self.layout.offsets[i], self.src[i], self.chan_base[i]
            cend = cb + self.channels[i] if kind else 0
            waste = -rl % TILE  # idle lanes of the row's last slice
            if one_channel and kind and rl >= TILE and rl % 64 == 0 and (
                    waste == 0 if FAST_WASTE == 0 else FAST_WASTE * waste <= rl):
                for c in range(self.channels[i]):
                    for j in range(0, rl, FAST_TILE):
                        e = c * rl + j
                        rows.append((off + e, src + e, min(FAST_TILE, rl - j), kind, cb + c, rl,
                                     j, cend))
                continue
            lt = LANE_TILE if lane_tile is None else lane_tile
            if lt == "adaptive" and kind and rl % 16 == 0:
                lt = _adaptive_lane_tile(rl, n)  # None: not a lane-tile tensor
            if kind and rl % 16 == 0 and lt is not None:
                for e in range(0, n, lt):
                    lane_rows.append((off + e, src + e, min(lt, n - e), kind, cb + e // rl,
                                      rl, e % rl, cend))
                continue
            if not kind:
                for e in range(0, n, F32_TILE):
                    f32_rows.append((off + e, src + e, min(F32_TILE, n - e), 0, 0, 1, 0, 0))
                continue
            if rl >= 4:
                # 1 KiB tiles from the tensor start; those inside one channel run on
                # the one-channel kernel, the others are cut into small tiles
                for e in range(0, n, TILE):
                    ln = min(TILE, n - e)
                    if e % rl + ln <= rl:
                        rows.append((off + e, src + e, ln, kind, cb + e // rl, rl, e % rl, cend))
                        continue
                    for e2 in range(e, e + ln, SMALL_TILE):
                        small_rows.append((off + e2, src + e2, min(SMALL_TILE, e + ln - e2), kind,
                                           cb + e2 // rl, rl, e2 % rl, cend))
                continue
            for e in range(0, n, TILE):
                rows.append((off + e, src + e, min(TILE, n - e), kind, cb + e // rl if kind else 0,
                             rl, e % rl if kind else 0, cend))

        def in_one_channel(r):
            return r[3] != 0 and r[6] + r[2] <= r[5]  # kind int, row_pos + len <= row_len

        def slices(r):
            return (r[2] + 63) // 64 * 64 // TILE + ((r[2] + 63) // 64 * 64 % TILE != 0)

        fast = [[r for r in rows if in_one_channel(r) and slices(r) == g] for g in (4, 3, 2, 1)]
        # group 4: lane tiles of 4 KiB slices or more (FMA tables: up to LANE_TILE_MAX)
        fast += [[r for r in lane_rows if min(slices(r), 4) == g] for g in (4, 3, 2, 1)]
        fast += [f32_rows, small_rows]
        rest = [r for r in rows if not in_one_channel(r)]
        assert all(r[2] <= TILE for r in rest)
        return (np.array([r for grp in fast for r in grp] + rest, dtype=QTILE_DTYPE),
                tuple(len(grp) for grp in fast))


class QuantizedClientStore:
    def __init__(self, payload, device, capacity=1):
        self.qlayout = QuantLayout(payload)
        self.layout = self.qlayout.layout
        self.device = torch.device(device)
        cap = max(1, capacity)
        ql = self.qlayout
        self.Q = torch.zeros((cap, ql.ldq), dtype=torch.uint8, device=self.device)
        self.F = torch.zeros((cap, ql.ldf), dtype=torch.float32, device=self.device)
        self.sz = torch.zeros((ql.C + 1, cap, 2), dtype=torch.float32, device=self.device)
        t, self.nfast = ql.tiles()
        self.ntiles = len(t)
        self.tiles = torch.from_numpy(t.view(np.uint8).copy()).to(self.device)
        tf, self.nfast_fma = ql.tiles(LANE_TILE_FMA, one_channel=FMA_ONE_CHANNEL)
        self.ntiles_fma = len(tf)
        self.tiles_fma = torch.from_numpy(tf.view(np.uint8).copy()).to(self.device)
        self._host_tables = {_native.FEDAVG_EXACT: (t, self.nfast),
                             _native.FEDAVG_FMA: (tf, self.nfast_fma)}
        self._col_tables = {}
        self._free = list(range(cap))[::-1]

    @property
    def capacity(self):
        return self.Q.shape[0]

    def acquire(self):
        if not self._free:
            old = (self.Q, self.F, self.sz)
            cap = 2 * old[0].shape[0]
            self.Q = torch.zeros((cap,) + tuple(old[0].shape[1:]), dtype=old[0].dtype,
                                 device=self.device)
            self.F = torch.zeros((cap,) + tuple(old[1].shape[1:]), dtype=old[1].dtype,
                                 device=self.device)
            self.sz = torch.zeros((old[2].shape[0], cap, 2), dtype=old[2].dtype,
                                  device=self.device)
            n = old[0].shape[0]
            self.Q[:n].copy_(old[0])
            self.F[:n].copy_(old[1])
            self.sz[:, :n].copy_(old[2])
            self._free = list(range(n, cap))[::-1]
        return self._free.pop()

    def release(self, row):
        self._free.append(row)

    def write(self, row, payload):
        ql = self.qlayout
        for i, (name, v) in enumerate(payload.items()):
            n = self.layout.numels[i]
            if ql.kinds[i]:
                w, scale, zp = v
                w = _int_repr(w)
                self.Q[row, ql.src[i]:ql.src[i] + n].copy_(
                    w.reshape(-1).view(torch.uint8), non_blocking=True)
                cb, C = ql.chan_base[i], ql.channels[i]
                # torch casts the 0-dim float64 scale / int64 zero point to fp32
                # before the fp32 ops (servers/fed_quant_server.py:31)
                s32 = torch.as_tensor(scale).reshape(-1).to(torch.float32)
                z32 = torch.as_tensor(zp).reshape(-1).to(torch.float32)
                self.sz[cb:cb + C, row, 0].copy_(s32, non_blocking=True)
                self.sz[cb:cb + C, row, 1].copy_(z32, non_blocking=True)
            else:
                self.F[row, ql.src[i]:ql.src[i] + n].copy_(v.reshape(-1).float(),
                                                           non_blocking=True)

    def fedavg(self, rows, ns, out=None, total=None, mode=_native.FEDAVG_EXACT, cols=None):
        """Dequant + weighted mean of the rows (dls_dequant_fedavg_mode): EXACT is
        bit-exact with the reference's dequant-then-average, FMA within 1e-6.

        ``rows`` / ``ns``: sequences, or device int32 / fp32 tensors (a caller that
        makes several calls over the same clients converts them once).  ``cols =
        (c0, c1)``: only the tiles whose first output element lies in [c0, c1)
        (``out`` is still the whole P-element row; a tile starting in the range may
        end past c1, so the range's elements are final once every range before it
        has run too) — the sharded server reduces the column chunks in order while
        the previous chunk's all-reduce is on the wire."""
        if out is None:
            out = torch.empty(self.layout.P, dtype=torch.float32, device=self.device)
        if torch.is_tensor(rows):
            rows_t = rows
        else:
            rows_t = torch.tensor(list(rows), dtype=torch.int32).to(self.device)
        if torch.is_tensor(ns):
            w_t = ns
            if total is None:
                total = float(ns.sum())
        else:
            w_t = torch.tensor([int(n) for n in ns], dtype=torch.float32).to(self.device)
            if total is None:
                total = sum(int(n) for n in ns)
        tiles, ntiles, nfast = self.table(mode, cols)
        if ntiles == 0:
            return out
        _native.dequant_fedavg(tiles, ntiles, nfast, self.Q, self.F, self.sz, rows_t, w_t,
                               float(total), out, mode=mode)
        return out

    def table(self, mode=_native.FEDAVG_EXACT, cols=None):
        """(tiles, ntiles, nfast) the fused kernel takes in this mode; ``cols``: the
        sub-table of the tiles starting in [c0, c1), groups kept in table order
        (built on the host once per (mode, range) and cached)."""
        if cols is None:
            if mode == _native.FEDAVG_FMA:
                return self.tiles_fma, self.ntiles_fma, self.nfast_fma
            return self.tiles, self.ntiles, self.nfast
        key = (int(mode), int(cols[0]), int(cols[1]))
        hit = self._col_tables.get(key)
        if hit is None:
            t, nfast = self._host_tables[int(mode)]
            ends = np.cumsum(list(nfast))
            group = np.searchsorted(ends, np.arange(len(t)), side="right")  # len(nfast): general
            keep = (t["dst"] >= cols[0]) & (t["dst"] < cols[1])
            sub = t[keep]
            nsub = tuple(int(np.count_nonzero(keep & (group == g))) for g in range(len(nfast)))
            dev = torch.from_numpy(sub.view(np.uint8).copy()).to(self.device)
            hit = self._col_tables[key] = (dev, len(sub), nsub)
        return hit

    def dequantize(self, row):
        """One client's fp32 dict (the reference's _process_client_parameter output)."""
        return self.layout.views(self.fedavg([row], [1]))

    def accepts(self, payload):
        return self.qlayout.matches(payload)

    def views(self, row):
        return self.dequantize(row)

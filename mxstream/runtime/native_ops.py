"""Native-backed DataStream operators.

``NativeWindowOp`` runs a keyed tumbling/sliding window with a field-wise aggregate (reduce that
sums one numeric field, ``sum/min/max(pos)``, builtin aggregate functions) on the native
``KeyedWindowOperator`` — the C++ twin on CPU or the gfx950 kernels on GPU — instead of the
per-record host WindowOperator. Semantics are identical (differential tests in
tests/test_api_native.py); the planner (api/planner.py) only selects it for shapes it can prove.

Records are columnarised per micro-batch: the key field becomes a 64-bit id (string keys via the
C++ StringDict), the aggregated field an int64 / float64 column, the timestamp an int64 column;
window results come back as (key id, value, count) rows and are rebuilt into tuples.
"""
from __future__ import annotations

import numpy as np
import torch

from ..api.tuples import Tuple
from ..ops import expr as E
from ..ops import kernels as K
from ..ops.text import FK_DOUBLE, FK_LONG, FK_STR
from ..utils.hashing import java_hash
from .columnar import ColumnBatch, DeviceColumnBatch, concat_device, expand_columns
from .operators import LONG_MAX, LONG_MIN, Operator, Rec, WM, WindowOp
from .window_operator import KeyedWindowOperator


class _ColumnInput:
    """Columnar input for the native keyed operators: a ColumnBatch's key column (dense
    dictionary ids of string keys, or integer keys) and value column go to the engine as they
    are; only keys seen for the first time build a keep-first template tuple."""

    def _cb_keys(self, cb: ColumnBatch) -> np.ndarray:
        kp = self.key_pos
        kk = cb.kinds[kp]
        col = cb.cols[kp]
        if kk == FK_STR:
            if self.str_keys is False:
                raise TypeError("mixed key types")
            self.str_keys = True
            if cb.strings is not self.dict:
                if len(self.dict) == 0 and not self.templates:
                    self.dict = cb.strings  # adopt the parser's dictionary: ids are shared
                else:
                    u, inv = np.unique(col, return_inverse=True)
                    names = cb.strings.strings()
                    ids = np.array([self.dict.intern(names[x]) for x in u.tolist()], dtype=np.int32)
                    return ids[inv]
            # Dictionary ids stay int32: the window operator's partition reads them as they are.
            return col.astype(np.int32, copy=False)
        if kk == FK_DOUBLE:
            raise TypeError("double keys on the native path")
        if self.str_keys is True:
            raise TypeError("mixed key types")
        self.str_keys = False
        if col.size and (int(col.min()) < 0 or int(col.max()) >= (1 << 63) - 2):
            raise TypeError("negative / reserved integer keys on the native path")
        return col.astype(np.int64, copy=False)

    def _cb_templates(self, cb: ColumnBatch, kid: np.ndarray) -> None:
        u, first = np.unique(kid, return_index=True)
        known = getattr(self, "_known", None)
        if known is not None and known.size:
            new = ~np.isin(u, known)
            u, first = u[new], first[new]
        if u.size:
            for k, i in zip(u.tolist(), first.tolist()):
                if k not in self.templates:
                    self.templates[k] = cb.value(i)
            self._known = u if known is None else np.union1d(known, u)

    def _template(self, k: int):
        """Keep-first template of key id k. Device batches never bring host rows: their
        template holds the key (its dictionary name) and leaves the other fields empty -- the
        planner only lowers a window whose other fields are dead downstream."""
        t = self.templates.get(k)
        if t is not None:
            return t
        lazy = getattr(self, "_lazy_tpl", None)
        if lazy is None:
            raise KeyError(k)
        t = lazy.get(k)
        if t is None:
            row = [None] * self._lazy_arity
            row[self.key_pos] = self.dict.get(k) if self.str_keys else k
            t = lazy[k] = Tuple(row)
        return t

    def _device_keys(self, cb: DeviceColumnBatch):
        """Key column of a device batch: dictionary ids (the batch's DeviceDict becomes this
        operator's dictionary) or non-negative integer keys."""
        kp = self.key_pos
        kk = cb.kinds[kp]
        col = cb.cols[kp][:cb.n]
        if kk == FK_STR:
            if self.str_keys is False:
                raise TypeError("mixed key types")
            if cb.strings is not self.dict:
                known = self.dict.strings() if len(self.dict) else []
                # (an empty dictionary needs no comparison: reading the parser's names back
                # would wait for the device -- a 7 ms stall in the first step of config 7)
                if not self.templates and (not known
                                           or cb.strings.strings()[:len(known)] == known):
                    # the parser's dictionary (after a restore: the same strings, same ids)
                    self.dict = cb.strings
                else:
                    raise TypeError("keys from a second dictionary")
            self.str_keys = True
            return col
        if kk == FK_DOUBLE:
            raise TypeError("double keys on the native path")
        if self.str_keys is True:
            raise TypeError("mixed key types")
        self.str_keys = False
        if cb.n and int(col.min()) < 0:
            raise TypeError("negative integer keys on the native path")
        return col

    @staticmethod
    def _cb_concat(batches: list) -> ColumnBatch:
        if len(batches) == 1:
            return batches[0]
        b0 = batches[0]
        if any(b.kinds != b0.kinds or b.strings is not b0.strings for b in batches):
            raise TypeError("incompatible column batches")
        cat = lambda xs: None if xs[0] is None else np.concatenate(xs)  # noqa: E731
        return ColumnBatch(sum(b.n for b in batches),
                           [np.concatenate([b.cols[j] for b in batches]) for j in range(len(b0.cols))],
                           b0.kinds, b0.strings, cat([b.ts for b in batches]),
                           cat([b.sub for b in batches]))


class NativeWindowOp(_ColumnInput, Operator):
    name = "Window(native)"
    accepts_columns = True

    def __init__(self, *, key_fn, key_pos: int, val_pos: int, kind: str, assigner, lateness: int,
                 late_tag, device: str, fallback_factory, map_prog=None, filter_prog=None,
                 result_builder=None, max_keys: int = 1 << 16, ok_arities=None):
        self.key_fn = key_fn
        self.key_pos = key_pos
        self.val_pos = val_pos
        self.kind = kind                      # sum | min | max | count | avg
        self.assigner = assigner
        self.lateness = lateness
        self.late_tag = late_tag
        self.device = device
        self.fallback_factory = fallback_factory
        self.result_builder = result_builder
        self.max_keys = max_keys
        self.ok_arities = ok_arities
        # Fused post-window map/filter (planner._fuse_window_epilogue): evaluated in the fire
        # kernel; fused_layout gives the output tuple (field index, or -1 = the mapped value).
        self.map_prog, self.filter_prog = map_prog, filter_prog
        self.fused_layout = None
        self.fused_scalar = False
        self._subs: dict = {}                 # key id -> output subtask
        self.op: KeyedWindowOperator | None = None
        self.fallback: WindowOp | None = None
        self.wm = LONG_MIN
        self.pending: list = []
        self.templates: dict = {}             # key id -> first record (keep-first fields)
        self.num_late_records_dropped = 0

    device_input = None  # planner: (column kinds, shared ingest state) for device-ingest input

    def open(self, ctx):
        super().open(ctx)
        from ..ops.native import load

        self.dict = load().StringDict()
        self.str_keys = None
        self.device_exchange = self.collective = False
        comm = getattr(ctx, "comm", None)
        if (comm is not None and comm.world > 1 and self.device_input is not None
                and self._exchange_ok):
            # Multi-rank with device-ingest input: the operator exchanges keys itself (local-
            # global partials or records over RCCL, key groups from the shared dictionary's Java
            # hashes) and runs one collective step per pass -- built now, identically on every
            # rank. Processing-time windows stamp and fire on the step's agreed clock (the
            # executor's MAX over the ranks' clocks), so every rank fires the same windows.
            kinds, shared = self.device_input
            vk = kinds[self.val_pos]
            if vk == FK_STR or (self.ok_arities and len(kinds) not in self.ok_arities):
                return
            if kinds[self.key_pos] == FK_DOUBLE:
                return
            self.dict = shared["dict"]
            self.str_keys = kinds[self.key_pos] == FK_STR
            self.comm = comm
            self.device_exchange = self.collective = True
            self._lazy_tpl, self._lazy_arity = {}, len(kinds)
            if not self._build(1.0 if vk == FK_DOUBLE else 1, dense=self.str_keys):
                self.device_exchange = self.collective = False
                self.op, self.comm = None, None
                self.dict, self.str_keys = load().StringDict(), None
                self._lazy_tpl = None

    _exchange_ok = True  # subclasses that cannot exchange their keys at G > 1 opt out
    scalar_result = False  # planner: the window emits the bare aggregate (a Double), no tuple

    def _jhash(self):
        """Java hashes of the dictionary ids (key groups of string keys at G > 1)."""
        jh = getattr(self.dict, "id_jh", None)
        return jh if jh is not None else torch.zeros(1, dtype=torch.int32,
                                                     device=torch.device(self.device))

    dense_budget = 1 << 27  # planner: ExecutionConfig.window_dense_max_keys
    _spill_state = False    # hashed keys + host-DRAM tier (a dictionary beyond dense_budget)

    def _ensure_capacity(self) -> None:
        """Dense state covers dictionary ids < max_keys: a growing dictionary regrows the state
        (snapshot -> larger operator -> restore). Beyond `dense_budget` ids the state moves to
        hashed keys of that HBM size with the host-DRAM tier: keys whose data is older than a
        window leave HBM (runtime/window_spill.py) instead of every id holding a slot. At G > 1
        every rank sees the same dictionary size, so every rank switches in the same pass (the
        restore is collective)."""
        if not (self.str_keys and self.op is not None and getattr(self.op, "dense_bits", 0)):
            return
        need = len(self.dict)
        if need <= (1 << self.op.dense_bits):
            return
        es = self.op.snapshot_state()
        budget = max(1024, int(self.dense_budget))
        if need > budget:
            self.max_keys = 1 << max(budget - 1, 1).bit_length()
            self._spill_state = True
            self._build(1.0 if self.is_float else 1, dense=False)
        else:
            self.max_keys = 1 << max(need - 1, 1).bit_length()
            self._build(1.0 if self.is_float else 1, dense=True)
        self.op.restore_state(es.columns, es.meta)

    def _local_columns(self, data: list):
        """This rank's (key id, timestamp, value bits) device columns of a pass (empty columns
        when it got no rows). Processing time: every row carries the step's agreed time."""
        dev = self.op.device if self.op is not None else torch.device(self.device)
        if any(not isinstance(b, DeviceColumnBatch) for b in data):
            raise TypeError("multi-rank native window: device-ingest batches expected")
        event = self.assigner.is_event_time()
        if data:
            cb = concat_device(data)
            n = cb.n
            kid = cb.cols[self.key_pos][:n]
            if event:
                ts = cb.ts[:n] if cb.ts is not None else torch.full((n,), LONG_MIN,
                                                                     dtype=torch.int64, device=dev)
            else:
                ts = torch.full((n,), self.ctx.clock(), dtype=torch.int64, device=dev)
            vals = cb.cols[self.val_pos][:n]
            vals = vals.view(torch.int64) if vals.dtype == torch.float64 else vals.to(torch.int64)
        else:
            kid = torch.empty(0, dtype=torch.int32 if self.str_keys else torch.int64, device=dev)
            ts = torch.empty(0, dtype=torch.int64, device=dev)
            vals = torch.empty(0, dtype=torch.int64, device=dev)
        return kid.contiguous(), ts.contiguous(), vals.contiguous()

    def _process_exchange(self, items) -> list:
        """G > 1 device exchange: one engine step per pass (an empty batch if this rank got no
        rows), then the merged watermark (identical on every rank) advances every rank (event
        time; processing-time windows fire in on_processing_time on the agreed clock)."""
        data = [it for it in items if not isinstance(it, WM)]
        wms = [it.ts for it in items if isinstance(it, WM)]
        self._ensure_capacity()
        self.op.jhash = self._jhash()
        kid, ts, vals = self._local_columns(data)
        if kid.dtype == torch.int32 and not self._key32_ok:
            kid = kid.to(torch.int64)
        late_before = self.op.metrics.num_late_records_dropped
        out = self._emit(self.op.process(kid, ts, vals))
        self.num_late_records_dropped += self.op.metrics.num_late_records_dropped - late_before
        event = self.assigner.is_event_time()
        for w in wms:
            self.wm = w
            if event:
                out.extend(self._emit(self.op.advance_watermark(w)))
            out.append(WM(w))
        return out

    # -- lazy construction on the first records (value type decides the aggregate kind) --
    def _build(self, sample_val, dense: bool = False) -> bool:
        is_float = isinstance(sample_val, float)
        if not isinstance(sample_val, (int, float)) or isinstance(sample_val, bool):
            return False
        agg = {("sum", False): K.AGG_SUM_I64, ("sum", True): K.AGG_SUM_F64,
               ("min", False): K.AGG_MIN_I64, ("min", True): K.AGG_MIN_F64,
               ("max", False): K.AGG_MAX_I64, ("max", True): K.AGG_MAX_F64,
               ("count", False): K.AGG_COUNT, ("count", True): K.AGG_COUNT,
               ("avg", False): K.AGG_AVG_I64, ("avg", True): K.AGG_AVG_F64}[(self.kind, is_float)]
        self.is_float = is_float
        a = self.assigner
        event = a.is_event_time()
        dev = torch.device(self.device)
        if dense:
            # Dense dictionary-id state sized to the dictionary (x2 headroom, regrown as it
            # grows): a firing sweeps every slot of its panes, so a 2^16-slot table for a
            # thousand channels would cost 64x the sweep (5 min / 5 s windows: 60 panes each).
            self.max_keys = max(2048, 1 << max(1, 2 * max(1, len(self.dict))).bit_length())
        cap_log2 = 12 if self.max_keys > 100_000 else (6 if self._spill_state else 9)
        comm = getattr(self, "comm", None)
        multi = comm is not None and comm.world > 1
        self.op = KeyedWindowOperator(
            size=a.size, slide=a.slide, offset=a.offset, lateness=self.lateness if event else 0,
            agg=agg, device=dev, max_keys=self.max_keys,
            parallelism=self.ctx.parallelism if multi else 1, comm=comm if multi else None,
            max_parallelism=self.ctx.max_parallelism if multi else 128,
            hash_mode=1 if (multi and self.str_keys) else 0,
            jhash_table=self._jhash() if (multi and self.str_keys) else None,
            exchange="partials" if multi else "auto", spill=self._spill_state,
            batch_capacity=max(1024, self.ctx.parallelism), cap_log2=cap_log2,
            time_mode="event" if event else "processing", external_watermark=True,
            side_output_late=self.late_tag is not None, clock=self.ctx.clock,
            dense_keys=dense, map_prog=self.map_prog or E.EMPTY,
            filter_prog=self.filter_prog or E.EMPTY,
            emit="key_value" if self._key_value_only() else "full")
        return True

    def _key_value_only(self) -> bool:
        """The output tuple reads only the key and the mapped value (no raw result, count or
        keep-first template field): fired rows can be 12-byte (key id, value) rows."""
        if self.fused_scalar:
            return True
        return self.fused_layout is not None and all(
            j < 0 or (j == self.key_pos and j != self.val_pos) for j in self.fused_layout)

    def _to_fallback(self):
        self.fallback = self.fallback_factory()
        self.fallback.open(self.ctx)

    def _key_id(self, k) -> int:
        if isinstance(k, str):
            if self.str_keys is False:
                raise TypeError("mixed key types")
            self.str_keys = True
            return self.dict.intern(k)
        if isinstance(k, int) and not isinstance(k, bool) and 0 <= k < (1 << 63) - 1:
            if self.str_keys is True:
                raise TypeError("mixed key types")
            self.str_keys = False
            return k
        raise TypeError("unsupported key type for the native path")

    def _flush_device(self, batches: list) -> list:
        """Device batches (device text ingest): key, timestamp and value columns go to the
        engine operator in place -- no host copy, no per-record Python."""
        try:
            cb = concat_device(batches)
            vk = cb.kinds[self.val_pos]
            if vk == FK_STR or (self.ok_arities and len(cb.kinds) not in self.ok_arities):
                raise TypeError("value column not numeric")
            kid = self._device_keys(cb)  # adopts the dictionary before the state is sized
            if self.op is None:
                dense = cb.kinds[self.key_pos] == FK_STR
                if not self._build(1.0 if vk == FK_DOUBLE else 1, dense=dense):
                    raise TypeError("unsupported value")
            elif (vk == FK_DOUBLE) != self.is_float:
                raise TypeError("mixed value types")
        except TypeError:
            if self.templates or getattr(self, "_lazy_tpl", None):
                raise
            recs = expand_columns(batches)
            self._to_fallback()
            return self.fallback.process(recs)
        if getattr(self, "_lazy_tpl", None) is None:
            self._lazy_tpl, self._lazy_arity = {}, len(cb.kinds)
        self._ensure_capacity()
        dev = self.op.device
        n = cb.n
        if self.assigner.is_event_time():
            ts = cb.ts[:n] if cb.ts is not None else torch.full((n,), LONG_MIN, dtype=torch.int64,
                                                                 device=dev)
        else:
            ts = torch.full((n,), self.ctx.clock(), dtype=torch.int64, device=dev)
        vals = cb.cols[self.val_pos][:n]
        vals = vals.view(torch.int64) if vals.dtype == torch.float64 else vals.to(torch.int64)
        if kid.dtype == torch.int32 and not self._key32_ok:
            kid = kid.to(torch.int64)
        late_before = self.op.metrics.num_late_records_dropped
        fired = self.op.process(kid.contiguous(), ts.contiguous(), vals.contiguous())
        if getattr(self.op, "late_side", None):
            host = cb.host()
            for idx in np.concatenate(self.op.late_side).tolist():
                self.side.setdefault(self.late_tag.tag_id, []).append(
                    Rec(host.value(idx), int(host.ts[idx]) if host.ts is not None else LONG_MIN,
                        int(host.sub[idx])))
            self.op.late_side.clear()
        elif self.late_tag is None:
            self.num_late_records_dropped += self.op.metrics.num_late_records_dropped - late_before
        return self._emit(fired)

    _key32_ok = True  # KeyedWindowOperator reads int32 dictionary ids as they are

    def _flush_columns(self, batches: list) -> list:
        """All pending items are ColumnBatches: no per-record Python on the input side."""
        if all(isinstance(b, DeviceColumnBatch) for b in batches):
            return self._flush_device(batches)
        batches = [b.host() if isinstance(b, DeviceColumnBatch) else b for b in batches]
        try:
            cb = self._cb_concat(batches)
            vk = cb.kinds[self.val_pos]
            if vk == FK_STR or (self.ok_arities and len(cb.kinds) not in self.ok_arities):
                raise TypeError("value column not numeric")
            if self.op is None:
                dense = cb.kinds[self.key_pos] == FK_STR
                if not self._build(1.0 if vk == FK_DOUBLE else 1, dense=dense):
                    raise TypeError("unsupported value")
            elif (vk == FK_DOUBLE) != self.is_float:
                raise TypeError("mixed value types")
            kid = self._cb_keys(cb)
        except TypeError:
            if self.templates:
                raise
            recs = expand_columns(batches)
            self._to_fallback()
            return self.fallback.process(recs)
        self._cb_templates(cb, kid)
        self._ensure_capacity()
        event = self.assigner.is_event_time()
        if event:
            tsa = cb.ts if cb.ts is not None else np.full(cb.n, LONG_MIN, dtype=np.int64)
        else:
            tsa = np.full(cb.n, self.ctx.clock(), dtype=np.int64)
        vv = cb.cols[self.val_pos].astype(np.float64 if self.is_float else np.int64, copy=False)
        dev = self.op.device
        late_before = self.op.metrics.num_late_records_dropped
        fired = self.op.process(torch.from_numpy(np.ascontiguousarray(kid)).to(dev),
                                torch.from_numpy(np.ascontiguousarray(tsa, dtype=np.int64)).to(dev),
                                torch.from_numpy(np.ascontiguousarray(vv).view(np.int64)).to(dev))
        if getattr(self.op, "late_side", None):
            for idx in np.concatenate(self.op.late_side).tolist():
                sub = int(cb.sub[idx]) if cb.sub is not None else 0
                ts = int(cb.ts[idx]) if cb.ts is not None else LONG_MIN
                self.side.setdefault(self.late_tag.tag_id, []).append(Rec(cb.value(idx), ts, sub))
            self.op.late_side.clear()
        elif self.late_tag is None:
            self.num_late_records_dropped += self.op.metrics.num_late_records_dropped - late_before
        return self._emit(fired)

    def _flush(self) -> list:
        recs = self.pending
        self.pending = []
        if not recs:
            return []
        if all(isinstance(r, ColumnBatch) for r in recs):
            return self._flush_columns(recs)
        recs = expand_columns(recs)
        if self.op is None:
            v0 = recs[0].value
            dense = (isinstance(v0, tuple) and len(v0) > self.key_pos
                     and isinstance(v0[self.key_pos], str))
            if (not isinstance(v0, tuple) or (self.ok_arities and len(v0) not in self.ok_arities)
                    or not self._build(v0[self.val_pos], dense=dense)):
                self._to_fallback()
                return self.fallback.process(recs)
        n = len(recs)
        try:
            kid = np.empty(n, dtype=np.int64)
            tsa = np.empty(n, dtype=np.int64)
            vv = np.empty(n, dtype=np.float64 if self.is_float else np.int64)
            now = self.ctx.clock()
            event = self.assigner.is_event_time()
            for i, r in enumerate(recs):
                v = r.value
                k = self._key_id(v[self.key_pos])
                kid[i] = k
                if k not in self.templates:
                    self.templates[k] = v
                tsa[i] = r.ts if event else now
                x = v[self.val_pos]
                if isinstance(x, float) != self.is_float:
                    raise TypeError("mixed value types")
                vv[i] = x
        except TypeError:
            # Unsupported data for the native path: switch to the exact host operator.
            self._to_fallback()
            return self.fallback.process(recs)
        dev = self.op.device
        kt = torch.from_numpy(kid).to(dev)
        tt = torch.from_numpy(tsa).to(dev)
        vt = torch.from_numpy(vv.view(np.int64)).to(dev)
        late_before = self.op.metrics.num_late_records_dropped
        fired = self.op.process(kt, tt, vt)
        if self.op.late_side:
            for idx in np.concatenate(self.op.late_side).tolist():
                r = recs[idx]
                self.side.setdefault(self.late_tag.tag_id, []).append(Rec(r.value, r.ts, r.subtask))
            self.op.late_side.clear()
        elif self.late_tag is None:
            self.num_late_records_dropped += self.op.metrics.num_late_records_dropped - late_before
        return self._emit(fired)

    def _out_layout(self):
        """(layout, scalar) of the output rows: field indices of the output tuple (-1 = the
        mapped value), or one column for a bare result / a map to a scalar."""
        if self.fused_scalar:
            return (-1,), True
        if self.fused_layout is None and self.scalar_result:
            return (self.val_pos,), True
        return self.fused_layout, False

    def _columnar_kinds(self):
        """Column kinds of the output rows when every field is the key, the window result or
        the mapped value (no keep-first template fields); None otherwise."""
        layout, _ = self._out_layout()
        if layout is None or self.str_keys is None:
            return None
        kinds = []
        for j in layout:
            if j < 0 or (j == self.val_pos and self.kind == "avg"):
                kinds.append(FK_DOUBLE)
            elif j == self.val_pos:
                kinds.append(FK_DOUBLE if self.is_float and self.kind != "count" else FK_LONG)
            elif j == self.key_pos:
                kinds.append(FK_STR if self.str_keys else FK_LONG)
            else:
                return None
        return tuple(kinds)

    def _subtasks(self, keys: np.ndarray) -> np.ndarray:
        """Output subtask of every key id (Java hash + murmur, cached per key). Dictionary keys
        of a device dictionary: one vectorised pass over the ids' Java hashes."""
        P, MP = self.ctx.parallelism, self.ctx.max_parallelism
        jh = getattr(self.dict, "jhash_table", None) if self.str_keys else None
        if jh is not None and keys.size:
            from ..utils.hashing import key_groups_of_java_hashes

            tab = getattr(self, "_sub_tab", None)
            need = int(keys.max()) + 1
            if tab is None or tab.size < need:
                hashes = jh()
                if hashes.size >= need:
                    tab = self._sub_tab = (key_groups_of_java_hashes(hashes, MP).astype(np.int64)
                                           * P // MP).astype(np.int32)
            if tab is not None and tab.size >= need:
                return tab[keys]
        u, inv = np.unique(keys, return_inverse=True)
        su = np.empty(u.size, dtype=np.int32)
        for i, k in enumerate(u.tolist()):
            sub = self._subs.get(k)
            if sub is None:
                from ..utils.hashing import flink_murmur

                key_obj = self.dict.get(k) if self.str_keys else k
                sub = self._subs[k] = (flink_murmur(java_hash(key_obj)) % MP) * P // MP
            su[i] = sub
        return su[inv.reshape(-1)]

    def _emit_columns(self, fired, kinds) -> list:
        """The fired rows of all windows as ONE ColumnBatch (window order, then row order --
        the order of the per-record path): a columnar sink (print) formats them in bulk,
        any other operator receives the same Recs through ColumnBatch.to_recs."""
        fired = [fr for fr in fired if fr.keys.size]
        if not fired:
            return []
        keys = np.concatenate([fr.keys for fr in fired])
        keys = keys.view(np.int64) if keys.dtype == np.uint64 else keys.astype(np.int64)
        cols = []
        layout, scalar = self._out_layout()
        for j, k in zip(layout, kinds):
            if j < 0 or (j == self.val_pos and self.kind == "avg"):
                cols.append(np.concatenate([fr.values for fr in fired]).astype(np.float64, copy=False))
            elif j == self.val_pos:
                if self.kind == "count":
                    cols.append(np.concatenate([fr.counts for fr in fired]).astype(np.int64))
                else:
                    raw = np.concatenate([fr.raw for fr in fired])
                    raw = raw.view(np.int64) if raw.dtype == np.uint64 else raw.astype(np.int64)
                    cols.append(raw.view(np.float64) if k == FK_DOUBLE else raw)
            else:
                cols.append(keys)
        ts = np.repeat(np.array([fr.window_end - 1 for fr in fired], dtype=np.int64),
                       [fr.keys.size for fr in fired])
        return [ColumnBatch(int(keys.size), cols, kinds, self.dict if self.str_keys else None,
                            ts, self._subtasks(keys), scalar)]

    def _emit(self, fired) -> list:
        kinds = self._columnar_kinds() if fired else None
        if kinds is not None:
            return self._emit_columns(fired, kinds)
        out = []
        P, MP = self.ctx.parallelism, self.ctx.max_parallelism
        for fr in fired:
            ts = fr.window_end - 1
            n = len(fr.keys)
            raws = fr.raw.tolist() if fr.raw is not None else [0] * n
            cnts = fr.counts.tolist() if fr.counts is not None else [0] * n
            for k, val, raw, cnt in zip(fr.keys.tolist(), fr.values.tolist(), raws, cnts):
                key_obj = self.dict.get(k) if self.str_keys else k
                if self.kind in ("sum", "min", "max"):
                    res = float(np.int64(raw).view(np.float64)) if self.is_float else int(raw)
                elif self.kind == "count":
                    res = int(cnt)
                else:
                    res = float(val)
                if self.fused_scalar:
                    value = float(val)
                elif self.fused_layout is not None:
                    tpl = self._template(k)
                    value = Tuple([float(val) if j < 0 else (res if j == self.val_pos else tpl[j])
                                   for j in self.fused_layout])
                else:
                    value = self.result_builder(self._template(k), res, key_obj)
                sub = self._subs.get(k)
                if sub is None:  # subtask of the key (Java hash + murmur): once per key
                    from ..utils.hashing import flink_murmur

                    sub = self._subs[k] = (flink_murmur(java_hash(key_obj)) % MP) * P // MP
                out.append(Rec(value, ts, sub))
        return out

    def process(self, items):
        if self.device_exchange:
            return self._process_exchange(items)
        if self.fallback is not None:
            return self.fallback.process(expand_columns(items))
        out = []
        for it in items:
            if isinstance(it, WM):
                out.extend(self._flush())
                if self.fallback is not None:
                    out.extend(self.fallback.process([it]))
                    continue
                self.wm = it.ts
                if self.op is not None and self.assigner.is_event_time():
                    out.extend(self._emit(self.op.advance_watermark(it.ts)))
                out.append(it)
            else:
                self.pending.append(it)
        out.extend(self._flush())
        return out

    def on_processing_time(self, now):
        if self.fallback is not None:
            return self.fallback.on_processing_time(now)
        if self.device_exchange:
            # collective on every rank and pass: `now` is the step's agreed time
            if self.assigner.is_event_time():
                return []
            return self._emit(self.op.advance_watermark(now))
        out = self._flush()
        if self.op is not None and not self.assigner.is_event_time():
            out.extend(self._emit(self.op.advance_watermark(now)))
        return out

    def finish(self):
        if self.fallback is not None:
            return self.fallback.finish()
        return self._flush()

    def snapshot(self) -> dict:
        """Engine state (key-grouped rows of the pane tables) + the host-side key dictionary and
        keep-first templates; or the exact host operator's state after a fallback."""
        if self.pending:
            raise RuntimeError("snapshot between micro-batches only (records pending)")
        if self.fallback is not None:
            return {"fallback": self.fallback.snapshot()}
        snap = {"wm": self.wm, "late": self.num_late_records_dropped, "str_keys": self.str_keys,
                "templates": dict(self.templates), "strings": list(self.dict.strings()),
                "lazy_arity": getattr(self, "_lazy_arity", None)
                if getattr(self, "_lazy_tpl", None) is not None else None}
        if self.op is not None:
            es = self.op.snapshot_state()
            snap["engine"] = {"columns": es.columns, "meta": es.meta, "is_float": self.is_float}
        return snap

    def restore(self, snap: dict) -> None:
        if "fallback" in snap:
            self._to_fallback()
            self.fallback.restore(snap["fallback"])
            return
        self.wm = snap["wm"]
        self.num_late_records_dropped = snap["late"]
        self.str_keys = snap["str_keys"]
        self.templates = dict(snap["templates"])
        for st in snap["strings"]:
            self.dict.intern(st)
        if snap.get("lazy_arity") is not None:
            self._lazy_tpl, self._lazy_arity = {}, snap["lazy_arity"]
        eng = snap.get("engine")
        if eng is not None:
            self._build(1.0 if eng["is_float"] else 1, dense=bool(self.str_keys))
            self.op.restore_state(eng["columns"], eng["meta"])

    def take_side(self, tag_id):
        if self.fallback is not None:
            return self.fallback.take_side(tag_id)
        return super().take_side(tag_id)


_ = LONG_MAX


class DeviceTemplates:
    """Keep-first template fields of a rolling aggregate's keys on the device (Flink's
    ``max(p)`` keeps the first record's other fields, ComputeCpuMax.java:26): one column per
    output field indexed by dictionary id, plus a `have` mask and each key's output subtask.

    A batch's first occurrence of every key without a template wins (scatter-amin of the row
    index, then masked selects over the table -- no host sync). At G > 1 the table is
    replicated: the winner of a key is the smallest (rank, row) over the ranks (one MIN
    all-reduce of the table's codes), and every field is merged by a SUM all-reduce of the
    winner's value (zeros elsewhere, so the sum is exact) -- the ranks' dictionary ids agree,
    so a key's template is the same row on every rank and the owner of the key finds it."""

    def __init__(self, kinds, key_pos: int, val_pos: int, device, comm):
        self.kinds = tuple(kinds)
        self.key_pos, self.val_pos = key_pos, val_pos
        self.device = device
        self.comm = comm if comm is not None and comm.world > 1 else None
        self.cap = 0
        self.have = None
        self.tpl: dict = {}
        self.sub = None
        self._sub_n = 0

    @staticmethod
    def _dtype(kind):
        return {FK_STR: torch.int32, FK_DOUBLE: torch.float64}.get(kind, torch.int64)

    def _grow(self, need: int) -> None:
        if need <= self.cap:
            return
        cap = max(1024, 1 << max(0, need - 1).bit_length())
        dev = self.device

        def grown(t, dt):
            g = torch.zeros(cap, dtype=dt, device=dev)
            if t is not None:
                g[:t.numel()] = t
            return g
        self.have = grown(self.have, torch.bool)
        for j, k in enumerate(self.kinds):
            if j not in (self.key_pos, self.val_pos):
                self.tpl[j] = grown(self.tpl.get(j), self._dtype(k))
        self.sub = grown(self.sub, torch.int32)
        self.cap = cap

    def _subtasks(self, nkeys: int, jhash, ctx) -> None:
        """Output subtask (Java hash -> murmur -> key group -> subtask) of new dictionary ids."""
        if nkeys <= self._sub_n:
            return
        ids = torch.arange(self._sub_n, nkeys, dtype=torch.int64, device=self.device)
        kg = K.keygroups(ids, max_parallelism=ctx.max_parallelism, hash_mode=1, jhash=jhash)
        P, MP = ctx.parallelism, ctx.max_parallelism
        self.sub[self._sub_n:nkeys] = ((kg.to(torch.int64) * P) // MP).to(torch.int32)
        self._sub_n = nkeys

    def update(self, cb, nkeys: int, jhash, ctx) -> None:
        """Take the templates of keys first seen in batch `cb` (None: no rows on this rank)."""
        self._grow(max(nkeys, 1))
        if jhash is not None:
            self._subtasks(nkeys, jhash, ctx)
        cap, dev = self.cap, self.device
        n = cb.n if cb is not None else 0
        first = torch.full((cap,), 1 << 62, dtype=torch.int64, device=dev)
        if n:
            kid = cb.cols[self.key_pos][:n].to(torch.int64)
            first.scatter_reduce_(0, kid, torch.arange(n, dtype=torch.int64, device=dev),
                                  reduce="amin")
        new = (first < (1 << 62)) & ~self.have
        if self.comm is None:
            if not n:
                return
            idx = torch.where(new, first, torch.zeros_like(first))
            for j, t in self.tpl.items():
                col = cb.cols[j][:n].to(t.dtype)
                self.tpl[j] = torch.where(new, col[idx], t)
            self.have |= new
            return
        # G > 1: the smallest (rank, row) over the ranks wins each new key
        code = torch.where(new, (self.comm.rank << 40) + first,
                           torch.full_like(first, K.I64_MAX))
        self.comm.allreduce_min_(code)
        won = code != K.I64_MAX
        if not bool(won.any()):  # (all ranks agree: the reduced codes are identical)
            return
        mine = won & ((code >> 40) == self.comm.rank)
        idx = torch.where(mine, code & ((1 << 40) - 1), torch.zeros_like(code))
        for j, t in self.tpl.items():
            if n:
                col = cb.cols[j][:n].to(t.dtype)
                part = torch.where(mine, col[idx.clamp(max=n - 1)], torch.zeros_like(t))
            else:
                part = torch.zeros_like(t)
            self.comm.allreduce_sum_(part)
            self.tpl[j] = torch.where(won, part, t)
        self.have |= won

    def rows(self, key: torch.Tensor, val: torch.Tensor) -> list:
        """Output columns of emitted rows (key id, value, templates gathered by key id)."""
        cols = []
        for j in range(len(self.kinds)):
            if j == self.key_pos:
                cols.append(key.to(torch.int32))
            elif j == self.val_pos:
                cols.append(val)
            else:
                cols.append(self.tpl[j][key])
        return cols

    def snapshot(self) -> dict:
        return {"kinds": list(self.kinds), "cap": self.cap,
                "have": None if self.have is None else self.have.cpu().numpy(),
                "tpl": {j: t.cpu().numpy() for j, t in self.tpl.items()}}

    def restore(self, snap: dict) -> None:
        if not snap["cap"]:
            return
        self._grow(int(snap["cap"]))
        n = len(snap["have"])
        self.have[:n] = torch.from_numpy(snap["have"]).to(self.device)
        for j, a in snap["tpl"].items():
            self.tpl[int(j)][:len(a)] = torch.from_numpy(a).to(self.device)
        self._sub_n = 0  # recomputed from the dictionary's Java hashes


class NativeRollingOp(_ColumnInput, Operator):
    """``keyBy(k).sum/min/max(p)`` (StreamGroupedReduce + ComparableAggregator,
    ComputeCpuMax.java:26) on the native ``KeyedRollingOperator``: per micro-batch the records
    are columnarised, the GPU (or C++ twin) returns the post-update value of every record in
    per-key arrival order, and the output tuples are rebuilt from each key's first record with
    field p replaced (Flink's ``max(p)`` keeps the other fields of the first record). Output order
    equals input order. Unsupported data (non-numeric field, mixed types, non-tuple records)
    switches to the exact host RollingReduceOp."""

    name = "Keyed Aggregation"
    accepts_columns = True

    def __init__(self, *, key_fn, key_pos: int, val_pos: int, kind: str, device: str,
                 fallback_factory, max_keys: int = 1 << 20):
        self.key_fn, self.key_pos, self.val_pos, self.kind = key_fn, key_pos, val_pos, kind
        self.device = device
        self.fallback_factory = fallback_factory
        self.max_keys = max_keys
        self.op = None
        self.fallback = None
        self.templates: dict = {}
        self.is_float = None
        self.str_keys = None

    device_input = None  # planner: (column kinds, shared ingest state) of a device-ingest input
    event_ts = True      # planner: the device-ingest rows carry event timestamps

    def open(self, ctx):
        super().open(ctx)
        from ..ops.native import load

        self.dict = load().StringDict()
        self.device_exchange = self.collective = False
        self.dtpl = None  # device keep-first templates (DeviceTemplates), device batches only
        comm = getattr(ctx, "comm", None)
        if comm is not None and comm.world > 1 and self.device_input is not None:
            # Multi-rank with device-ingest input and dictionary keys: the rolling operator
            # partitions by key group and exchanges the records itself (RCCL all-to-all), the
            # keep-first templates are a replicated device table merged by two all-reduces, and
            # the per-record emit stays a device column batch -- nothing is pickled. (Rows with
            # event timestamps keep the executor's exchange: the owner could not stamp them.)
            kinds, shared = self.device_input
            if (kinds[self.key_pos] != FK_STR or kinds[self.val_pos] == FK_STR
                    or len(kinds) <= max(self.key_pos, self.val_pos) or self.event_ts):
                return
            self.dict = shared["dict"]
            self.str_keys = True
            self.comm = comm
            if not self._build(1.0 if kinds[self.val_pos] == FK_DOUBLE else 1):
                return
            self.device_exchange = self.collective = True
            self.dtpl = DeviceTemplates(kinds, self.key_pos, self.val_pos, self.op.device, comm)

    def _to_fallback(self):
        self.fallback = self.fallback_factory()
        self.fallback.open(self.ctx)
        if self.templates or self.dtpl is not None:
            raise RuntimeError("native rolling state cannot be handed to the host operator")

    def _build(self, v) -> bool:
        from .rolling_operator import KeyedRollingOperator

        if isinstance(v, bool) or not isinstance(v, (int, float)):
            return False
        self.is_float = isinstance(v, float)
        agg = {("sum", False): K.AGG_SUM_I64, ("sum", True): K.AGG_SUM_F64,
               ("max", False): K.AGG_MAX_I64, ("max", True): K.AGG_MAX_F64,
               ("min", False): K.AGG_MIN_I64, ("min", True): K.AGG_MIN_F64}[(self.kind, self.is_float)]
        comm = getattr(self, "comm", None)
        multi = comm is not None and comm.world > 1
        self.op = KeyedRollingOperator(agg=agg, device=torch.device(self.device),
                                       max_keys=self.max_keys, comm=comm if multi else None,
                                       parallelism=self.ctx.parallelism if multi else 1,
                                       max_parallelism=self.ctx.max_parallelism if multi else 128,
                                       batch_capacity=1024)
        return True

    def _run_device(self, batches: list) -> list:
        """Device-ingest batches with dictionary keys (G = 1, or every pass at G > 1): keys and
        values go to the engine in place, the post-update value of every record comes back as
        device rows, and the output is ONE device column batch -- key ids, keep-first template
        fields gathered by key id, the value column, the key's subtask -- in arrival order
        ((source rank, row) at G > 1). The print sink formats it natively."""
        dev = self.op.device if self.op is not None else torch.device(self.device)
        cb = concat_device(batches) if batches else None
        n = cb.n if cb is not None else 0
        if cb is not None:
            kid = cb.cols[self.key_pos][:n].to(torch.int64)
            v = cb.cols[self.val_pos][:n]
            vals = v.view(torch.int64) if v.dtype == torch.float64 else v.to(torch.int64)
        else:
            kid = torch.empty(0, dtype=torch.int64, device=dev)
            vals = torch.empty(0, dtype=torch.int64, device=dev)
        self.dtpl.update(cb, len(self.dict), self._jhash_dev(), self.ctx)
        self.op.process(kid.contiguous(), vals.contiguous(), to_host=False)
        k = min(self.op.check(), self.op.out_key.numel())
        if k == 0:
            return []
        tag = self.op.out_tag[:k]
        order = torch.argsort(tag)  # (source rank, row): arrival order
        key = self.op.out_key[:k][order]
        val = self.op.out_val[:k][order]
        ts = None
        if cb is not None and cb.ts is not None and self.comm_world() == 1:
            ts = cb.ts[:n][(tag[order] & 0xFFFFFFFF)]
        cols = self.dtpl.rows(key, val.view(torch.float64) if self.is_float else val)
        return [DeviceColumnBatch(k, cols, self.dtpl.kinds, self.dict, ts,
                                  sub_dev=self.dtpl.sub[key])]

    def comm_world(self) -> int:
        c = getattr(self, "comm", None)
        return c.world if c is not None else 1

    def _jhash_dev(self):
        jh = getattr(self.dict, "id_jh", None)
        return jh

    def _key_id(self, k) -> int:
        if isinstance(k, str):
            if self.str_keys is False:
                raise TypeError("mixed key types")
            self.str_keys = True
            return self.dict.intern(k)
        if isinstance(k, int) and not isinstance(k, bool) and 0 <= k < (1 << 63) - 2:
            if self.str_keys is True:
                raise TypeError("mixed key types")
            self.str_keys = False
            return k
        raise TypeError("unsupported key type for the native path")

    def _device_ok(self, batches: list) -> bool:
        """Device batches of dictionary keys and a numeric value (the device emit path)."""
        if not batches or not all(isinstance(b, DeviceColumnBatch) for b in batches):
            return False
        kinds = batches[0].kinds
        if len(kinds) <= max(self.key_pos, self.val_pos) or kinds[self.key_pos] != FK_STR \
                or kinds[self.val_pos] == FK_STR or self.templates:
            return False
        if self.str_keys is False:
            return False
        return True

    def _run_columns(self, batches: list) -> list:
        """ColumnBatch input: key/value columns straight to the engine; the output (one row per
        input record, Flink's rolling emit) is built per row only for the host sink."""
        if self._device_ok(batches):
            b0 = batches[0]
            if b0.strings is not self.dict:
                if len(self.dict) and self.dtpl is None:
                    batches = [b.host() for b in batches]
                    return self._run_columns(batches)
                self.dict = b0.strings
            self.str_keys = True
            vk = b0.kinds[self.val_pos]
            if self.op is None and not self._build(1.0 if vk == FK_DOUBLE else 1):
                raise TypeError("unsupported value")
            if (vk == FK_DOUBLE) != self.is_float:
                raise TypeError("mixed value types")
            if self.dtpl is None:
                self.dtpl = DeviceTemplates(b0.kinds, self.key_pos, self.val_pos, self.op.device,
                                            None)
            return self._run_device(batches)
        # One output row per input record goes to a host sink anyway: device batches come over.
        batches = [b.host() if isinstance(b, DeviceColumnBatch) else b for b in batches]
        try:
            cb = self._cb_concat(batches)
            vk = cb.kinds[self.val_pos]
            if vk == FK_STR or len(cb.kinds) <= max(self.key_pos, self.val_pos):
                raise TypeError("value column not numeric")
            if self.op is None:
                if not self._build(1.0 if vk == FK_DOUBLE else 1):
                    raise TypeError("unsupported value")
            elif (vk == FK_DOUBLE) != self.is_float:
                raise TypeError("mixed value types")
            kid = self._cb_keys(cb)
        except TypeError:
            if self.templates:
                raise
            recs = expand_columns(batches)
            self._to_fallback()
            return self.fallback.process(recs)
        self._cb_templates(cb, kid)
        vv = cb.cols[self.val_pos].astype(np.float64 if self.is_float else np.int64, copy=False)
        dev = self.op.device
        rows = self.op.process(torch.from_numpy(np.ascontiguousarray(kid, dtype=np.int64)).to(dev),
                               torch.from_numpy(np.ascontiguousarray(vv).view(np.int64)).to(dev))
        ts = cb.ts.tolist() if cb.ts is not None else None
        return self._rows_out(rows, (lambda i: ts[i]) if ts is not None else (lambda i: LONG_MIN))

    def _result(self, raw: int):
        return float(np.int64(raw).view(np.float64)) if self.is_float else raw

    def _value(self, k: int, res):
        from ..api.tuples import Tuple

        row = list(self.templates[k])
        row[self.val_pos] = res
        return Tuple(row)

    def _out_ts(self, ts: int) -> int:
        return ts

    def _rows_out(self, rows, ts_of) -> list:
        """Engine rows -> output records in input order (by arrival tag)."""
        from ..utils.hashing import flink_murmur

        order = np.argsort(rows.tags & 0xFFFFFFFF, kind="stable")  # back to input order
        P, MP = self.ctx.parallelism, self.ctx.max_parallelism
        keys = rows.keys[order].tolist()
        raws = rows.values[order].tolist()
        idx = (rows.tags[order] & 0xFFFFFFFF).tolist()
        subs: dict = {}
        out = []
        for k, raw, i in zip(keys, raws, idx):
            sub = subs.get(k)
            if sub is None:
                key_obj = self.dict.get(k) if self.str_keys else k
                sub = subs[k] = (flink_murmur(java_hash(key_obj)) % MP) * P // MP
            out.append(Rec(self._value(k, self._result(raw)), self._out_ts(ts_of(i)), sub))
        return out

    def _run(self, recs: list) -> list:
        if not recs:
            return []
        if all(isinstance(r, ColumnBatch) for r in recs):
            return self._run_columns(recs)
        recs = expand_columns(recs)
        if self.op is None:
            v0 = recs[0].value
            if not isinstance(v0, tuple) or len(v0) <= max(self.key_pos, self.val_pos) \
                    or not self._build(v0[self.val_pos]):
                self._to_fallback()
                return self.fallback.process(recs)
        n = len(recs)
        try:
            kid = np.empty(n, dtype=np.int64)
            vv = np.empty(n, dtype=np.float64 if self.is_float else np.int64)
            ar = len(recs[0].value)
            for i, r in enumerate(recs):
                v = r.value
                if not isinstance(v, tuple) or len(v) != ar:
                    raise TypeError("record shape")
                k = self._key_id(v[self.key_pos])
                kid[i] = k
                if k not in self.templates:
                    self.templates[k] = v
                x = v[self.val_pos]
                if isinstance(x, bool) or isinstance(x, float) != self.is_float or \
                        not isinstance(x, (int, float)):
                    raise TypeError("mixed value types")
                vv[i] = x
        except TypeError:
            if self.templates:
                raise
            self._to_fallback()
            return self.fallback.process(recs)
        dev = self.op.device
        rows = self.op.process(torch.from_numpy(kid).to(dev),
                               torch.from_numpy(vv.view(np.int64)).to(dev))
        return self._rows_out(rows, lambda i: recs[i].ts)

    def process(self, items):
        if self.fallback is not None:
            return self.fallback.process(expand_columns(items))
        if self.device_exchange:
            # one collective engine step per pass (empty if this rank got no rows)
            data = [it for it in items if not isinstance(it, WM)]
            if any(not isinstance(b, DeviceColumnBatch) for b in data):
                raise TypeError("multi-rank native rolling: device-ingest batches expected")
            return self._run_device(data) + [it for it in items if isinstance(it, WM)]
        out, pending = [], []
        for it in items:
            if isinstance(it, WM):
                out.extend(self._run(pending))
                pending = []
                out.append(it)
            else:
                pending.append(it)
        out.extend(self._run(pending))
        return out

    def snapshot(self) -> dict:
        if self.fallback is not None:
            return {"fallback": self.fallback.snapshot()}
        snap = {"templates": dict(self.templates), "strings": list(self.dict.strings()),
                "str_keys": self.str_keys, "is_float": self.is_float}
        if self.op is not None:
            es = self.op.snapshot_state()
            snap["engine"] = {"columns": es.columns, "meta": es.meta}
        if self.dtpl is not None:
            snap["device_templates"] = self.dtpl.snapshot()
        return snap

    def restore(self, snap: dict) -> None:
        if "fallback" in snap:
            self.fallback = self.fallback_factory()
            self.fallback.open(self.ctx)
            self.fallback.restore(snap["fallback"])
            return
        self.templates = dict(snap["templates"])
        self.str_keys = snap["str_keys"]
        for st in snap["strings"]:
            self.dict.intern(st)
        if "engine" in snap and self.op is None:
            self._build(1.0 if snap["is_float"] else 1)
        if "engine" in snap:
            self.op.restore_state(snap["engine"]["columns"], snap["engine"]["meta"])
        dt = snap.get("device_templates")
        if dt is not None:
            if self.dtpl is None:
                self.dtpl = DeviceTemplates(tuple(dt["kinds"]), self.key_pos, self.val_pos,
                                            self.op.device, None)
            self.dtpl.restore(dt)


class NativeCountWindowOp(NativeRollingOp):
    """``keyBy(k).countWindow(n)`` with an incremental sum/min/max/reduce or (count, sum) average
    (GlobalWindows + PurgingTrigger(CountTrigger(n)); countWindow in chapter2/README.md:78 and
    chapter3/README.md:4) on the native ``KeyedRollingOperator`` in count-window mode: the
    segmented wave scan emits one row per completed window, in input order of the completing
    elements, with the GlobalWindow's timestamp (Long.MAX_VALUE). Only lowered when the fields
    other than key and value are dead downstream (planner), like the time windows."""

    name = "Window(native count)"

    def __init__(self, *, count: int, result_builder, ok_arities=None, **kw):
        super().__init__(**kw)
        self.count = int(count)
        self.result_builder = result_builder
        self.ok_arities = ok_arities

    def _build(self, v) -> bool:
        from .rolling_operator import KeyedRollingOperator

        if isinstance(v, bool) or not isinstance(v, (int, float)):
            return False
        self.is_float = isinstance(v, float)
        agg = {("sum", False): K.AGG_SUM_I64, ("sum", True): K.AGG_SUM_F64,
               ("max", False): K.AGG_MAX_I64, ("max", True): K.AGG_MAX_F64,
               ("min", False): K.AGG_MIN_I64, ("min", True): K.AGG_MIN_F64,
               ("count", False): K.AGG_COUNT, ("count", True): K.AGG_COUNT,
               ("avg", False): K.AGG_AVG_I64, ("avg", True): K.AGG_AVG_F64}[(self.kind, self.is_float)]
        self.op = KeyedRollingOperator(agg=agg, device=torch.device(self.device),
                                       max_keys=self.max_keys, parallelism=1,
                                       batch_capacity=1024, count_window=self.count)
        return True

    def _result(self, raw: int):
        if self.kind == "count":
            return int(raw)
        if self.kind == "avg":
            s = float(np.int64(raw).view(np.float64)) if self.is_float else float(raw)
            return s / self.count
        return super()._result(raw)

    def _value(self, k: int, res):
        key_obj = self.dict.get(k) if self.str_keys else k
        return self.result_builder(self.templates[k], res, key_obj)

    def _out_ts(self, ts: int) -> int:
        return LONG_MAX  # GlobalWindow.maxTimestamp()

    def _run_columns(self, batches: list) -> list:
        if self.ok_arities and self.op is None and len(batches[0].kinds) not in self.ok_arities:
            self._to_fallback()
            return self.fallback.process(expand_columns(batches))
        return super()._run_columns(batches)

    def _run(self, recs: list) -> list:
        if recs and self.ok_arities and self.op is None:
            v0 = expand_columns(recs[:1])[0].value if not isinstance(recs[0], ColumnBatch) else None
            if v0 is not None and (not isinstance(v0, tuple) or len(v0) not in self.ok_arities):
                self._to_fallback()
                return self.fallback.process(expand_columns(recs))
        return super()._run(recs)


class NativeSessionOp(NativeWindowOp):
    """``window(EventTimeSessionWindows.withGap(g))`` with a field-wise aggregate on the native
    ``KeyedSessionOperator`` (GPU slot table + host store, or the C++ store on CPU). Results are
    emitted at the session's maxTimestamp like Flink's WindowOperator."""

    _key32_ok = False

    def _build(self, sample_val, dense: bool = False) -> bool:
        from .session_operator import KeyedSessionOperator

        is_float = isinstance(sample_val, float)
        if not isinstance(sample_val, (int, float)) or isinstance(sample_val, bool):
            return False
        agg = {("sum", False): K.AGG_SUM_I64, ("sum", True): K.AGG_SUM_F64,
               ("min", False): K.AGG_MIN_I64, ("min", True): K.AGG_MIN_F64,
               ("max", False): K.AGG_MAX_I64, ("max", True): K.AGG_MAX_F64,
               ("count", False): K.AGG_COUNT, ("count", True): K.AGG_COUNT,
               ("avg", False): K.AGG_AVG_I64, ("avg", True): K.AGG_AVG_F64}[(self.kind, is_float)]
        self.is_float = is_float
        comm = getattr(self, "comm", None)
        multi = comm is not None and comm.world > 1
        # G > 1: the session operator partitions by key group and exchanges its records itself
        # (RCCL all-to-all inside process()); firing is local to each key's owner.
        self.op = KeyedSessionOperator(gap=self.assigner.gap, lateness=self.lateness, agg=agg,
                                       device=torch.device(self.device), max_keys=self.max_keys,
                                       comm=comm if multi else None,
                                       parallelism=self.ctx.parallelism if multi else 1,
                                       max_parallelism=self.ctx.max_parallelism if multi else 128,
                                       batch_capacity=max(1024, self.ctx.parallelism),
                                       external_watermark=True)
        return True

    def _result_column(self, raw: np.ndarray, values: np.ndarray, counts: np.ndarray):
        """(column, kind) of the window result of fired rows."""
        if self.kind in ("sum", "min", "max"):
            r = raw.view(np.int64) if raw.dtype == np.uint64 else raw.astype(np.int64)
            return (r.view(np.float64), FK_DOUBLE) if self.is_float else (r, FK_LONG)
        if self.kind == "count":
            return counts.astype(np.int64), FK_LONG
        return values.astype(np.float64, copy=False), FK_DOUBLE

    def _emit(self, rows) -> list:
        if not len(rows):
            return []
        if self.scalar_result:
            col, k = self._result_column(np.asarray(rows.raw), np.asarray(rows.values),
                                         np.asarray(rows.counts))
            keys = np.asarray(rows.keys)
            keys = keys.view(np.int64) if keys.dtype == np.uint64 else keys.astype(np.int64)
            return [ColumnBatch(int(keys.size), [col], (k,), None,
                                np.asarray(rows.end, dtype=np.int64) - 1, self._subtasks(keys),
                                True)]
        out = []
        P, MP = self.ctx.parallelism, self.ctx.max_parallelism
        from ..utils.hashing import flink_murmur

        for k, end, val, raw, cnt in zip(rows.keys.tolist(), rows.end.tolist(),
                                         rows.values.tolist(), rows.raw.tolist(),
                                         rows.counts.tolist()):
            key_obj = self.dict.get(k) if self.str_keys else k
            if self.kind in ("sum", "min", "max"):
                res = float(np.int64(raw).view(np.float64)) if self.is_float else int(raw)
            elif self.kind == "count":
                res = int(cnt)
            else:
                res = float(val)
            value = self.result_builder(self._template(k), res, key_obj)
            sub = (flink_murmur(java_hash(key_obj)) % MP) * P // MP
            out.append(Rec(value, end - 1, sub))
        return out


class NativeMedianOp(NativeWindowOp):
    """``process(<median>)`` windows (ComputeCpuMiddle.java:34-48) on the device list-window
    operator (runtime/list_window_operator.py): elements stay in a device pane arena, a firing
    counting-sorts the window by key id and a kernel selects each key's median.
    Checkpoints carry the live panes' elements (NativeWindowOp.snapshot -> snapshot_state)."""

    _key32_ok = False

    def _build(self, sample_val, dense: bool = False) -> bool:
        from .list_window_operator import KeyedListWindowOperator

        if not isinstance(sample_val, float):
            return False  # the reference's values are Double; anything else: host operator
        self.is_float = True
        a = self.assigner
        self.op = KeyedListWindowOperator(
            size=a.size, slide=a.slide, offset=a.offset,
            lateness=self.lateness if a.is_event_time() else 0, device=torch.device(self.device),
            time_mode="event" if a.is_event_time() else "processing")
        comm = getattr(self, "comm", None)
        if comm is not None and comm.world > 1:
            # G > 1: the pane arena holds this rank's key groups; records reach their owner by
            # one row all-to-all per pass (parallel/exchange.py), firing is local
            P, MP = self.ctx.parallelism, self.ctx.max_parallelism
            kgd = [((kg * P // MP) * comm.world) // P for kg in range(MP)]
            self._kg_dest = torch.tensor(kgd, dtype=torch.int64, device=torch.device(self.device))
        return True

    def _process_exchange(self, items) -> list:
        """G > 1: this rank's (key id, ts, value) rows to the owners of their key groups, the
        owner's pane arena folds them; the merged watermark fires each rank's own keys."""
        from ..parallel.exchange import exchange_rows

        data = [it for it in items if not isinstance(it, WM)]
        wms = [it.ts for it in items if isinstance(it, WM)]
        kid, ts, vals = self._local_columns(data)
        kid = kid.to(torch.int64)
        kg = K.keygroups(kid, max_parallelism=self.ctx.max_parallelism,
                         hash_mode=1 if self.str_keys else 0,
                         jhash=self._jhash() if self.str_keys else None)
        kid, ts, vals = exchange_rows(self.comm, self._kg_dest[kg.to(torch.int64)],
                                      [kid, ts, vals])
        late_before = self.op.metrics.num_late_records_dropped
        out = self._emit(self.op.process(kid, ts, vals)) if kid.numel() else []
        self.num_late_records_dropped += self.op.metrics.num_late_records_dropped - late_before
        event = self.assigner.is_event_time()
        for w in wms:
            self.wm = w
            if event:
                out.extend(self._emit(self.op.advance_watermark(w)))
            out.append(WM(w))
        return out

    def _emit(self, fired) -> list:
        fired = [f for f in fired if len(f[2])]
        if not fired:
            return []
        if self.scalar_result:
            keys = np.concatenate([np.asarray(f[2]) for f in fired]).astype(np.int64)
            med = np.concatenate([np.asarray(f[3]) for f in fired]).astype(np.float64)
            ts = np.repeat(np.array([f[1] - 1 for f in fired], dtype=np.int64),
                           [len(f[2]) for f in fired])
            return [ColumnBatch(int(keys.size), [med], (FK_DOUBLE,), None, ts,
                                self._subtasks(keys), True)]
        out = []
        P, MP = self.ctx.parallelism, self.ctx.max_parallelism
        from ..utils.hashing import flink_murmur

        for s, e, keys, med in fired:
            for k, v in zip(keys.tolist(), med.tolist()):
                key_obj = self.dict.get(k) if self.str_keys else k
                value = self.result_builder(self._template(k), float(v), key_obj)
                sub = (flink_murmur(java_hash(key_obj)) % MP) * P // MP
                out.append(Rec(value, e - 1, sub))
        return out


class NativeVectorWindowOp(NativeWindowOp):
    """``timeWindow(..).aggregate(VectorSumAggregate / VectorAvgAggregate(field))``: per-key
    element-wise sum / average of a metric-vector field on the native vector-window operator
    (runtime/vector_window_operator.py: MFMA segmented sums on the GPU, C++ twin on the CPU).
    Vectors are zero-padded to the kernel width (a multiple of 32); results are cut back to the
    input length. Windows and watermarks behave exactly as in NativeWindowOp."""

    name = "VectorWindow(native)"
    _exchange_ok = False  # no device ingest of vectors: the host-record exchange below instead

    def open(self, ctx):
        super().open(ctx)
        comm = getattr(ctx, "comm", None)
        if comm is not None and comm.world > 1 and self.scalar_result and self.late_tag is None:
            # G > 1: the operator takes this rank's records as they are and moves (key id, ts,
            # row) records plus their vectors to the key's owner inside VectorWindowOperator's
            # all-to-all (RCCL). Only the pass's NEW key strings travel as objects, so every
            # rank interns them in the same order and the ids agree (the key groups come from
            # the ids' Java hashes). The result is the aggregate alone (no keep-first
            # template), so the owner needs nothing else from the record's source rank.
            self.comm = comm
            self.device_exchange = self.collective = True
            self._vknown: set = set()  # key strings interned (identically on every rank)

    def _process_exchange(self, items) -> list:
        """One collective step per pass: agree on new keys and the vector length, then the
        engine step (records and vectors exchanged inside), then the merged watermark."""
        recs = [r for r in expand_columns([it for it in items if not isinstance(it, WM)])
                if isinstance(r, Rec)]
        wms = [it.ts for it in items if isinstance(it, WM)]
        err, new, seen_new, vlen, kind = None, [], set(), None, None
        try:
            for r in recs:
                v = r.value
                if not isinstance(v, tuple) or (self.ok_arities and len(v) not in self.ok_arities):
                    raise TypeError("vector window input must be a tuple")
                k, x = v[self.key_pos], v[self.val_pos]
                if not isinstance(x, (list, tuple)):
                    raise TypeError("metric vector field must be a list")
                vlen = len(x) if vlen is None else vlen
                if isinstance(k, str):
                    kind = kind or "str"
                    if k not in seen_new and k not in self._vknown:
                        seen_new.add(k)
                        new.append(k)
                elif isinstance(k, int) and not isinstance(k, bool) and 0 <= k < (1 << 63) - 1:
                    kind = kind or "int"
                else:
                    raise TypeError("unsupported key type for the native path")
        except TypeError as e:
            err = str(e)
        # Steady state (no new key string, no error, the known vector length and key kind on
        # every rank): one packed int64 all-reduce; the object gather runs only otherwise.
        from ..parallel.comm import control_reduce

        kc = {"str": 1, "int": 2}.get(kind, 0)
        vl = -1 if vlen is None else vlen
        (vmin, kmin), (nnew, bad, vmax, kmax) = control_reduce(
            self.comm, mins=[vl if vl >= 0 else (1 << 62), kc or 3],
            maxs=[len(new), int(err is not None), vl, kc])
        known_k = None if self.str_keys is None else (1 if self.str_keys else 2)
        quiet = (nnew == 0 and not bad and getattr(self, "_vjh_t", None) is not None
                 and (vmax < 0 or (self.op is not None and vmin == vmax == self.vlen))
                 and (kmax == 0 or (kmin == kmax == known_k)))
        if quiet:
            got = [([], None, None, None)]
        else:
            got = self.comm.all_gather_object((new, vlen, kind, err))
        errs = [e for *_, e in got if e]
        if errs:
            raise TypeError(f"native vector window at G > 1: {errs[0]}")
        kinds = {k for _, _, k, _ in got if k} | ({"str" if self.str_keys else "int"}
                                                 if self.str_keys is not None else set())
        if len(kinds) > 1:
            raise TypeError("mixed key types")
        if kinds:
            self.str_keys = kinds.pop() == "str"
        lens = {n for _, n, _, _ in got if n is not None}
        if self.op is not None:
            lens.add(self.vlen)
        if len(lens) > 1:
            raise TypeError("metric vectors must all have the first vector's length")
        grew = False
        for strs, *_ in got:  # rank order: identical interning on every rank
            for st in strs:
                if st not in self._vknown:
                    self._vknown.add(st)
                    self.dict.intern(st)
                    grew = True
        if grew or getattr(self, "_vjh_t", None) is None:
            self._vjh_t = torch.from_numpy(self.dict.jhash_table())
        if self.op is None and lens:
            if not self._build([0.0] * lens.pop()):
                raise TypeError("metric vectors wider than the kernel")
        out = []
        if self.op is not None:
            if self.str_keys:
                self.op.jhash = self._vjh_t.to(self.op.device)
            n, dim = len(recs), self.op.dim
            kid = np.empty(n, dtype=np.int64)
            tsa = np.empty(n, dtype=np.int64)
            vv = np.zeros((n, dim), dtype=np.float32)
            event = self.assigner.is_event_time()
            now = self.ctx.clock()
            for i, r in enumerate(recs):
                v = r.value
                k = v[self.key_pos]
                kid[i] = self.dict.intern(k) if self.str_keys else k  # agreed id
                tsa[i] = r.ts if event else now
                vv[i, :self.vlen] = v[self.val_pos]
            dev = self.op.device
            late_before = self.op.metrics.num_late_records_dropped
            out = self._emit(self.op.process(torch.from_numpy(kid).to(dev),
                                             torch.from_numpy(tsa).to(dev),
                                             torch.from_numpy(vv).to(dev)))
            self.num_late_records_dropped += self.op.metrics.num_late_records_dropped - late_before
        for w in wms:
            self.wm = w
            if self.op is not None and self.assigner.is_event_time():
                out.extend(self._emit(self.op.advance_watermark(w)))
            out.append(WM(w))
        return out

    def on_processing_time(self, now):
        if self.device_exchange and self.op is None:
            return []  # collective: no rank has built the operator yet (agreed in the pass)
        return super().on_processing_time(now)

    def _build(self, sample_val, dense: bool = False) -> bool:
        if not isinstance(sample_val, (list, tuple)) or not sample_val \
                or not all(isinstance(x, (int, float)) and not isinstance(x, bool)
                           for x in sample_val):
            return False
        from .vector_window_operator import VectorWindowOperator

        self.vlen = len(sample_val)
        self.is_float = True
        dim = max(32, -(-self.vlen // 32) * 32)
        if dim > 256:
            return False
        a = self.assigner
        event = a.is_event_time()
        comm = getattr(self, "comm", None)
        multi = comm is not None and comm.world > 1
        self.op = VectorWindowOperator(
            dim=dim, avg=self.kind == "vavg", size=a.size, slide=a.slide, offset=a.offset,
            lateness=self.lateness if event else 0, device=torch.device(self.device),
            max_keys=self.max_keys, parallelism=self.ctx.parallelism if multi else 1,
            comm=comm if multi else None,
            max_parallelism=self.ctx.max_parallelism if multi else 128,
            hash_mode=1 if (multi and self.str_keys) else 0,
            jhash_table=self._vjh_t if (multi and self.str_keys) else None,
            batch_capacity=max(1024, self.ctx.parallelism),
            cap_log2=9, time_mode="event" if event else "processing", external_watermark=True,
            side_output_late=self.late_tag is not None, clock=self.ctx.clock)
        return True

    def _flush(self) -> list:
        recs = expand_columns(self.pending)
        self.pending = []
        if not recs:
            return []
        if self.op is None:
            v0 = recs[0].value
            if (not isinstance(v0, tuple) or (self.ok_arities and len(v0) not in self.ok_arities)
                    or not self._build(v0[self.val_pos])):
                self._to_fallback()
                return self.fallback.process(recs)
        n = len(recs)
        dim = self.op.dim
        try:
            kid = np.empty(n, dtype=np.int64)
            tsa = np.empty(n, dtype=np.int64)
            vv = np.zeros((n, dim), dtype=np.float32)
            now = self.ctx.clock()
            event = self.assigner.is_event_time()
            for i, r in enumerate(recs):
                v = r.value
                k = self._key_id(v[self.key_pos])
                kid[i] = k
                if k not in self.templates:
                    self.templates[k] = v
                tsa[i] = r.ts if event else now
                x = v[self.val_pos]
                if not isinstance(x, (list, tuple)) or len(x) != self.vlen:
                    raise TypeError("metric vectors must all have the first vector's length")
                vv[i, :self.vlen] = x
        except (TypeError, ValueError):
            self._to_fallback()
            return self.fallback.process(recs)
        dev = self.op.device
        fired = self.op.process(torch.from_numpy(kid).to(dev), torch.from_numpy(tsa).to(dev),
                                torch.from_numpy(vv).to(dev))
        if self.op.late_side:
            for idx in np.concatenate(self.op.late_side).tolist():
                r = recs[idx]
                self.side.setdefault(self.late_tag.tag_id, []).append(Rec(r.value, r.ts, r.subtask))
            self.op.late_side.clear()
        return self._emit(fired)

    def _emit(self, fired) -> list:
        from ..utils.hashing import flink_murmur

        out = []
        P, MP = self.ctx.parallelism, self.ctx.max_parallelism
        for fr in fired:
            ts = fr.window_end - 1
            for k, vec in zip(fr.keys.tolist(), fr.values):
                key_obj = self.dict.get(k) if self.str_keys else k
                res = [float(x) for x in vec[:self.vlen]]
                # a bare aggregate result reads no template (none exists off the source rank)
                tpl = None if self.scalar_result else self._template(k)
                value = self.result_builder(tpl, res, key_obj)
                sub = (flink_murmur(java_hash(key_obj)) % MP) * P // MP
                out.append(Rec(value, ts, sub))
        return out

    def snapshot(self) -> dict:
        snap = super().snapshot()
        if "engine" in snap:
            snap["engine"]["vlen"] = self.vlen
        return snap

    def restore(self, snap: dict) -> None:
        eng = snap.get("engine")
        if eng is None or "fallback" in snap:
            return super().restore(snap)
        self.wm = snap["wm"]
        self.num_late_records_dropped = snap["late"]
        self.str_keys = snap["str_keys"]
        self.templates = dict(snap["templates"])
        for st in snap["strings"]:
            self.dict.intern(st)
        if self.device_exchange:
            self._vknown.update(snap["strings"])
            self._vjh_t = torch.from_numpy(self.dict.jhash_table())
        self._build([0.0] * eng["vlen"])
        self.op.restore_state(eng["columns"], eng["meta"])

"""print() rows of a device column batch formatted on the device (csrc/row_format.h,
csrc/format_hip.hip; the C++ twin on the CPU).

A keyed operator's columnar emit stays on the device up to its text: one lane per row computes
the row's length (subtask prefix, Tuple.toString, String / Long / Double.toString fields --
strings straight from the device dictionary's arena), a device scan gives every row its offset,
a workgroup per 256 rows writes them through LDS with 16-byte stores, and ONE copy moves the
finished bytes to pinned host memory. A batch with a value the device cannot format exactly
(a double needing more than 15 significant digits or scientific notation) is reported and the
caller formats it on the host (PrintSinkOp's host path).
"""
from __future__ import annotations

import numpy as np
import torch

from .native import load
from .text import FK_DOUBLE, FK_INT, FK_LONG, FK_STR


class RowFormatter:
    """Per-sink buffers of the device formatter (device output, pinned host copy, prefixes)."""

    def __init__(self):
        self._m = load()
        self._out = None
        self._pin = None
        self._pfx_key = None
        self._pfx = None

    def _prefix_table(self, prefixes: list[str], dev):
        key = (tuple(prefixes), str(dev))
        if self._pfx_key != key:
            enc = [p.encode() for p in prefixes]
            off = np.zeros(len(enc) + 1, dtype=np.int32)
            off[1:] = np.cumsum([len(b) for b in enc])
            raw = np.frombuffer(b"".join(enc) or b"\0", dtype=np.uint8)
            self._pfx = (torch.from_numpy(raw.copy()).to(dev), torch.from_numpy(off).to(dev))
            self._pfx_key = key
        return self._pfx

    def format(self, cb, prefixes: list[str], as_tuple: bool):
        """The rows of DeviceColumnBatch `cb` as Java prints them (a memoryview valid until the
        next call), or None when the batch needs the host formatter."""
        n = cb.n
        if getattr(cb, "_parts", None):  # a concatenation: subtasks live in the parts
            return None
        if n == 0 or not cb.cols or len(cb.cols) > 8 or (not as_tuple and len(cb.cols) != 1):
            return None
        dev = cb.cols[0].device
        gpu = dev.type == "cuda"
        cols, keep = [], []
        for c, k in zip(cb.cols, cb.kinds):
            if c.device != dev:
                return None
            c = c[:n].contiguous()
            if k == FK_STR and c.dtype in (torch.int32, torch.int64):
                cols.append((0, c.element_size(), c.data_ptr()))
            elif k == FK_DOUBLE and c.dtype == torch.float64:
                cols.append((1, 8, c.data_ptr()))
            elif k in (FK_LONG, FK_INT) and c.dtype in (torch.int32, torch.int64):
                cols.append((2, c.element_size(), c.data_ptr()))
            else:
                return None
            keep.append(c)
        d = {"cols": cols, "as_tuple": bool(as_tuple), "arena": 0, "id_off": 0, "id_len": 0,
             "n_ids": 0, "sub": 0, "sub0": 0, "par": 1, "npfx": 0, "pfx": 0, "pfx_off": 0}
        if FK_STR in cb.kinds:
            s = cb.strings
            arena = getattr(s, "arena", None)
            if arena is None or arena.device != dev:
                return None
            d.update(arena=arena.data_ptr(), id_off=s.id_off.data_ptr(),
                     id_len=s.id_len.data_ptr(), n_ids=int(s.n_ids))
        if any(prefixes):
            pfx, off = self._prefix_table(prefixes, dev)
            d.update(npfx=len(prefixes), pfx=pfx.data_ptr(), pfx_off=off.data_ptr())
            if cb.sub_dev is not None:
                sub = cb.sub_dev[:n].to(torch.int32).contiguous()
            elif cb.line_idx is not None:
                sub = ((cb.line_idx[:n].to(torch.int64) + cb.sub0)
                       % max(1, cb.parallelism)).to(torch.int32)
            else:
                sub = None
                d.update(sub0=int(cb.sub0), par=max(1, int(cb.parallelism)))
            if sub is not None:
                keep.append(sub)
                d["sub"] = sub.data_ptr()
        st = torch.cuda.current_stream(dev).cuda_stream if gpu else 0
        ln = torch.empty(n, dtype=torch.int64, device=dev)
        bad = torch.zeros(1, dtype=torch.int32, device=dev)
        self._m.format_rows_len(gpu, d, n, ln.data_ptr(), bad.data_ptr(), st)
        end = torch.cumsum(ln, 0)
        total, flag = torch.stack([end[-1], bad[0].to(torch.int64)]).tolist()
        if flag:
            return None
        if self._out is None or self._out.numel() < total or self._out.device != dev:
            self._out = torch.empty(max(total, 1 << 16) * 5 // 4, dtype=torch.uint8, device=dev)
        self._m.format_rows_write(gpu, d, n, end.data_ptr(), self._out.data_ptr(), st)
        if not gpu:
            return memoryview(self._out.numpy())[:total]
        if self._pin is None or self._pin.numel() < total:
            self._pin = torch.empty(max(total, 1 << 16) * 5 // 4, dtype=torch.uint8,
                                    pin_memory=True)
        self._pin[:total].copy_(self._out[:total], non_blocking=True)
        torch.cuda.current_stream(dev).synchronize()
        del keep
        return memoryview(self._pin.numpy())[:total]

"""Keyed windows that need every element (``process`` windows: ComputeCpuMiddle.java:34-48).

Flink keeps a ListState per (key, window) and hands the full Iterable to the ProcessWindowFunction.
Here the elements of each pane (pane = gcd(size, slide)) stay on the device as columns
(key id, value bits); when a window fires its panes are concatenated, radix-sorted by
(key, order-preserving value bits) -- two stable passes, value first -- and reduced per key
segment by a kernel (median: csrc/kernels_hip.hip ``segment_median``). Late data
within the allowed lateness re-fires the touched windows, like the pane operator.

Runs on one device (the DataStream API's logical subtasks map onto it); the all-to-all path of the
pane operator is not needed for the reference's process-window job.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..ops import kernels as K
from .window_operator import OperatorMetrics, java_window_start

I64_MIN, I64_MAX = K.I64_MIN, K.I64_MAX


class KeyedListWindowOperator:
    def __init__(self, *, size: int, slide: int | None = None, offset: int = 0,
                 lateness: int = 0, device="cpu", time_mode: str = "event", func: str = "median"):
        slide = size if slide is None else slide
        if func != "median":
            raise ValueError("supported list-window functions: median")
        self.size, self.slide, self.offset, self.lateness = int(size), int(slide), int(offset), int(lateness)
        self.pane = math.gcd(self.size, self.slide)
        self.device = K.resolve_device(device)
        self.time_mode = time_mode
        self.wm = I64_MIN
        self.panes: dict[int, list[tuple[torch.Tensor, torch.Tensor]]] = {}
        self.next_fire_start: int | None = None
        self.metrics = OperatorMetrics()
        self.late_side: list = []

    def _pane_of(self, t):
        return (t - self.offset) // self.pane

    def _late_ts(self) -> int:
        if self.wm == I64_MIN or self.time_mode != "event":
            return I64_MIN
        s = self._align_up(self.wm - self.size - self.lateness + 2)
        return s

    def _align_up(self, t: int) -> int:
        ls = java_window_start(t, self.offset, self.slide)
        return ls if ls >= t else ls + self.slide

    def process(self, keys: torch.Tensor, ts: torch.Tensor, vals_f64: torch.Tensor) -> list:
        """keys int64 (or int32 dictionary ids), ts int64, vals: f64 bit patterns (int64).
        Returns fired rows."""
        out = []
        keys = keys.to(torch.int64)
        if keys.numel():
            late_ts = self._late_ts()
            keep = ts >= late_ts
            self.metrics.num_late_records_dropped += int((~keep).sum().item())
            keys, ts, vals_f64 = keys[keep], ts[keep], vals_f64[keep]
        if keys.numel():
            panes = torch.div(ts - self.offset, self.pane, rounding_mode="floor")
            pu = torch.unique(panes).tolist()
            for p in pu:
                sel = panes == p
                self.panes.setdefault(int(p), []).append((keys[sel], vals_f64[sel]))
            first = self._first_start_containing(self.offset + min(pu) * self.pane)
            if self.wm > I64_MIN:
                first = max(first, self._align_up(self.wm - self.size + 2))
            self.next_fire_start = first if self.next_fire_start is None else min(self.next_fire_start, first)
            # Late-but-allowed data: re-fire, for the keys that received it, the windows that
            # already fired and contain those panes (EventTimeTrigger.onElement per key).
            if self.wm > I64_MIN:
                for p in pu:
                    touched = torch.unique(keys[panes == p])
                    s = self._first_start_containing(self.offset + p * self.pane)
                    while s <= self.offset + p * self.pane:
                        if s + self.size - 1 <= self.wm < s + self.size - 1 + self.lateness:
                            out += self._fire_window(s, only_keys=touched)
                        s += self.slide
        return out

    def _first_start_containing(self, t: int) -> int:
        ls = java_window_start(t, self.offset, self.slide)
        return ls - ((ls - (t - self.size + 1)) // self.slide) * self.slide

    def advance_watermark(self, wm: int) -> list:
        if wm <= self.wm:
            return []
        self.wm = wm
        out = []
        if self.next_fire_start is not None:
            s = self.next_fire_start
            # Windows after the last pane hold no data: never iterate past it (wm may be MAX).
            last_pane = max(self.panes) if self.panes else None
            while s + self.size - 1 <= wm and last_pane is not None \
                    and self._pane_of(s) <= last_pane:
                out += self._fire_window(s)
                s += self.slide
            if s + self.size - 1 <= wm:  # caught up: resume at the first window not yet due
                s = self._align_up(wm - self.size + 2) if wm < I64_MAX - self.size else s
            self.next_fire_start = s
        self._purge()
        return out

    def _purge(self) -> None:
        if self.wm == I64_MAX:
            self.panes.clear()
            return
        keep_from = self._pane_of(self._align_up(self.wm - self.size - self.lateness + 2))
        for p in [p for p in self.panes if p < keep_from]:
            del self.panes[p]

    def _fire_window(self, s: int, only_keys: torch.Tensor | None = None) -> list:
        p0 = self._pane_of(s)
        parts = [c for p in range(p0, p0 + self.size // self.pane) for c in self.panes.get(p, [])]
        if not parts:
            return []
        keys = torch.cat([k for k, _ in parts])
        vals = torch.cat([v for _, v in parts])
        if only_keys is not None:
            sel = torch.isin(keys, only_keys)
            keys, vals = keys[sel], vals[sel]
            if not keys.numel():
                return []
        ordv = K.f64_order_bits(vals.contiguous())
        # One radix sort by key over the used key bits (dictionary ids / small ints sort as they
        # are; anything else through dense ids), the values ride along unsorted; the median of
        # each key segment is then selected per segment (LDS bitonic sort / radix select) -- no
        # 64-bit sort of every value of the window.
        kmin, kmax = (int(x) for x in torch.aminmax(keys))
        if kmin >= 0 and kmax < (1 << 40):
            uniq, ids = None, keys.contiguous()
            kbits = max(1, kmax.bit_length())
        else:
            uniq, ids = torch.unique(keys, return_inverse=True)
            kbits = max(1, int(uniq.numel() - 1).bit_length())
        ids, ordv = K.sort_pairs(ids.contiguous(), ordv, bits=kbits)
        heads = torch.nonzero(torch.cat([torch.ones(1, dtype=torch.bool, device=ids.device),
                                         ids[1:] != ids[:-1]])).flatten()
        med = K.segment_median(heads.contiguous(), ordv, sorted_values=False)
        out_keys = ids[heads] if uniq is None else uniq[ids[heads]]
        return [(s, s + self.size, out_keys.cpu().numpy(), med.cpu().numpy())]

"""Record-at-a-time reference model of the Flink 1.8 semantics the reference relies on.

This is the semantics oracle of SURVEY.md §4.2 (not an execution engine): the native CPU/GPU
engine is differential-tested against it. Modelled behaviour (citations are Flink 1.8 classes
the reference triggers, with the reference call site):

* WindowOperator + EventTimeTrigger / ProcessingTimeTrigger (BandwidthMonitor.java:34,
  BandwidthMonitorWithEventTime.java:46): assignment, per-window state, FIRE on timer
  (``maxTs <= wm``), FIRE on element when the window is already past its maxTs but within the
  allowed lateness, cleanup at ``maxTs + allowedLateness``, late drop (all windows late),
  ``numLateRecordsDropped``, optional late side output.
* StreamGroupedReduce (ComputeCpuMax.java:26 ``max(2)``): emit on every element.
* BoundedOutOfOrdernessTimestampExtractor (BandwidthMonitorWithEventTime.java:30-35):
  ``wm = maxTs - bound`` emitted at batch boundaries (the engine's periodic-watermark points).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Callable

from ..utils.hashing import subtask_of

LONG_MIN = -(1 << 63)
LONG_MAX = (1 << 63) - 1


def java_rem(a: int, b: int) -> int:
    r = abs(a) % abs(b)
    return -r if a < 0 else r


def window_start(ts: int, offset: int, size: int) -> int:
    return ts - java_rem(ts - offset + size, size)


def assign_windows(ts: int, size: int, slide: int, offset: int = 0) -> list[tuple[int, int]]:
    """SlidingEventTimeWindows.assignWindows (tumbling when slide == size)."""
    out = []
    last = window_start(ts, offset, slide)
    s = last
    while s > ts - size:
        out.append((s, s + size))
        s -= slide
    return out


@dataclass
class Emission:
    window: tuple[int, int]
    key: Any
    value: Any
    on_element: bool = False  # fired by a late element (allowed lateness) rather than a timer


@dataclass
class WindowOracle:
    size: int
    slide: int | None = None
    offset: int = 0
    lateness: int = 0
    add: Callable[[Any, Any], Any] = lambda acc, v: v if acc is None else acc + v
    result: Callable[[Any, list], Any] = lambda acc, elems: acc
    keep_elements: bool = False  # ProcessWindowFunction: buffer the raw elements (ListState)
    wm: int = LONG_MIN
    state: dict = field(default_factory=dict)  # (key, window) -> [acc, elements]
    late_dropped: int = 0
    late_side: list = field(default_factory=list)

    def __post_init__(self):
        if self.slide is None:
            self.slide = self.size

    def _emit(self, key, w, on_element=False) -> Emission:
        acc, elems = self.state[(key, w)]
        return Emission(w, key, self.result(acc, elems), on_element)

    def element(self, key, ts: int, value) -> list[Emission]:
        out = []
        skipped = True
        for w in assign_windows(ts, self.size, self.slide, self.offset):
            cleanup = w[1] - 1 + self.lateness
            if cleanup <= self.wm:
                continue  # isWindowLate
            skipped = False
            st = self.state.setdefault((key, w), [None, []])
            st[0] = self.add(st[0], value)
            if self.keep_elements:
                st[1].append(value)
            if w[1] - 1 <= self.wm:  # EventTimeTrigger.onElement: already past maxTs -> FIRE
                out.append(self._emit(key, w, True))
        if skipped:
            self.late_dropped += 1
            self.late_side.append((key, ts, value))
        return out

    def watermark(self, wm: int) -> list[Emission]:
        if wm <= self.wm:
            return []
        old = self.wm
        self.wm = wm
        out = []
        # Event timers at maxTs fire in timestamp order (ties: any order — compare as multisets).
        for (key, w) in sorted(self.state, key=lambda kw: (kw[1][1], kw[1][0])):
            if old < w[1] - 1 <= wm:
                out.append(self._emit(key, w))
        for kw in [kw for kw in self.state if kw[1][1] - 1 + self.lateness <= wm]:
            del self.state[kw]
        return out

    def processing_time(self, now: int) -> list[Emission]:
        """ProcessingTimeTrigger: fire windows whose maxTs passed; no cleanup delay."""
        return self.watermark(now)


@dataclass
class RollingOracle:
    """keyBy(..).reduce / max / sum: emit the post-update value for every element."""

    reduce: Callable[[Any, Any], Any]
    state: dict = field(default_factory=dict)

    def element(self, key, value):
        if key in self.state:
            self.state[key] = self.reduce(self.state[key], value)
        else:
            self.state[key] = value
        return self.state[key]


def flink_max_field(pos: int) -> Callable[[tuple, tuple], tuple]:
    """ComparableAggregator(MAX) for `max(pos)`: replace only field `pos` (first record's other
    fields are kept), ComputeCpuMax.java:26."""

    def red(acc: tuple, new: tuple) -> tuple:
        if new[pos] > acc[pos]:
            acc = acc[:pos] + (new[pos],) + acc[pos + 1:]
        return acc

    return red


def flink_min_field(pos: int):
    def red(acc: tuple, new: tuple) -> tuple:
        if new[pos] < acc[pos]:
            acc = acc[:pos] + (new[pos],) + acc[pos + 1:]
        return acc

    return red


def flink_sum_field(pos: int):
    def red(acc: tuple, new: tuple) -> tuple:
        return acc[:pos] + (acc[pos] + new[pos],) + acc[pos + 1:]

    return red


class BoundedOutOfOrderness:
    """BoundedOutOfOrdernessTimestampExtractor: currentMax starts at Long.MIN_VALUE + bound."""

    def __init__(self, bound: int):
        self.bound = bound
        self.current_max = LONG_MIN + bound
        self.last_emitted = LONG_MIN

    def observe(self, ts: int) -> None:
        if ts > self.current_max:
            self.current_max = ts

    def current_watermark(self) -> int:
        return self.current_max - self.bound


def prefix_for(key, parallelism: int, max_parallelism: int = 128) -> int:
    """1-based print prefix of the subtask that owns `key`."""
    return subtask_of(key, parallelism, max_parallelism) + 1

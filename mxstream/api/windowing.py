"""Window assigners, windows, triggers and evictors (Flink 1.8 ``streaming.api.windowing``).

Reference uses: ``timeWindow(Time.minutes(1))`` (tumbling: ComputeCpuAvg.java:29,
BandwidthMonitor.java:34), ``timeWindow(Time.minutes(5), Time.seconds(5))`` (sliding:
BandwidthMonitorWithEventTime.java:46), sessions and count windows are described in
chapter3/README.md:4,412-428 and chapter2/README.md:78.
"""
from __future__ import annotations

import enum
from dataclasses import dataclass

from .time import to_ms

LONG_MIN = -(1 << 63)
LONG_MAX = (1 << 63) - 1


def _jrem(a: int, b: int) -> int:
    r = abs(a) % abs(b)
    return -r if a < 0 else r


def get_window_start_with_offset(ts: int, offset: int, size: int) -> int:
    """TimeWindow.getWindowStartWithOffset (Java truncated remainder)."""
    return ts - _jrem(ts - offset + size, size)


@dataclass(frozen=True, order=True)
class TimeWindow:
    start: int
    end: int

    def max_timestamp(self) -> int:
        return self.end - 1

    maxTimestamp = max_timestamp

    def get_start(self) -> int:
        return self.start

    def get_end(self) -> int:
        return self.end

    getStart = get_start
    getEnd = get_end

    def intersects(self, other: "TimeWindow") -> bool:
        return self.start <= other.end and self.end >= other.start

    def cover(self, other: "TimeWindow") -> "TimeWindow":
        return TimeWindow(min(self.start, other.start), max(self.end, other.end))

    def __str__(self):
        return f"TimeWindow{{start={self.start}, end={self.end}}}"


@dataclass(frozen=True)
class GlobalWindow:
    def max_timestamp(self) -> int:
        return LONG_MAX

    maxTimestamp = max_timestamp

    def __str__(self):
        return "GlobalWindow"


GLOBAL_WINDOW = GlobalWindow()


def merge_time_windows(windows):
    """TimeWindow.mergeWindows: sort by start, merge overlapping -> list of (merged, members)."""
    ws = sorted(windows, key=lambda w: w.start)
    out = []
    cur, members = None, []
    for w in ws:
        if cur is None:
            cur, members = w, [w]
        elif cur.intersects(w):
            cur = cur.cover(w)
            members.append(w)
        else:
            out.append((cur, members))
            cur, members = w, [w]
    if cur is not None:
        out.append((cur, members))
    return out


# ---- assigners ----------------------------------------------------------------------------

class WindowAssigner:
    event_time: bool = True
    merging: bool = False

    def assign_windows(self, element, timestamp: int, now: int) -> list:
        raise NotImplementedError

    def default_trigger(self) -> "Trigger":
        return EventTimeTrigger() if self.event_time else ProcessingTimeTrigger()

    def is_event_time(self) -> bool:
        return self.event_time


class TumblingEventTimeWindows(WindowAssigner):
    def __init__(self, size: int, offset: int = 0):
        if offset < 0 or offset >= size or size <= 0:
            raise ValueError("TumblingEventTimeWindows parameters must satisfy 0 <= offset < size")
        self.size, self.offset = size, offset

    @staticmethod
    def of(size, offset=0) -> "TumblingEventTimeWindows":
        return TumblingEventTimeWindows(to_ms(size), to_ms(offset))

    def assign_windows(self, element, timestamp, now):
        if timestamp <= LONG_MIN:
            raise RuntimeError("Record has Long.MIN_VALUE timestamp (= no timestamp marker). "
                               "Is the time characteristic set to 'ProcessingTime', or did you "
                               "forget to call 'DataStream.assignTimestampsAndWatermarks(...)'?")
        s = get_window_start_with_offset(timestamp, self.offset, self.size)
        return [TimeWindow(s, s + self.size)]

    # window geometry used by the native planner
    @property
    def slide(self):
        return self.size


class TumblingProcessingTimeWindows(TumblingEventTimeWindows):
    event_time = False

    @staticmethod
    def of(size, offset=0) -> "TumblingProcessingTimeWindows":
        return TumblingProcessingTimeWindows(to_ms(size), to_ms(offset))

    def assign_windows(self, element, timestamp, now):
        s = get_window_start_with_offset(now, self.offset, self.size)
        return [TimeWindow(s, s + self.size)]


class SlidingEventTimeWindows(WindowAssigner):
    def __init__(self, size: int, slide: int, offset: int = 0):
        if abs(offset) >= slide or size <= 0 or slide <= 0:
            raise ValueError("SlidingEventTimeWindows parameters must satisfy abs(offset) < slide and size > 0")
        self.size, self.slide, self.offset = size, slide, offset

    @staticmethod
    def of(size, slide, offset=0) -> "SlidingEventTimeWindows":
        return SlidingEventTimeWindows(to_ms(size), to_ms(slide), to_ms(offset))

    def _assign(self, ts):
        out = []
        last = get_window_start_with_offset(ts, self.offset, self.slide)
        s = last
        while s > ts - self.size:
            out.append(TimeWindow(s, s + self.size))
            s -= self.slide
        return out

    def assign_windows(self, element, timestamp, now):
        if timestamp <= LONG_MIN:
            raise RuntimeError("Record has Long.MIN_VALUE timestamp (= no timestamp marker).")
        return self._assign(timestamp)


class SlidingProcessingTimeWindows(SlidingEventTimeWindows):
    event_time = False

    @staticmethod
    def of(size, slide, offset=0) -> "SlidingProcessingTimeWindows":
        return SlidingProcessingTimeWindows(to_ms(size), to_ms(slide), to_ms(offset))

    def assign_windows(self, element, timestamp, now):
        return self._assign(now)


class EventTimeSessionWindows(WindowAssigner):
    merging = True

    def __init__(self, gap: int):
        if gap <= 0:
            raise ValueError("session gap must be > 0")
        self.gap = gap

    @staticmethod
    def with_gap(gap) -> "EventTimeSessionWindows":
        return EventTimeSessionWindows(to_ms(gap))

    withGap = with_gap

    def assign_windows(self, element, timestamp, now):
        return [TimeWindow(timestamp, timestamp + self.gap)]


class ProcessingTimeSessionWindows(EventTimeSessionWindows):
    event_time = False

    @staticmethod
    def with_gap(gap) -> "ProcessingTimeSessionWindows":
        return ProcessingTimeSessionWindows(to_ms(gap))

    withGap = with_gap

    def assign_windows(self, element, timestamp, now):
        return [TimeWindow(now, now + self.gap)]


class GlobalWindows(WindowAssigner):
    event_time = False

    @staticmethod
    def create() -> "GlobalWindows":
        return GlobalWindows()

    def assign_windows(self, element, timestamp, now):
        return [GLOBAL_WINDOW]

    def default_trigger(self):
        return NeverTrigger()


# ---- triggers -----------------------------------------------------------------------------

class TriggerResult(enum.Enum):
    CONTINUE = (False, False)
    FIRE = (True, False)
    PURGE = (False, True)
    FIRE_AND_PURGE = (True, True)

    @property
    def is_fire(self):
        return self.value[0]

    @property
    def is_purge(self):
        return self.value[1]


class Trigger:
    """on_element / on_event_time / on_processing_time / clear, with a TriggerContext."""

    def on_element(self, element, timestamp, window, ctx) -> TriggerResult:
        return TriggerResult.CONTINUE

    def on_event_time(self, time, window, ctx) -> TriggerResult:
        return TriggerResult.CONTINUE

    def on_processing_time(self, time, window, ctx) -> TriggerResult:
        return TriggerResult.CONTINUE

    def can_merge(self) -> bool:
        return False

    def on_merge(self, window, ctx) -> None:
        raise NotImplementedError

    def clear(self, window, ctx) -> None:
        pass


class EventTimeTrigger(Trigger):
    def on_element(self, element, timestamp, window, ctx):
        if window.max_timestamp() <= ctx.get_current_watermark():
            return TriggerResult.FIRE  # late element within allowed lateness: fire immediately
        ctx.register_event_time_timer(window.max_timestamp())
        return TriggerResult.CONTINUE

    def on_event_time(self, time, window, ctx):
        return TriggerResult.FIRE if time == window.max_timestamp() else TriggerResult.CONTINUE

    def can_merge(self):
        return True

    def on_merge(self, window, ctx):
        if window.max_timestamp() > ctx.get_current_watermark():
            ctx.register_event_time_timer(window.max_timestamp())

    def clear(self, window, ctx):
        ctx.delete_event_time_timer(window.max_timestamp())

    @staticmethod
    def create():
        return EventTimeTrigger()


class ProcessingTimeTrigger(Trigger):
    def on_element(self, element, timestamp, window, ctx):
        ctx.register_processing_time_timer(window.max_timestamp())
        return TriggerResult.CONTINUE

    def on_processing_time(self, time, window, ctx):
        return TriggerResult.FIRE

    def can_merge(self):
        return True

    def on_merge(self, window, ctx):
        ctx.register_processing_time_timer(window.max_timestamp())

    def clear(self, window, ctx):
        ctx.delete_processing_time_timer(window.max_timestamp())

    @staticmethod
    def create():
        return ProcessingTimeTrigger()


class CountTrigger(Trigger):
    """Fires when the window holds `count` elements (countWindow, chapter2/README.md:78)."""

    def __init__(self, count: int):
        self.count = count

    @staticmethod
    def of(count: int) -> "CountTrigger":
        return CountTrigger(count)

    def on_element(self, element, timestamp, window, ctx):
        c = ctx.get_partitioned_state("count", 0) + 1
        if c >= self.count:
            ctx.set_partitioned_state("count", 0)
            return TriggerResult.FIRE
        ctx.set_partitioned_state("count", c)
        return TriggerResult.CONTINUE

    def can_merge(self):
        return True

    def on_merge(self, window, ctx):
        pass

    def clear(self, window, ctx):
        ctx.set_partitioned_state("count", 0)


class PurgingTrigger(Trigger):
    def __init__(self, nested: Trigger):
        self.nested = nested

    @staticmethod
    def of(nested: Trigger) -> "PurgingTrigger":
        return PurgingTrigger(nested)

    @staticmethod
    def _p(r: TriggerResult) -> TriggerResult:
        return TriggerResult.FIRE_AND_PURGE if r.is_fire else r

    def on_element(self, element, timestamp, window, ctx):
        return self._p(self.nested.on_element(element, timestamp, window, ctx))

    def on_event_time(self, time, window, ctx):
        return self._p(self.nested.on_event_time(time, window, ctx))

    def on_processing_time(self, time, window, ctx):
        return self._p(self.nested.on_processing_time(time, window, ctx))

    def can_merge(self):
        return self.nested.can_merge()

    def on_merge(self, window, ctx):
        self.nested.on_merge(window, ctx)

    def clear(self, window, ctx):
        self.nested.clear(window, ctx)


class NeverTrigger(Trigger):
    pass


# ---- evictors -----------------------------------------------------------------------------

class Evictor:
    def evict_before(self, elements: list, size: int, window, ctx) -> list:
        return elements

    def evict_after(self, elements: list, size: int, window, ctx) -> list:
        return elements


class CountEvictor(Evictor):
    def __init__(self, max_count: int, do_evict_after: bool = False):
        self.max_count, self.after = max_count, do_evict_after

    @staticmethod
    def of(max_count: int, do_evict_after: bool = False) -> "CountEvictor":
        return CountEvictor(max_count, do_evict_after)

    def _ev(self, elements):
        if len(elements) <= self.max_count:
            return elements
        return elements[len(elements) - self.max_count:]

    def evict_before(self, elements, size, window, ctx):
        return elements if self.after else self._ev(elements)

    def evict_after(self, elements, size, window, ctx):
        return self._ev(elements) if self.after else elements


class TimeEvictor(Evictor):
    """Keeps elements with timestamp >= max(timestamp) - window_size. Elements are (value, ts)."""

    def __init__(self, window_size: int, do_evict_after: bool = False):
        self.window_size, self.after = window_size, do_evict_after

    @staticmethod
    def of(window_size, do_evict_after: bool = False) -> "TimeEvictor":
        return TimeEvictor(to_ms(window_size), do_evict_after)

    def _ev(self, elements):
        if not elements:
            return elements
        mx = max(ts for _, ts in elements)
        cut = mx - self.window_size
        return [(v, ts) for v, ts in elements if ts > cut]

    def evict_before(self, elements, size, window, ctx):
        return elements if self.after else self._ev(elements)

    def evict_after(self, elements, size, window, ctx):
        return self._ev(elements) if self.after else elements

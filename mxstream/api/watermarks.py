"""Timestamp extractors / watermark assigners (Flink 1.8 ``functions.timestamps``).

``BoundedOutOfOrdernessTimestampExtractor`` is the reference's assigner
(BandwidthMonitorWithEventTime.java:30-35; its Flink source is quoted in chapter3/README.md:
342-397): ``currentMaxTimestamp`` starts at ``Long.MIN_VALUE + bound`` and the periodic
watermark is ``currentMax - bound`` (emitted only when it increases).
"""
from __future__ import annotations

from typing import Callable

from .time import to_ms

LONG_MIN = -(1 << 63)
LONG_MAX = (1 << 63) - 1


class Watermark:
    MAX_WATERMARK = None  # set below

    def __init__(self, timestamp: int):
        self.timestamp = timestamp

    def get_timestamp(self) -> int:
        return self.timestamp

    getTimestamp = get_timestamp

    def __repr__(self):
        return f"Watermark @ {self.timestamp}"

    def __eq__(self, o):
        return isinstance(o, Watermark) and o.timestamp == self.timestamp


Watermark.MAX_WATERMARK = Watermark(LONG_MAX)


class TimestampAssigner:
    def extract_timestamp(self, element, previous_element_timestamp: int) -> int:
        raise NotImplementedError


class AssignerWithPeriodicWatermarks(TimestampAssigner):
    periodic = True

    def get_current_watermark(self) -> Watermark | None:
        raise NotImplementedError


class AssignerWithPunctuatedWatermarks(TimestampAssigner):
    periodic = False

    def check_and_get_next_watermark(self, last_element, extracted_timestamp: int) -> Watermark | None:
        raise NotImplementedError


class BoundedOutOfOrdernessTimestampExtractor(AssignerWithPeriodicWatermarks):
    """Subclass and implement ``extract_timestamp(element)``, or pass ``extractor=``."""

    def __init__(self, max_out_of_orderness, extractor: Callable | None = None):
        bound = to_ms(max_out_of_orderness)
        if bound < 0:
            raise ValueError("Tried to set the maximum allowed lateness to a negative value")
        self.max_out_of_orderness = bound
        self.current_max_timestamp = LONG_MIN + bound
        self.last_emitted_watermark = LONG_MIN
        self._extractor = extractor

    def get_max_out_of_orderness_in_millis(self) -> int:
        return self.max_out_of_orderness

    def extract(self, element) -> int:  # user hook (Java: extractTimestamp(T))
        if self._extractor is not None:
            return int(self._extractor(element))
        return int(self.extractTimestamp(element))

    def extractTimestamp(self, element) -> int:  # noqa: N802 - Java-style override point
        raise NotImplementedError("implement extract(element) / extractTimestamp(element)")

    def extract_timestamp(self, element, previous_element_timestamp: int = LONG_MIN) -> int:
        ts = self.extract(element)
        if ts > self.current_max_timestamp:
            self.current_max_timestamp = ts
        return ts

    def get_current_watermark(self) -> Watermark:
        potential = self.current_max_timestamp - self.max_out_of_orderness
        if potential >= self.last_emitted_watermark:
            self.last_emitted_watermark = potential
        return Watermark(self.last_emitted_watermark)


class AscendingTimestampExtractor(AssignerWithPeriodicWatermarks):
    """Monotonously ascending timestamps: watermark = current timestamp - 1."""

    def __init__(self, extractor: Callable | None = None):
        self.current_timestamp = LONG_MIN
        self._extractor = extractor

    def extract_ascending_timestamp(self, element) -> int:
        if self._extractor is None:
            raise NotImplementedError
        return int(self._extractor(element))

    def extract_timestamp(self, element, previous_element_timestamp: int = LONG_MIN) -> int:
        ts = self.extract_ascending_timestamp(element)
        if ts >= self.current_timestamp:
            self.current_timestamp = ts
        # Flink's default violation handler only logs; the timestamp is kept.
        return ts

    def get_current_watermark(self) -> Watermark:
        return Watermark(LONG_MIN if self.current_timestamp == LONG_MIN else self.current_timestamp - 1)


class PunctuatedAssigner(AssignerWithPunctuatedWatermarks):
    """Convenience punctuated assigner from two callables."""

    def __init__(self, extract: Callable, watermark_for: Callable):
        self._extract = extract
        self._wm = watermark_for

    def extract_timestamp(self, element, previous_element_timestamp: int = LONG_MIN) -> int:
        return int(self._extract(element))

    def check_and_get_next_watermark(self, last_element, extracted_timestamp):
        w = self._wm(last_element, extracted_timestamp)
        if w is None:
            return None
        return w if isinstance(w, Watermark) else Watermark(int(w))


class IngestionTimeAssigner(AssignerWithPeriodicWatermarks):
    """TimeCharacteristic.IngestionTime: timestamp = source clock, watermark = clock - 1."""

    def __init__(self, clock: Callable[[], int]):
        self.clock = clock
        self.last = LONG_MIN

    def extract_timestamp(self, element, previous_element_timestamp: int = LONG_MIN) -> int:
        self.last = max(self.last, self.clock())
        return self.last

    def get_current_watermark(self) -> Watermark:
        now = self.clock()
        return Watermark(now - 1)

"""Time values and the time characteristic (Flink 1.8 ``Time`` / ``TimeCharacteristic``).

Reference call sites: ``Time.minutes(1)`` (ComputeCpuAvg.java:29, BandwidthMonitor.java:34),
``Time.minutes(5), Time.seconds(5)`` (BandwidthMonitorWithEventTime.java:46),
``env.setStreamTimeCharacteristic(TimeCharacteristic.EventTime)`` (…WithEventTime.java:27).
"""
from __future__ import annotations

import enum


class TimeCharacteristic(enum.Enum):
    ProcessingTime = "ProcessingTime"
    IngestionTime = "IngestionTime"
    EventTime = "EventTime"

    # pythonic aliases
    PROCESSING_TIME = "ProcessingTime"
    INGESTION_TIME = "IngestionTime"
    EVENT_TIME = "EventTime"


class Time:
    """A duration in milliseconds."""

    __slots__ = ("ms",)

    def __init__(self, ms: int):
        self.ms = int(ms)

    @staticmethod
    def milliseconds(n) -> "Time":
        return Time(n)

    @staticmethod
    def seconds(n) -> "Time":
        return Time(int(n) * 1000)

    @staticmethod
    def minutes(n) -> "Time":
        return Time(int(n) * 60_000)

    @staticmethod
    def hours(n) -> "Time":
        return Time(int(n) * 3_600_000)

    @staticmethod
    def days(n) -> "Time":
        return Time(int(n) * 86_400_000)

    @staticmethod
    def of(n, unit: str) -> "Time":
        mult = {"ms": 1, "s": 1000, "min": 60_000, "h": 3_600_000, "d": 86_400_000}[unit]
        return Time(int(n) * mult)

    def to_milliseconds(self) -> int:
        return self.ms

    toMilliseconds = to_milliseconds

    def __eq__(self, o):
        return isinstance(o, Time) and o.ms == self.ms

    def __hash__(self):
        return hash(self.ms)

    def __repr__(self):
        return f"Time({self.ms} ms)"


def to_ms(t) -> int:
    if isinstance(t, Time):
        return t.ms
    return int(t)

"""Java-semantics helpers for user functions ported from the reference's Java jobs.

``split`` = ``String.split(" ")`` (trailing empty strings removed), ``parse_double`` =
``Double.parseDouble``, ``parse_long`` = ``Long.parseLong``, ``iso_epoch_seconds`` =
``(int) LocalDateTime.parse(s).toEpochSecond(ZoneOffset.ofHours(h))`` — backed by the C++ runtime
(csrc/runtime.cpp) so the host path and the native parsers agree exactly. Reference call sites:
Main.java:21-24, BandwidthMonitor.java:28-30, BandwidthMonitorWithEventTime.java:33,41.
"""
from __future__ import annotations

from ..ops.native import load


def _traced(x) -> bool:
    """A tracing proxy (mxstream.api.textplan): the planner is recording the parse plan."""
    from .textplan import is_proxy

    return is_proxy(x)


class NumberFormatException(ValueError):
    pass


class ArrayIndexOutOfBoundsException(IndexError):
    pass


def split(s: str, sep: str = " ") -> list[str]:
    if _traced(s):
        return s.split(sep)
    return load().java_split(s, sep)


def _parsed(s, kind: int, offset_s: int = 0):
    from .textplan import FieldProxy, ParsedProxy, TraceError

    if not isinstance(s, FieldProxy):
        raise TraceError("parse of something other than a split field")
    return ParsedProxy(s.sep, s.idx, kind, offset_s)


def parse_double(s: str) -> float:
    if _traced(s):
        return _parsed(s, 1)  # FK_DOUBLE
    try:
        return load().java_parse_double(s)
    except Exception as e:  # ParseError
        raise NumberFormatException(str(e)) from None


def parse_long(s: str) -> int:
    if _traced(s):
        return _parsed(s, 2)  # FK_LONG
    neg = s.startswith("-")
    body = s[1:] if s[:1] in "+-" else s
    if not body or not body.isdigit() or not body.isascii():
        raise NumberFormatException(f'For input string: "{s}"')
    v = int(body)
    v = -v if neg else v
    if not -(1 << 63) <= v < (1 << 63):
        raise NumberFormatException(f'For input string: "{s}"')
    return v


def parse_int(s: str) -> int:
    if _traced(s):
        return _parsed(s, 5)  # FK_INT
    v = parse_long(s)
    if not -(1 << 31) <= v < (1 << 31):
        raise NumberFormatException(f'For input string: "{s}"')
    return v


def iso_epoch_millis(s: str, offset_hours: int = 0) -> int:
    if _traced(s):
        return _parsed(s, 4, int(offset_hours) * 3600)  # FK_TS_MS
    try:
        return load().iso_to_epoch_ms(s, offset_hours * 3600)
    except Exception as e:
        raise ValueError(f"DateTimeParseException: Text '{s}' could not be parsed") from e


def iso_epoch_seconds(s: str, offset_hours: int = 0) -> int:
    """(int) LocalDateTime.parse(s).toEpochSecond(ZoneOffset.ofHours(h)) — int32 wrap."""
    if _traced(s):
        return _parsed(s, 7, int(offset_hours) * 3600)  # FK_ISO_SEC
    v = iso_epoch_millis(s, offset_hours) // 1000
    v &= 0xFFFFFFFF
    return v - (1 << 32) if v & 0x80000000 else v


def get(items: list, i: int):
    """items[i] with Java's ArrayIndexOutOfBoundsException (no negative indexing)."""
    if _traced(items):
        return items[i]
    if i < 0 or i >= len(items):
        raise ArrayIndexOutOfBoundsException(str(i))
    return items[i]

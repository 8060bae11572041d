"""Metrics registry and exporters.

The reference relies on Flink's built-in operator metrics (unused by its jobs) and prints results;
mxstream keeps Flink's metric names where one exists and adds the engine's own:

  Flink names   numRecordsIn, numRecordsOut, numLateRecordsDropped, currentInputWatermark,
                numberOfCompletedCheckpoints, lastCheckpointDuration, numRestarts
  engine        events_per_sec, alert_latency_ms{p50,p99}, state_bytes_hbm, state_bytes_host,
                spill_bytes, a2a_bytes, step_ms{stage}

Metrics live in a process-wide :class:`MetricRegistry` under scoped names
(``<job>.<operator>.<metric>``). Exporters write JSON lines (one object per report) and the
Prometheus text exposition format (``mxs_<metric>{job=..,operator=..}``). Per-stage step timings
come from :class:`StageTimer`, which brackets GPU work with HIP events so the numbers are device
time, not launch time.
"""
from __future__ import annotations

import json
import math
import re
import threading
import time
from collections import defaultdict
from typing import Callable

import torch


class Counter:
    def __init__(self):
        self.value = 0

    def inc(self, n: int = 1) -> None:
        self.value += n

    def get(self):
        return self.value


class Gauge:
    def __init__(self, fn: Callable[[], float]):
        self.fn = fn

    def get(self):
        return self.fn()


class Histogram:
    """Reservoir of the last `size` samples; reports count/mean/p50/p99/max."""

    def __init__(self, size: int = 4096):
        self.size = size
        self.samples: list[float] = []
        self.count = 0
        self._i = 0

    def update(self, v: float) -> None:
        self.count += 1
        if len(self.samples) < self.size:
            self.samples.append(float(v))
        else:
            self.samples[self._i] = float(v)
            self._i = (self._i + 1) % self.size

    def quantile(self, q: float) -> float | None:
        if not self.samples:
            return None
        s = sorted(self.samples)
        return s[min(len(s) - 1, int(math.ceil(q * len(s))) - 1 if q > 0 else 0)]

    def get(self):
        if not self.samples:
            return {"count": self.count}
        return {"count": self.count, "mean": sum(self.samples) / len(self.samples),
                "p50": self.quantile(0.5), "p99": self.quantile(0.99), "max": max(self.samples)}


class MetricRegistry:
    def __init__(self):
        self._m: dict[str, object] = {}
        self._lock = threading.Lock()

    def _get(self, name: str, factory):
        with self._lock:
            m = self._m.get(name)
            if m is None:
                m = factory()
                self._m[name] = m
            return m

    def counter(self, name: str) -> Counter:
        return self._get(name, Counter)

    def histogram(self, name: str, size: int = 4096) -> Histogram:
        return self._get(name, lambda: Histogram(size))

    def gauge(self, name: str, fn: Callable[[], float]) -> Gauge:
        with self._lock:
            g = Gauge(fn)
            self._m[name] = g
            return g

    def register_object(self, scope: str, obj, fields: dict[str, str]) -> None:
        """Expose attributes of an engine object (e.g. OperatorMetrics) as gauges:
        fields = {metric name: attribute name}."""
        for metric, attr in fields.items():
            self.gauge(f"{scope}.{metric}", lambda o=obj, a=attr: getattr(o, a))

    def snapshot(self) -> dict:
        with self._lock:
            items = list(self._m.items())
        return {k: m.get() for k, m in items}

    def clear(self) -> None:
        with self._lock:
            self._m.clear()


REGISTRY = MetricRegistry()

# Flink operator metric names for the engine operators' metric objects.
OPERATOR_FIELDS = {"numRecordsIn": "num_records_in", "numRecordsOut": "num_records_out",
                   "numLateRecordsDropped": "num_late_records_dropped",
                   "currentInputWatermark": "current_watermark"}


def register_operator(scope: str, op, registry: MetricRegistry = REGISTRY) -> None:
    """Flink-named gauges for a KeyedWindow/Rolling/Session operator (plus state sizes)."""
    m = getattr(op, "metrics", None)
    if m is not None:
        registry.register_object(scope, m, {k: v for k, v in OPERATOR_FIELDS.items()
                                            if hasattr(m, v)})
    if hasattr(op, "state_bytes"):
        registry.gauge(f"{scope}.state_bytes_hbm", lambda o=op: o.state_bytes()
                       - (o.host_bytes() if hasattr(o, "host_bytes") else 0))
    if hasattr(op, "host_bytes"):
        registry.gauge(f"{scope}.state_bytes_host", op.host_bytes)


# ---- exporters ----------------------------------------------------------------------------------
def to_json_line(registry: MetricRegistry = REGISTRY, **extra) -> str:
    return json.dumps({"ts_ms": int(time.time() * 1000), **extra, "metrics": registry.snapshot()},
                      default=float)


_BAD = re.compile(r"[^a-zA-Z0-9_]")


def _prom_name(metric: str) -> str:
    return "mxs_" + _BAD.sub("_", metric)


def to_prometheus(registry: MetricRegistry = REGISTRY) -> str:
    """Prometheus text exposition format. Scoped names `<job>.<op>.<metric>` become
    `mxs_<metric>{job="..",operator=".."}`; histograms export quantiles."""
    lines, typed = [], set()
    for name, val in sorted(registry.snapshot().items()):
        parts = name.split(".")
        metric = parts[-1]
        labels = {}
        if len(parts) >= 3:
            labels = {"job": parts[0], "operator": ".".join(parts[1:-1])}
        elif len(parts) == 2:
            labels = {"scope": parts[0]}
        pname = _prom_name(metric)
        lab = ",".join(f'{k}="{v}"' for k, v in labels.items())
        if isinstance(val, dict):
            if pname not in typed:
                lines.append(f"# TYPE {pname} summary")
                typed.add(pname)
            for q, key in ((0.5, "p50"), (0.99, "p99")):
                if val.get(key) is not None:
                    ql = f'{lab},quantile="{q}"' if lab else f'quantile="{q}"'
                    lines.append(f"{pname}{{{ql}}} {val[key]}")
            lines.append(f"{pname}_count{{{lab}}} {val.get('count', 0)}")
            continue
        if val is None:
            continue
        if pname not in typed:
            lines.append(f"# TYPE {pname} gauge")
            typed.add(pname)
        lines.append(f"{pname}{{{lab}}} {float(val)}")
    return "\n".join(lines) + "\n"


class Reporter:
    """Periodic JSON-lines / Prometheus-file reporter (call `maybe_report()` once per step)."""

    def __init__(self, *, json_path: str | None = None, prom_path: str | None = None,
                 interval_ms: int = 1000, registry: MetricRegistry = REGISTRY):
        self.json_path, self.prom_path = json_path, prom_path
        self.interval = interval_ms / 1000.0
        self.registry = registry
        self._last = 0.0

    def maybe_report(self, force: bool = False, **extra) -> None:
        now = time.monotonic()
        if not force and now - self._last < self.interval:
            return
        self._last = now
        if self.json_path:
            with open(self.json_path, "a") as f:
                f.write(to_json_line(self.registry, **extra) + "\n")
        if self.prom_path:
            tmp = self.prom_path + ".tmp"
            with open(tmp, "w") as f:
                f.write(to_prometheus(self.registry))
            import os

            os.replace(tmp, self.prom_path)


class StageTimer:
    """Per-stage step timings. On a GPU the stages are bracketed by HIP events (device time,
    read lazily); on the CPU by the host clock. Results go to `<scope>.step_ms.<stage>`
    histograms."""

    def __init__(self, scope: str, device, registry: MetricRegistry = REGISTRY,
                 enabled: bool = True):
        self.scope = scope
        self.gpu = torch.device(device).type == "cuda"
        self.registry = registry
        self.enabled = enabled
        self._pending: list[tuple[str, object, object]] = []

    def stage(self, name: str):
        timer = self

        class _Ctx:
            def __enter__(self_inner):
                from . import trace

                self_inner.tr = trace.active()
                if self_inner.tr:
                    trace.load().trace_push(f"{timer.scope}.{name}", "stage")
                if not timer.enabled:
                    return self_inner
                if timer.gpu:
                    self_inner.a = torch.cuda.Event(enable_timing=True)
                    self_inner.a.record()
                else:
                    self_inner.t0 = time.perf_counter()
                return self_inner

            def __exit__(self_inner, *exc):
                if self_inner.tr:
                    from . import trace

                    trace.load().trace_pop()
                if not timer.enabled:
                    return False
                if timer.gpu:
                    b = torch.cuda.Event(enable_timing=True)
                    b.record()
                    timer._pending.append((name, self_inner.a, b))
                else:
                    timer.registry.histogram(f"{timer.scope}.step_ms.{name}").update(
                        (time.perf_counter() - self_inner.t0) * 1e3)
                return False

        return _Ctx()

    def add(self, name: str, ms: float) -> None:
        """A stage time measured elsewhere (the native window step's own stage clocks)."""
        self.registry.histogram(f"{self.scope}.step_ms.{name}").update(ms)

    def flush(self) -> None:
        """Resolve recorded GPU events (call after a sync point)."""
        from . import trace

        tr = self.gpu and trace.enabled()
        keep = []
        for name, a, b in self._pending:
            if b.query():
                self.registry.histogram(f"{self.scope}.step_ms.{name}").update(a.elapsed_time(b))
                if tr:
                    trace.gpu_span(f"{self.scope}.{name}", a, b)
            else:
                keep.append((name, a, b))
        self._pending = keep


def stage_table(registry: MetricRegistry = REGISTRY, scope: str | None = None) -> dict:
    """{stage: mean ms} from the step_ms histograms (optionally one scope)."""
    out = defaultdict(float)
    for name, val in registry.snapshot().items():
        if ".step_ms." in name and isinstance(val, dict) and "mean" in val:
            sc, stage = name.split(".step_ms.")
            if scope is None or sc == scope:
                out[stage] = val["mean"]
    return dict(out)

"""The reference's six pipelines on the mxstream DataStream API (same operators, same order).

Each ``build_*`` takes an environment and a ``DataStream[str]`` of text lines (the reference
always reads ``env.socketTextStream("localhost", 8080)``), wires the job, and returns the final
stream; ``main()`` functions run them against the socket exactly like the Java ``main`` methods.

| function | reference |
|---|---|
| build_cpu_alert              | chapter1/src/main/java/me/zjy/Main.java:16-34 |
| build_compute_cpu_max        | chapter2/src/main/java/me/zjy/ComputeCpuMax.java:15-27 |
| build_compute_cpu_avg        | chapter2/src/main/java/me/zjy/ComputeCpuAvg.java:17-60 |
| build_compute_cpu_middle     | chapter2/src/main/java/me/zjy/ComputeCpuMiddle.java:24-50 |
| build_bandwidth_monitor      | chapter3/src/main/java/me/zjy/BandwidthMonitor.java:20-42 |
| build_bandwidth_event_time   | chapter3/src/main/java/me/zjy/BandwidthMonitorWithEventTime.java:25-57 |
"""
from __future__ import annotations

import sys

from ..api import java as J
from ..api.environment import StreamExecutionEnvironment
from ..api.functions import AggregateFunction, FilterFunction, MapFunction, ProcessWindowFunction
from ..api.time import Time, TimeCharacteristic
from ..api.tuples import Tuple2, Tuple3
from ..api.watermarks import BoundedOutOfOrdernessTimestampExtractor


# ---- chapter 1 ----------------------------------------------------------------------------

class ParseCpu(MapFunction):
    """Main.java:18-26: "ts ip cpuN usage" -> Tuple3<host, cpu, usage>."""

    def map(self, value):
        items = J.split(value, " ")
        host = J.get(items, 1)
        cpu = J.get(items, 2)
        usage = J.parse_double(J.get(items, 3))
        return Tuple3(host, cpu, usage)


class HighUsage(FilterFunction):
    """Main.java:27-32: keep usage > 90."""

    def filter(self, value):
        return value.f2 > 90


def build_cpu_alert(env, text, with_filter: bool = True):
    s = text.map(ParseCpu())
    if with_filter:
        s = s.filter(HighUsage())
    s.print()
    return s


# ---- chapter 2 ----------------------------------------------------------------------------

def build_compute_cpu_max(env, text):
    s = text.map(ParseCpu()).key_by(0).max(2)
    s.print()
    return s


class ParseHostUsage(MapFunction):
    """ComputeCpuAvg.java:19-26: -> Tuple2<host, usage>."""

    def map(self, value):
        items = J.split(value, " ")
        return Tuple2(J.get(items, 1), J.parse_double(J.get(items, 3)))


class AvgUsage(AggregateFunction):
    """ComputeCpuAvg.java:31-58: accumulator Tuple2<Integer count, Double sum>."""

    def create_accumulator(self):
        return Tuple2(0, 0.0)

    def add(self, value, accumulator):
        return Tuple2(accumulator.f0 + 1, accumulator.f1 + value.f1)

    def get_result(self, accumulator):
        return 0.0 if accumulator.f0 == 0 else accumulator.f1 / accumulator.f0

    def merge(self, a, b):
        return Tuple2(a.f0 + b.f0, a.f1 + b.f1)


def build_compute_cpu_avg(env, text, aggregate=None):
    s = (text.map(ParseHostUsage()).key_by(0)
         .time_window(Time.minutes(1))
         .aggregate(aggregate or AvgUsage()))
    s.print()
    return s


class MedianUsage(ProcessWindowFunction):
    """ComputeCpuMiddle.java:34-48: buffer, sort, median (0.0 when empty).

    ``native`` tells the planner this is the median of field 1, so the window can run on the
    device list-window operator (sort + segment-median kernels); this method is the exact host
    implementation used otherwise."""

    native = ("median", 1)

    def process(self, key, context, elements, out):
        values = sorted(t.f1 for t in elements)
        if not values:
            out.collect(0.0)
        elif len(values) % 2 != 0:
            out.collect(values[len(values) // 2])
        else:
            out.collect((values[len(values) // 2] + values[len(values) // 2 - 1]) / 2)


def build_compute_cpu_middle(env, text):
    s = text.map(ParseHostUsage()).key_by(0).time_window(Time.minutes(1)).process(MedianUsage())
    s.print()
    return s


# ---- chapter 3 ----------------------------------------------------------------------------

class ParseChannelFlow(MapFunction):
    """BandwidthMonitor.java:25-31: "time channel bytes" -> Tuple2<channel, Long bytes>."""

    def map(self, s):
        items = J.split(s, " ")
        return Tuple2(J.get(items, 1), J.parse_long(J.get(items, 2)))


def build_bandwidth_monitor(env, text, slide=None):
    env.set_stream_time_characteristic(TimeCharacteristic.ProcessingTime)
    keyed = text.map(ParseChannelFlow()).key_by(0)
    w = keyed.time_window(Time.minutes(1)) if slide is None else keyed.time_window(Time.minutes(1), slide)
    s = (w.reduce(lambda a, b: Tuple2(a.f0, a.f1 + b.f1))
         .filter(lambda t: t.f1 * 8.0 / 60 / 1024 / 1024 < 100))
    s.print()
    return s


class EventTimeExtractor(BoundedOutOfOrdernessTimestampExtractor):
    """BandwidthMonitorWithEventTime.java:30-35: ISO time at UTC+8, (int) seconds * 1000L."""

    def __init__(self):
        super().__init__(Time.minutes(1))

    def extractTimestamp(self, element):  # noqa: N802 (Java override name)
        return J.iso_epoch_seconds(J.split(element, " ")[0], 8) * 1000


class ParseTimedFlow(MapFunction):
    """…WithEventTime.java:36-45: -> Tuple3<Integer time, channel, Long flow>."""

    def map(self, s):
        items = J.split(s, " ")
        time = J.iso_epoch_seconds(J.get(items, 0), 8)
        return Tuple3(time, J.get(items, 1), J.parse_long(J.get(items, 2)))


def build_bandwidth_event_time(env, text):
    env.set_stream_time_characteristic(TimeCharacteristic.EventTime)
    s = (text.assign_timestamps_and_watermarks(EventTimeExtractor())
         .map(ParseTimedFlow())
         .key_by(1)
         .time_window(Time.minutes(5), Time.seconds(5))
         .reduce(lambda a, b: Tuple3(a.f0, a.f1, a.f2 + b.f2))
         .map(lambda t: Tuple2(t.f1, t.f2 * 8.0 / 60 / 1024 / 1024))
         .filter(lambda t: t.f1 < 100.0))
    s.print()
    return s


JOBS = {
    "Main": (build_cpu_alert, "Window WordCount"),
    "ComputeCpuMax": (build_compute_cpu_max, "ComputeCpuMax"),
    "ComputeCpuAvg": (build_compute_cpu_avg, "ComputeCpuAvg"),
    "ComputeCpuMiddle": (build_compute_cpu_middle, "ComputeCpuMiddle"),
    "BandwidthMonitor": (build_bandwidth_monitor, "BandwidthMonitor"),
    "BandwidthMonitorWithEventTime": (build_bandwidth_event_time, "BandwidthMonitorWithEventTime"),
}


def main(argv=None) -> int:
    """python -m mxstream.models.chapters <Job> [host] [port] [--conf k=v ...]
    (defaults: localhost 8080; engine keys: mxstream/utils/config.py)."""
    from ..utils.config import apply_to_env, load_config, strip_conf_args

    argv = sys.argv[1:] if argv is None else argv
    cfg = load_config(argv)
    argv = strip_conf_args(argv)
    if not argv or argv[0] not in JOBS:
        print(f"usage: python -m mxstream.models.chapters {{{'|'.join(JOBS)}}} [host] [port]"
              " [--conf key=value ...]")
        return 2
    build, name = JOBS[argv[0]]
    host = argv[1] if len(argv) > 1 else "localhost"
    port = int(argv[2]) if len(argv) > 2 else 8080
    env = StreamExecutionEnvironment.get_execution_environment()
    apply_to_env(cfg, env)
    build(env, env.socket_text_stream(host, port))
    env.execute(name)
    return 0


if __name__ == "__main__":
    sys.exit(main())

"""Golden tests: the reference's six jobs on README inputs.

Processing-time jobs run against a ManualClock (lines "typed" one per second, then the source
stays open past the window end, like waiting a minute before closing `nc`).
"""
from collections import Counter

import pytest

from mxstream.api.environment import StreamExecutionEnvironment
from mxstream.models import chapters as C
from mxstream.runtime.executor import JobExecutionException, ManualClock


def run(build, lines, *, end_time=None, p=4, rebalance_start=0, native="auto", **kw):
    out = []
    env = StreamExecutionEnvironment(p, clock=ManualClock(0)).set_output(out.append)
    env.config.rebalance_start = rebalance_start
    env.config.native = native
    src = env.from_timed_collection([(1000 * (i + 1), l) for i, l in enumerate(lines)],
                                    end_time=end_time)
    build(env, src, **kw)
    env.execute("test")
    return out


# A.1 -- chapter1/README.md:72-84 (map + print) and :114-123 (with the > 90 filter)
def test_chapter1_map_print_readme():
    lines = ["1563452056 10.8.22.1 cpu0 80.5", "1563452051 10.8.22.1 cpu2 10.5",
             "1563452051 10.8.22.1 cpu2 10.5"]
    # Round-robin from channel 2 reproduces the README's 3>, 4>, 1> exactly.
    out = run(C.build_cpu_alert, lines, rebalance_start=2, with_filter=False)
    assert out == ["3> (10.8.22.1,cpu0,80.5)", "4> (10.8.22.1,cpu2,10.5)",
                   "1> (10.8.22.1,cpu2,10.5)"]


def test_chapter1_filter_readme():
    out = run(C.build_cpu_alert, ["1563452051 10.8.22.1 cpu2 10.5", "1563452051 10.8.22.1 cpu2 99.2"],
              rebalance_start=0)
    assert out == ["2> (10.8.22.1,cpu2,99.2)"]


def test_chapter1_malformed_line_fails_job():
    # ArrayIndexOutOfBounds in the map fails the job (no restart strategy).
    with pytest.raises(JobExecutionException):
        run(C.build_cpu_alert, ["1563452056 10.8.22.1"])


# A.2 -- chapter2/README.md:54-66
def test_compute_cpu_max_readme():
    lines = ["1563452056 10.8.22.1 cpu0 80.5", "1563452050 10.8.22.1 cpu0 78.4",
             "1563452056 10.8.22.1 cpu0 99.9"]
    assert run(C.build_compute_cpu_max, lines) == [
        "3> (10.8.22.1,cpu0,80.5)", "3> (10.8.22.1,cpu0,80.5)", "3> (10.8.22.1,cpu0,99.9)"]


# A.3 -- chapter2/README.md:153-164 (avg) and :236-248 (median), processing time
AVG_LINES = ["1563452056 10.8.22.1 cpu0 80.5", "1563452050 10.8.22.1 cpu0 78.4",
             "1563452056 10.8.22.1 cpu0 99.9", "1563452056 10.8.22.2 cpu1 20.2"]


def test_compute_cpu_avg_readme():
    out = run(C.build_compute_cpu_avg, AVG_LINES, end_time=61_000)
    assert sorted(out) == ["3> 20.2", "3> 86.26666666666667"]


def test_compute_cpu_avg_not_fired_before_window_end():
    # Processing-time windows are not fired at end of input (source closed before 60 s).
    assert run(C.build_compute_cpu_avg, AVG_LINES, end_time=30_000) == []


def test_compute_cpu_middle_readme():
    out = run(C.build_compute_cpu_middle, AVG_LINES, end_time=61_000)
    assert sorted(out) == ["3> 20.2", "3> 80.5"]


# A.4 -- chapter3/README.md:71-81 (processing-time tumbling / sliding)
BW_LINES = ["2019-08-28T10:00:00 www.163.com 10000", "2019-08-28T10:01:00 www.163.com 100",
            "2019-08-28T10:02:00 www.163.com 100", "2019-08-28T10:03:00 www.163.com 1000"]


def test_bandwidth_monitor_tumbling_readme():
    assert run(C.build_bandwidth_monitor, BW_LINES, end_time=61_000) == ["2> (www.163.com,11200)"]


def test_bandwidth_monitor_sliding_readme():
    from mxstream.api.time import Time

    out = run(C.build_bandwidth_monitor, BW_LINES, end_time=16_000, slide=Time.seconds(15))
    # First output after ~15 s: the 1 min / 15 s window [-45 s, 15 s) holds all four lines.
    assert out == ["2> (www.163.com,11200)"]


# A.4 -- chapter3/README.md:284-297 (event time, sliding 5 min / 5 s, bound 1 min)
EV_LINES = ["2019-08-28T10:00:00 www.163.com 10000", "2019-08-28T10:01:00 www.163.com 100",
            "2019-08-28T10:02:00 www.163.com 100", "2019-08-28T09:01:00 www.163.com 100",
            "2019-08-28T10:06:00 www.163.com 100"]


@pytest.mark.parametrize("native", ["off", "auto"])
def test_bandwidth_event_time_readme(native):
    out = run(C.build_bandwidth_event_time, EV_LINES, native=native)
    first = out[:60]
    c = Counter(first)
    assert c == Counter({"2> (www.163.com,0.0012715657552083333)": 12,
                         "2> (www.163.com,0.0012842814127604167)": 12,
                         "2> (www.163.com,0.0012969970703125)": 36})
    # README shows the first and last distinct values of the live run (:295-296).
    assert first[0] == "2> (www.163.com,0.0012715657552083333)"
    assert first[-1] == "2> (www.163.com,0.0012969970703125)"
    # End of input (socket closed) fires the 72 windows that stay open in the README run.
    assert len(out) == 60 + 72

"""Columnar text ingest behind the DataStream API (api/textplan.py, runtime/columnar.py).

The planner traces each reference job's parse map (and extractor / filter) and lowers
source -> [timestamps] -> map -> [filter] to one TextParseOp over raw line batches: the C++
parser fills columns, the native keyed operators consume them. These tests check that the
user's parse function is never called per record, that results equal the per-record host
path (native='off') on multi-line batches, and that parse errors still fail the job.
"""
import random
from collections import Counter

import pytest

from mxstream.api.environment import StreamExecutionEnvironment
from mxstream.api.textplan import LineProxy
from mxstream.models import chapters as C
from mxstream.runtime.executor import JobExecutionException, ManualClock


def _lines_cpu(n, seed=1):
    rng = random.Random(seed)
    return [f"{1563452000 + i} 10.8.{rng.randint(0, 3)}.{rng.randint(1, 40)} cpu{rng.randint(0, 7)} "
            f"{rng.uniform(0, 100):.1f}" for i in range(n)]


def _lines_bw(n, seed=2):
    rng = random.Random(seed)
    out = []
    for i in range(n):
        sec = 36000 + i // 3 + rng.randint(-50, 5)
        out.append(f"2019-08-28T{sec // 3600:02d}:{sec // 60 % 60:02d}:{sec % 60:02d} "
                   f"ch{rng.randint(0, 30)}.com {rng.randint(0, 20000)}")
    return out


def _run_file(tmp_path, build, lines, native, p=4, **kw):
    path = tmp_path / "in.txt"
    path.write_text("\n".join(lines) + "\n")
    out = []
    env = StreamExecutionEnvironment(p, clock=ManualClock(0)).set_output(out.append)
    env.config.native = native
    env.config.batch_size = 4096
    build(env, env.read_text_file(str(path)), **kw)
    env.execute("file")
    return out


@pytest.mark.parametrize("job", ["BandwidthMonitorWithEventTime", "ComputeCpuMax", "Main"])
def test_file_jobs_columnar_equal_host(tmp_path, job):
    build = C.JOBS[job][0]
    lines = _lines_bw(20_000) if job.startswith("Bandwidth") else _lines_cpu(20_000)
    host = _run_file(tmp_path, build, lines, "off")
    col = _run_file(tmp_path, build, lines, "auto")
    assert len(host) > 0
    assert Counter(col) == Counter(host)


def test_user_parse_functions_not_called_per_record(monkeypatch):
    calls = Counter()

    def wrap(cls):
        orig = cls.map

        def counted(self, value):
            if not isinstance(value, LineProxy):
                calls[cls.__name__] += 1
            return orig(self, value)
        monkeypatch.setattr(cls, "map", counted)

    for cls in (C.ParseCpu, C.ParseHostUsage, C.ParseChannelFlow, C.ParseTimedFlow):
        wrap(cls)
    cpu = _lines_cpu(300)
    bw = _lines_bw(300)
    for name, (build, _) in C.JOBS.items():
        out = []
        env = StreamExecutionEnvironment(4, clock=ManualClock(0)).set_output(out.append)
        env.config.native = "auto"
        lines = bw if name.startswith("Bandwidth") else cpu
        src = env.from_timed_collection([(1000 * (i + 1), l) for i, l in enumerate(lines)],
                                        end_time=400_000)
        build(env, src)
        env.execute(name)
        assert out, name
    assert sum(calls.values()) == 0, calls


def test_columnar_parse_error_fails_job(tmp_path):
    lines = _lines_cpu(5000)
    lines[3210] = "1563452056 10.8.22.1 cpu0 eighty"
    with pytest.raises(JobExecutionException, match="NumberFormatException"):
        _run_file(tmp_path, C.build_cpu_alert, lines, "auto")
    lines[3210] = "1563452056 10.8.22.1"
    with pytest.raises(JobExecutionException, match="ArrayIndexOutOfBounds"):
        _run_file(tmp_path, C.build_cpu_alert, lines, "auto")


def test_deferred_device_ingest_equals_synchronous():
    """Deferred device ingest (each batch's parse result read one pass later, TextParseOp
    defer) prints exactly what the synchronous ingest prints, in the same order -- event-time
    sliding windows (BandwidthMonitorWithEventTime) and the rolling max (ComputeCpuMax)."""
    from mxstream.api.environment import StreamExecutionEnvironment
    from mxstream.models import chapters as C

    bw = [f"2019-08-28T10:{(i // 60) % 60:02d}:{i % 60:02d} www.ch{(i * 7) % 13}.com "
          f"{40 + i % 11 if i % 5 == 0 else 9_000_000 + i}" for i in range(3000)]
    cpu = [f"{1563452000 + i} 10.8.{i % 37}.1 cpu{i % 4} {(i * 37 % 400) / 4.0}"
           for i in range(3000)]

    def run(build, lines, defer):
        out = []
        env = StreamExecutionEnvironment(4).set_output(out.append)
        env.config.native = "auto"
        env.config.device = "cpu"
        env.config.text_ingest = "device"
        env.config.ingest_defer = defer
        build(env, env.from_collection(lines, batch_size=256))
        env.execute("defer")
        return out

    for build, lines in ((C.build_bandwidth_event_time, bw), (C.build_compute_cpu_max, cpu)):
        ref = run(build, lines, False)
        assert len(ref) > 10
        assert run(build, lines, True) == ref

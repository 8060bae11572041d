"""Golden fixture: the out-of-order stream of chapter3/img/stream_watermark_out_of_order.svg
(SURVEY.md D4 / Appendix A.4), replayed through the event-time window path.

The figure's stream arrives right to left:  7 11 15 9 12 W(11) 14 17 12 22 17 20 W(17) 19 21.
Reading its labels' x positions gives exactly that order; the watermarks are punctuated at
the positions shown. The test asserts Flink's semantics on it with 4 ms tumbling windows:
  * W(11) fires [4,8) = {7} and [8,12) = {11, 9}; nothing after W(11) is late (all > 11);
  * W(17) fires [12,16) = {15, 12, 14, 12}; [16,20) stays open (maxTs 19 > 17);
  * end of input (Long.MAX_VALUE watermark) fires [16,20) = {17, 17, 19} and [20,24) =
    {22, 20, 21}; no element is dropped.
It also checks the periodic BoundedOutOfOrderness assigner (bound 4) reproduces the figure's
first watermark: after the first five elements the current watermark is W(11).
"""
import pytest

from mxstream.api.environment import StreamExecutionEnvironment
from mxstream.api.functions import ProcessWindowFunction
from mxstream.api.time import Time, TimeCharacteristic
from mxstream.api.tuples import Tuple3
from mxstream.api.watermarks import (BoundedOutOfOrdernessTimestampExtractor, PunctuatedAssigner,
                                     Watermark)

# (arrival index, event timestamp); watermarks follow arrival indices 4 (W11) and 11 (W17).
STREAM = [7, 11, 15, 9, 12, 14, 17, 12, 22, 17, 20, 19, 21]
WM_AFTER = {4: 11, 10: 17}
LONG_MAX = (1 << 63) - 1


def test_figure_order_from_svg_labels():
    # Flink docs figure labels (x position, text) as drawn; the stream flows right to left.
    labels = [(511.9, "7"), (481.1, "11"), (439.3, "15"), (417.5, "9"), (379.2, "12"),
              (356.5, "W(11)"), (344.8, "14"), (311.7, "17"), (284.4, "12"), (257.9, "22"),
              (213.9, "17"), (183.7, "20"), (145.1, "W(17)"), (134.5, "19"), (98.1, "21")]
    seq = [t for _x, t in sorted(labels, reverse=True)]
    events = [int(t) for t in seq if not t.startswith("W")]
    assert events == STREAM
    wpos = {}
    n = 0
    for t in seq:
        if t.startswith("W"):
            wpos[n - 1] = int(t[2:-1])
        else:
            n += 1
    assert wpos == WM_AFTER


class _Tag(ProcessWindowFunction):
    def process(self, key, context, elements, out):
        for e in elements:
            w = context.window()
            out.collect((w.start, w.end, e.f1, e.f2, context.current_watermark()))


def _run(native):
    out = []
    env = StreamExecutionEnvironment(1).set_output(out.append)
    env.config.native = native
    env.set_stream_time_characteristic(TimeCharacteristic.EventTime)
    items = [(i, ts) for i, ts in enumerate(STREAM)]
    assigner = PunctuatedAssigner(lambda e: e[1], lambda e, ts: WM_AFTER.get(e[0]))
    (env.from_collection(items, batch_size=1)
     .assign_timestamps_and_watermarks(assigner)
     .map(lambda e: Tuple3("k", e[1], 1))
     .key_by(0)
     .time_window(Time.milliseconds(4))
     .reduce(lambda a, b: Tuple3(a.f0, a.f1 + b.f1, a.f2 + b.f2), _Tag())
     .print())
    env.execute("watermark figure")
    return out


def test_figure_windows_fire_at_their_watermarks():
    rows = [eval(line) for line in _run("off")]  # noqa: S307 - our own tuple repr
    assert rows == [(4, 8, 7, 1, 11), (8, 12, 20, 2, 11), (12, 16, 53, 4, 17),
                    (16, 20, 53, 3, LONG_MAX), (20, 24, 63, 3, LONG_MAX)]


@pytest.mark.parametrize("native", ["off", "auto"])
def test_figure_window_sums_native_and_host(native):
    out = []
    env = StreamExecutionEnvironment(1).set_output(out.append)
    env.config.native = native
    env.set_stream_time_characteristic(TimeCharacteristic.EventTime)
    items = [(i, ts) for i, ts in enumerate(STREAM)]
    assigner = PunctuatedAssigner(lambda e: e[1], lambda e, ts: WM_AFTER.get(e[0]))
    (env.from_collection(items, batch_size=1)
     .assign_timestamps_and_watermarks(assigner)
     .map(lambda e: Tuple3("k", e[1], 1))
     .key_by(0)
     .time_window(Time.milliseconds(4))
     .reduce(lambda a, b: Tuple3(a.f0, a.f1 + b.f1, a.f2 + b.f2))
     .print())
    env.execute("watermark figure")
    assert out == ["(k,7,1)", "(k,20,2)", "(k,53,4)", "(k,53,3)", "(k,63,3)"]


def test_bounded_out_of_orderness_reproduces_w11():
    a = BoundedOutOfOrdernessTimestampExtractor(Time.milliseconds(4), extractor=lambda ts: ts)
    for ts in STREAM[:5]:
        a.extract_timestamp(ts)
    assert a.get_current_watermark() == Watermark(11)
    for ts in STREAM[5:11]:
        a.extract_timestamp(ts)
    # The figure's second watermark is drawn at 17; a bound-4 periodic assigner would be at
    # 22 - 4 = 18 there: the figure's watermarks are punctuated, not derived from one bound.
    assert a.get_current_watermark() == Watermark(18)

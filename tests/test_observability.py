"""Metrics (Flink names + engine metrics, JSON lines / Prometheus text), stage timers, logging and
the engine configuration precedence."""
import json

import torch

from mxstream.api.environment import StreamExecutionEnvironment
from mxstream.ops import kernels as K
from mxstream.runtime.window_operator import KeyedWindowOperator
from mxstream.utils import metrics as M
from mxstream.utils.config import EngineConfig, apply_to_env, load_config, strip_conf_args
from mxstream.utils.log import get_logger


def test_registry_histogram_and_prometheus():
    r = M.MetricRegistry()
    c = r.counter("job.op.numRecordsIn")
    c.inc(5)
    h = r.histogram("job.op.alert_latency_ms")
    for v in range(1, 101):
        h.update(v)
    r.gauge("job.op.currentInputWatermark", lambda: 1234)
    snap = r.snapshot()
    assert snap["job.op.numRecordsIn"] == 5
    assert snap["job.op.alert_latency_ms"]["p50"] == 50 and snap["job.op.alert_latency_ms"]["p99"] == 99
    text = M.to_prometheus(r)
    assert 'mxs_numRecordsIn{job="job",operator="op"} 5.0' in text
    assert 'mxs_alert_latency_ms{job="job",operator="op",quantile="0.5"} 50' in text
    assert "# TYPE mxs_currentInputWatermark gauge" in text
    line = json.loads(M.to_json_line(r, step=3))
    assert line["step"] == 3 and line["metrics"]["job.op.numRecordsIn"] == 5


def test_operator_metrics_and_stage_timer():
    r = M.MetricRegistry()
    op = KeyedWindowOperator(size=1000, agg=K.AGG_SUM_I64, device="cpu", max_keys=1000,
                             batch_capacity=1000)
    M.register_operator("bench.window", op, r)
    op.timer = M.StageTimer("bench.window", "cpu", r)
    k = torch.arange(100, dtype=torch.int64) % 7
    t = torch.arange(100, dtype=torch.int64) * 30
    op.process(k, t, torch.ones(100, dtype=torch.int64))
    op.advance_watermark(10_000)
    snap = r.snapshot()
    assert snap["bench.window.numRecordsIn"] == 100
    assert snap["bench.window.currentInputWatermark"] == 10_000
    assert snap["bench.window.state_bytes_hbm"] > 0
    stages = M.stage_table(r, "bench.window")
    assert {"partition", "window_agg", "fire"} <= set(stages)


def test_job_counts_and_reporter(tmp_path):
    out = []
    env = StreamExecutionEnvironment(2)
    env.config.metrics_json = str(tmp_path / "m.jsonl")
    env.config.metrics_prometheus = str(tmp_path / "m.prom")
    env.from_collection(list(range(10))).map(lambda x: x * 2).filter(lambda x: x > 4).collect(out)
    res = env.execute("obs")
    assert res.metrics["Map.numRecordsIn"] == 10 and res.metrics["Filter.numRecordsOut"] == 7
    lines = (tmp_path / "m.jsonl").read_text().strip().splitlines()
    final = json.loads(lines[-1])
    assert final["final"] is True and final["job"] == "obs"
    assert any(k.endswith("numRecordsIn") for k in final["metrics"])
    assert "mxs_numRecordsIn" in (tmp_path / "m.prom").read_text()


def test_config_precedence(tmp_path):
    f = tmp_path / "c.yaml"
    f.write_text("parallelism: 3\nbatch_events: 4096\nlog_level: INFO\n")
    cfg = load_config(["--conf", "batch_events=8192", "x"],
                      env={"MXS_CONF_FILE": str(f), "MXS_LOG_LEVEL": "ERROR",
                           "MXS_CHECKPOINT_INTERVAL_MS": "250"})
    assert cfg.parallelism == 3            # file
    assert cfg.log_level == "ERROR"        # env beats file
    assert cfg.batch_events == 8192        # --conf beats both
    assert cfg.checkpoint_interval_ms == 250
    assert strip_conf_args(["--conf", "a=1", "job", "--conf=b=2", "9"]) == ["job", "9"]
    env = StreamExecutionEnvironment()
    cfg.checkpoint_dir = str(tmp_path)
    cfg.device = "cpu"
    apply_to_env(cfg, env)
    assert env.get_parallelism() == 3 and env.checkpoint_config.interval_ms == 250
    assert env.config.batch_size == 8192


def test_logger_layout(capsys):
    log = get_logger("test")
    log.error("hello %d", 7)
    err = capsys.readouterr().err
    assert "ERROR mxstream.test" in err and "hello 7" in err


def test_engine_config_defaults():
    c = EngineConfig()
    assert c.parallelism == 4 and c.max_parallelism == 128 and c.resolved_device() in ("cpu", "cuda")

"""Engine configuration.

The reference hard-codes everything (host/port, thresholds, window sizes, out-of-orderness,
timezone; ``main(args)`` ignores its arguments). mxstream keeps those defaults in the job code and
adds one engine configuration with a fixed precedence:

    defaults  <  config file (MXS_CONF_FILE: YAML or JSON)  <  MXS_<KEY> environment  <  --conf k=v

Keys (all optional):

| key | meaning | default |
|---|---|---|
| parallelism | logical subtasks of the DataStream API | 4 (README parity) |
| max_parallelism | key groups | 128 |
| device | cpu / cuda for native operators | cuda if available else cpu |
| batch_events | events per GPU per micro-batch | 16777216 |
| checkpoint_dir | checkpoint root (FsStateBackend path) | none |
| checkpoint_interval_ms | checkpoint period; <= 0 disables | -1 |
| checkpoints_retained | completed checkpoints kept | 1 |
| log_level | DEBUG / INFO / WARN / ERROR | WARN |
| metrics_json | JSON-lines metrics file | none |
| metrics_prometheus | Prometheus text file (rewritten each report) | none |
| metrics_interval_ms | reporter period | 1000 |
| fault | fault injection spec "op:records[:attempts]" | none |
| host_budget_bytes | host-DRAM budget of spilled session state (exceeding it fails the job) | unlimited |
| trace_path | Chrome-trace JSON of the job's stage spans (utils/trace.py) | none |
| step_timeout_ms | watchdog: a DAG pass slower than this fails the job (runtime/health.py) | off |
"""
from __future__ import annotations

import json
import os
from dataclasses import asdict, dataclass, fields


@dataclass
class EngineConfig:
    parallelism: int = 4
    max_parallelism: int = 128
    device: str = "auto"
    batch_events: int = 1 << 24
    checkpoint_dir: str | None = None
    checkpoint_interval_ms: int = -1
    checkpoints_retained: int = 1
    log_level: str = "WARN"
    metrics_json: str | None = None
    metrics_prometheus: str | None = None
    metrics_interval_ms: int = 1000
    fault: str | None = None
    host_budget_bytes: int | None = None
    trace_path: str | None = None
    step_timeout_ms: int = 0

    def resolved_device(self) -> str:
        if self.device != "auto":
            return self.device
        import torch

        return "cuda" if torch.cuda.is_available() else "cpu"

    def as_dict(self) -> dict:
        return asdict(self)


def _coerce(name: str, raw):
    f = {x.name: x for x in fields(EngineConfig)}.get(name)
    if f is None:
        raise KeyError(f"unknown config key {name!r}")
    if raw is None or not isinstance(raw, str):
        return raw
    t = str(f.type)
    if raw.lower() in ("none", "null", ""):
        return None
    if "bool" in t:
        return raw.lower() in ("1", "true", "yes", "on")
    if "int" in t:
        return int(raw)
    return raw


def load_config(argv: list[str] | None = None, env: dict | None = None) -> EngineConfig:
    """Build the effective configuration; `argv` may contain `--conf k=v` pairs (other arguments
    are ignored and left to the caller)."""
    env = os.environ if env is None else env
    cfg = EngineConfig()
    path = env.get("MXS_CONF_FILE")
    if path:
        with open(path) as f:
            text = f.read()
        if path.endswith((".yaml", ".yml")):
            import yaml

            data = yaml.safe_load(text) or {}
        else:
            data = json.loads(text)
        for k, v in data.items():
            setattr(cfg, k, _coerce(k, v if not isinstance(v, (int, float, bool)) else v))
    for f in fields(EngineConfig):
        v = env.get("MXS_" + f.name.upper())
        if v is not None:
            setattr(cfg, f.name, _coerce(f.name, v))
    args = list(argv or [])
    for i, a in enumerate(args):
        kv = None
        if a == "--conf" and i + 1 < len(args):
            kv = args[i + 1]
        elif a.startswith("--conf="):
            kv = a[len("--conf="):]
        if kv is not None:
            k, _, v = kv.partition("=")
            setattr(cfg, k.strip(), _coerce(k.strip(), v.strip()))
    return cfg


def strip_conf_args(argv: list[str]) -> list[str]:
    out, skip = [], False
    for i, a in enumerate(argv):
        if skip:
            skip = False
            continue
        if a == "--conf":
            skip = True
            continue
        if a.startswith("--conf="):
            continue
        out.append(a)
    return out


def apply_to_env(cfg: EngineConfig, env) -> None:
    """Apply an EngineConfig to a StreamExecutionEnvironment."""
    env.set_parallelism(cfg.parallelism)
    env.set_max_parallelism(cfg.max_parallelism)
    env.config.device = cfg.resolved_device()
    env.config.batch_size = cfg.batch_events
    env.config.fault_injection = cfg.fault
    env.config.metrics_json = cfg.metrics_json
    env.config.metrics_prometheus = cfg.metrics_prometheus
    env.config.metrics_interval_ms = cfg.metrics_interval_ms
    if cfg.trace_path:
        env.config.trace_path = cfg.trace_path
    if cfg.step_timeout_ms:
        env.config.step_timeout_ms = cfg.step_timeout_ms
    if cfg.checkpoint_interval_ms and cfg.checkpoint_interval_ms > 0:
        env.enable_checkpointing(cfg.checkpoint_interval_ms)
        env.checkpoint_config.checkpoint_dir = cfg.checkpoint_dir
        env.checkpoint_config.max_retained = cfg.checkpoints_retained
    from .log import set_level

    set_level(cfg.log_level)

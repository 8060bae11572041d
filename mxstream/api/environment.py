"""StreamExecutionEnvironment (Flink 1.8 ``streaming.api.environment``).

``getExecutionEnvironment()`` returns a local environment whose default parallelism matches the
reference's observed runs (4 subtasks: the README ``N>`` prefixes) unless set.
``execute(name)`` builds the DAG and runs it on the micro-batch executor (host operators for
arbitrary Python functions, native CPU/GPU operators for the recognised hot shapes).
Reference: Main.java:16,34 and the first/last line of every job.
"""
from __future__ import annotations

import os
import sys
from dataclasses import dataclass, field

from ..runtime.executor import Executor, ManualClock, SystemClock, Transformation
from ..runtime import sources as S
from ..utils.hashing import default_max_parallelism
from .datastream import DataStream, _ids
from .time import TimeCharacteristic, to_ms


@dataclass
class ExecutionConfig:
    auto_watermark_interval: int = 0        # ms; set to 200 by EventTime (Flink default)
    rebalance_start: int = 0                # first channel of round-robin rebalance
    native: str = "auto"                    # auto | off | force  (native keyed operators)
    # cpu | cuda: where native operators run (MXS_DEVICE overrides the default)
    device: str = field(default_factory=lambda: os.environ.get("MXS_DEVICE", "cpu"))
    batch_size: int = 1 << 16
    # Text jobs whose parse map traces (api/textplan.py): "device" parses on `device` with the
    # device string dictionary (ops/ingest.py; the C++ twins when device is "cpu"), "host" with
    # the multi-threaded host parser, "auto" = device on a GPU. MXS_TEXT_INGEST overrides.
    text_ingest: str = field(default_factory=lambda: os.environ.get("MXS_TEXT_INGEST", "auto"))
    # Device ingest, one rank: read each batch's parse result one pass later (the host's work on
    # batch i overlaps the GPU's parse of batch i + 1). Applied only where a pass's delay cannot
    # be observed (planner._defer_safe); MXS_INGEST_DEFER=0 turns it off.
    ingest_defer: bool = field(default_factory=lambda: os.environ.get("MXS_INGEST_DEFER", "1") != "0")
    # Native keyed windows over dictionary ids: dense id-addressed HBM state up to this many
    # ids; a dictionary that outgrows it moves the state to hashed keys with the host-DRAM tier
    # (cold keys leave HBM). MXS_WINDOW_DENSE_MAX_KEYS.
    window_dense_max_keys: int = field(default_factory=lambda: int(
        os.environ.get("MXS_WINDOW_DENSE_MAX_KEYS", str(1 << 27))))
    global_job_parameters: dict = field(default_factory=dict)
    # "<operator name>:<records>[:<attempts>]" (tests / chaos runs); default from MXS_FAULT.
    fault_injection: str | None = field(default_factory=lambda: os.environ.get("MXS_FAULT"))
    metrics_json: str | None = field(default_factory=lambda: os.environ.get("MXS_METRICS_JSON"))
    metrics_prometheus: str | None = field(
        default_factory=lambda: os.environ.get("MXS_METRICS_PROMETHEUS"))
    metrics_interval_ms: int = 1000
    # Chrome-trace JSON of the job's stage spans (utils/trace.py); MXS_TRACE_PATH.
    trace_path: str | None = field(default_factory=lambda: os.environ.get("MXS_TRACE_PATH"))
    # Failure detection (runtime/health.py): a pass over the DAG taking longer than this fails
    # the job with StepTimeout (restartable like any failure); <= 0 disables. MXS_STEP_TIMEOUT_MS.
    step_timeout_ms: int = field(
        default_factory=lambda: int(os.environ.get("MXS_STEP_TIMEOUT_MS", "0")))

    def set_auto_watermark_interval(self, ms: int) -> "ExecutionConfig":
        self.auto_watermark_interval = int(ms)
        return self

    def get_auto_watermark_interval(self) -> int:
        return self.auto_watermark_interval

    def set_global_job_parameters(self, params: dict) -> None:
        self.global_job_parameters = dict(params)

    setAutoWatermarkInterval = set_auto_watermark_interval
    getAutoWatermarkInterval = get_auto_watermark_interval


@dataclass
class CheckpointConfig:
    interval_ms: int = -1
    mode: str = "EXACTLY_ONCE"
    checkpoint_dir: str | None = None
    max_retained: int = 1
    externalized: bool = False

    def is_checkpointing_enabled(self) -> bool:
        return self.interval_ms > 0


class MemoryStateBackend:
    """Flink's default: keyed state on the heap (host operators) / in HBM (native operators);
    checkpoints need a directory set on the CheckpointConfig."""

    checkpoint_path: str | None = None


class FsStateBackend(MemoryStateBackend):
    """Checkpoints to `<checkpoint_path>/<jobId>/chk-<n>/` (Flink FsStateBackend layout)."""

    def __init__(self, checkpoint_path: str):
        self.checkpoint_path = str(checkpoint_path)


class HbmStateBackend(FsStateBackend):
    """MI355X engine backend: keyed state in HBM hash tables, cold state spilled to host DRAM
    (up to `host_budget_bytes`), checkpoints under `checkpoint_path`."""

    def __init__(self, checkpoint_path: str, spill_dir: str | None = None,
                 host_budget_bytes: int | None = None):
        super().__init__(checkpoint_path)
        self.spill_dir = spill_dir
        self.host_budget_bytes = host_budget_bytes


class RestartStrategies:
    @staticmethod
    def no_restart():
        return ("none",)

    @staticmethod
    def fixed_delay_restart(attempts: int, delay_ms: int):
        return ("fixed_delay", int(attempts), int(delay_ms))

    noRestart = no_restart
    fixedDelayRestart = fixed_delay_restart


class _StdoutWriter:
    """print() sink target: one line per call, or a whole column batch in one write."""

    def __call__(self, s: str) -> None:
        print(s, flush=True)

    @staticmethod
    def many(lines: list) -> None:
        if lines:
            sys.stdout.write("\n".join(lines) + "\n")
            sys.stdout.flush()

    @staticmethod
    def raw(data: bytes, nlines: int | None = None) -> None:
        """A column batch already formatted as `nlines` newline-terminated lines (native
        formatter)."""
        if data:
            buf = getattr(sys.stdout, "buffer", None)
            if buf is None:  # a text-only stream (captured stdout)
                sys.stdout.write(bytes(data).decode())
                sys.stdout.flush()
                return
            sys.stdout.flush()
            buf.write(data)
            buf.flush()


class StreamExecutionEnvironment:
    DEFAULT_PARALLELISM = 4

    def __init__(self, parallelism: int | None = None, clock=None):
        env_p = os.environ.get("MXS_PARALLELISM")
        self.parallelism = parallelism or (int(env_p) if env_p else self.DEFAULT_PARALLELISM)
        self._max_parallelism: int | None = None
        self.time_characteristic = TimeCharacteristic.ProcessingTime
        self.config = ExecutionConfig()
        self.checkpoint_config = CheckpointConfig()
        self.restart_strategy = RestartStrategies.no_restart()
        self.clock = clock or SystemClock()
        self._sinks: list[Transformation] = []
        self._writer = _StdoutWriter()
        self.rank = int(os.environ.get("RANK", "0"))
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.state_backend = None

    # ---- construction ----
    @staticmethod
    def get_execution_environment(parallelism: int | None = None) -> "StreamExecutionEnvironment":
        return StreamExecutionEnvironment(parallelism)

    @staticmethod
    def create_local_environment(parallelism: int | None = None, clock=None) -> "StreamExecutionEnvironment":
        return StreamExecutionEnvironment(parallelism, clock)

    # ---- configuration ----
    def set_parallelism(self, p: int) -> "StreamExecutionEnvironment":
        if p < 1:
            raise ValueError("parallelism must be at least one")
        self.parallelism = int(p)
        return self

    def get_parallelism(self) -> int:
        return self.parallelism

    def set_max_parallelism(self, p: int) -> "StreamExecutionEnvironment":
        if not 0 < p <= 32768:
            raise ValueError("maxParallelism must be in (0, 32768]")
        self._max_parallelism = int(p)
        return self

    @property
    def max_parallelism(self) -> int:
        return self._max_parallelism or default_max_parallelism(self.parallelism)

    def get_max_parallelism(self) -> int:
        return self.max_parallelism

    def set_stream_time_characteristic(self, tc: TimeCharacteristic) -> None:
        self.time_characteristic = tc
        if tc == TimeCharacteristic.ProcessingTime:
            self.config.auto_watermark_interval = 0
        elif self.config.auto_watermark_interval == 0:
            self.config.auto_watermark_interval = 200

    def get_stream_time_characteristic(self) -> TimeCharacteristic:
        return self.time_characteristic

    def get_config(self) -> ExecutionConfig:
        return self.config

    def enable_checkpointing(self, interval_ms: int, mode: str = "EXACTLY_ONCE") -> "StreamExecutionEnvironment":
        self.checkpoint_config.interval_ms = int(interval_ms)
        self.checkpoint_config.mode = mode
        return self

    def get_checkpoint_config(self) -> CheckpointConfig:
        return self.checkpoint_config

    def set_restart_strategy(self, strategy) -> None:
        self.restart_strategy = strategy

    def set_state_backend(self, backend) -> "StreamExecutionEnvironment":
        self.state_backend = backend
        return self

    def set_clock(self, clock) -> "StreamExecutionEnvironment":
        """Inject a processing-time clock (ManualClock in tests)."""
        self.clock = clock
        return self

    def set_output(self, writer) -> "StreamExecutionEnvironment":
        """Where print() writes lines (default: stdout)."""
        self._writer = writer
        return self

    # ---- sources ----
    def _source(self, name: str, factory, text: bool = False) -> DataStream:
        t = Transformation(next(_ids), name, "source", [], factory, 1)
        # text: the source can emit raw line batches (planner: columnar text ingest)
        t.meta = {"kind": "source", "text": text}
        return DataStream(self, t)

    def socket_text_stream(self, hostname: str, port: int, delimiter: str = "\n",
                           max_retry: int = 0) -> DataStream:
        return self._source("Socket Stream",
                            lambda: S.SocketTextSource(hostname, port, delimiter, max_retry),
                            text=delimiter == "\n")

    def from_collection(self, values, batch_size: int | None = None) -> DataStream:
        vals = list(values)
        return self._source("Collection Source", lambda: S.CollectionSource(vals, batch_size),
                            text=bool(vals) and all(isinstance(v, str) and "\n" not in v
                                                    for v in vals))

    def from_elements(self, *values) -> DataStream:
        return self.from_collection(values)

    def from_timed_collection(self, timed, end_time: int | None = None) -> DataStream:
        """[(processing_time_ms, value), ...] arriving one per micro-batch at those times."""
        items = list(timed)
        return self._source("Timed Source", lambda: S.TimedCollectionSource(items, end_time),
                            text=bool(items) and all(isinstance(v, str) and "\n" not in v
                                                     for _, v in items))

    def read_text_file(self, path: str) -> DataStream:
        return self._source("Text File Source", lambda: S.TextFileSource(path, self.config.batch_size),
                            text=True)

    def generate_sequence(self, start: int, end: int) -> DataStream:
        return self._source("Sequence Source", lambda: S.SequenceSource(start, end))

    def add_source(self, fn, name: str = "Custom Source") -> DataStream:
        return self._source(name, lambda: S.FunctionSource(fn))

    # ---- execution ----
    def get_stream_graph(self) -> list[Transformation]:
        return Executor._topo(self._sinks)

    def get_execution_plan(self) -> str:
        import json

        nodes = [{"id": t.id, "type": t.name, "pact": t.kind,
                  "parallelism": t.parallelism or (1 if t.kind == "source" else self.parallelism),
                  "predecessors": [p.id for p in t.parents]} for t in self.get_stream_graph()]
        return json.dumps({"nodes": nodes}, indent=2)

    def execute(self, job_name: str = "Flink Streaming Job"):
        if not self._sinks:
            raise RuntimeError("No operators defined in streaming topology. Cannot execute.")
        from .planner import plan

        import secrets

        sinks = plan(self, list(self._sinks))
        job_id = secrets.token_hex(16)
        comm = getattr(self, "_comm", None)  # injected (LoopbackComm: virtual ranks in tests)
        if comm is not None:
            self.rank, self.world = comm.rank, comm.world
            job_id = comm.broadcast_object(job_id, src=0)
        elif getattr(self, "world", 1) > 1:
            # All ranks of a multi-process job share one job id (checkpoint directory).
            from ..parallel.comm import init_distributed

            job_id = init_distributed("cpu").broadcast_object(job_id, src=0)
        attempts = 0
        restore = None
        while True:
            try:
                result = Executor(self, sinks, job_name, job_id=job_id, restore_from=restore,
                                  attempt=attempts, comm=comm).run()
                break
            except Exception as e:
                kind = self.restart_strategy[0]
                if kind == "fixed_delay" and attempts < self.restart_strategy[1]:
                    attempts += 1
                    from ..utils.log import get_logger

                    get_logger("api.environment").warning(
                        "Job %s failed (%s: %s); restart %d of %d", job_name, type(e).__name__, e,
                        attempts, self.restart_strategy[1])
                    import time as _t

                    _t.sleep(self.restart_strategy[2] / 1000.0)
                    # Restart from the latest completed checkpoint (replayable sources rewind to
                    # their checkpointed offsets); without checkpoints the job starts over.
                    restore = None
                    if self.checkpoint_config.is_checkpointing_enabled():
                        from ..runtime.checkpoint import CheckpointStorage

                        root = (self.checkpoint_config.checkpoint_dir
                                or getattr(self.state_backend, "checkpoint_path", None))
                        restore = CheckpointStorage(root, job_id).latest()
                    continue
                raise
        result.metrics["numRestarts"] = attempts
        self._sinks = []
        return result

    def execute_from_savepoint(self, path: str, job_name: str = "Flink Streaming Job"):
        """Run the job graph starting from a checkpoint/savepoint directory (`flink run -s`)."""
        from .planner import plan

        sinks = plan(self, list(self._sinks))
        comm = getattr(self, "_comm", None)  # injected (LoopbackComm: virtual ranks in tests)
        if comm is not None:
            self.rank, self.world = comm.rank, comm.world
        # The checkpoint may come from another world size: the executor re-splits keyed state
        # by key group and source positions by partition (checkpoint.read_host_checkpoint).
        result = Executor(self, sinks, job_name, restore_from=path, comm=comm).run()
        self._sinks = []
        return result

    # camelCase aliases
    getExecutionEnvironment = get_execution_environment
    createLocalEnvironment = create_local_environment
    setParallelism = set_parallelism
    getParallelism = get_parallelism
    setMaxParallelism = set_max_parallelism
    getMaxParallelism = get_max_parallelism
    setStreamTimeCharacteristic = set_stream_time_characteristic
    getStreamTimeCharacteristic = get_stream_time_characteristic
    getConfig = get_config
    enableCheckpointing = enable_checkpointing
    getCheckpointConfig = get_checkpoint_config
    setRestartStrategy = set_restart_strategy
    setStateBackend = set_state_backend
    socketTextStream = socket_text_stream
    fromCollection = from_collection
    fromElements = from_elements
    readTextFile = read_text_file
    generateSequence = generate_sequence
    addSource = add_source
    getExecutionPlan = get_execution_plan


_ = (sys, to_ms, ManualClock)

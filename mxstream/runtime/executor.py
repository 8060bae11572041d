"""Micro-batch executor of a DataStream job graph (replaces Flink's StreamGraph -> JobGraph ->
MiniCluster path).

The job is a DAG of transformations. Each *tick*: every source is polled once (one micro-batch),
its records are pushed through the DAG in topological order, each operator receives its inputs'
items (records and watermarks in stream order), and processing-time timers up to the clock's
``now`` fire. After the last tick, event-time jobs see ``Long.MAX_VALUE`` (end of input fires all
event-time windows); processing-time windows are not fired at end of input (Flink 1.8).

Multi-rank (``torchrun`` with WORLD_SIZE > 1, one process per GPU): every rank runs the same
graph on its source partition. Every tick is step-synchronous across ranks: a keyed edge
(an operator built on a KeyedStream) exchanges its records so that each key group's records
reach the rank that owns it. Subtask s of P lives on rank s * world // P, like the engine
operators' key-group map. Watermarks crossing a keyed edge are merged to the minimum over the
ranks, like Flink's minimum over input channels. A parallelism-1 operator (windowAll) gathers
its input on rank 0. The job ends when every rank's sources are finished. The record exchange
runs over the gloo process group with pickled records; it is the host-level data path. The
engines' GPU-scale exchange is the RCCL all-to-all inside the keyed operators (bench path).
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import Any, Callable

from ..utils import trace
from ..utils.log import get_logger
from .health import StepTimeout, Watchdog
from .operators import LONG_MAX, OpContext, Operator, Rec, UnionOp, WM
from .sources import Source

log = get_logger("runtime.executor")


class ManualClock:
    """Injectable processing-time clock (Flink's TestProcessingTimeService analogue)."""

    def __init__(self, start: int = 0):
        self.now = int(start)

    def __call__(self) -> int:
        return self.now

    def advance_to(self, t: int) -> None:
        self.now = max(self.now, int(t))


class SystemClock:
    def __call__(self) -> int:
        return int(time.time() * 1000)


@dataclass
class Transformation:
    id: int
    name: str
    kind: str                          # source | op | union | side | sink
    parents: list = field(default_factory=list)
    factory: Callable[[], Any] | None = None   # -> Operator (or Source for kind=source)
    parallelism: int | None = None
    side_tag: Any = None
    uid: str | None = None
    meta: dict = field(default_factory=dict)   # planner hints (op kind, user fn, window spec)
    key_fn_in: Any = None              # set when the input is a KeyedStream (hash-partitioned edge)

    def __hash__(self):
        return self.id


class JobExecutionResult:
    def __init__(self, job_name: str, runtime_ms: float, metrics: dict):
        self.job_name = job_name
        self.net_runtime_ms = runtime_ms
        self.metrics = metrics

    def get_net_runtime(self) -> float:
        return self.net_runtime_ms

    getNetRuntime = get_net_runtime


class JobExecutionException(RuntimeError):
    """Job failed (no restart strategy): wraps the user/operator exception."""


class InjectedFault(RuntimeError):
    """Raised by the fault injector (``MXS_FAULT`` / ExecutionConfig.fault_injection)."""


def parse_fault(spec: str | None):
    """"<operator name substring>:<records>[:<attempts>]" -> (name, n, attempts) or None.
    The fault fires when the operator has received `records` records, on the first `attempts`
    executions of the job (default 1: the restarted job runs clean)."""
    if not spec:
        return None
    parts = spec.split(":")
    if len(parts) not in (2, 3):
        raise ValueError(f"bad fault spec {spec!r} (name:records[:attempts])")
    return parts[0], int(parts[1]), int(parts[2]) if len(parts) == 3 else 1


class Executor:
    """Micro-batch DAG executor. Checkpoints are step-aligned: taken between two passes over the
    DAG, when no record is in flight (every pass drains the inboxes to the sinks), so operator
    snapshots plus source positions form a consistent cut -- Flink's aligned barrier without
    alignment buffering. Layout: runtime/checkpoint.py (chk-<n>/_metadata + one state file per
    operator)."""

    def __init__(self, env, sinks: list[Transformation], job_name: str, *, job_id: str | None = None,
                 restore_from=None, attempt: int = 0, comm=None):
        self.env = env
        self.job_name = job_name
        self.job_id = job_id
        self.restore_from = restore_from
        self.attempt = attempt
        self.fault = parse_fault(getattr(env.config, "fault_injection", None))
        self._fault_count = 0
        self._counts: dict[int, dict[str, int]] = {}
        self.nodes = self._topo(sinks)
        self.children: dict[int, list[Transformation]] = {n.id: [] for n in self.nodes}
        for n in self.nodes:
            for p in n.parents:
                self.children[p.id].append(n)
        self.clock = env.clock
        self.ops: dict[int, Any] = {}
        self.metrics: dict[str, int] = {}
        self._rr: dict = {}
        self._trace = False
        self.comm = None
        self._wm_in: dict = {}  # keyed node -> latest watermark received from every rank
        self._failure: Exception | None = None  # multi-rank: first operator failure of this rank
        self.dev_comm = None  # device collectives of the native operators (G > 1)
        self._step_now = None  # G > 1: the step's agreed processing time (_step_begin)
        if comm is not None and comm.world > 1:
            # Injected communicator (LoopbackComm: G virtual ranks in one process, tests).
            self.comm = self.dev_comm = comm
        elif getattr(env, "world", 1) > 1:
            import os

            import torch

            from ..parallel.comm import TorchComm, init_distributed

            cuda = str(env.config.device).startswith("cuda") and torch.cuda.is_available()
            if cuda:
                torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))  # one GPU per rank
            self.comm = init_distributed("cpu")
            if cuda:
                # Device tensors of the native operators travel over RCCL (xGMI); host objects
                # (records, control) over the gloo group.
                import torch.distributed as dist

                self.dev_comm = TorchComm(dist.new_group(backend="nccl"))
            else:
                self.dev_comm = self.comm

    @staticmethod
    def _topo(sinks):
        seen, order = set(), []

        def visit(t):
            if t.id in seen:
                return
            seen.add(t.id)
            for p in t.parents:
                visit(p)
            order.append(t)

        for s in sinks:
            visit(s)
        return order

    # ------------------------------------------------------------------------------------
    def _open(self):
        env = self.env
        tc = env.time_characteristic.value
        for n in self.nodes:
            p = n.parallelism or env.parallelism
            if n.kind == "source":
                src: Source = n.factory()
                if self.comm is not None and hasattr(type(src), "comm"):
                    src.comm = self.comm  # K18: the source spreads its batches over the ranks
                src.open(env.rank, env.world, self.clock)
                self.ops[n.id] = src
            elif n.kind == "union":
                op = UnionOp(len(n.parents))
                op.open(OpContext(n.name, p, env.max_parallelism, self.clock, tc))
                self.ops[n.id] = op
            elif n.kind == "side":
                op = Operator()
                op.open(OpContext(n.name, p, env.max_parallelism, self.clock, tc))
                self.ops[n.id] = op
            else:
                op = n.factory()
                op.open(OpContext(n.name, p, env.max_parallelism, self._op_clock, tc,
                                  comm=self.dev_comm, ctrl=self.comm))
                self.ops[n.id] = op

    def _push(self, inbox: dict[int, list], now: int | None) -> None:
        """One pass over the DAG in topological order."""
        from .columnar import expand_columns, rows_in

        for n in self.nodes:
            if n.kind == "source":
                out = inbox.pop(n.id, [])
            elif n.kind == "union":
                op: UnionOp = self.ops[n.id]
                out = []
                for idx, p in enumerate(n.parents):
                    out.extend(op.process_input(idx, inbox.pop((n.id, p.id), [])))
            else:
                items = []
                for p in n.parents:
                    items.extend(inbox.pop((n.id, p.id), []))
                op = self.ops[n.id]
                if self.comm is not None:
                    items = self._exchange(n, items)
                if self.comm is not None:
                    # Multi-rank: a failing operator must not leave the other ranks blocked in
                    # this pass's exchanges. The rank records the failure, keeps joining the
                    # collectives with no work, and every rank learns it at the step's control
                    # gather (_control) and fails together -> coordinated restart.
                    if self._failure is not None:
                        items = []
                    try:
                        out = self._run_op(n, op, items, now)
                    except Exception as e:  # noqa: BLE001 -- re-raised by _control
                        self._record_failure(e)
                        out = []
                else:
                    out = self._run_op(n, op, items, now)
                if items or out:
                    c = self._counts.setdefault(n.id, {"numRecordsIn": 0, "numRecordsOut": 0})
                    c["numRecordsIn"] += rows_in(items)
                    c["numRecordsOut"] += rows_in(out)
            for c in self.children[n.id]:
                if c.kind == "side":
                    side = [it for it in self.ops[n.id].take_side(c.side_tag.tag_id)] \
                        if n.kind not in ("source", "union") else []
                    side = side + [it for it in out if isinstance(it, WM)]
                    inbox.setdefault((c.id, n.id), []).extend(side)
                else:
                    inbox.setdefault((c.id, n.id), []).extend(out)

    def _run_op(self, n: Transformation, op, items: list, now: int | None) -> list:
        from .columnar import expand_columns

        if not getattr(op, "accepts_columns", False):
            items = expand_columns(items)
        if self.fault is not None and items:
            self._maybe_fault(n, items)
        # Collective operators (multi-rank device exchange) run every pass, with or without
        # input: each call is one step of their collectives on every rank.
        run = bool(items) or getattr(op, "collective", False)
        if run and self._trace:
            with trace.span(n.name, "operator"):
                out = op.process(items)
        else:
            out = op.process(items) if run else []
        if now is not None:
            out.extend(op.on_processing_time(now))
        return out

    def _record_failure(self, e: Exception) -> None:
        """Multi-rank: keep the first failure of this rank for the next _control (which raises
        it on every rank); single rank: raise right away."""
        if self.comm is None:
            raise e
        if self._failure is None:
            self._failure = e

    def _control(self, want_ckpt: bool) -> bool:
        """End-of-step agreement between ranks: a failure anywhere fails every rank (the
        restart strategy then restarts all of them from the same checkpoint), and a checkpoint
        is taken when any rank's interval elapsed (ranks' clocks need not agree). Multi-rank:
        one packed int64 all-reduce (control_reduce); the failure text moves only when a rank
        failed."""
        if self.comm is None:
            return want_ckpt
        from ..parallel.comm import control_reduce

        _, (want, failed) = control_reduce(self.comm, maxs=[int(want_ckpt),
                                                            int(self._failure is not None)])
        if failed:
            self._raise_agreed_failure()
        return bool(want)

    def _raise_agreed_failure(self) -> None:
        """Some rank failed (agreed by the control all-reduce): gather the failure texts (the
        only object collective of the control plane) and fail every rank."""
        got = self.comm.all_gather_object(None if self._failure is None else
                                          f"{type(self._failure).__name__}: {self._failure}")
        failed = [(r, f) for r, f in enumerate(got) if f is not None]
        if self._failure is not None:
            raise self._failure
        raise JobExecutionException(f"Job '{self.job_name}' failed on rank(s) "
                                    f"{[r for r, _ in failed]}: {failed[0][1] if failed else '?'}")

    # ---- multi-rank exchange ---------------------------------------------------------------
    def _exchange(self, n: Transformation, items: list) -> list:
        """Route this rank's input items of node n to their owner ranks (keyed edge: the key's
        subtask; parallelism 1: rank 0; anything else stays). Collective: every rank calls it for
        every node in the same order, with or without items."""
        from ..utils.hashing import flink_murmur, java_hash
        from .columnar import expand_columns

        world, rank = self.comm.world, self.comm.rank
        p = n.parallelism or self.env.parallelism
        keyed = n.key_fn_in is not None
        if not keyed and p != 1:
            return items
        if keyed and getattr(self.ops.get(n.id), "device_exchange", False):
            # The operator exchanges its keys itself (RCCL all-to-all inside the native keyed
            # operator): its data stays on this rank; only the watermarks are merged here.
            data = [it for it in items if not isinstance(it, WM)]
            wms = [it.ts for it in items if isinstance(it, WM)]
            return data + self._merge_watermarks(n, wms[-1] if wms else None)
        mp = self.env.max_parallelism
        outs: list[list] = [[] for _ in range(world)]
        last_wm = None
        try:
            for it in expand_columns(items):
                if isinstance(it, WM):
                    last_wm = it.ts
                    continue
                if not isinstance(it, Rec):
                    outs[rank].append(it)
                    continue
                if keyed:
                    sub = (flink_murmur(java_hash(n.key_fn_in(it.value))) % mp) * p // mp
                    outs[sub * world // p].append(it)
                else:
                    outs[0].append(it)
        except Exception as e:  # noqa: BLE001 -- a user key selector failed: agreed in _control
            self._record_failure(e)
            outs, last_wm = [[] for _ in range(world)], None
        from ..parallel.exchange import NotExchangeable, exchange_records

        # Typed, code-free columnar exchange (statecodec words through exchange_rows): each rank
        # receives only its own records. Values without a typed encoding (arbitrary user objects)
        # make every rank fall back to the object collective together.
        try:
            recv, wms = exchange_records(self.comm, outs, last_wm)
            return recv + self._merge_watermarks(n, last_wm, wms)
        except NotExchangeable:
            self.metrics["objectExchangeFallbacks"] = self.metrics.get("objectExchangeFallbacks", 0) + 1
        got = self.comm.all_gather_object((outs, last_wm))
        recv: list = []
        for r_outs, _ in got:
            recv.extend(r_outs[rank])
        return recv + self._merge_watermarks(n, last_wm, [w for _, w in got])

    def _merge_watermarks(self, n: Transformation, last_wm, got_wms=None) -> list:
        """Watermarks across a keyed edge: the minimum over the ranks of the latest watermark
        each one has sent (Flink's StatusWatermarkValve over the input channels). Without
        `got_wms` (device-exchange edges) this is collective: each rank keeps the max of what it
        sent and one MIN all-reduce of (sent anything?, that max) gives the valve's minimum."""
        world = self.comm.world
        if got_wms is None:
            from ..parallel.comm import I64_MIN, control_reduce

            mine = self._wm_in.get((n.id, "self"))
            if last_wm is not None:
                mine = last_wm if mine is None else max(mine, last_wm)
                self._wm_in[(n.id, "self")] = mine
            (has, low), _ = control_reduce(self.comm, mins=[int(mine is not None),
                                                            I64_MIN if mine is None else mine])
            if not has:
                return []
            wm = low
        else:
            seen = self._wm_in.setdefault(n.id, [None] * world)
            for r, w in enumerate(got_wms):
                if w is not None:
                    seen[r] = w if seen[r] is None else max(seen[r], w)
            if not all(w is not None for w in seen):
                return []
            wm = min(seen)
        prev = self._wm_in.get((n.id, "emitted"))
        if prev is None or wm > prev:
            self._wm_in[(n.id, "emitted")] = wm
            return [WM(wm)]
        return []

    def _op_clock(self) -> int:
        """Processing time as operators see it: one rank reads its clock; several ranks read the
        step's agreed time (_step_begin), so every rank stamps and fires the same windows."""
        if self.comm is None or self._step_now is None:
            return self.clock()
        return self._step_now

    def _step_begin(self, finished: dict, sources: list, manual: bool,
                    want_ckpt: bool = False) -> tuple[bool, int]:
        """(every source finished on every rank, the step's processing time). Multi-rank: ONE
        packed int64 all-reduce per pass (parallel/comm.control_reduce) carries done (MIN),
        the clock (MAX: the step's time, which a manual clock advances to), and the previous
        pass's control words -- checkpoint request and failure flag (MAX). A failure fails
        every rank here; a requested checkpoint is taken here, at the cut between the previous
        pass and this one, before the clock moves."""
        nxt_t = None
        if manual:
            nxt = [self.ops[n.id].next_event_time() for n in sources if not finished[n.id]]
            nxt = [t for t in nxt if t is not None]
            if nxt:
                nxt_t = min(nxt)
        done = all(finished.values())
        if self.comm is None:
            if nxt_t is not None:
                self.clock.advance_to(nxt_t)
            return done, self.clock()
        from ..parallel.comm import control_reduce

        now = self.clock() if nxt_t is None else max(self.clock(), nxt_t)
        (all_done,), (now, want, failed) = control_reduce(
            self.comm, mins=[int(done)],
            maxs=[now, int(want_ckpt), int(self._failure is not None)])
        if failed:
            self._raise_agreed_failure()
        if want:
            self._checkpoint(finished)
            self._last_ckpt = self.clock()
        if manual:
            self.clock.advance_to(now)
        self._step_now = now
        return bool(all_done), now

    # ---- checkpoints ---------------------------------------------------------------------
    def _storage(self):
        from .checkpoint import CheckpointStorage

        cfg = self.env.checkpoint_config
        root = cfg.checkpoint_dir or getattr(self.env.state_backend, "checkpoint_path", None)
        if root is None:
            raise ValueError("checkpointing needs a directory: set_state_backend(FsStateBackend(path))"
                             " or get_checkpoint_config().checkpoint_dir")
        return CheckpointStorage(root, self.job_id)

    def _checkpoint(self, finished: dict) -> None:
        from .checkpoint import write_host_checkpoint, write_host_states

        t0 = time.perf_counter()
        storage = self._storage()
        storage.init_job_dirs()
        n = self._next_ckpt

        def snap_all():
            return {self._uid(nd): self.ops[nd.id].snapshot() for nd in self.nodes
                    if nd.id in self.ops}

        extra = {
            "clock": self.clock() if isinstance(self.clock, ManualClock) else None,
            "rr": [[self._uid(self._node[a]), self._uid(self._node[b]), v]
                   for (a, b), v in self._rr.items()],
            "finished": {self._uid(nd): finished[nd.id] for nd in self.nodes if nd.id in finished},
            "nodes": {self._uid(nd): nd.name for nd in self.nodes}}
        d = storage.checkpoint_dir(n)
        if self.comm is None:
            write_host_checkpoint(d, job_id=storage.job_id, checkpoint_id=n, states=snap_all(),
                                  extra=extra)
        else:
            # Every rank writes its own state files; rank 0 completes the checkpoint (_metadata)
            # once all of them have, so a crash mid-write leaves no completed checkpoint.
            try:
                files, err = write_host_states(d, snap_all(), self.comm.rank), None
            except Exception as e:  # noqa: BLE001 -- agreed on below, raised on every rank
                files, err = None, f"{type(e).__name__}: {e}"
            ranks = self.comm.all_gather_object({"host_operators": files, "extra": extra,
                                                 "error": err})
            bad = [(r, x["error"]) for r, x in enumerate(ranks) if x.get("error")]
            if bad:
                raise JobExecutionException(f"Job '{self.job_name}': checkpoint {n} failed on "
                                            f"rank(s) {[r for r, _ in bad]}: {bad[0][1]}")
            if self.comm.rank == 0:
                write_host_checkpoint(d, job_id=storage.job_id, checkpoint_id=n, states={},
                                      extra=extra, ranks=ranks)
            self.comm.barrier()
        if self.comm is None or self.comm.rank == 0:
            for old in storage.completed_checkpoints()[:-max(1, self.env.checkpoint_config.max_retained)]:
                import shutil

                shutil.rmtree(old, ignore_errors=True)
        self._next_ckpt += 1
        self.metrics["numberOfCompletedCheckpoints"] = self.metrics.get("numberOfCompletedCheckpoints", 0) + 1
        self.metrics["lastCheckpointDuration"] = (time.perf_counter() - t0) * 1e3
        self.metrics["lastCheckpointPath"] = str(storage.checkpoint_dir(n))
        log.info("Completed checkpoint %d for job %s (%.1f ms)", n, storage.job_id,
                 self.metrics["lastCheckpointDuration"])

    def _restore(self, path, finished: dict) -> None:
        from .checkpoint import read_host_checkpoint

        rank, world = (self.comm.rank, self.comm.world) if self.comm is not None else (0, 1)
        meta, states = read_host_checkpoint(
            path, rank, world, self.env.parallelism, self.env.max_parallelism,
            node_parallelism={self._uid(nd): nd.parallelism for nd in self.nodes
                              if nd.parallelism})
        names = meta["extra"]["nodes"]
        for nd in self.nodes:
            key = self._uid(nd)
            if key not in states or names.get(key) != nd.name:
                raise ValueError(f"checkpoint {path} does not match the job graph ({nd.name})")
            self.ops[nd.id].restore(states[key])
        ex = meta["extra"]
        if ex.get("clock") is not None and isinstance(self.clock, ManualClock):
            self.clock.advance_to(ex["clock"])
        by_uid = {self._uid(nd): nd.id for nd in self.nodes}
        self._rr = {(by_uid[a], by_uid[b]): v for a, b, v in ex.get("rr", [])}
        for k, v in ex.get("finished", {}).items():
            finished[by_uid[k]] = v
        self._next_ckpt = int(meta["checkpoint_id"]) + 1
        self.metrics["restoredCheckpointId"] = int(meta["checkpoint_id"])
        log.info("Restored job %s from %s", self.job_name, path)

    def _reporter(self):
        c = self.env.config
        if not (getattr(c, "metrics_json", None) or getattr(c, "metrics_prometheus", None)):
            return None
        from ..utils.metrics import REGISTRY, Reporter

        for n in self.nodes:
            cnt = self._counts.setdefault(n.id, {"numRecordsIn": 0, "numRecordsOut": 0})
            scope = f"{self.job_name}.{self._uid(n)}"
            for k in ("numRecordsIn", "numRecordsOut"):
                REGISTRY.gauge(f"{scope}.{k}", lambda d=cnt, k=k: d[k])
            op = self.ops.get(n.id)
            if op is not None and hasattr(op, "num_late_records_dropped"):
                REGISTRY.gauge(f"{scope}.numLateRecordsDropped",
                               lambda o=op: o.num_late_records_dropped)
            if op is not None and hasattr(op, "wm"):
                REGISTRY.gauge(f"{scope}.currentInputWatermark", lambda o=op: o.wm)
        return Reporter(json_path=c.metrics_json, prom_path=c.metrics_prometheus,
                        interval_ms=c.metrics_interval_ms)

    def _uid(self, nd) -> str:
        """Stable operator id across job submissions: the user's .uid(), else the position in
        the topological order + name (Flink hashes the graph structure the same way)."""
        if nd.uid:
            return nd.uid
        if not hasattr(self, "_pos"):
            self._pos = {n.id: i for i, n in enumerate(self.nodes)}
            self._node = {n.id: n for n in self.nodes}
        return f"{self._pos[nd.id]}-{nd.name}"

    def _maybe_fault(self, node, items) -> None:
        f = self.fault
        if f is None or self.attempt >= f[2] or f[0] not in node.name:
            return
        from .columnar import rows_in

        self._fault_count += rows_in(items)
        if self._fault_count >= f[1]:
            raise InjectedFault(f"injected fault in {node.name} after {self._fault_count} records"
                                f" (attempt {self.attempt})")

    def run(self) -> JobExecutionResult:
        t0 = time.perf_counter()
        self._open()
        sources = [n for n in self.nodes if n.kind == "source"]
        finished = {n.id: False for n in sources}
        manual = isinstance(self.clock, ManualClock)
        cfg = self.env.checkpoint_config
        self._next_ckpt = 1
        self._uid(self.nodes[0])  # builds the position / node maps
        if self.restore_from is not None:
            self._restore(self.restore_from, finished)
        elif cfg.is_checkpointing_enabled():
            done = self._storage().completed_checkpoints()
            if done:
                self._next_ckpt = int(done[-1].name[4:]) + 1
        self._last_ckpt = self.clock()
        reporter = self._reporter()
        cfg_x = self.env.config
        trace_path = getattr(cfg_x, "trace_path", None)
        if trace_path:
            trace.enable(True)
        self._trace = trace.active()
        wd = None
        if getattr(cfg_x, "step_timeout_ms", 0) and cfg_x.step_timeout_ms > 0:
            wd = Watchdog(cfg_x.step_timeout_ms, name=self.job_name).start()
        try:
            want = False
            while True:
                done, now = self._step_begin(finished, sources, manual, want)
                if done:
                    break
                inbox: dict = {}
                for n in sources:
                    if finished[n.id]:
                        continue
                    try:
                        items, done = self.ops[n.id].poll(now)
                        finished[n.id] = done
                        for c in self.children[n.id]:
                            inbox.setdefault((c.id, n.id), []).extend(self._rebalance(n, c, items))
                    except Exception as e:  # noqa: BLE001 -- multi-rank: re-raised by _control
                        self._record_failure(e)
                self._push(inbox, now)
                if wd is not None:
                    wd.beat()
                want = (cfg.is_checkpointing_enabled()
                        and self.clock() - self._last_ckpt >= cfg.interval_ms)
                if self.comm is None and want:
                    self._checkpoint(finished)
                    self._last_ckpt = self.clock()
                    want = False
                # (multi-rank: the request and any failure are agreed at the next _step_begin)
                if reporter is not None:
                    reporter.maybe_report(job=self.job_name)
            # End of input: MAX watermark (event time), then operators' finish hooks.
            inbox = {}
            for n in sources:
                for c in self.children[n.id]:
                    inbox.setdefault((c.id, n.id), []).append(WM(LONG_MAX))
            self._push(inbox, None)
            # Multi-rank: the end-of-input firing (MAX watermark) and the finish hooks run under
            # the same record-then-agree protocol as every step, so a failure in either fails
            # every rank instead of being swallowed or leaving the peers in a collective.
            self._control(False)
            self._finish()
            self._control(False)
        except (JobExecutionException, InjectedFault):
            raise
        except KeyboardInterrupt:
            if wd is not None and wd.expired:
                raise JobExecutionException(f"Job '{self.job_name}' failed: StepTimeout: no "
                                            f"progress for {cfg_x.step_timeout_ms} ms") \
                    from StepTimeout(self.job_name)
            raise
        except Exception as e:
            raise JobExecutionException(f"Job '{self.job_name}' failed: {type(e).__name__}: {e}") from e
        finally:
            if wd is not None:
                wd.stop()
            if trace_path:
                trace.dump(trace_path, self.env.rank)
            for n in self.nodes:
                op = self.ops.get(n.id)
                if op is not None:
                    try:
                        op.close()
                    except Exception:
                        pass
        for n in self.nodes:
            op = self.ops.get(n.id)
            if op is not None and hasattr(op, "num_late_records_dropped"):
                self.metrics[f"{n.name}.numLateRecordsDropped"] = op.num_late_records_dropped
        for n in self.nodes:
            for k, v in self._counts.get(n.id, {}).items():
                self.metrics[f"{n.name}.{k}"] = v
        if reporter is not None:
            reporter.maybe_report(force=True, job=self.job_name, final=True)
        return JobExecutionResult(self.job_name, (time.perf_counter() - t0) * 1e3, self.metrics)

    def _rebalance(self, src: Transformation, child: Transformation, items: list) -> list:
        """Source (parallelism 1) -> parallel operator: RebalancePartitioner round robin."""
        p = child.parallelism or self.env.parallelism
        key = (src.id, child.id)
        nxt = self._rr.get(key, self.env.config.rebalance_start)
        from .columnar import TextBatch

        out = []
        for it in items:
            if isinstance(it, Rec):
                out.append(Rec(it.value, it.ts, nxt % p))
                nxt += 1
            elif isinstance(it, TextBatch):
                out.append(TextBatch(it.data, it.n, nxt % p, p, it.token, it.ready))
                nxt += it.n
            else:
                out.append(it)
        self._rr[key] = nxt
        return out

    def _finish(self):
        inbox: dict = {}
        for n in self.nodes:
            if n.kind in ("source", "union", "side"):
                out = []
                if n.kind == "union":
                    for p in n.parents:
                        out.extend(inbox.pop((n.id, p.id), []))
            else:
                items = []
                for p in n.parents:
                    items.extend(inbox.pop((n.id, p.id), []))
                op = self.ops[n.id]
                if self.comm is not None:
                    items = self._exchange(n, items)
                    if self._failure is not None:
                        items = []
                if not getattr(op, "accepts_columns", False):
                    from .columnar import expand_columns

                    items = expand_columns(items)
                try:
                    out = op.process(items) if (items or getattr(op, "collective", False)) else []
                    out.extend(op.finish())
                except Exception as e:  # noqa: BLE001 -- multi-rank: re-raised by _control
                    if self.comm is None:
                        raise
                    self._record_failure(e)
                    out = []
            for c in self.children[n.id]:
                inbox.setdefault((c.id, n.id), []).extend(out)


_ = Rec

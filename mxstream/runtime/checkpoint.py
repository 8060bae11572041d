"""Checkpoints and savepoints with Flink's FsStateBackend directory layout.

Flink 1.8 (promised but not implemented by the reference,
chapter3/README.md:454-456) stores

  <checkpoint dir>/<jobId>/chk-<n>/_metadata        (+ <jobId>/shared/, <jobId>/taskowned/)
  <savepoint dir>/savepoint-<jobId[:6]>-<12 hex>/_metadata

with keyed state partitioned by *key group* so that a job can be restored at another parallelism.
This module mirrors that layout; the file contents are mxstream's own (documented below), not
Flink's binary MetadataV2.

* One state file per (operator uid, rank): ``<uid>-<rank>.kg`` written by the C++ runtime
  (csrc/runtime.cpp ``write_kg_file``): magic ``MXSKG001`` | JSON header | key-group range |
  per-key-group row offsets | columns sorted by key group. A reader asks for a key-group range and
  gets exactly those rows (restore at a different world size reads the slices it now owns from
  every old rank's file).
* ``_metadata`` (JSON) is written last, atomically (write + rename), by rank 0 after every rank
  finished its files (barrier): checkpoint id, job id, world size, max parallelism, per-operator
  file list and scalar metadata (watermark, fire cursor, ...), source offsets, user extras.
  A directory without ``_metadata`` is an incomplete checkpoint and is never restored.

Snapshots are step-aligned: between two micro-batches every rank is at the same step, so the
checkpoint barrier needs no alignment buffering (the engine's analogue of Flink's aligned
barriers). The device tables are exported by ``keygroups`` + gathers on the GPU and copied to the
host once per checkpoint.
"""
from __future__ import annotations

import json
import os
import secrets
import shutil
import time
from dataclasses import dataclass, field
from pathlib import Path

import numpy as np

from ..ops.native import load

META = "_metadata"
FORMAT = "mxstream-checkpoint-v1"


@dataclass
class OperatorSnapshot:
    """What an operator hands to the coordinator: key-grouped rows + scalar metadata."""
    kg: np.ndarray                         # int32 key group per row
    columns: dict[str, np.ndarray]         # equal-length columns (fixed-width dtypes)
    meta: dict = field(default_factory=dict)


def freeze_operator(op, tensor_names: tuple[str, ...], post=None):
    """Synchronous phase of an async snapshot: a shallow copy of ``op`` whose state tensors are
    device-side clones (HBM-speed copies enqueued on the current stream, ordered after every
    kernel that wrote the state) and whose metrics are copied. Returns a thunk that runs the
    operator's ordinary ``snapshot_state`` on the frozen copy — safe to call from another thread
    on another stream while ``op`` keeps processing micro-batches."""
    import copy

    import torch

    frozen = copy.copy(op)
    frozen.metrics = copy.copy(op.metrics)
    for name in tensor_names:
        setattr(frozen, name, getattr(op, name).clone())
    if post is not None:
        post(frozen)  # host-side state the export reads (e.g. the spill tier): private copies
    ev = None
    dev = getattr(op, "device", None)
    if dev is not None and torch.device(dev).type == "cuda":
        ev = torch.cuda.Event()
        ev.record()

    def run():
        if ev is not None:
            torch.cuda.current_stream().wait_event(ev)
        return type(op).snapshot_state(frozen)

    return run


def _dtype_str(a: np.ndarray) -> str:
    return np.dtype(a.dtype).str


class CheckpointStorage:
    """Directory layout of one job's checkpoints (and of savepoints)."""

    def __init__(self, root: str | os.PathLike, job_id: str | None = None):
        self.root = Path(root)
        self.job_id = job_id or secrets.token_hex(16)

    @property
    def job_dir(self) -> Path:
        return self.root / self.job_id

    def checkpoint_dir(self, n: int) -> Path:
        return self.job_dir / f"chk-{n}"

    def init_job_dirs(self) -> None:
        for d in (self.job_dir, self.job_dir / "shared", self.job_dir / "taskowned"):
            d.mkdir(parents=True, exist_ok=True)

    def new_savepoint_dir(self, target: str | os.PathLike | None = None) -> Path:
        base = Path(target) if target is not None else self.root
        return base / f"savepoint-{self.job_id[:6]}-{secrets.token_hex(6)}"

    def completed_checkpoints(self) -> list[Path]:
        if not self.job_dir.exists():
            return []
        out = []
        for d in self.job_dir.iterdir():
            if d.name.startswith("chk-") and (d / META).exists():
                out.append(d)
        return sorted(out, key=lambda d: int(d.name[4:]))

    def latest(self) -> Path | None:
        done = self.completed_checkpoints()
        return done[-1] if done else None


def write_operator_file(directory: Path, uid: str, rank: int, snap: OperatorSnapshot,
                        max_parallelism: int) -> str:
    """Write one operator's key-grouped rows for this rank; returns the file name."""
    m = load()
    name = f"{uid}-{rank}.kg"
    cols = list(snap.columns.items())
    n = len(snap.kg)
    for k, v in cols:
        if len(v) != n:
            raise ValueError(f"column {k}: {len(v)} rows, expected {n}")
    header = json.dumps({"uid": uid, "rank": rank,
                         "columns": [[k, _dtype_str(v)] for k, v in cols]})
    m.write_kg_file(str(directory / name), header, 0, max_parallelism - 1,
                    np.ascontiguousarray(snap.kg, dtype=np.int32),
                    [np.ascontiguousarray(v) for _, v in cols])
    return name


def read_operator_rows(directory: Path, files: list[str], kg_lo: int, kg_hi: int) -> dict:
    """Rows of key groups [kg_lo, kg_hi] from every listed file, concatenated per column."""
    m = load()
    parts: dict[str, list[np.ndarray]] = {}
    order: list[tuple[str, str]] = []
    for fname in files:
        path = directory / fname
        head, _lo, _hi, _offs, _c, _n = m.read_kg_file(str(path), [], 0, 0)
        cols = json.loads(bytes(head).decode())["columns"]
        if not order:
            order = [tuple(c) for c in cols]
        sizes = [np.dtype(dt).itemsize for _, dt in cols]
        head, _lo, _hi, _offs, raw, nrows = m.read_kg_file(str(path), sizes, kg_lo, kg_hi)
        for (cname, dt), buf in zip(cols, raw):
            parts.setdefault(cname, []).append(np.asarray(buf).view(np.dtype(dt)))
    def join(c, dt):
        p = parts.get(c)
        return np.zeros(0, np.dtype(dt)) if not p else p[0] if len(p) == 1 else np.concatenate(p)

    return {c: join(c, dt) for c, dt in order}


def _atomic_write_json(path: Path, obj: dict) -> None:
    tmp = path.with_name(path.name + ".inprogress")
    with open(tmp, "w") as f:
        json.dump(obj, f, indent=1, sort_keys=True)
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, path)


def read_metadata(path: str | os.PathLike) -> dict:
    d = Path(path)
    with open(d / META) as f:
        meta = json.load(f)
    if meta.get("format") != FORMAT:
        raise ValueError(f"{d}: not an mxstream checkpoint ({meta.get('format')})")
    return meta


class CheckpointCoordinator:
    """Triggers step-aligned checkpoints of a set of engine operators across ranks.

    ``operators``: {uid: operator} where each operator implements ``snapshot_state() ->
    OperatorSnapshot`` and ``restore_state(rows: dict, meta: dict)`` and exposes ``comm`` (all
    operators of a job share one communicator) and ``max_parallelism``.
    """

    def __init__(self, storage: CheckpointStorage, operators: dict, *, comm=None,
                 interval_steps: int | None = None, retain: int = 1):
        self.storage = storage
        self.ops = operators
        first = next(iter(operators.values()))
        self.comm = comm if comm is not None else first.comm
        self.world, self.rank = self.comm.world, self.comm.rank
        self.max_parallelism = first.max_parallelism
        self.interval_steps = interval_steps
        self.retain = max(1, retain)
        self.next_id = 1
        done = storage.completed_checkpoints()
        if done:
            self.next_id = int(done[-1].name[4:]) + 1
        self.stats: list[dict] = []
        self._pending: dict | None = None

    # ---- triggering --------------------------------------------------------------------
    def maybe_trigger(self, step: int, sources: dict | None = None) -> Path | None:
        if self.interval_steps and step > 0 and step % self.interval_steps == 0:
            return self.trigger(step, sources)
        return None

    def trigger(self, step: int, sources: dict | None = None, extra: dict | None = None) -> Path:
        """Checkpoint chk-<next id> (all ranks call this at the same step)."""
        self.complete_pending()
        if self.rank == 0:
            self.storage.init_job_dirs()
        d = self.storage.checkpoint_dir(self.next_id)
        self._write(d, "checkpoint", step, sources, extra)
        self.next_id += 1
        if self.rank == 0:
            self._prune()
        return d

    def savepoint(self, step: int, target: str | None = None, sources: dict | None = None,
                  extra: dict | None = None) -> Path:
        """Savepoint (all ranks must pass the same `target`; rank 0's directory name wins)."""
        self.complete_pending()
        d = self.storage.new_savepoint_dir(target)
        if self.world > 1:
            # the communicator's group (not the default one): operators may run on a subgroup
            d = d.parent / self.comm.broadcast_object(d.name, src=0)
        self._write(d, "savepoint", step, sources, extra)
        return d

    def _write(self, d: Path, kind: str, step: int, sources, extra) -> dict | None:
        t0 = time.perf_counter()
        d.mkdir(parents=True, exist_ok=True)
        op_meta, nbytes = {}, 0
        for uid, op in self.ops.items():
            snap = op.snapshot_state()
            fname = write_operator_file(d, uid, self.rank, snap, self.max_parallelism)
            nbytes += sum(v.nbytes for v in snap.columns.values())
            op_meta[uid] = {"meta": snap.meta, "rows": int(len(snap.kg)), "file": fname}
        gathered = self._gather({"rank": self.rank, "ops": op_meta, "sources": sources or {},
                                 "bytes": nbytes})
        meta = None
        if self.rank == 0:
            ops_all = {}
            for uid in self.ops:
                ops_all[uid] = {
                    "files": [g["ops"][uid]["file"] for g in gathered],
                    "rows": [g["ops"][uid]["rows"] for g in gathered],
                    "meta": gathered[0]["ops"][uid]["meta"],
                }
            meta = {"format": FORMAT, "type": kind, "job_id": self.storage.job_id,
                    "checkpoint_id": self.next_id if kind == "checkpoint" else None,
                    "step": int(step), "timestamp_ms": int(time.time() * 1000),
                    "world": self.world, "max_parallelism": self.max_parallelism,
                    "operators": ops_all, "sources": [g["sources"] for g in gathered],
                    "extra": extra or {}}
            _atomic_write_json(d / META, meta)
        self.comm.barrier()
        self.stats.append({"dir": str(d), "type": kind, "step": step,
                           "ms": (time.perf_counter() - t0) * 1e3, "bytes": nbytes})
        return meta

    # ---- asynchronous checkpoints (SURVEY.md §5.4 "async mode") -----------------------------
    def trigger_async(self, step: int, sources: dict | None = None,
                      extra: dict | None = None) -> None:
        """Start chk-<next id> without stalling the step loop.

        Synchronous part (this call, between two micro-batches): every operator freezes its
        state (``snapshot_state_async``: device-to-device copies of the tables at HBM speed, plus
        the host bookkeeping). Asynchronous part (a worker thread, on its own HIP stream): the
        key-group export, the D2H copies and the state files, overlapped with the next steps.
        ``complete_pending()`` (called by the next trigger, or explicitly at a step boundary /
        end of job) joins the worker and runs the cross-rank acknowledgement — metadata gather,
        ``_metadata`` written atomically by rank 0, barrier — on the calling thread, so the
        process group is never used from two threads. Until then the checkpoint has no
        ``_metadata`` and is not restorable (Flink's pending checkpoint)."""
        import threading

        self.complete_pending()
        t0 = time.perf_counter()
        if self.rank == 0:
            self.storage.init_job_dirs()
        d = self.storage.checkpoint_dir(self.next_id)
        d.mkdir(parents=True, exist_ok=True)
        frozen = {uid: (op.snapshot_state_async() if hasattr(op, "snapshot_state_async")
                        else (lambda s=op.snapshot_state(): s))
                  for uid, op in self.ops.items()}
        result: dict = {}
        cuda_dev = next((op.device for op in self.ops.values()
                         if getattr(getattr(op, "device", None), "type", "cpu") == "cuda"), None)

        def work():
            import contextlib

            try:
                op_meta, nbytes = {}, 0
                ctx = contextlib.ExitStack()
                if cuda_dev is not None:
                    import torch

                    # The current device is per thread: pin it, then export on a side stream.
                    ctx.enter_context(torch.cuda.device(cuda_dev))
                    ctx.enter_context(torch.cuda.stream(torch.cuda.Stream(cuda_dev)))
                with ctx:
                    for uid, fn in frozen.items():
                        snap = fn()
                        fname = write_operator_file(d, uid, self.rank, snap, self.max_parallelism)
                        # make the data durable here, off the step loop, so the _metadata
                        # fsync in complete_pending() does not flush it on the caller's thread
                        fd = os.open(d / fname, os.O_RDONLY)
                        try:
                            os.fsync(fd)
                        finally:
                            os.close(fd)
                        nbytes += sum(v.nbytes for v in snap.columns.values())
                        op_meta[uid] = {"meta": snap.meta, "rows": int(len(snap.kg)),
                                        "file": fname}
                result.update(op_meta=op_meta, nbytes=nbytes, t_done=time.perf_counter())
            except BaseException as e:  # surfaced by complete_pending()
                result["error"] = e

        th = threading.Thread(target=work, name=f"mxs-ckpt-{self.next_id}", daemon=True)
        th.start()
        self._pending = {"thread": th, "result": result, "dir": d, "step": step,
                         "sources": sources, "extra": extra, "id": self.next_id, "t0": t0,
                         "sync_ms": (time.perf_counter() - t0) * 1e3}
        self.next_id += 1

    def pending_done(self) -> bool:
        """True when this rank's export of the pending checkpoint has finished (local only:
        ranks must still agree on the step at which they call ``complete_pending``)."""
        return self._pending is not None and not self._pending["thread"].is_alive()

    def complete_pending(self) -> Path | None:
        """Finish the pending async checkpoint (if any); returns its directory."""
        import threading

        p = getattr(self, "_pending", None)
        if p is None:
            return None
        self._pending = None
        p["thread"].join()
        res = p["result"]
        d = p["dir"]
        # Every rank joins the acknowledgement, failed or not, so a rank whose export failed
        # (disk error, ...) does not leave the others blocked in the collective until its
        # timeout: all ranks learn the failure together, nobody writes _metadata, all raise.
        err = res.get("error")
        gathered = self._gather({"rank": self.rank, "error": repr(err) if err else None,
                                 "ops": res.get("op_meta"), "sources": p["sources"] or {},
                                 "bytes": res.get("nbytes", 0)})
        failed = [(g["rank"], g["error"]) for g in gathered if g.get("error")]
        if failed:
            self.comm.barrier()
            msg = f"async checkpoint {p['id']} failed on rank(s) {failed}"
            if err is not None:
                raise RuntimeError(msg) from err
            raise RuntimeError(msg)
        if self.rank == 0:
            ops_all = {uid: {"files": [g["ops"][uid]["file"] for g in gathered],
                             "rows": [g["ops"][uid]["rows"] for g in gathered],
                             "meta": gathered[0]["ops"][uid]["meta"]} for uid in self.ops}
            meta = {"format": FORMAT, "type": "checkpoint", "job_id": self.storage.job_id,
                    "checkpoint_id": p["id"], "step": int(p["step"]),
                    "timestamp_ms": int(time.time() * 1000), "world": self.world,
                    "max_parallelism": self.max_parallelism, "operators": ops_all,
                    "sources": [g["sources"] for g in gathered], "extra": p["extra"] or {},
                    "async": True}
            _atomic_write_json(d / META, meta)
        self.comm.barrier()
        if self.rank == 0:
            threading.Thread(target=self._prune, name="mxs-ckpt-prune", daemon=True).start()
        self.stats.append({"dir": str(d), "type": "checkpoint-async", "step": p["step"],
                           "ms": (time.perf_counter() - p["t0"]) * 1e3,
                           "sync_ms": p["sync_ms"], "bytes": res["nbytes"],
                           "export_ms": (res["t_done"] - p["t0"]) * 1e3})
        return d

    def _gather(self, obj: dict) -> list[dict]:
        if self.world == 1:
            return [obj]
        return self.comm.all_gather_object(obj)

    def _prune(self) -> None:
        done = self.storage.completed_checkpoints()
        for old in done[:-self.retain]:
            shutil.rmtree(old, ignore_errors=True)

    # ---- restore -----------------------------------------------------------------------
    def restore(self, path: str | os.PathLike | None = None) -> dict:
        """Restore every operator from a completed checkpoint/savepoint (default: latest).

        Works at any world size: each rank reads the key groups it now owns from all old files.
        Returns the metadata (source offsets etc. are the caller's to apply)."""
        self.complete_pending()
        d = Path(path) if path is not None else self.storage.latest()
        if d is None:
            raise FileNotFoundError("no completed checkpoint")
        meta = read_metadata(d)
        if meta["max_parallelism"] != self.max_parallelism:
            raise ValueError("max parallelism changed: key groups cannot be remapped")
        for uid, op in self.ops.items():
            om = meta["operators"].get(uid)
            if om is None:
                raise KeyError(f"operator {uid!r} not in checkpoint {d}")
            lo, hi = op.owned_key_groups()
            rows = read_operator_rows(d, om["files"], lo, hi)
            op.restore_state(rows, om["meta"])
        if meta.get("checkpoint_id") is not None and d.parent == self.storage.job_dir:
            self.next_id = max(self.next_id, int(meta["checkpoint_id"]) + 1)
        return meta


def owned_key_groups(rank: int, world: int, parallelism: int, max_parallelism: int) -> tuple[int, int]:
    """Contiguous key-group range of a rank (subtasks laid out in blocks over ranks):
    kg -> subtask = kg * P // maxP -> rank = subtask * G // P."""
    kgs = [kg for kg in range(max_parallelism)
           if (kg * parallelism // max_parallelism) * world // parallelism == rank]
    if not kgs:
        return 1, 0  # empty range
    return kgs[0], kgs[-1]


# ---- host executor checkpoints (DataStream API jobs) ------------------------------------------
# Host operators hold Python values (user tuples, accumulators, timers); their state files use the
# typed, code-free encoding of runtime/statecodec.py (JSON + an allow_pickle=False npz), never
# pickle: restoring a checkpoint directory runs no code from it. Keyed state inside them is
# partitioned by key group (HeapKeyedStateBackend.snapshot), which lets a restore at another
# world size re-split it (rescale_host_state).
def write_host_states(d: Path, states: dict[str, dict], rank: int = 0) -> dict[str, str]:
    """One state file per operator of this rank (``op<i>-<rank>.state.json`` [+ ``.npz``]);
    returns uid -> file."""
    from .statecodec import write_state

    d.mkdir(parents=True, exist_ok=True)
    files = {}
    for i, (node_id, st) in enumerate(states.items()):
        name = f"op{i:03d}-{rank}.state.json"  # uid -> file map lives in _metadata
        write_state(d / name, st)
        files[node_id] = name
    return files


def write_host_checkpoint(d: Path, *, job_id: str, checkpoint_id: int, states: dict[str, dict],
                          extra: dict, kind: str = "checkpoint",
                          ranks: list[dict] | None = None) -> None:
    """Single-process host checkpoint, or (``ranks``: every rank's ``{"host_operators",
    "extra"}``, files already written by write_host_states) the metadata of a multi-rank one."""
    files = write_host_states(d, states) if ranks is None else ranks[0]["host_operators"]
    meta = {"format": FORMAT, "type": kind, "job_id": job_id, "checkpoint_id": checkpoint_id,
            "timestamp_ms": int(time.time() * 1000), "host_operators": files,
            "state_encoding": "mxs-typed-v1",
            "extra": extra if ranks is None else ranks[0]["extra"]}
    if ranks is not None:
        meta["world"] = len(ranks)
        meta["ranks"] = ranks
    _atomic_write_json(d / META, meta)


def read_host_checkpoint(path: str | os.PathLike, rank: int = 0, world: int = 1,
                         parallelism: int | None = None, max_parallelism: int = 128,
                         node_parallelism: dict[str, int] | None = None
                         ) -> tuple[dict, dict[str, dict]]:
    """Metadata (with this rank's ``extra``) and this rank's operator states. At the world size
    that wrote the checkpoint every rank reads its own files; at another world size every rank
    reads all of them and keeps the key groups it now owns (rescale_host_state).

    node_parallelism: uid -> the operator's own parallelism where it differs from the
    environment's (``set_parallelism``): the executor routes a key with the parallelism of its
    node (executor.py ``_exchange``), so each operator's owned key-group range is computed with
    that node's parallelism, not one range for every operator."""
    from .statecodec import read_state

    d = Path(path)
    meta = read_metadata(d)
    if meta.get("state_encoding") != "mxs-typed-v1":
        raise ValueError(f"checkpoint {d}: unsupported host state encoding "
                         f"{meta.get('state_encoding')!r} (only mxs-typed-v1 is read)")
    w = int(meta.get("world", 1))
    per_rank = ([r["host_operators"] for r in meta["ranks"]] if "ranks" in meta
                else [meta["host_operators"]])
    extras = [r["extra"] for r in meta["ranks"]] if "ranks" in meta else [meta["extra"]]
    if w == world:
        states = {nid: read_state(d / name) for nid, name in per_rank[rank].items()}
        return dict(meta, extra=extras[rank]), states
    old = [{nid: read_state(d / name) for nid, name in files.items()} for files in per_rank]
    node_parallelism = node_parallelism or {}

    def kg_range(nid: str) -> tuple[int, int]:
        return owned_key_groups(rank, world, node_parallelism.get(nid) or parallelism or world,
                                max_parallelism)

    states = {nid: rescale_host_state([o[nid] for o in old], rank, world, kg_range(nid),
                                      max_parallelism)
              for nid in per_rank[0]}
    return dict(meta, extra=rescale_extra(extras, rank, world)), states


_KEYED_PARTS = ("keyed", "timers", "wm", "merging", "trigger_state")


def rescale_host_state(snaps: list[dict], rank: int, world: int, kg_range: tuple[int, int],
                       max_parallelism: int) -> dict:
    """One operator's state at a new rank from every old rank's snapshot.

    * keyed operators (``keyed`` / ``timers`` / ``wm`` / ``merging`` / ``trigger_state``): the
      key groups in ``kg_range`` from every old rank, timers and merging/trigger entries of
      those keys, the minimum watermark;
    * sources (``{"rescale": ...}``): the source merges its old positions itself
      (Source.restore_rescaled);
    * stateless operators ({}): nothing;
    * anything else (a parallelism-1 operator's state lives on rank 0): rank 0's snapshot at
      the new rank 0 only."""
    from ..utils.hashing import key_group

    if not any(snaps):
        return {}
    if all(not s or set(s) <= set(_KEYED_PARTS) for s in snaps):
        lo, hi = kg_range
        out: dict = {"keyed": {}}

        def mine(key) -> bool:
            return lo <= key_group(key, max_parallelism) <= hi

        for s in snaps:
            for kg, tables in s.get("keyed", {}).items():
                if lo <= int(kg) <= hi:
                    dst = out["keyed"].setdefault(int(kg), {})
                    for name, entries in tables.items():
                        dst.setdefault(name, {}).update(entries)
        if any("timers" in s for s in snaps):
            out["timers"] = {kind: sorted(t for s in snaps for t in s.get("timers", {}).get(kind, [])
                                          if mine(t[1]))
                             for kind in ("event", "proc")}
        wms = [s["wm"] for s in snaps if "wm" in s]
        if wms:
            out["wm"] = min(wms)
        for part in ("merging", "trigger_state"):
            if any(part in s for s in snaps):
                out[part] = {}
                for s in snaps:
                    for k, v in s.get(part, {}).items():
                        kk = k[0] if part == "trigger_state" and isinstance(k, tuple) else k
                        if mine(kk):
                            out[part][k] = v
        return out
    if all("rescale" in s for s in snaps if s):
        return {"rescaled": [s["rescale"] for s in snaps], "rank": rank, "world": world}
    if rank == 0:
        if any(snaps[1:]):
            raise ValueError("host checkpoint: an operator with state on several ranks that is "
                             "not keyed cannot be restored at another world size")
        return snaps[0]
    return {}


def rescale_extra(extras: list[dict], rank: int, world: int) -> dict:
    """Executor bookkeeping at a new world size: the clock is the maximum (the ranks agree on a
    step clock), round-robin counters restart, a source is finished only if it was everywhere."""
    ex = dict(extras[0])
    clocks = [e.get("clock") for e in extras if e.get("clock") is not None]
    ex["clock"] = max(clocks) if clocks else None
    ex["rr"] = []
    fin = {}
    for e in extras:
        for k, v in e.get("finished", {}).items():
            fin[k] = fin.get(k, True) and bool(v)
    ex["finished"] = fin
    return ex

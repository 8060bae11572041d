"""bench.py under torch.distributed.run (the driver's multi-GPU launch), rehearsed on the CPU
with gloo: 2 ranks, tiny batches, long enough for window firings inside the timed region."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _ranks_stderr(r):
    """Both ranks' stderr as torchrun relayed it (faulthandler stacks of an aborting rank
    included) -- not just the launcher's summary at the end."""
    return f"rc={r.returncode}\n--- stderr ---\n{r.stderr[-20000:]}\n--- stdout ---\n{r.stdout[-4000:]}"


def test_bench_two_ranks_gloo():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2",
           "--device", "cpu", "--batch", "32768", "--keys", "5000", "--steps", "14",
           "--warmup", "1"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, _ranks_stderr(r)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 prints one JSON line
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 14 and d["warmup"] == 1
    assert d["config"]["exchange"] == "partials"
    assert d["config"]["global_batch"] == 2 * 32768
    assert d["alerts"] > 0 and d["value"] > 0
    assert abs(d["value"] - 2 * 32768 * 14 / (d["ms_per_step"] * 14 / 1e3)) / d["value"] < 1e-6
    # the per-event keyBy shuffle is measured next to the local-global headline
    assert d["records_events_per_s"] > 0 and d["records_ms_per_step"] > 0


def test_bench_two_ranks_records_exchange():
    """--exchange records: the headline itself is the per-event all-to-all (hashed state)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2",
           "--device", "cpu", "--batch", "32768", "--keys", "5000", "--steps", "14",
           "--warmup", "1", "--exchange", "records"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, _ranks_stderr(r)
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert d["config"]["exchange"] == "records" and d["config"]["keyed_state"] == "hashed"
    assert d["alerts"] > 0 and "records_events_per_s" not in d

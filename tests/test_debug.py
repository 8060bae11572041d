"""Race/corruption detection: keyed-state invariant checker (GPU kernel + C++
twin), MXS_DEBUG per-step checks, and the ASan/UBSan host harness over the C++ twins."""
import subprocess

import pytest
import torch

from mxstream.ops import debug as D
from mxstream.ops import kernels as K
from mxstream.runtime.window_operator import KeyedWindowOperator


def _populated_op(dev, nkeys=3000):
    op = KeyedWindowOperator(size=2000, agg=K.AGG_SUM_I64, device=dev, max_keys=nkeys,
                             batch_capacity=1 << 14, ooo_bound=100, cap_log2=8)
    keys = torch.empty(1 << 14, dtype=torch.int64, device=dev)
    ts = torch.empty_like(keys)
    vals = torch.empty_like(keys)
    K.gen_events(keys, ts, vals, seed=1, stream_id=0, idx0=0, nkeys=nkeys, ts_base=0,
                 ts_span=1000, disorder=0, val_lo=0, val_span=10)
    op.process(keys, ts, vals)
    op.expected_live = int(torch.unique(keys).numel())
    return op


def _check(op):
    return D.check_table(op.keys_g, nsub=op.nsub, nsub_log2=op.nsub_log2, cap_log2=op.cap_log2)


def test_clean_table_passes():
    op = _populated_op("cpu")
    r = _check(op)
    assert r["live"] == op.expected_live and r["misplaced"] == r["broken_chain"] == r["duplicate"] == 0


def test_corruptions_are_detected():
    op = _populated_op("cpu")
    keys = op.keys_g
    live = torch.nonzero(keys != -1).flatten()
    # 1. a duplicate: copy a key into the next empty slot after it in the same sub-table
    cap = 1 << op.cap_log2
    s0 = int(live[0])
    sub0 = s0 // cap
    j = s0 + 1
    while keys[j] != -1:
        j = sub0 * cap + ((j - sub0 * cap + 1) % cap)
    keys[j] = keys[s0]
    r = _check(op)
    assert r["duplicate"] >= 1
    keys[j] = -1
    # 2. a key moved to another sub-table
    other = (sub0 + 1) % op.nsub
    k = int(keys[s0])
    keys[s0] = -1
    free = (keys[other * cap:(other + 1) * cap] == -1).nonzero().flatten()
    keys[other * cap + int(free[0])] = k
    r = _check(op)
    assert r["misplaced"] >= 1
    # (emptying s0 may also break other keys' probe chains)
    with pytest.raises(D.StateCorruption):
        D.assert_table_ok(keys, nsub=op.nsub, nsub_log2=op.nsub_log2, cap_log2=op.cap_log2)


def test_debug_mode_checks_every_step(monkeypatch):
    """MXS_DEBUG: the native step checks the table invariants after every aggregation; a corrupted
    table (a key moved to another sub-table) stops the next step with the step number."""
    monkeypatch.setenv("MXS_DEBUG", "1")
    op = _populated_op("cpu")  # clean steps pass the check
    keys = op.keys_g
    live = torch.nonzero(keys != -1).flatten()
    cap = 1 << op.cap_log2
    s0 = int(live[0])
    other = (s0 // cap + 1) % op.nsub
    free = (keys[other * cap:(other + 1) * cap] == -1).nonzero().flatten()
    keys[other * cap + int(free[0])] = keys[s0]
    keys[s0] = -1
    k = torch.full((16,), 7, dtype=torch.int64)
    t = torch.full((16,), 500, dtype=torch.int64)
    with pytest.raises(RuntimeError, match="invariant violated after step 2"):
        op.process(k, t, torch.ones(16, dtype=torch.int64))


def test_host_sanitizer_harness():
    from mxstream.build import build_sanitize

    exe = build_sanitize()
    res = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert res.returncode == 0, res.stderr[-3000:]
    assert "ERROR: AddressSanitizer" not in res.stderr
    assert "runtime error" not in res.stderr
    assert "sanitize_main ok" in res.stdout


def test_thread_sanitizer_harness():
    """ThreadSanitizer over the threaded host code: pinned-slot file reader, socket source
    (incl. close() from another thread while recv() blocks), the session store's spill-worker
    hand-off and concurrent key-group checkpoint writers (csrc/tests/tsan_main.cpp)."""
    import os

    from mxstream.build import build_tsan

    exe = build_tsan()
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1")
    res = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    assert "ThreadSanitizer" not in res.stderr, res.stderr[-4000:]
    assert res.returncode == 0, res.stderr[-3000:]
    assert "tsan_main ok" in res.stdout


@pytest.mark.gpu
def test_gpu_checker_matches_cpu(gpu_device):
    op = _populated_op(gpu_device)
    g = _check(op)
    cpu_keys = op.keys_g.cpu()
    c = D.check_table(cpu_keys, nsub=op.nsub, nsub_log2=op.nsub_log2, cap_log2=op.cap_log2)
    assert g == c and g["live"] == op.expected_live and g["duplicate"] == 0
    k = op.keys_g
    live = torch.nonzero(k != -1).flatten()
    k[int(live[0])] = k[int(live[1])]  # duplicate / misplaced key
    assert _check(op) == D.check_table(k.cpu(), nsub=op.nsub, nsub_log2=op.nsub_log2,
                                       cap_log2=op.cap_log2)

"""Every bench config runs end to end on the CPU at a tiny size and prints one JSON line
(mxstream/models/bench_configs.py; the GPU runs use the same code paths at full size)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CASES = {
    "1": ["--config", "1", "--batch", "65536"],
    "2": ["--config", "2", "--batch", "65536", "--keys", "1000"],
    "2-spill": ["--config", "2", "--spill", "--batch", "65536"],
    "4": ["--config", "4", "--batch", "65536"],
    "4-latency": ["--config", "4", "--batch", "65536", "--latency-fire", "8"],
    "4-spill": ["--config", "4", "--spill", "--batch", "65536"],
    "5": ["--config", "5", "--batch", "65536"],
    "6": ["--config", "6", "--batch", "65536"],
    "7": ["--config", "7", "--lines", "200000", "--batch", "65536"],
    "8": ["--config", "8", "--batch", "65536"],
    "9": ["--config", "9", "--lines", "200000", "--batch", "65536"],
}


@pytest.mark.parametrize("name", list(CASES))
def test_bench_config_runs_on_cpu(name):
    cmd = [sys.executable, "-m", "mxstream.models.bench_configs", *CASES[name], "--device", "cpu",
           "--steps", "2", "--warmup", "1"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, OMP_NUM_THREADS="2"))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["value"] > 0 and d["metric"]

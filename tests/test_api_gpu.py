"""The DataStream API with native operators on the GPU: the reference jobs' README outputs and
differential checks against the exact host operators (native off)."""
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _cuda_device(monkeypatch, gpu_device):
    monkeypatch.setenv("MXS_DEVICE", "cuda")


def test_reference_jobs_on_gpu():
    import test_reference_jobs as R

    R.test_compute_cpu_max_readme()
    R.test_compute_cpu_avg_readme()
    R.test_compute_cpu_middle_readme()
    R.test_bandwidth_monitor_tumbling_readme()
    R.test_bandwidth_monitor_sliding_readme()
    for native in ("off", "auto"):
        R.test_bandwidth_event_time_readme(native)


def test_native_operators_match_host_on_gpu():
    from collections import Counter

    import numpy as np

    import test_api_native as N

    rng = np.random.default_rng(4)
    keys = ["a", "b", "c", "d", "www.163.com"]
    for trial in range(6):
        ev = [(keys[int(rng.integers(0, 5))], int(rng.integers(0, 1000)), int(rng.integers(0, 20_000)))
              for _ in range(int(rng.integers(5, 40)))]
        assert Counter(N._run(ev, 2400, 1200, 500, 0, "auto")) == \
            Counter(N._run(ev, 2400, 1200, 500, 0, "off"))
        assert N._run_rolling(ev, "max", "auto") == N._run_rolling(ev, "max", "off")
        assert Counter(N._run_sessions(ev, 1500, 500, 2000, "auto")) == \
            Counter(N._run_sessions(ev, 1500, 500, 2000, "off"))
        assert Counter(N._run_median(ev, 4000, 2000, 1000, 3000, "auto")) == \
            Counter(N._run_median(ev, 4000, 2000, 1000, 3000, "off"))


def test_native_count_windows_match_host_on_gpu():
    from collections import Counter

    import numpy as np

    import test_api_native as N

    rng = np.random.default_rng(7)
    keys = ["a", "b", "c", "10.8.22.1"]
    for trial in range(8):
        ev = [(keys[int(rng.integers(0, 4))], int(rng.integers(0, 1000)))
              for _ in range(int(rng.integers(5, 80)))]
        n = int(rng.integers(1, 7))
        for agg in ("reduce", "max", "sum", "avg"):
            assert Counter(N._run_count(ev, n, "auto", agg)) == \
                Counter(N._run_count(ev, n, "off", agg))

"""K5 gate statistics (ops/gatestats.py + gatestats.hip) and K6 storm counts (storm.hip)."""

import numpy as np
import pytest

from llm_slo_ebpf_toolkit_amd.correlation.retry_storm import RetryStormDetector
from llm_slo_ebpf_toolkit_amd.evaluation import releasegate as rg
from llm_slo_ebpf_toolkit_amd.ops import gatestats as gs
from llm_slo_ebpf_toolkit_amd.ops import storm


def _samples(seed=0, ties=False):
    rng = np.random.default_rng(seed)
    x, y = rng.normal(100, 10, 57), rng.normal(104, 12, 43)
    if ties:
        x, y = np.round(x / 5) * 5, np.round(y / 5) * 5
    return x, y


@pytest.mark.parametrize("ties", [False, True])
def test_rank_counts_reproduce_mann_whitney_and_cliffs(ties):
    x, y = _samples(1, ties)
    p, d, _ = gs.stats_from_rank_counts(gs.rank_counts_np(x, y), len(x), len(y))
    assert p == pytest.approx(rg.mann_whitney_p(x, y), rel=1e-12, abs=1e-15)
    assert d == pytest.approx(rg.cliffs_delta(x, y), rel=1e-12)


def test_bootstrap_np_matches_explicit_resampling():
    x, y = _samples(2)
    q = gs.bootstrap_quantiles_np(x, y, 0.95, 64, 42)
    # explicit definition: resample with the counter stream, sort, REF linear quantile
    for set_id, v in enumerate((np.sort(x), np.sort(y))):  # indices address the sorted sample
        idx = gs._indices_np(len(v), set_id, 64, 42)
        for it in range(64):
            r = np.sort(v[idx[it]])
            pos = 0.95 * (len(r) - 1)
            lo, hi = int(np.floor(pos)), int(np.ceil(pos))
            ref = r[lo] * (1 - (pos - lo)) + r[hi] * (pos - lo)
            assert q[set_id, it] == ref


def test_bootstrap_ci_deterministic_and_brackets_delta():
    x, y = _samples(3)
    a = rg.bootstrap_delta_ci(x, y, 0.95, 1000, 42)
    b = rg.bootstrap_delta_ci(x, y, 0.95, 1000, 42)
    assert a == b and a[0] <= a[1]
    assert a[0] <= rg.quantile(list(x), 0.95) - rg.quantile(list(y), 0.95) + 25


def test_storm_oracle_matches_streaming_detector():
    rng = np.random.default_rng(4)
    pods = rng.integers(0, 5, 400)
    ts = np.sort(rng.integers(0, 60_000_000_000, 400))
    counts, n_storm = storm.windowed_counts_np(pods, ts)
    det = RetryStormDetector()
    order = np.lexsort((ts, pods))
    exp = np.empty(400, dtype=np.int64)
    for i in order:
        det.record(str(pods[i]), int(ts[i]))
        exp[i] = det.count(str(pods[i]), int(ts[i]))
    np.testing.assert_array_equal(counts, exp)
    assert n_storm == int((exp >= 5).sum())


@pytest.mark.gpu
def test_gpu_bootstrap_bit_identical():
    for seed in (42, 7):
        x, y = _samples(seed)
        np.testing.assert_array_equal(gs.bootstrap_quantiles(x, y, 0.95, 1000, seed),
                                      gs.bootstrap_quantiles_np(x, y, 0.95, 1000, seed))
    x, y = _samples(9)
    np.testing.assert_array_equal(gs.bootstrap_quantiles(x[:1], y, 0.5, 10, 1),
                                  gs.bootstrap_quantiles_np(x[:1], y, 0.5, 10, 1))


@pytest.mark.gpu
@pytest.mark.parametrize("ties", [False, True])
def test_gpu_rank_counts(ties):
    x, y = _samples(5, ties)
    np.testing.assert_array_equal(gs.rank_counts(x, y), gs.rank_counts_np(x, y))


@pytest.mark.gpu
def test_gpu_storm_counts():
    rng = np.random.default_rng(6)
    pods = rng.integers(0, 50, 20000)
    ts = rng.integers(0, 120_000_000_000, 20000)
    c_gpu, n_gpu = storm.windowed_counts(pods, ts)
    c_np, n_np = storm.windowed_counts_np(pods, ts)
    np.testing.assert_array_equal(c_gpu, c_np)
    assert n_gpu == n_np

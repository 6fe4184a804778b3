"""Session replay over slot groups (gw_session.hip seg_run): on large tables the radix sort
groups records by slot >> gshift (24 sort bits, 3 passes) and one thread replays the
interleaved runs of up to 2^gshift slots, each in arrival order; punted runs continue in
the wide pass from the slot's first record of the group.  GW_SESSION_SORT_BITS=4 forces
16-slot groups on the small tables of these tests; results equal the oracle's."""
import numpy as np
import pytest

from gpu_helpers import compare, random_stream, run_gpu, run_oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def grouped(monkeypatch):
    monkeypatch.setenv("GW_SESSION_SORT_BITS", "4")


@pytest.mark.parametrize("agg", ["count", "sum_i64", "avg_f64", "max_f64"])
@pytest.mark.parametrize("gap,lateness", [(100, 0), (1500, 0), (100, 2000)])
def test_grouped_sessions_match_oracle(oracle_lib, agg, gap, lateness):
    kw = dict(assigner="session", gap=gap, agg=agg, lateness=lateness)
    keys, ts, vals, batches = random_stream(seed=gap + lateness, n=30000, num_keys=3000, n_batches=15,
                                            disorder=1500 + lateness, wm_lag=300, agg=agg)
    g, glate, _ = run_gpu(kw, keys, ts, vals, batches, capacity_hint=8192)
    o, olate = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert glate == olate
    assert compare(g, o, agg in ("avg_f64", "sum_f64")) == []


def test_grouped_sessions_many_in_flight(oracle_lib):
    """Keys with many sessions in one group: lists outgrow the lane, runs move to the wide
    table mid-group while the group's other slots stay inline."""
    kw = dict(assigner="session", gap=100, agg="sum_i64")
    rng = np.random.default_rng(8)
    n = 6000
    keys = rng.integers(0, 300, n).astype(np.int64)
    ts = rng.integers(0, 600_000, n).astype(np.int64)
    vals = rng.integers(0, 100, n).astype(np.int64)
    batches = [(0, 2000, -1), (2000, 4000, 50_000), (4000, 6000, 300_000)]
    g, glate, _ = run_gpu(kw, keys, ts, vals, batches, capacity_hint=1024)
    o, olate = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert glate == olate
    assert compare(g, o, False) == []

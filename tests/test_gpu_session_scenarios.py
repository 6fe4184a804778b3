"""Session ingest (gw_session.hip: k_sess_prep / gw_sort.hip radix sort by slot /
k_sess_segment / k_sess_migrate / k_sess_wide) against the oracle on the shapes that stress it:

* batches of 1.2M records over 60k keys (runs of many records per key, the table grown under
  the batch), every session aggregate, with and without allowed lateness;
* a 2^25-slot table under small batches (26 sorted slot bits: three radix passes);
* a hot key carrying 40% of the records (one long run) and the sentinel key Long.MIN_VALUE
  (the table's empty marker) among ordinary keys, on a table grown from 1024 slots;
* keys that open many sessions within one batch: they outgrow the thread's lane and the slot,
  migrate to the wide table, and later batches replay them there -- under allowed lateness and
  the late side output too;
* more keys than a small starting table has slots.
Parity: bit-exact for integer aggregates, 1e-6 relative for f64 averages (MergingWindowSet.java:153-224,
WindowOperator.java:303-403)."""
import numpy as np
import pytest

from flink_amd import _native as N
from flink_amd import windowing as W
from gpu_helpers import compare, random_stream, run_gpu, run_oracle

pytestmark = pytest.mark.gpu

AGGS = ["count", "sum_i64", "avg_f64", "max_f64", "min_i64"]


@pytest.mark.parametrize("agg", AGGS)
@pytest.mark.parametrize("gap,lateness", [(100, 0), (2000, 0), (300, 1500)])
def test_large_batches_match_oracle(oracle_lib, agg, gap, lateness):
    kw = dict(assigner="session", gap=gap, agg=agg, lateness=lateness)
    keys, ts, vals, batches = random_stream(seed=gap * 7 + lateness, n=2_400_000, num_keys=60_000, n_batches=2,
                                            ts_step=1, disorder=800 + lateness, wm_lag=400, agg=agg)
    g, glate, _ = run_gpu(kw, keys, ts, vals, batches, capacity_hint=2048, max_batch=1 << 21)
    o, olate = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert glate == olate
    assert compare(g, o, agg in ("avg_f64", "sum_f64")) == []


@pytest.mark.parametrize("agg", ["sum_i64", "avg_f64"])
def test_large_table_small_batches(oracle_lib, agg):
    kw = dict(assigner="session", gap=400, agg=agg)
    keys, ts, vals, batches = random_stream(seed=21, n=480_000, num_keys=90_000, n_batches=4, ts_step=1,
                                            disorder=300, wm_lag=300, agg=agg)
    g, glate, _ = run_gpu(kw, keys, ts, vals, batches, capacity_hint=20_000_000)
    o, olate = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert glate == olate
    assert compare(g, o, agg == "avg_f64") == []


@pytest.mark.parametrize("agg", ["sum_i64", "avg_f64", "sum_f64"])
def test_hot_key_and_sentinel(oracle_lib, agg):
    kw = dict(assigner="session", gap=50, agg=agg)
    keys, ts, vals, batches = random_stream(seed=8, n=300_000, num_keys=20_000, n_batches=3, ts_step=1,
                                            disorder=200, wm_lag=200, agg=agg)
    rng = np.random.default_rng(9)
    keys[rng.random(keys.size) < 0.4] = 77
    keys[::89] = W.LONG_MIN
    g, glate, _ = run_gpu(kw, keys, ts, vals, batches, capacity_hint=1024)
    o, olate = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert glate == olate
    assert compare(g, o, agg == "avg_f64") == []


@pytest.mark.parametrize("lateness,side", [(0, False), (2000, False), (2000, True)])
def test_many_sessions_per_key_mid_batch(oracle_lib, lateness, side):
    kw = dict(assigner="session", gap=100, agg="sum_i64", lateness=lateness)
    rng = np.random.default_rng(11)
    n = 60_000
    keys = rng.integers(0, 500, n).astype(np.int64)
    ts = np.sort(rng.integers(0, 3_000_000, n)).astype(np.int64) - rng.integers(0, 5000, n)
    vals = rng.integers(0, 1000, n).astype(np.int64)
    batches = [(0, 20_000, 400_000), (20_000, 40_000, 1_500_000), (40_000, 60_000, 2_000_000)]
    flags = N.FLAG_LATE_SIDE_OUTPUT if side else 0
    op = W.GpuWindowOperator(W.EventTimeSessionWindows.with_gap(100), "sum_i64", allowed_lateness=lateness,
                             capacity_hint=1024, flags=flags).open()
    ora = oracle_lib.OracleOperator(oracle_lib.make_config(**kw, flags=flags))
    g, o = [], []
    try:
        for lo, hi, wm in batches + [(n, n, W.LONG_MAX)]:
            if hi > lo:
                op.process_batch(keys[lo:hi], ts[lo:hi], vals[lo:hi])
                ora.process_batch(keys[lo:hi], ts[lo:hi], vals[lo:hi])
            op.advance_watermark(wm)
            ora.process_watermark(wm)
            k, s, e, r = op.drain()
            g.append((k, s, e, r.view(np.int64)))
            o.append(ora.drain())
        if side:
            gl = sorted(zip(*[x.tolist() for x in op.drain_late()]))
            ol = sorted(zip(*[x.tolist() for x in ora.drain_late()]))
            assert gl == ol
        assert op.num_late_records_dropped == ora.late_dropped
    finally:
        op.close()
        ora.close()
    assert compare(g, o, False) == []


def test_more_keys_than_slots(oracle_lib):
    kw = dict(assigner="session", gap=30, agg="sum_i64")
    keys, ts, vals, batches = random_stream(seed=9, n=120_000, num_keys=4000, n_batches=6, ts_step=1,
                                            disorder=100, wm_lag=100)
    keys[::97] = W.LONG_MIN
    g, glate, _ = run_gpu(kw, keys, ts, vals, batches, capacity_hint=1024)
    o, olate = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert glate == olate
    assert compare(g, o, False) == []

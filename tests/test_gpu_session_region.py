"""Bucketed session ingest (gw_session.hip k_sb_part P1 / k_sb_cols / k_sb_part P2 /
k_sb_replay; GW_SESSION_PATH=region, opt-in: the sort path is the default) against the oracle:

* buckets holding many records of a batch (a small table under large batches: hundreds to
  thousands of records per bucket, so the LDS radix sort, the ordered head list and runs of
  several records per home slot all work at more than one wave's worth), with and without
  the second partition pass (P2 runs when a batch needs more than 2^6 buckets);
* a large table under a small batch (the bucket count set by the sort key's home-bit limit);
* home slots shared by several keys (more keys than home slots in a bucket);
* a hot key whose bucket exceeds kSbCap (1024) records in one batch: the bucket goes to the
  punt list and the sort path replays it (stats()["session_punted"] counts it);
* keys that need the wide table mid-batch (more sessions than the lane holds), under allowed
  lateness and the late side output too;
* the sentinel key Long.MIN_VALUE among ordinary keys.
Parity: bit-exact for integer aggregates, 1e-6 relative for f64 (MergingWindowSet.java:153-224,
WindowOperator.java:303-403)."""
import numpy as np
import pytest

from flink_amd import _native as N
from flink_amd import windowing as W
from gpu_helpers import compare, random_stream, run_gpu, run_oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def region_path(monkeypatch):
    monkeypatch.setenv("GW_SESSION_PATH", "region")

AGGS = ["count", "sum_i64", "avg_f64", "max_f64", "min_i64"]


@pytest.mark.parametrize("agg", AGGS)
@pytest.mark.parametrize("gap,lateness", [(100, 0), (2000, 0), (300, 1500)])
def test_dense_buckets_match_oracle(oracle_lib, agg, gap, lateness):
    kw = dict(assigner="session", gap=gap, agg=agg, lateness=lateness)
    # 1.2M records per batch: the table grows to 2^21 slots, 1024 buckets of ~1170 records
    keys, ts, vals, batches = random_stream(seed=gap * 7 + lateness, n=2_400_000, num_keys=60_000, n_batches=2,
                                            ts_step=1, disorder=800 + lateness, wm_lag=400, agg=agg)
    g, glate, st = run_gpu(kw, keys, ts, vals, batches, capacity_hint=2048, max_batch=1 << 21)
    o, olate = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert glate == olate
    assert compare(g, o, agg in ("avg_f64", "sum_f64")) == []


@pytest.mark.parametrize("agg", ["sum_i64", "avg_f64"])
def test_large_table_small_batches(oracle_lib, agg):
    """2^25 slots, 120k-record batches: 2^7 buckets (the home bits per bucket are capped), so
    both partition passes run on a batch the mean-size rule alone would single-pass."""
    kw = dict(assigner="session", gap=400, agg=agg)
    keys, ts, vals, batches = random_stream(seed=21, n=480_000, num_keys=90_000, n_batches=4, ts_step=1,
                                            disorder=300, wm_lag=300, agg=agg)
    g, glate, st = run_gpu(kw, keys, ts, vals, batches, capacity_hint=20_000_000)
    o, olate = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert glate == olate
    assert compare(g, o, agg == "avg_f64") == []


@pytest.mark.parametrize("agg", ["sum_i64", "avg_f64"])
def test_hot_key_bucket_goes_to_sort_path(oracle_lib, agg):
    """One key carries 40% of 100k records per batch: its bucket exceeds kSbCap records."""
    kw = dict(assigner="session", gap=50, agg=agg)
    keys, ts, vals, batches = random_stream(seed=5, n=300_000, num_keys=20_000, n_batches=3, ts_step=1,
                                            disorder=200, wm_lag=200, agg=agg)
    rng = np.random.default_rng(6)
    keys[rng.random(keys.size) < 0.4] = 77
    g, glate, st = run_gpu(kw, keys, ts, vals, batches, capacity_hint=32768)
    o, olate = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert glate == olate
    assert compare(g, o, agg == "avg_f64") == []
    assert st["session_punted"] >= 3 * 16384


@pytest.mark.parametrize("lateness,side", [(0, False), (2000, False), (2000, True)])
def test_many_sessions_per_key_mid_batch(oracle_lib, lateness, side):
    """Sparse timestamps: keys open many sessions within one batch, outgrow the lane and the
    slot, migrate to the wide table and punt their later records."""
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
        assert op.stats()["session_punted"] > 0
    finally:
        op.close()
        ora.close()
    assert compare(g, o, False) == []


def test_sentinel_key_and_shared_home_slots(oracle_lib):
    """Long.MIN_VALUE (the table's empty marker) as a key, and 4x more keys than home slots."""
    kw = dict(assigner="session", gap=30, agg="sum_i64")
    keys, ts, vals, batches = random_stream(seed=9, n=120_000, num_keys=4000, n_batches=6, ts_step=1,
                                            disorder=100, wm_lag=100)
    keys[::97] = W.LONG_MIN
    g, glate, _ = run_gpu(kw, keys, ts, vals, batches, capacity_hint=1024)
    o, olate = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert glate == olate
    assert compare(g, o, False) == []


def test_f64_sessions_take_no_punts(oracle_lib):
    """Keys that never hold two sessions at once (records ~3 s apart, gap 60 s) never leave the
    bucketed path.  (A key with more sessions in flight than its slot holds -- one for averages --
    lives in the wide table from then on, and its records take the sort path; so does every
    key of a bucket beyond kSbCap records, which enough keys per bucket keep away.)"""
    kw = dict(assigner="session", gap=60_000, agg="avg_f64")
    keys, ts, vals, batches = random_stream(seed=13, n=80_000, num_keys=3000, n_batches=5, ts_step=1,
                                            disorder=300, wm_lag=300, agg="avg_f64")
    g1, _, s1 = run_gpu(kw, keys, ts, vals, batches, capacity_hint=4096)
    o, _ = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert compare(g1, o, True) == []
    assert s1["session_punted"] == 0

"""Keyed sort session ingest (gw_session.hip k_sess_kprep / radix sort by key code /
k_sess_kseg; the default path) against the oracle:

* every key's records form one run of the sorted codes, replayed in arrival order;
* code collisions: GW_SESSION_KEY_BITS=4 sorts only 4 bits of the code, so each run mixes
  thousands of keys and sp_run replays every key of a run in order of its first record
  (the default sorts lcap + 2 bits or more, where two keys share a run only by chance);
* keys that outgrow the lane or live in the wide table are punted with their records and the
  slot sort path replays them at the next sync (stats()["session_punted"]);
* a hot key, the sentinel key Long.MIN_VALUE, a table grown under the batch;
* allowed lateness and the late side output (the ingest then syncs at once).
Parity: bit-exact for integer aggregates, 1e-6 relative for f64 (MergingWindowSet.java:153-224,
WindowOperator.java:303-403)."""
import numpy as np
import pytest

from flink_amd import _native as N
from flink_amd import windowing as W
from gpu_helpers import compare, random_stream, run_gpu, run_oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def keyed_path(monkeypatch):
    monkeypatch.setenv("GW_SESSION_PATH", "keyed")


AGGS = ["count", "sum_i64", "avg_f64", "max_f64", "min_i64"]


@pytest.mark.parametrize("agg", AGGS)
@pytest.mark.parametrize("gap,lateness", [(100, 0), (2000, 0), (300, 1500)])
def test_keyed_matches_oracle(oracle_lib, agg, gap, lateness):
    kw = dict(assigner="session", gap=gap, agg=agg, lateness=lateness)
    keys, ts, vals, batches = random_stream(seed=gap * 5 + lateness, n=1_200_000, num_keys=60_000, n_batches=3,
                                            ts_step=1, disorder=800 + lateness, wm_lag=400, agg=agg)
    g, glate, st = run_gpu(kw, keys, ts, vals, batches, capacity_hint=2048, max_batch=1 << 20)
    o, olate = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert glate == olate
    assert compare(g, o, agg in ("avg_f64", "sum_f64")) == []


@pytest.mark.parametrize("agg", ["sum_i64", "avg_f64", "max_f64"])
def test_colliding_codes_mix_keys_in_runs(oracle_lib, monkeypatch, agg):
    """4 sorted code bits: 16 runs per batch, each holding thousands of keys interleaved."""
    monkeypatch.setenv("GW_SESSION_KEY_BITS", "4")
    kw = dict(assigner="session", gap=200, agg=agg)
    keys, ts, vals, batches = random_stream(seed=31, n=60_000, num_keys=3000, n_batches=4, ts_step=1,
                                            disorder=300, wm_lag=300, agg=agg)
    g, glate, _ = run_gpu(kw, keys, ts, vals, batches, capacity_hint=4096)
    o, olate = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert glate == olate
    assert compare(g, o, agg == "avg_f64") == []


@pytest.mark.parametrize("lateness,side", [(0, False), (2000, False), (2000, True)])
def test_punts_to_the_wide_table(oracle_lib, lateness, side):
    """Sparse timestamps: keys open many sessions within one batch, outgrow the lane and the
    slot, migrate to the wide table; their later batches punt to the slot sort path."""
    kw = dict(assigner="session", gap=100, agg="sum_i64", lateness=lateness)
    rng = np.random.default_rng(17)
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


@pytest.mark.parametrize("agg", ["sum_i64", "avg_f64"])
def test_hot_key_and_sentinel(oracle_lib, agg):
    """One key carries 40% of the records (one long run), Long.MIN_VALUE is a key too, and the
    table grows from 1024 slots under the first batch."""
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


def test_keyed_equals_slot_sort(oracle_lib, monkeypatch):
    """The two sort paths fire the same rows on the same stream (f64 sums bit-equal: both
    fold each key's records in arrival order)."""
    kw = dict(assigner="session", gap=500, agg="sum_f64")
    keys, ts, vals, batches = random_stream(seed=41, n=400_000, num_keys=50_000, n_batches=4, ts_step=1,
                                            disorder=400, wm_lag=400, agg="sum_f64")
    g1, l1, _ = run_gpu(kw, keys, ts, vals, batches, capacity_hint=65536)
    monkeypatch.setenv("GW_SESSION_PATH", "sort")
    g2, l2, _ = run_gpu(kw, keys, ts, vals, batches, capacity_hint=65536)
    assert l1 == l2
    assert compare(g1, g2, False) == []

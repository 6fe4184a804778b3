"""Narrow region-path records (gw_pane.hip kFmtNar: the 32-bit key itself + a 28-bit value
beside the ring position, 8 B per record, 4 B for COUNT) against the oracle:

* every integer aggregate, tumbling / sliding / allowed lateness, single- and two-pass tables;
* records that do not fit -- keys beyond 32 bits or negative, values beyond 28 bits, COUNT keys
  beyond 28 bits -- go to the deferred list (exact); a few of them keep narrow records, many
  of them switch the handle to compact records after the window;
* spills (records of a full region) leave the buffer through k_rgn_collect_nar.
Parity: bit-exact for integer results, 1e-6 relative for averages."""
import numpy as np
import pytest

from flink_amd import _native as N
from flink_amd import windowing as W
from gpu_helpers import compare, make_assigner

pytestmark = pytest.mark.gpu


def stream(seed, n, num_keys, n_batches, key_hi=1 << 31, odd_frac=0.0, odd="key", disorder=400, wm_lag=500):
    rng = np.random.default_rng(seed)
    keys = rng.integers(0, key_hi, num_keys).astype(np.int64)[rng.integers(0, num_keys, n)]
    ts = np.arange(n, dtype=np.int64) * 20_000 // n - rng.integers(0, disorder + 1, n)
    vals = rng.integers(-(10 ** 6), 10 ** 6, n).astype(np.int64)
    m = rng.random(n) < odd_frac
    if odd == "key":  # keys that do not fit: beyond 32 bits, or negative
        keys[m] = np.where(rng.random(int(m.sum())) < 0.5, rng.integers(1 << 32, 1 << 60, int(m.sum())),
                           -rng.integers(1, 1 << 40, int(m.sum())))
    elif odd == "val":  # values beyond the 28-bit field
        vals[m] = np.where(rng.random(int(m.sum())) < 0.5, rng.integers(1 << 27, 1 << 40, int(m.sum())),
                           -rng.integers((1 << 27) + 1, 1 << 40, int(m.sum())))
    elif odd == "edge":  # exactly at the limits
        vals[m] = rng.choice(np.array([(1 << 27) - 1, -(1 << 27), 1 << 27, -(1 << 27) - 1], np.int64), int(m.sum()))
        keys[m] = rng.choice(np.array([0, (1 << 32) - 1, 1 << 32, (1 << 28) - 1, 1 << 28], np.int64), int(m.sum()))
    cuts = np.linspace(0, n, n_batches + 1).astype(np.int64)
    batches = [(int(cuts[b]), int(cuts[b + 1]), int(ts[:cuts[b + 1]].max()) - wm_lag - 1) for b in range(n_batches)]
    return keys, ts, vals, batches


def run(oracle_lib, kw, keys, ts, vals, batches, capacity_hint, flags=0):
    op = W.GpuWindowOperator(make_assigner(kw), kw["agg"], kw.get("lateness", 0), capacity_hint=capacity_hint,
                             flags=N.FLAG_FORCE_REGION | flags).open()
    ora = oracle_lib.OracleOperator(oracle_lib.make_config(**kw))
    g, o, fmts = [], [], []
    try:
        for lo, hi, wm in batches:
            op.process_batch(keys[lo:hi], ts[lo:hi], vals[lo:hi])
            fmts.append(op.stats()["region_format"])
            op.advance_watermark(wm)
            k, s, e, r = op.drain()
            g.append((k, s, e, r.view(np.int64)))
            ora.process_batch(keys[lo:hi], ts[lo:hi], vals[lo:hi])
            ora.process_watermark(wm)
            o.append(ora.drain())
        op.advance_watermark(W.LONG_MAX)
        k, s, e, r = op.drain()
        g.append((k, s, e, r.view(np.int64)))
        ora.process_watermark(W.LONG_MAX)
        o.append(ora.drain())
        assert op.num_late_records_dropped == ora.late_dropped
    finally:
        op.close()
        ora.close()
    return g, o, fmts


CFGS = [dict(assigner="tumbling", size=1000, slide=1000), dict(assigner="sliding", size=2000, slide=500),
        dict(assigner="sliding", size=1500, slide=500, lateness=300)]  # ring 6 <= 8
AGGS = ["count", "sum_i64", "sum_i32", "min_i64", "max_i64", "avg_i64"]


@pytest.mark.parametrize("kw", CFGS, ids=["tumbling", "sliding", "lateness"])
@pytest.mark.parametrize("agg", AGGS)
@pytest.mark.parametrize("cap", [1 << 14, 1 << 19], ids=["single-pass", "two-pass"])
def test_narrow_records_against_oracle(oracle_lib, kw, agg, cap):
    kw = dict(kw, agg=agg)
    keys, ts, vals, batches = stream(7, 120_000, 9_000, 10, key_hi=(1 << 28) - 1)
    g, o, fmts = run(oracle_lib, kw, keys, ts, vals, batches, cap)
    assert compare(g, o, agg == "avg_i64") == []
    assert 2 in fmts  # narrow records ran


@pytest.mark.parametrize("odd,frac", [("key", 0.005), ("key", 0.5), ("val", 0.005), ("val", 0.6), ("edge", 0.2)])
@pytest.mark.parametrize("agg", ["count", "sum_i64", "max_i64", "avg_i64"])
def test_records_beyond_narrow_are_exact(oracle_lib, odd, frac, agg):
    kw = dict(assigner="sliding", size=2000, slide=500, agg=agg)
    keys, ts, vals, batches = stream(19, 150_000, 12_000, 12, key_hi=(1 << 32) - 1, odd_frac=frac, odd=odd)
    g, o, fmts = run(oracle_lib, kw, keys, ts, vals, batches, 1 << 19)
    assert compare(g, o, agg == "avg_i64") == []
    if frac > 0.1 and not (odd == "val" and agg == "count"):
        # too many misfits: compact records from the next window (and wide ones after that
        # when the values do not fit compact records' 32 bits either)
        assert fmts[0] == 2 and 1 in fmts and fmts[-1] == (0 if odd == "val" else 1)


def test_narrow_spills_and_growth(oracle_lib):
    """A tiny table: regions fill, spilled narrow records go to the deferred list, the table grows."""
    kw = dict(assigner="sliding", size=2000, slide=500, agg="sum_i64")
    keys, ts, vals, batches = stream(23, 200_000, 60_000, 8, key_hi=(1 << 32) - 1)
    g, o, fmts = run(oracle_lib, kw, keys, ts, vals, batches, 1 << 13)
    assert compare(g, o, False) == []


@pytest.mark.parametrize("agg", ["count", "sum_i64"])
def test_no_narrow_flag_keeps_compact(oracle_lib, agg):
    kw = dict(assigner="sliding", size=2000, slide=500, agg=agg)
    keys, ts, vals, batches = stream(29, 80_000, 5_000, 6)
    g, o, fmts = run(oracle_lib, kw, keys, ts, vals, batches, 1 << 19, flags=N.FLAG_NO_NARROW)
    assert compare(g, o, False) == []
    assert set(fmts) <= {-1, 1}


@pytest.mark.parametrize("agg", ["sum_i64", "count"])
def test_narrow_two_pass_regions_fill_and_spill(oracle_lib, agg):
    """A two-pass table (2^19 slots: 256 regions, P2 by (super-region, ring position), the
    k_rgn_apply_nar flush) that one buffered window overfills with new keys: full regions
    leave records unapplied, the spill pass marks them, k_rgn_collect_nar2 parks them on the
    deferred list, the table grows and the merge applies them -- exact against the oracle."""
    kw = dict(assigner="sliding", size=2000, slide=500, agg=agg)
    rng = np.random.default_rng(41)
    n = 1_400_000
    keys = rng.integers(0, 720_000, n).astype(np.int64)
    ts = np.arange(n, dtype=np.int64) * 6_000 // n - rng.integers(0, 300, n)
    vals = rng.integers(-(10 ** 6), 10 ** 6, n).astype(np.int64)
    cuts = [0, 1_000_000, 1_200_000, n]  # the first batch alone brings ~540K distinct keys
    batches = [(cuts[b], cuts[b + 1], int(ts[:cuts[b + 1]].max()) - 400) for b in range(3)]
    g, o, fmts = run(oracle_lib, kw, keys, ts, vals, batches, 1 << 19)
    assert compare(g, o, False) == []
    assert fmts[0] == 2

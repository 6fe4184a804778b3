"""Compact region-path records (gw_pane.hip cmp_pack: the key's hash word with the ring
position in its bucket bits + a 32-bit value, 12 B per record, 8 B for COUNT) against
the oracle, on tables large enough for them (>= 16 regions; two-pass and buffered at
>= 256 regions):

* every integer aggregate, tumbling / sliding / allowed lateness, single- and two-pass;
* values beyond 32 bits go to the deferred list (exact), a few of them (compact records
  stay on) or nearly all of them (the operator turns compact records off after a flush);
* spills (records of a full region) leave the buffer through k_rgn_collect_cmp.
Parity: bit-exact for integer results, 1e-6 relative for averages."""
import zlib

import numpy as np
import pytest

from flink_amd import _native as N
from flink_amd import windowing as W
from gpu_helpers import compare, make_assigner

pytestmark = pytest.mark.gpu


def stream(seed, n, num_keys, n_batches, wide_frac=0.0, disorder=400, wm_lag=500):
    rng = np.random.default_rng(seed)
    keys = rng.integers(-(1 << 62), 1 << 62, num_keys).astype(np.int64)[rng.integers(0, num_keys, n)]
    ts = np.arange(n, dtype=np.int64) * 20_000 // n - rng.integers(0, disorder + 1, n)
    vals = rng.integers(-(10 ** 6), 10 ** 6, n).astype(np.int64)
    wide = rng.random(n) < wide_frac
    vals[wide] = rng.integers(-(1 << 50), 1 << 50, int(wide.sum()))
    cuts = np.linspace(0, n, n_batches + 1).astype(np.int64)
    batches = [(int(cuts[b]), int(cuts[b + 1]), int(ts[:cuts[b + 1]].max()) - wm_lag - 1) for b in range(n_batches)]
    return keys, ts, vals, batches


def run(oracle_lib, kw, keys, ts, vals, batches, capacity_hint):
    op = W.GpuWindowOperator(make_assigner(kw), kw["agg"], kw.get("lateness", 0), capacity_hint=capacity_hint,
                             flags=N.FLAG_FORCE_REGION).open()
    ora = oracle_lib.OracleOperator(oracle_lib.make_config(**kw))
    vb = vals.view(np.int64) if vals.dtype == np.float64 else vals
    g, o = [], []
    try:
        for lo, hi, wm in batches:
            op.process_batch(keys[lo:hi], ts[lo:hi], vals[lo:hi])
            op.advance_watermark(wm)
            k, s, e, r = op.drain()
            g.append((k, s, e, r.view(np.int64)))
            ora.process_batch(keys[lo:hi], ts[lo:hi], vb[lo:hi])
            ora.process_watermark(wm)
            o.append(ora.drain())
        op.advance_watermark(W.LONG_MAX)
        k, s, e, r = op.drain()
        g.append((k, s, e, r.view(np.int64)))
        ora.process_watermark(W.LONG_MAX)
        o.append(ora.drain())
        assert op.num_late_records_dropped == ora.late_dropped
        stats = op.stats()
    finally:
        op.close()
        ora.close()
    return g, o, stats


INT_AGGS = ["count", "sum_i64", "sum_i32", "min_i64", "max_i64", "avg_i64"]
CFGS = [dict(assigner="tumbling", size=2000, slide=2000),
        dict(assigner="sliding", size=4000, slide=1000),
        dict(assigner="sliding", size=3000, slide=1000, lateness=2500)]


@pytest.mark.parametrize("agg", INT_AGGS)
@pytest.mark.parametrize("cfg", CFGS, ids=lambda c: "-".join(str(v) for v in c.values()))
@pytest.mark.parametrize("keys_n,cap", [(40_000, 65_536), (200_000, 400_000)], ids=["single_pass", "two_pass"])
def test_compact_records_match_oracle(oracle_lib, cfg, agg, keys_n, cap):
    kw = dict(cfg, agg=agg)
    n = 600_000 if keys_n < 100_000 else 2_000_000
    keys, ts, vals, batches = stream(zlib.crc32(f"{agg}{keys_n}".encode()) & 0xffff, n, keys_n, 12)
    if agg == "sum_i32":
        vals = vals.astype(np.int32).astype(np.int64)
    g, o, stats = run(oracle_lib, kw, keys, ts, vals, batches, cap)
    assert compare(g, o, agg in N.DOUBLE_RESULT) == []


@pytest.mark.parametrize("wide_frac", [0.001, 0.9])
@pytest.mark.parametrize("agg", ["sum_i64", "min_i64", "max_i64", "avg_i64"])
def test_values_beyond_32_bits(oracle_lib, agg, wide_frac):
    kw = dict(assigner="sliding", size=4000, slide=1000, agg=agg)
    keys, ts, vals, batches = stream(5, 2_000_000, 200_000, 12, wide_frac=wide_frac)
    g, o, _ = run(oracle_lib, kw, keys, ts, vals, batches, 400_000)
    assert compare(g, o, agg in N.DOUBLE_RESULT) == []


def test_compact_spills_of_full_regions(oracle_lib):
    """A table hinted far too small: regions fill, their records spill to the deferred
    list (k_rgn_collect_cmp) and the table grows; results stay exact."""
    kw = dict(assigner="sliding", size=4000, slide=1000, agg="sum_i64")
    keys, ts, vals, batches = stream(9, 1_200_000, 150_000, 6)
    g, o, stats = run(oracle_lib, kw, keys, ts, vals, batches, 40_000)
    assert compare(g, o, False) == []
    assert stats["rehashes"] > 0


def test_f64_aggregates_keep_wide_records(oracle_lib):
    kw = dict(assigner="sliding", size=4000, slide=1000, agg="avg_f64")
    keys, ts, vals, batches = stream(3, 1_000_000, 100_000, 8)
    fv = (vals.astype(np.float64) / 7.0)
    g, o, _ = run(oracle_lib, kw, keys, ts, fv, batches, 200_000)
    assert compare(g, o, True) == []

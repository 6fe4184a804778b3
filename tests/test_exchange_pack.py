"""Packed exchange records (include/gpuwin.h gw_pack_geom; gw_common.h pack_word), on the CPU:

* gw_pack_records against a numpy restatement of the packing rule (key in [0, 2^32), value in
  [-2^27, 2^27), pane within 16 of the base pane, |ts| and |offset| below 2^62), edge values
  included, and the round trip through gw_unpack_records (key and value exact, ts = the start
  of the record's pane);
* the claim the packing rests on: replacing a record's timestamp by its pane's start changes
  no row and no late count of the reference operator (the oracle) for tumbling and sliding
  windows with size >= slide (pane = gcd(size, slide)), with offsets and allowed lateness --
  WindowOperator.processElement decides by assignWindows / isWindowLate / cleanupTime, which
  depend on the pane alone (TimeWindow.getWindowStartWithOffset, SlidingEventTimeWindows
  .assignWindows, WindowOperator.java:303-403, 440-446);
* the protocol at world size 2 and 4 over gloo (KeyByExchange.exchange_packed: the same
  partition order, messages and plans as gw_exchange_batch): the union of the ranks' rows
  equals one operator's over the original stream, and most records travel packed."""
import multiprocessing as mp
import random

import numpy as np
import pytest

from flink_amd import _native as N
from tests.gpu_helpers import random_stream

LIM = 1 << 62


def np_pack(keys, ts, vals, pane, offset, base):
    """Restatement of the packing rule: (words, fits)."""
    keys, ts = np.asarray(keys, np.int64), np.asarray(ts, np.int64)
    ok = (keys >= 0) & (keys < (1 << 32)) & (ts >= -LIM) & (ts < LIM) & (-LIM <= offset < LIM)
    rel = np.where(ok, ts - offset, 0)
    q = rel // pane  # numpy floor division
    d = q - base
    ok &= (d >= 0) & (d < 16)
    v = np.zeros_like(keys) if vals is None else np.asarray(vals, np.int64)
    if vals is not None:
        ok &= (v >= -(1 << 27)) & (v < (1 << 27))
    hi = ((v.astype(np.int64) << 4) | np.where(ok, d, 0)) & 0xFFFFFFFF
    w = (keys & 0xFFFFFFFF).astype(np.uint64) | (hi.astype(np.uint64) << np.uint64(32))
    return np.where(ok, w, np.uint64(0)), ok


@pytest.mark.parametrize("size,slide,offset", [(1000, 1000, 0), (1000, 250, 0), (900, 600, -70), (5, 5, 3)])
@pytest.mark.parametrize("with_values", [True, False])
def test_pack_rule_and_round_trip(size, slide, offset, with_values):
    rng = np.random.default_rng(size + slide)
    wm = int(rng.integers(-10_000, 10_000))
    g = N.pack_geom(size, slide, offset, wm)
    pane = int(np.gcd(size, slide))
    assert g.pane == pane and g.base_pane == (wm - offset) // pane
    n = 20_000
    keys = rng.integers(-(1 << 33), 1 << 33, n)
    keys[::3] = rng.integers(0, 1 << 32, keys[::3].size)
    keys[:4] = [0, (1 << 32) - 1, 1 << 32, -1]
    ts = wm + rng.integers(-3 * pane, 20 * pane, n)
    ts[4:8] = [np.iinfo(np.int64).min, -LIM - 1, LIM, wm]
    vals = rng.integers(-(1 << 28), 1 << 28, n)
    vals[8:12] = [-(1 << 27), (1 << 27) - 1, 1 << 27, -(1 << 27) - 1]
    v = vals if with_values else None
    w, fits = N.pack_records(keys, ts, v, g)
    ew, efits = np_pack(keys, ts, v, pane, offset, g.base_pane)
    assert np.array_equal(fits, efits)
    assert np.array_equal(w[fits], ew[fits])
    assert 0.1 < fits.mean() < 0.9
    k, t, uv = N.unpack_records(w[fits], g, with_values)
    assert np.array_equal(k, keys[fits])
    assert np.array_equal(t, ts[fits] - (ts[fits] - offset) % pane)
    if with_values:
        assert np.array_equal(uv, vals[fits])


@pytest.mark.parametrize("pane,offset,wm", [(1 << 40, -(1 << 45) + 3, (1 << 61) - 12345),
                                             (1 << 58, 17, -(1 << 61)),
                                             ((1 << 59) + 7, -5, (1 << 61) + 99),  # 16 * pane overflows
                                             (3, -(1 << 61), -(1 << 61) + 10),
                                             (999_983, (1 << 61) - 1, -(1 << 61))])
def test_pack_rule_extreme_geometry(pane, offset, wm):
    """The pane offset without a 64-bit division (compares against base_pane * pane + k * pane)
    equals floor division, and the division path where those products overflow."""
    rng = np.random.default_rng(pane % 1000)
    g = N.pack_geom(pane, pane, offset, wm)
    assert g.pane == pane and g.base_pane == (wm - offset) // pane
    n = 20_000
    keys = rng.integers(0, 1 << 32, n)
    start = g.base_pane * pane + offset if abs(g.base_pane) < (1 << 62) // pane else wm
    span = min(pane, 1 << 40)
    ts = np.clip(start + rng.integers(-2 * span, 18 * span, n, dtype=np.int64) * max(pane // span, 1)
                 + rng.integers(-2, 3, n), -LIM - 2, LIM + 2).astype(np.int64)
    ts[:6] = [start, start - 1, start + 16 * pane - 1 if 16 * pane < LIM else LIM - 1, LIM - 1, -LIM, wm]
    w, fits = N.pack_records(keys, ts, None, g)
    ew, efits = np_pack(keys, ts, None, pane, offset, g.base_pane)
    assert np.array_equal(fits, efits)
    assert np.array_equal(w[fits], ew[fits])
    assert 0.1 < fits.mean() < 0.9


def test_geometry_that_does_not_pack():
    assert N.pack_geom(100, 300, 0, 5000) is None  # size < slide: gaps between windows
    assert N.pack_geom(100, 100, 0, -(1 << 63)) is None  # no watermark yet


CFGS = [dict(assigner="tumbling", size=1000, agg="count"),
        dict(assigner="sliding", size=1000, slide=250, agg="sum_i64"),
        dict(assigner="sliding", size=900, slide=300, offset=-120, agg="max_i64", lateness=500),
        dict(assigner="tumbling", size=700, offset=55, agg="min_i64", lateness=300),
        dict(assigner="sliding", size=1200, slide=400, agg="avg_i64")]


@pytest.mark.parametrize("cfg", CFGS, ids=lambda c: f"{c['assigner']}_{c['agg']}")
def test_pane_start_changes_no_window_decision(oracle_lib, cfg):
    keys, ts, vals, batches = random_stream(seed=31, n=60_000, num_keys=700, n_batches=15, disorder=4000,
                                            wm_lag=300, agg=cfg["agg"])
    pane = int(np.gcd(cfg["size"], cfg.get("slide", cfg["size"])))
    off = cfg.get("offset", 0)
    ts2 = ts - (ts - off) % pane
    outs = []
    for t in (ts, ts2):
        op = oracle_lib.OracleOperator(oracle_lib.make_config(**cfg))
        rows = []
        for lo, hi, wm in batches:
            op.process_batch(keys[lo:hi], t[lo:hi], vals[lo:hi])
            op.process_watermark(wm)
            rows.append(op.drain())
        op.process_watermark((1 << 63) - 1)
        rows.append(op.drain())
        outs.append((sorted(row for r in rows for row in zip(*[x.tolist() for x in r])), op.late_dropped))
    assert outs[0][1] > 0 or cfg.get("lateness")  # the stream has late records
    assert outs[0] == outs[1]
    assert len(outs[0][0]) > 0


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("cfg", [dict(assigner="sliding", size=1000, slide=250, agg="sum_i64"),
                                 dict(assigner="tumbling", size=500, agg="count", lateness=200)],
                         ids=["sliding_sum", "tumbling_count_lateness"])
def test_packed_exchange_over_gloo_equals_single_operator(oracle_lib, world, cfg):
    from tests.dist_worker import worker_packed
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = random.randint(20000, 40000)
    procs = [ctx.Process(target=worker_packed, args=(r, world, port, cfg, 17, q)) for r in range(world)]
    for p in procs:
        p.start()
    gathered = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(g[1] == 0 for g in gathered)  # every record reached its key group's owner
    packed = sum(g[3] for g in gathered)
    total = sum(g[4] for g in gathered)
    assert total == 24000 and packed > 0.7 * total
    union = sorted(row for g in gathered for row in g[0])
    keys, ts, vals, batches = random_stream(seed=17, n=24000, num_keys=500, n_batches=12, ts_step=1, agg=cfg["agg"])
    op = oracle_lib.OracleOperator(oracle_lib.make_config(**cfg))
    single = []
    for lo, hi, wm in batches:
        op.process_batch(keys[lo:hi], ts[lo:hi], vals[lo:hi])
        op.process_watermark(wm)
        single.append(op.drain())
    op.process_watermark((1 << 63) - 1)
    single.append(op.drain())
    ref = sorted(row for r in single for row in zip(*[x.tolist() for x in r]))
    assert sum(g[2] for g in gathered) == op.late_dropped
    assert len(union) == len(ref) > 0
    assert union == ref

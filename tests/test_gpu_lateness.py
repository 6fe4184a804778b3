"""GPU parity with allowed lateness > 0: windows keep their state
until max timestamp + lateness (WindowOperator.cleanupTime, WindowOperator.java:670-677),
a late record of a fired window that is not cleaned yet fires it again with the updated
contents (EventTimeTrigger.onElement, EventTimeTrigger.java:37-45; WindowOperator.java:
408-446), PurgingTrigger emits the late record alone, and records of cleaned windows are
dropped and counted (isElementLate :620-624).  The CPU oracle (oracle/flink_oracle.c)
replays the reference record by record; rows are compared per watermark as multisets."""
import zlib

import numpy as np
import pytest

from flink_amd import _native as N
from tests.gpu_helpers import compare, gpu_operator, random_stream, run_gpu, run_oracle

pytestmark = pytest.mark.gpu

TOL_AGGS = {"sum_f64", "avg_f64"}

CFGS = [
    dict(assigner="tumbling", size=1000, slide=1000),
    dict(assigner="tumbling", size=700, slide=700, offset=-300),
    dict(assigner="sliding", size=1000, slide=250),
    dict(assigner="sliding", size=1000, slide=300, offset=-50),
    dict(assigner="sliding", size=10000, slide=2000),
]


def _cmp(g, o, agg):
    return compare(g, o, agg in TOL_AGGS)


def _late_stream(seed, agg, cfg, lateness, n=20000, num_keys=60, n_batches=40):
    # disorder well beyond the watermark lag: records land in fired windows, some
    # within the lateness, some beyond it
    disorder = max(2500, 3 * cfg["size"]) + lateness
    return random_stream(seed=seed, n=n, num_keys=num_keys, n_batches=n_batches, disorder=disorder, wm_lag=200,
                         agg=agg)


@pytest.mark.parametrize("agg", ["count", "sum_i64", "min_f64", "avg_f64", "sum_i32"])
@pytest.mark.parametrize("lateness", [300, 2000])
@pytest.mark.parametrize("cfg", CFGS, ids=lambda c: "-".join(str(v) for v in c.values()))
@pytest.mark.parametrize("flags", [N.FLAG_NO_REGION, N.FLAG_FORCE_REGION], ids=["direct", "region"])
def test_lateness_refires_vs_oracle(oracle_lib, cfg, lateness, agg, flags):
    kw = dict(cfg, agg=agg, lateness=lateness)
    keys, ts, vals, batches = _late_stream(zlib.crc32(f"lat{agg}{cfg}{lateness}".encode()) & 0xffff, agg, cfg,
                                           lateness)
    g, glate, _ = run_gpu(kw, keys, ts, vals, batches, flags=flags)
    o, olate = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert olate > 0
    assert glate == olate
    assert _cmp(g, o, agg) == []
    # re-fires happened: more rows than (key, window) pairs
    rows = sum(len(x[0]) for x in o)
    pairs = len({(int(k), int(s)) for x in o for k, s in zip(x[0], x[1])})
    assert rows > pairs


@pytest.mark.parametrize("agg", ["sum_i64", "max_i64", "avg_i64"])
@pytest.mark.parametrize("cfg", CFGS, ids=lambda c: "-".join(str(v) for v in c.values()))
def test_lateness_purging_trigger_vs_oracle(oracle_lib, cfg, agg):
    """PurgingTrigger: every re-fire row holds the late record alone."""
    kw = dict(cfg, agg=agg, lateness=1500, trigger="purging_event_time")
    keys, ts, vals, batches = _late_stream(zlib.crc32(f"purge{agg}{cfg}".encode()) & 0xffff, agg, cfg, 1500)
    g, glate, _ = run_gpu(kw, keys, ts, vals, batches, flags=0)
    o, olate = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert glate == olate
    assert _cmp(g, o, agg) == []


@pytest.mark.parametrize("cfg", CFGS[:4], ids=lambda c: "-".join(str(v) for v in c.values()))
@pytest.mark.parametrize("flags", [N.FLAG_FORCE_REGION, N.FLAG_FORCE_REGION | N.FLAG_NO_BUFFER],
                         ids=["buffered", "unbuffered"])
def test_lateness_two_pass_region_table(oracle_lib, cfg, flags):
    """A two-pass (buffered) region table: late records leave the P1 buckets for the
    re-fire list; far-future records are parked as before."""
    kw = dict(cfg, agg="sum_i64", lateness=1200)
    keys, ts, vals, batches = random_stream(seed=41, n=60000, num_keys=20000, n_batches=40,
                                            disorder=max(4000, 3 * cfg["size"]), wm_lag=200, agg="sum_i64")
    rng = np.random.default_rng(9)
    far = rng.choice(len(ts), 300, replace=False)
    ts[far] += rng.integers(50_000, 2_000_000, 300)
    g, glate, _ = run_gpu(kw, keys, ts, vals, batches, flags=flags, capacity_hint=600_000)
    o, olate = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert glate == olate
    assert compare(g, o, False) == []


@pytest.mark.parametrize("flags", [0, N.FLAG_FORCE_REGION], ids=["auto", "region"])
def test_lateness_watermark_jumps(oracle_lib, flags):
    """Watermark jumps fire and clean many windows in one call; records land all over."""
    kw = dict(assigner="sliding", size=1000, slide=250, agg="count", lateness=1700)
    rng = np.random.default_rng(6)
    n = 9000
    keys = rng.integers(0, 40, n).astype(np.int64)
    ts = rng.integers(0, 400_000, n).astype(np.int64)
    vals = np.zeros(n, np.int64)
    batches = [(0, 2000, -1), (2000, 4000, 50_000), (4000, 6000, 51_000), (6000, 7500, 200_000),
               (7500, 9000, 200_900)]
    g, glate, _ = run_gpu(kw, keys, ts, vals, batches, flags=flags)
    o, olate = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert glate == olate
    assert compare(g, o, False) == []


def test_lateness_preaggregation_path(oracle_lib):
    """Few keys, many records per batch: the LDS pre-aggregation path with re-fires."""
    kw = dict(assigner="tumbling", size=1000, slide=1000, agg="sum_i64", lateness=800)
    keys, ts, vals, batches = random_stream(seed=3, n=40000, num_keys=5, n_batches=20, disorder=3000, wm_lag=200)
    g, glate, stats = run_gpu(kw, keys, ts, vals, batches, flags=N.FLAG_FORCE_LDS_PREAGG)
    o, olate = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert stats["preagg_batches"] > 0
    assert glate == olate
    assert compare(g, o, False) == []


# ------------------------------------------------------------------ session windows
# Merging windows with allowed lateness (WindowOperator.java:303-403 merging branch):
# a session keeps its state until max timestamp + lateness; a late element that lands in
# or merges with it fires the merged window at once (EventTimeTrigger.onElement FIRE),
# a merge that ends beyond the watermark re-arms the timer (onMerge), and elements whose
# window would be cleaned already are dropped and counted.  Parity against the oracle's
# record-by-record MergingWindowSet replay (no reference golden vector covers this case).
@pytest.mark.parametrize("agg", ["count", "sum_i64", "max_f64", "avg_f64", "avg_i64"])
@pytest.mark.parametrize("lateness", [300, 2000])
@pytest.mark.parametrize("gap", [100, 1500])
def test_session_lateness_vs_oracle(oracle_lib, gap, lateness, agg):
    kw = dict(assigner="session", gap=gap, agg=agg, lateness=lateness)
    keys, ts, vals, batches = random_stream(seed=zlib.crc32(f"sl{agg}{gap}{lateness}".encode()) & 0xffff, n=20000,
                                            num_keys=60, n_batches=40, disorder=2500 + lateness, wm_lag=200, agg=agg)
    g, glate, _ = run_gpu(kw, keys, ts, vals, batches)
    o, olate = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert olate > 0
    assert glate == olate
    assert _cmp(g, o, agg) == []
    # elements fired windows at once: some (key, start) pairs come out more than once
    rows = sum(len(x[0]) for x in o)
    assert rows > len({(int(k), int(s), int(e)) for x in o for k, s, e in zip(x[0], x[1], x[2])}) or gap == 100


def test_session_lateness_many_sessions_per_key(oracle_lib):
    """Late elements on a few keys with many fired-but-kept sessions: the slot widens."""
    kw = dict(assigner="session", gap=50, agg="sum_i64", lateness=600)
    keys, ts, vals, batches = random_stream(seed=77, n=6000, num_keys=20, n_batches=30, disorder=1500, wm_lag=100,
                                            agg="sum_i64")
    g, glate, st = run_gpu(kw, keys, ts, vals, batches)
    o, olate = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert glate == olate
    assert _cmp(g, o, "sum_i64") == []


@pytest.mark.parametrize("agg", ["count", "sum_i64", "min_f64", "avg_f64"])
@pytest.mark.parametrize("lateness", [300, 2000])
def test_session_lateness_purging_trigger_vs_oracle(oracle_lib, lateness, agg):
    """PurgingTrigger(EventTimeTrigger) with lateness: every firing purges, the session stays
    (empty) in the merging window set until cleanup, and a later merge folds into nothing."""
    kw = dict(assigner="session", gap=1500, agg=agg, lateness=lateness, trigger="purging_event_time")
    keys, ts, vals, batches = random_stream(seed=zlib.crc32(f"slp{agg}{lateness}".encode()) & 0xffff, n=20000,
                                            num_keys=60, n_batches=40, disorder=2500 + lateness, wm_lag=200, agg=agg)
    g, glate, _ = run_gpu(kw, keys, ts, vals, batches)
    o, olate = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert glate == olate
    assert _cmp(g, o, agg) == []


# ------------------------------------------------------------------ late-data side output
# WindowedStream.sideOutputLateData: a skipped late element goes to the side output instead
# of numLateRecordsDropped (WindowOperator.java:440-446, sideOutput :587-588).  Rows and the
# side output are compared with the oracle per watermark; nothing is counted as dropped.
@pytest.mark.parametrize("agg", ["sum_i64", "avg_f64"])
@pytest.mark.parametrize("kw", [
    dict(assigner="tumbling", size=1000, slide=1000),
    dict(assigner="sliding", size=1000, slide=300, offset=-50),
    dict(assigner="sliding", size=1000, slide=250, lateness=700),
    dict(assigner="session", gap=300),
    dict(assigner="session", gap=800, lateness=500),
], ids=lambda c: "-".join(str(v) for v in c.values()))
@pytest.mark.parametrize("flags", [0, N.FLAG_FORCE_REGION], ids=["auto", "region"])
def test_late_side_output_vs_oracle(oracle_lib, kw, agg, flags):
    if flags and kw["assigner"] == "session":
        pytest.skip("sessions have one ingest path")
    o = oracle_lib
    kw = dict(kw, agg=agg)
    keys, ts, vals, batches = random_stream(seed=zlib.crc32(f"so{kw}".encode()) & 0xffff, n=20000, num_keys=80,
                                            n_batches=30, disorder=4000, wm_lag=200, agg=agg)
    op = gpu_operator(kw, flags=flags | N.FLAG_LATE_SIDE_OUTPUT)
    ora = o.OracleOperator(o.make_config(**kw, flags=N.FLAG_LATE_SIDE_OUTPUT))
    vb = vals.view(np.int64) if vals.dtype == np.float64 else vals
    g_rows, o_rows, g_side, o_side = [], [], [], []
    for lo, hi, wm in batches:
        op.process_batch(keys[lo:hi], ts[lo:hi], vals[lo:hi])
        op.advance_watermark(wm)
        k, s, e, r = op.drain()
        g_rows.append((k, s, e, r.view(np.int64)))
        g_side.append(op.drain_late())
        ora.process_batch(keys[lo:hi], ts[lo:hi], vb[lo:hi])
        ora.process_watermark(wm)
        o_rows.append(ora.drain())
        o_side.append(ora.drain_late())
    assert op.num_late_records_dropped == 0 and ora.late_dropped == 0
    assert _cmp(g_rows, o_rows, agg) == []
    n_side = 0
    for b, (gs, os_) in enumerate(zip(g_side, o_side)):
        got = sorted(zip(*[c.tolist() for c in gs]))
        exp = sorted(zip(*[c.tolist() for c in os_]))
        assert got == exp, f"side output differs at watermark #{b}"
        n_side += len(exp)
    assert n_side > 0
    op.close()
    ora.close()

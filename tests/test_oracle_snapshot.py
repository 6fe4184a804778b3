"""The oracle's snapshot / restore in the heap backend's per-key-group layout (blob version 4),
and the restore semantics of the reference it restates:

* state, merging window sets and timers are written per key group (HeapSnapshotStrategy.java:
  97-154, CopyOnWriteStateMapSnapshot.writeState :127-149, InternalTimerServiceImpl.
  snapshotTimersForKeyGroup :350-360) and read back unchanged;
* the watermark is not state: a restored operator starts at Long.MIN_VALUE
  (InternalTimerServiceImpl.java:72), so a record of an already fired window that arrives
  before the next watermark is NOT late -- it creates that window's state again and fires it
  at the next watermark (WindowOperator.processElement :405-433, EventTimeTrigger.onElement
  :37-47).  An uninterrupted operator drops the same record as late.
"""
import numpy as np
import pytest

from gpu_helpers import random_stream
from heapsnap import parse

CFGS = [
    dict(assigner="tumbling", size=1000, slide=1000, agg="sum_i64"),
    dict(assigner="sliding", size=1000, slide=300, offset=-50, agg="avg_f64"),
    dict(assigner="sliding", size=900, slide=300, agg="min_f64", lateness=700),
    dict(assigner="session", gap=200, agg="count"),
    dict(assigner="session", gap=150, agg="sum_i32", lateness=400),
    dict(assigner="tumbling", size=500, slide=500, agg="max_i64", lateness=1000, trigger="purging_event_time"),
]


def feed(op, keys, ts, vals, batches):
    outs = []
    for lo, hi, wm in batches:
        op.process_batch(keys[lo:hi], ts[lo:hi], vals[lo:hi])
        op.process_watermark(wm)
        outs.append(op.drain())
    return outs


def rows_sorted(outs):
    rows = [tuple(int(x) for x in r) for o in outs for r in zip(*o)]
    return sorted(rows)


@pytest.mark.parametrize("kw", CFGS, ids=lambda c: "-".join(str(v) for v in c.values()))
def test_oracle_snapshot_round_trip(oracle_lib, kw):
    o = oracle_lib
    keys, ts, vals, batches = random_stream(3, 8000, 300, 8, disorder=900, wm_lag=300, agg=kw["agg"])
    a = o.OracleOperator(o.make_config(**kw))
    feed(a, keys, ts, vals, batches[:5])
    blob = a.snapshot()
    b = o.OracleOperator(o.make_config(**kw))
    b.restore(blob)
    assert b.snapshot() == blob
    # per key-group blobs restore to the same state
    parts = [a.snapshot((kg, kg)) for kg in range(128)]
    c = o.OracleOperator(o.make_config(**kw))
    c.restore(parts)
    assert c.snapshot() == blob
    dec = parse(blob, kw["agg"])
    assert sum(len(v["state"]) for v in dec.values()) == a.state_entries
    assert sum(len(v["timers"]) for v in dec.values()) > 0
    if kw["assigner"] == "session":
        assert sum(len(v["sets"]) for v in dec.values()) > 0


@pytest.mark.parametrize("kw", CFGS[:3] + CFGS[5:], ids=lambda c: "-".join(str(v) for v in c.values()))
def test_restore_resets_the_watermark(oracle_lib, kw):
    """Records of already fired windows, arriving after a restore but before the next
    watermark, are accepted and fire again at that watermark (not dropped as late)."""
    o = oracle_lib
    keys, ts, vals, batches = random_stream(5, 6000, 200, 6, disorder=100, wm_lag=200, agg=kw["agg"])
    a = o.OracleOperator(o.make_config(**kw))
    feed(a, keys, ts, vals, batches)
    blob = a.snapshot()
    wm_last = batches[-1][2]
    # old records: timestamps well before the last watermark (their windows have fired)
    n_old = 300
    ok = keys[:n_old].copy()
    ot = ts[:n_old].copy()
    ov = vals[:n_old].copy()
    cont = o.OracleOperator(o.make_config(**kw))  # the uninterrupted operator
    feed(cont, keys, ts, vals, batches)
    late0 = cont.late_dropped
    cont.process_batch(ok, ot, ov)
    cont.process_watermark(wm_last + 1)
    r_cont = rows_sorted([cont.drain()])
    b = o.OracleOperator(o.make_config(**kw))
    b.restore(blob)
    b.process_batch(ok, ot, ov)
    assert b.late_dropped == 0  # nothing is late at Long.MIN_VALUE
    b.process_watermark(wm_last + 1)
    r_rest = rows_sorted([b.drain()])
    assert cont.late_dropped > late0  # the uninterrupted operator drops (some of) them
    assert len(r_rest) > len(r_cont)  # the restored one fires their windows again
    # every window fired again holds exactly the old records of its key in it
    if kw.get("lateness", 0) == 0:
        for k, s, e, r in r_rest:
            m = (ok == k) & (ot >= s) & (ot < e)
            assert m.any()

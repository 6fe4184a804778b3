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


@pytest.mark.parametrize("agg", ["count", "sum_i64", "max_f64", "avg_i64"])
def test_oracle_count_window_heap_layout(oracle_lib, agg):
    """countWindow(size) (PurgingTrigger(CountTrigger)) in the heap layout: per key group the
    reduced contents under the GlobalWindow and CountTrigger's "count" (CountTrigger.java:39-40),
    no timers; a key right after its FIRE_AND_PURGE holds none.  A restored operator fires
    every window at the same element as the uninterrupted one with the same result: the count
    carries the trigger, the reduced state the contents (ordinals restart at the count)."""
    import struct
    O = oracle_lib
    size = 6
    kw = dict(assigner="count_tumbling", size=size, slide=size, agg=agg)
    keys, _, vals, _ = random_stream(71, 30_000, 400, 1, agg=agg)
    vb = vals.view(np.int64) if vals.dtype == np.float64 else vals
    zeros = np.zeros(keys.size, np.int64)
    cut = 13_001
    a = O.OracleOperator(O.make_config(**kw))
    a.process_batch(keys[:cut], zeros[:cut], vb[:cut])
    a.drain()
    blob = a.snapshot()
    # layout: per key group n x (0, key, acc) then n x (0, key, be64 count) then 0 timers
    nk = 128
    offs = struct.unpack_from(f"<{nk + 1}q", blob, 96)
    pay0 = 96 + 8 * (nk + 1)
    acc = 16 if agg.startswith("avg") else 8
    counts = {}
    for g in range(nk):
        p = pay0 + offs[g]
        n = struct.unpack_from(">i", blob, p)[0]
        p += 4 + n * (9 + acc)
        assert struct.unpack_from(">i", blob, p)[0] == n
        p += 4
        for i in range(n):
            assert blob[p] == 0
            k, c = struct.unpack_from(">qq", blob, p + 1)
            counts[k] = c
            p += 17
        assert struct.unpack_from(">i", blob, p)[0] == 0 and p + 4 == pay0 + offs[g + 1]
    seen = np.bincount(np.unique(keys[:cut], return_inverse=True)[1])
    expect = {int(k): int(c) % size for k, c in zip(np.unique(keys[:cut]), seen) if c % size}
    assert counts == expect
    b = O.OracleOperator(O.make_config(**kw))
    b.restore(blob)
    a.process_batch(keys[cut:], zeros[cut:], vb[cut:])
    b.process_batch(keys[cut:], zeros[cut:], vb[cut:])
    ka, sa, ea, ra = a.drain()
    kb, sb, eb, rb = b.drain()
    assert np.array_equal(ka, kb) and np.array_equal(ra, rb) and np.array_equal(ea - sa, eb - sb) and len(ka) > 1000
    assert np.all(eb - sb == size)

"""Session-window checkpoints in the heap backend's per-key-group layout,
GPU against the oracle.

The reference writes, per key group (HeapSnapshotStrategy.java:97-154):
* the "window-contents" entries (CopyOnWriteStateMapSnapshot.writeState :127-149): one per
  session holding state, under the session's *state window* -- one of the windows it grew
  from (MergingWindowSet.addWindow :188-201);
* the "merging-window-set" ListState (MergingWindowSet.persist :99-106): window -> state window;
* the event-time timers (InternalTimerServiceImpl.java:350-360): maxTimestamp while a session
  has not fired, its cleanup time under allowed lateness.

libgpuwin keeps a session's state under the session itself, so its blob names each session
as its own state window.  The tests therefore compare the two blobs after filing every entry
under its window through the blob's own merging window set (tests/heapsnap.py
normalize_sessions): entries, sets and timers must then be equal -- accumulators bit-exact,
f64 sums within 1e-6 -- and a blob written by either side restores into the other.
"""
import numpy as np
import pytest

from flink_amd import _native as N
from flink_amd import windowing as W
from tests import refsnap
from tests.gpu_helpers import REL_TOL, compare, gpu_operator, random_stream
from tests.heapsnap import normalize_sessions, parse

pytestmark = pytest.mark.gpu

SESSION_AGGS = ["count", "sum_i64", "max_f64", "avg_f64", "avg_i64"]
DBL = ("sum_f64", "avg_f64")


def _vb(vals):
    return vals.view(np.int64) if vals.dtype == np.float64 else vals


def _drain(op, outs):
    k, s, e, r = op.drain()
    outs.append((k, s, e, r.view(np.int64)))


def _same_session_state(gblob, oblob, agg):
    g, o = parse(gblob, agg), parse(oblob, agg)
    assert g.keys() == o.keys()
    for kg in g:
        gst, gsets = normalize_sessions(g[kg])
        ost, osets = normalize_sessions(o[kg])
        assert gsets == osets, f"key group {kg}: merging window sets differ"
        # the GPU names each session as its own state window
        for x in g[kg]["sets"]:
            assert all((w[0], w[1]) == (w[2], w[3]) for w in x[1])
        assert [x[:3] for x in gst] == [x[:3] for x in ost], f"key group {kg}: entries differ"
        for a, b in zip(gst, ost):
            if agg in DBL:  # (sum bits, count): the sum within 1e-6, the count exact
                fa, fb = (np.array([x[3]], np.int64).view(np.float64)[0] for x in (a, b))
                assert fa == fb or abs(fa - fb) <= REL_TOL * max(abs(fa), abs(fb)), (a, b)
                assert a[4:] == b[4:], (a, b)
            else:
                assert a[3:] == b[3:], (a, b)
        assert g[kg]["timers"] == o[kg]["timers"], f"key group {kg}: timers differ"


CFGS = [
    dict(gap=300),
    dict(gap=1500, lateness=2000),
    dict(gap=1500, lateness=2000, trigger="purging_event_time"),
]


def _stream(seed, agg, lateness):
    if lateness:  # disorder beyond the watermark lag: late merges, immediate firings, drops
        return random_stream(seed, 16000, 120, 16, disorder=4500, wm_lag=200, agg=agg)
    return random_stream(seed, 16000, 400, 16, agg=agg)


@pytest.mark.parametrize("agg", SESSION_AGGS)
@pytest.mark.parametrize("cfg", CFGS, ids=lambda c: "-".join(f"{k}{v}" for k, v in c.items()))
def test_session_blob_equals_oracle_blob(oracle_lib, cfg, agg):
    if cfg.get("trigger") and agg not in ("sum_i64", "avg_f64"):
        pytest.skip("PurgingTrigger: two aggregates")
    kw = dict(cfg, assigner="session", agg=agg)
    keys, ts, vals, batches = _stream(3, agg, cfg.get("lateness", 0))
    op = gpu_operator(kw, capacity_hint=4096)
    ora = oracle_lib.OracleOperator(oracle_lib.make_config(**kw))
    go, oo = [], []
    done = 0
    for cut in (5, 11):
        for lo, hi, wm in batches[done:cut]:
            op.process_batch(keys[lo:hi], ts[lo:hi], vals[lo:hi])
            op.advance_watermark(wm)
            _drain(op, go)
            ora.process_batch(keys[lo:hi], ts[lo:hi], _vb(vals)[lo:hi])
            ora.process_watermark(wm)
            oo.append(ora.drain())
        done = cut
        hi = batches[cut - 1][1]
        extra = slice(hi, hi + 400)  # records after the watermark, before the snapshot
        op.process_batch(keys[extra], ts[extra], vals[extra])
        ora.process_batch(keys[extra], ts[extra], _vb(vals)[extra])
        gb = op.snapshot_state()
        _drain(op, go)
        oo.append(ora.drain())
        _same_session_state(gb, ora.snapshot(), agg)
    op.close()
    ora.close()
    assert compare(go, oo, agg in DBL) == []


def _resume(kind, o, kw, blob, keys, ts, vals, batches, key_hashes=None):
    outs = []
    if kind == "gpu":
        op = gpu_operator(kw, capacity_hint=4096)
        op.initialize_state(blob)
        for lo, hi, wm in batches:
            kh = None if key_hashes is None else key_hashes[lo:hi]
            op.process_batch(keys[lo:hi], ts[lo:hi], vals[lo:hi], key_hashes=kh)
            op.advance_watermark(wm)
            _drain(op, outs)
        op.advance_watermark(W.LONG_MAX)
        _drain(op, outs)
        late = op.num_late_records_dropped
        snap = None
        op.close()
        return outs, late
    op = o.OracleOperator(o.make_config(**kw))
    op.restore(blob)
    for lo, hi, wm in batches:
        op.process_batch(keys[lo:hi], ts[lo:hi], _vb(vals)[lo:hi])
        op.process_watermark(wm)
        outs.append(op.drain())
    op.process_watermark(W.LONG_MAX)
    outs.append(op.drain())
    late = op.late_dropped
    op.close()
    return outs, late


@pytest.mark.parametrize("agg", ["count", "sum_i64", "avg_f64"])
@pytest.mark.parametrize("cfg", CFGS, ids=lambda c: "-".join(f"{k}{v}" for k, v in c.items()))
@pytest.mark.parametrize("writer", ["oracle", "gpu"])
def test_session_blob_restores_both_ways(oracle_lib, cfg, agg, writer):
    """A blob written by `writer` (the oracle's state windows differ from its windows wherever
    sessions merged) restores into both; both continue identically, and both restored
    operators snapshot to the same normalized state right after the restore."""
    o = oracle_lib
    kw = dict(cfg, assigner="session", agg=agg)
    keys, ts, vals, batches = _stream(17, agg, cfg.get("lateness", 0))
    cut = 7
    if writer == "gpu":
        op = gpu_operator(kw, capacity_hint=4096)
        for lo, hi, wm in batches[:cut]:
            op.process_batch(keys[lo:hi], ts[lo:hi], vals[lo:hi])
            op.advance_watermark(wm)
        op.drain()
        blob = op.snapshot_state()
        op.close()
    else:
        op = o.OracleOperator(o.make_config(**kw))
        for lo, hi, wm in batches[:cut]:
            op.process_batch(keys[lo:hi], ts[lo:hi], _vb(vals)[lo:hi])
            op.process_watermark(wm)
        op.drain()
        blob = op.snapshot()
        op.close()
    if writer == "oracle":  # the oracle's blob does name merged state windows
        assert any((w[0], w[1]) != (w[2], w[3]) for sec in parse(blob, agg).values()
                   for x in sec["sets"] for w in x[1])
    # right after the restore both hold the same state
    g = gpu_operator(kw, capacity_hint=4096)
    g.initialize_state(blob)
    r = o.OracleOperator(o.make_config(**kw))
    r.restore(blob)
    _same_session_state(g.snapshot_state(), r.snapshot(), agg)
    g.close()
    r.close()
    gout, glate = _resume("gpu", o, kw, blob, keys, ts, vals, batches[cut:])
    rout, rlate = _resume("oracle", o, kw, blob, keys, ts, vals, batches[cut:])
    assert compare(gout, rout, agg in DBL) == []
    assert glate == rlate


def test_hashed_session_sets_carry_the_key_hash(oracle_lib):
    """Keys fed with a key_hash column (String / Integer / ... keys as caller ids): every
    merging-window-set record carries the key's hash, so a key whose sessions all fired and
    were purged (no state entry) is still filed under its key group on restore."""
    kw = dict(assigner="session", gap=1500, lateness=2000, trigger="purging_event_time", agg="sum_i64")
    keys, ts, vals, batches = _stream(29, "sum_i64", 2000)
    kh = (keys * 1_000_003 + 7).astype(np.int32)  # not Long.hashCode
    o = oracle_lib
    op = gpu_operator(kw, capacity_hint=4096)
    ora = o.OracleOperator(o.make_config(**kw))
    ora.set_key_hashes(np.unique(keys), (np.unique(keys) * 1_000_003 + 7).astype(np.int32))
    cut = 9
    for lo, hi, wm in batches[:cut]:
        op.process_batch(keys[lo:hi], ts[lo:hi], vals[lo:hi], key_hashes=kh[lo:hi])
        op.advance_watermark(wm)
        ora.process_batch(keys[lo:hi], ts[lo:hi], vals[lo:hi])
        ora.process_watermark(wm)
    op.drain()
    ora.drain()
    gb = op.snapshot_state()
    op.close()
    ob = ora.snapshot()
    ora.close()
    _same_session_state(gb, ob, "sum_i64")
    got = parse(gb, "sum_i64")
    purged_only = 0
    for kg, sec in got.items():
        with_state = {x[2] for x in sec["state"]}
        for x in sec["sets"]:
            k, h = x[0], x[2]
            assert h == int(np.int32(k * 1_000_003 + 7)) and N.lib().gw_key_group_for_hash(h, 128) == kg
            purged_only += k not in with_state
    assert purged_only > 0  # the case the hash in the set record is for
    for blob in (gb, ob):
        gout, glate = _resume("gpu", o, kw, blob, keys, ts, vals, batches[cut:], key_hashes=kh)
        rout, rlate = _resume("oracle", o, kw, blob, keys, ts, vals, batches[cut:])
        assert compare(gout, rout, False) == []
        assert glate == rlate


# ----------------------------------------------- the reference's own session snapshot
SESSION_FIXTURES = refsnap.migration_fixtures("session-with-stateful-trigger")
IDS = {"key1": 0, "key2": 1}


def test_gpu_restores_the_reference_merging_window_set():
    """win-op-migration-test-session-with-stateful-trigger-flink2.2-snapshot
    (WindowOperatorMigrationTest.java:97-152): key1's session [10, 4000) keeps its state under
    [10, 3010), key2's [0, 6500) under [0, 3000).  Filed into a gpuwin blob as sums, it restores
    into libgpuwin; the restore test's records (:200-214) then merge key1 into [10, 10000) with
    sum 22 -- the reference's expected ("key1-22", 10, 10000)@9999 (:216).  key2's purged state
    (CountTrigger(4) fired on its 4th element) has no entry and its trigger timer is still
    set: libgpuwin refuses such a session (a trigger outside EventTimeTrigger / PurgingTrigger)."""
    ref = refsnap.parse(open(SESSION_FIXTURES["2.2"], "rb").read(), refsnap.list_value)
    assert ref[0]["sets"] == [("key2", [((0, 6500), (0, 3000))]), ("key1", [((10, 4000), (10, 3010))])]
    op = W.GpuWindowOperator(W.EventTimeSessionWindows.with_gap(refsnap.SESSION_MIGRATION_GAP), "sum_i32",
                             max_parallelism=1, capacity_hint=64).open()
    blob = refsnap.to_gpuwin_session_blob(ref, IDS, W.java_string_hash, N.AGGS["sum_i32"],
                                          N.ASSIGNERS["session"], refsnap.SESSION_MIGRATION_GAP)
    with pytest.raises(N.GpuWinError) as ei:
        op.initialize_state(W.pack_keyed_snapshot(blob, {v: k for k, v in IDS.items()}))
    assert ei.value.code == N.GW_E_UNSUPPORTED
    op.close()
    # the same with key2's state as EventTimeTrigger keeps it (1 + 2 + 3 + 4 under [0, 3000))
    ref[0]["state"].append((0, 3000, "key2", [("key2", 10)]))
    blob = refsnap.to_gpuwin_session_blob(ref, IDS, W.java_string_hash, N.AGGS["sum_i32"],
                                          N.ASSIGNERS["session"], refsnap.SESSION_MIGRATION_GAP)
    op = W.GpuWindowOperator(W.EventTimeSessionWindows.with_gap(refsnap.SESSION_MIGRATION_GAP), "sum_i32",
                             max_parallelism=1, capacity_hint=64).open()
    try:
        op.initialize_state(W.pack_keyed_snapshot(blob, {v: k for k, v in IDS.items()}))
        for k, v, t in [("key1", 3, 2500), ("key1", 1, 6000), ("key1", 2, 6500), ("key1", 3, 7000),
                        ("key1", 10, 4500)]:
            op.process_element(W.StreamRecord((k, v), t))
        op.process_watermark(W.LONG_MAX)
        rows = sorted((r.value[0], int(r.value[1]), int(r.value[2]), int(r.value[3]), r.timestamp)
                      for r in op.get_output() if isinstance(r, W.StreamRecord))
        assert rows == [("key1", 10, 10000, 22, 9999), ("key2", 0, 6500, 10, 6499)]
    finally:
        op.close()

"""Heap-layout snapshots of the tumbling / sliding window state and the reference's restore
semantics, GPU against the oracle:

* what libgpuwin writes (blob version 4: per key group the "window-contents" entries
  (window, key, accumulator) and the event-time timers, CopyOnWriteStateMapSnapshot.writeState
  :127-149, TimerSerializer.serialize :147-152) equals what the oracle's WindowOperator
  restatement writes for the same stream: the same (key, window) entries and accumulators
  (f64 within 1e-6), the same timers;
* a blob written by either side restores into the other, and both continue identically;
* after a restore the watermark is Long.MIN_VALUE (InternalTimerServiceImpl.java:72): records
  of already fired windows that arrive before the next watermark are accepted and fire those
  windows again (the uninterrupted operator drops them as late) -- at allowed lateness 0 and
  > 0, with EventTimeTrigger and PurgingTrigger.
"""
import numpy as np
import pytest

from flink_amd import _native as N
from flink_amd import windowing as W
from gpu_helpers import REL_TOL, compare, gpu_operator, random_stream
from heapsnap import parse

pytestmark = pytest.mark.gpu

CFGS = [
    dict(assigner="tumbling", size=1000, slide=1000),
    dict(assigner="sliding", size=1000, slide=300, offset=-50),
    dict(assigner="sliding", size=2000, slide=500, lateness=1200),
    dict(assigner="tumbling", size=700, slide=700, lateness=900, trigger="purging_event_time"),
    dict(assigner="sliding", size=900, slide=300, lateness=600, trigger="purging_event_time"),
]
AGGS = ["count", "sum_i64", "sum_i32", "min_f64", "max_i64", "avg_f64", "avg_i64"]
DBL = ("sum_f64", "avg_f64", "avg_i64")


def ids(c):
    return "-".join(str(v) for v in c.values())


def drain(op, outs):
    k, s, e, r = op.drain()
    outs.append((k, s, e, r.view(np.int64)))


def feed_gpu(op, keys, ts, vals, batches, outs):
    for lo, hi, wm in batches:
        op.process_batch(keys[lo:hi], ts[lo:hi], vals[lo:hi])
        op.advance_watermark(wm)
        drain(op, outs)


def feed_oracle(op, keys, ts, vals, batches, outs):
    vb = vals.view(np.int64) if vals.dtype == np.float64 else vals
    for lo, hi, wm in batches:
        op.process_batch(keys[lo:hi], ts[lo:hi], vb[lo:hi])
        op.process_watermark(wm)
        outs.append(op.drain())


def same_state(gblob, oblob, agg):
    g, o = parse(gblob, agg), parse(oblob, agg)
    assert g.keys() == o.keys()
    for kg in g:
        gs, os_ = g[kg]["state"], o[kg]["state"]
        assert [x[:3] for x in gs] == [x[:3] for x in os_], f"key group {kg}: (window, key) entries differ"
        for a, b in zip(gs, os_):
            if agg in ("sum_f64", "avg_f64", "min_f64", "max_f64"):
                fa = np.array([a[3]], np.int64).view(np.float64)[0]
                fb = np.array([b[3]], np.int64).view(np.float64)[0]
                assert fa == fb or abs(fa - fb) <= REL_TOL * max(abs(fa), abs(fb)), (a, b)
                assert a[4:] == b[4:]
            else:
                assert a[3:] == b[3:], (a, b)
        # timers of windows with state (a purged window's leftover cleanup timer carries
        # no state: nothing observable, the GPU does not keep it)
        live = {(x[0], x[1], x[2]) for x in gs}
        ot = [t for t in o[kg]["timers"] if (t[2], t[3], t[1]) in live]
        assert g[kg]["timers"] == ot, f"key group {kg}: timers differ"


def stream(seed, agg, n=24000, keys=400, batches=12):
    # disorder beyond the watermark lag: some records are late
    return random_stream(seed, n, keys, batches, disorder=1500, wm_lag=300, agg=agg)


@pytest.mark.parametrize("agg", AGGS)
@pytest.mark.parametrize("cfg", CFGS, ids=ids)
def test_heap_snapshot_equals_oracle_snapshot(oracle_lib, cfg, agg):
    kw = dict(cfg, agg=agg)
    keys, ts, vals, batches = stream(7, agg)
    op = gpu_operator(kw, capacity_hint=4096)
    ora = oracle_lib.OracleOperator(oracle_lib.make_config(**kw))
    go, oo = [], []
    for cut in (4, 9):
        lo_b = 0 if cut == 4 else 4
        feed_gpu(op, keys, ts, vals, batches[lo_b:cut], go)
        feed_oracle(ora, keys, ts, vals, batches[lo_b:cut], oo)
        hi = batches[cut - 1][1]
        # records after the watermark, before the snapshot (some late)
        extra = slice(hi, hi + 300)
        op.process_batch(keys[extra], ts[extra], vals[extra])
        ora.process_batch(keys[extra], ts[extra], (vals.view(np.int64) if vals.dtype == np.float64 else vals)[extra])
        gb = op.snapshot_state()
        drain(op, go)  # rows of late records (fired on the element) emitted by the snapshot's flush
        oo.append(ora.drain())
        same_state(gb, ora.snapshot(), agg)
    op.close()
    ora.close()
    assert compare(go, oo, agg in DBL) == []


def resume(kind, o, kw, blob, keys, ts, vals, batches, old):
    """Restore `blob` into a fresh GPU operator or oracle, feed `old` records (timestamps of
    windows that fired before the snapshot) before the first watermark, then the batches."""
    outs = []
    if kind == "gpu":
        op = gpu_operator(kw, capacity_hint=4096)
        op.initialize_state(blob)
        op.process_batch(keys[old], ts[old], vals[old])
        assert op.num_late_records_dropped == 0  # nothing is late at Long.MIN_VALUE
        feed_gpu(op, keys, ts, vals, batches, outs)
        op.advance_watermark(W.LONG_MAX)
        drain(op, outs)
        late = op.num_late_records_dropped
        snap = None
        op.close()
    else:
        op = o.OracleOperator(o.make_config(**kw))
        op.restore(blob)
        vb = vals.view(np.int64) if vals.dtype == np.float64 else vals
        op.process_batch(keys[old], ts[old], vb[old])
        assert op.late_dropped == 0
        feed_oracle(op, keys, ts, vals, batches, outs)
        op.process_watermark(W.LONG_MAX)
        outs.append(op.drain())
        late = op.late_dropped
        op.close()
        snap = None
    return outs, late, snap


@pytest.mark.parametrize("agg", ["count", "sum_i64", "min_f64", "avg_f64"])
@pytest.mark.parametrize("cfg", CFGS, ids=ids)
@pytest.mark.parametrize("writer", ["oracle", "gpu"])
def test_restore_accepts_records_of_fired_windows(oracle_lib, cfg, agg, writer):
    """Blob written by `writer`, restored into both; after the restore, records of fired
    windows arrive before the first watermark: both accept them and fire those windows
    again; afterwards the streams continue identically."""
    o = oracle_lib
    kw = dict(cfg, agg=agg)
    keys, ts, vals, batches = stream(11, agg)
    cut = 6
    if writer == "gpu":
        op = gpu_operator(kw, capacity_hint=4096)
        feed_gpu(op, keys, ts, vals, batches[:cut], [])
        blob = op.snapshot_state()
        op.close()
    else:
        op = o.OracleOperator(o.make_config(**kw))
        feed_oracle(op, keys, ts, vals, batches[:cut], [])
        blob = op.snapshot()
        op.close()
    old = np.arange(0, batches[2][1], 7)  # records of the first batches: their windows fired
    g, glate, _ = resume("gpu", o, kw, blob, keys, ts, vals, batches[cut:], old)
    r, rlate, _ = resume("oracle", o, kw, blob, keys, ts, vals, batches[cut:], old)
    assert compare(g, r, agg in DBL) == []
    assert glate == rlate
    # the first watermark after the restore fires windows of the old records again
    k0, s0, e0, _ = g[0]
    ots = ts[old]
    assert any(((s0 <= t) & (t < e0)).any() for t in ots[:50])


def test_rescale_heap_blobs_per_key_group(oracle_lib):
    """Per-key-group slices of one subtask's heap blob (gw_snapshot_slice) restore into two
    subtasks; each continues like the oracle restored from the same slices."""
    from tests.dist_worker import owners
    o = oracle_lib
    kw = dict(assigner="sliding", size=1000, slide=250, agg="sum_i64", lateness=500)
    keys, ts, vals, batches = stream(13, "sum_i64")
    cut = 5
    op = gpu_operator(kw, capacity_hint=4096)
    feed_gpu(op, keys, ts, vals, batches[:cut], [])
    blob = op.snapshot_state()
    op.close()
    own = owners(keys, 128, 2)
    for r in range(2):
        lo, hi = W.compute_key_group_range_for_operator_index(128, 2, r)
        parts = [N.snapshot_slice(blob, kg) for kg in range(lo, hi + 1)]
        g = W.GpuWindowOperator(W.SlidingEventTimeWindows.of(1000, 250), "sum_i64", allowed_lateness=500,
                                capacity_hint=4096, parallelism=2, operator_index=r).open()
        g.initialize_state(parts)
        ora = o.OracleOperator(o.make_config(**dict(kw, parallelism=2, operator_index=r)))
        ora.restore(parts)
        go, oo = [], []
        for blo, bhi, wm in batches[cut:]:
            sel = np.arange(blo, bhi)
            sel = sel[own[blo:bhi] == r]
            g.process_batch(keys[sel], ts[sel], vals[sel])
            g.advance_watermark(wm)
            drain(g, go)
            ora.process_batch(keys[sel], ts[sel], vals[sel])
            ora.process_watermark(wm)
            oo.append(ora.drain())
        g.advance_watermark(W.LONG_MAX)
        drain(g, go)
        ora.process_watermark(W.LONG_MAX)
        oo.append(ora.drain())
        assert compare(go, oo, False) == []
        assert g.num_late_records_dropped == ora.late_dropped
        g.close()
        ora.close()


def test_restore_after_processing_is_rejected():
    kw = dict(assigner="tumbling", size=100, slide=100, agg="sum_i64")
    a = gpu_operator(kw)
    a.process_batch(np.arange(10, dtype=np.int64), np.arange(10, dtype=np.int64), np.ones(10, np.int64))
    blob = a.snapshot_state()
    with pytest.raises(N.GpuWinError) as ei:
        a.initialize_state(blob)
    assert ei.value.code == -8
    a.close()


def test_region_path_restore_q5_shape(oracle_lib):
    """A restored 200k-key Q5-shaped state continued on the region (bucketed) ingest path, the
    table growing from its 4096-slot hint (the restored keys are re-attached after the rehash)."""
    o = oracle_lib
    kw = dict(assigner="sliding", size=10000, slide=2000, agg="sum_i64")
    rng = np.random.default_rng(3)
    n = 1_200_000  # 100k records per batch: the region path
    keys = rng.integers(0, 200_000, n).astype(np.int64)
    ts = (np.arange(n, dtype=np.int64) * 20_000) // n - rng.integers(0, 100, n)
    vals = rng.integers(0, 10 ** 6, n).astype(np.int64)
    cuts = np.linspace(0, n, 13).astype(np.int64)
    batches = [(int(cuts[b]), int(cuts[b + 1]), int(ts[:cuts[b + 1]].max()) - 101) for b in range(12)]
    ora = o.OracleOperator(o.make_config(**kw))
    feed_oracle(ora, keys, ts, vals, batches[:6], [])
    blob = ora.snapshot()
    ora.close()
    old = np.arange(0, batches[1][1], 11)
    g, glate, _ = resume("gpu", o, kw, blob, keys, ts, vals, batches[6:], old)
    r, rlate, _ = resume("oracle", o, kw, blob, keys, ts, vals, batches[6:], old)
    assert compare(g, r, False) == []


@pytest.mark.parametrize("kw", [dict(assigner="sliding", size=1000, slide=250, agg="sum_i64"),
                                dict(assigner="sliding", size=1000, slide=10, agg="sum_i64")],  # 2 window classes
                         ids=["one-table", "window-classes"])
def test_rejected_blob_leaves_the_handle_unchanged(oracle_lib, kw):
    """A blob that fails part-way through (a bad window in its LAST non-empty key group, after
    the earlier groups parsed) raises GW_E_INVALID and leaves nothing behind: the good blob
    restored next continues exactly like the oracle restored from it alone (no duplicated
    windows from the rejected attempt) -- also when the handle splits its windows into classes
    and a later class rejects its part after earlier classes restored theirs."""
    import struct
    o = oracle_lib
    keys, ts, vals, batches = stream(21, "sum_i64")
    cut = 5
    src = o.OracleOperator(o.make_config(**kw))
    feed_oracle(src, keys, ts, vals, batches[:cut], [])
    good = src.snapshot()
    src.close()
    kg_lo, kg_hi = struct.unpack_from("<ii", good, 60)
    nk = kg_hi - kg_lo + 1
    offs = np.frombuffer(good[96:96 + 8 * (nk + 1)], np.int64)
    pay0 = 96 + 8 * (nk + 1)
    last = max(g for g in range(nk) if offs[g + 1] - offs[g] > 40)
    assert last > 0
    bad = bytearray(good)
    bad[pay0 + int(offs[last]) + 4 + 7] ^= 1  # first entry's window start, low byte
    g = gpu_operator(kw, capacity_hint=4096)
    with pytest.raises(N.GpuWinError) as ei:
        g.initialize_state(bytes(bad))
    assert ei.value.code == -1  # GW_E_INVALID
    g.initialize_state(good)
    ora = o.OracleOperator(o.make_config(**kw))
    ora.restore(good)
    go, oo = [], []
    feed_gpu(g, keys, ts, vals, batches[cut:], go)
    feed_oracle(ora, keys, ts, vals, batches[cut:], oo)
    g.advance_watermark(W.LONG_MAX)
    drain(g, go)
    ora.process_watermark(W.LONG_MAX)
    oo.append(ora.drain())
    assert compare(go, oo, False) == []
    g.close()
    ora.close()


def test_rejected_hashed_blob_leaves_no_key_hashes_behind(oracle_lib):
    """A blob whose key carries two different Java hashCodes (two window entries of one key)
    is refused before anything changes -- not its entries, not its (key, hash) pairs in the
    handle's key-hash map (a stale pair would refuse the good blob or file a key's state under
    the wrong key group).  The handle that refused it then behaves exactly like a fresh handle
    restored from the good blob: same rows at every watermark, same snapshot."""
    import struct
    kw = dict(CFGS[1], agg="sum_i64")
    keys, ts, vals, batches = random_stream(seed=31, n=6000, num_keys=60, n_batches=16, ts_step=3,
                                            disorder=200, wm_lag=250, agg="sum_i64")
    hashes = ((keys * 7919 + 13) % 1000003).astype(np.int32)
    cut = 7
    a = gpu_operator(kw, capacity_hint=4096)
    for lo, hi, wm in batches[:cut]:
        a.process_batch(keys[lo:hi], ts[lo:hi], vals[lo:hi], key_hashes=hashes[lo:hi])
        a.advance_watermark(wm)
        a.clear_rows()
    good = a.snapshot_state()
    a.close()
    assert struct.unpack_from("<q", good, 48)[0] & 1  # flags: entries carry key hashes
    kg_lo, kg_hi = struct.unpack_from("<ii", good, 60)
    nk = kg_hi - kg_lo + 1
    offs = np.frombuffer(good[96:96 + 8 * (nk + 1)], np.int64)
    pay0 = 96 + 8 * (nk + 1)
    eb = 24 + 4 + 8
    bad = None
    for g in range(nk):  # a key group holding two entries of one key
        p = pay0 + int(offs[g])
        n = struct.unpack_from(">i", good, p)[0]
        ks = [struct.unpack_from(">q", good, p + 4 + i * eb + 16)[0] for i in range(n)]
        dup = [i for i in range(1, n) if ks[i] in ks[:i]]
        if dup:
            bad = bytearray(good)
            bad[p + 4 + dup[0] * eb + 24 + 3] ^= 1  # its hash, low byte
            break
    assert bad is not None
    b = gpu_operator(kw, capacity_hint=4096)
    c = gpu_operator(kw, capacity_hint=4096)
    try:
        with pytest.raises(N.GpuWinError) as ei:
            b.initialize_state(bytes(bad))
        assert ei.value.code == N.GW_E_INVALID
        outs = {}
        for name, op in (("b", b), ("c", c)):
            op.initialize_state(good)
            outs[name] = []
            for lo, hi, wm in batches[cut:] + [(len(keys), len(keys), W.LONG_MAX)]:
                op.process_batch(keys[lo:hi], ts[lo:hi], vals[lo:hi], key_hashes=hashes[lo:hi])
                op.advance_watermark(wm)
                drain(op, outs[name])
        assert compare(outs["b"], outs["c"], False) == []
        assert b.snapshot_state() == c.snapshot_state()
    finally:
        b.close()
        c.close()

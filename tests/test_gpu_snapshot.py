"""Checkpoint / restore of the GPU window state: gw_snapshot /
gw_restore per key-group range, checked against the CPU oracle run without any
interruption (the reference's snapshot/restore is transparent to the output,
WindowOperatorTest.java:169-177), including rescaling 2 -> 1 and 1 -> 2 subtasks."""
import numpy as np
import pytest

from flink_amd import _native as N
from flink_amd import windowing as W
from tests.dist_worker import owners
from tests.gpu_helpers import compare, gpu_operator, random_stream, run_oracle
from tests.heapsnap import parse

pytestmark = pytest.mark.gpu

CFGS = [
    dict(assigner="tumbling", size=1000, slide=1000),
    dict(assigner="sliding", size=1000, slide=300, offset=-50),
    dict(assigner="sliding", size=10000, slide=2000),
]


def _rows(op, outs):
    k, s, e, r = op.drain()
    outs.append((k, s, e, r.view(np.int64)))


@pytest.mark.parametrize("agg", ["count", "sum_i64", "min_f64", "avg_f64"])
@pytest.mark.parametrize("cfg", CFGS, ids=lambda c: "-".join(str(v) for v in c.values()))
@pytest.mark.parametrize("flags", [N.FLAG_NO_REGION, N.FLAG_FORCE_REGION], ids=["direct", "region"])
def test_snapshot_restore_mid_stream(oracle_lib, cfg, agg, flags):
    kw = dict(cfg, agg=agg)
    keys, ts, vals, batches = random_stream(seed=41, n=40000, num_keys=3000, n_batches=16, agg=agg)
    opkw = dict(flags=flags, capacity_hint=600_000 if flags == N.FLAG_FORCE_REGION else 4096)
    op = gpu_operator(kw, **opkw)
    outs = []
    for i, (lo, hi, wm) in enumerate(batches):
        op.process_batch(keys[lo:hi], ts[lo:hi], vals[lo:hi])
        if i in (5, 11):  # snapshot after the records, before the watermark
            blob = op.snapshot_state()
            op.close()
            op = gpu_operator(kw, **opkw)
            op.initialize_state(blob)
        op.advance_watermark(wm)
        _rows(op, outs)
    op.advance_watermark(W.LONG_MAX)
    _rows(op, outs)
    op.close()
    o, _ = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert compare(outs, o, agg in ("sum_f64", "avg_f64")) == []


@pytest.mark.parametrize("agg", ["sum_i64", "max_f64"])
def test_rescale_two_to_one_and_one_to_two(oracle_lib, agg):
    """Key groups move between subtasks (KeyGroupRangeAssignment.java:93-106): two
    subtasks' snapshots restore into one, and one subtask's snapshot splits into two
    key-group ranges restored into two subtasks."""
    kw = dict(assigner="sliding", size=1000, slide=250, agg=agg)
    keys, ts, vals, batches = random_stream(seed=5, n=30000, num_keys=2000, n_batches=12, agg=agg)
    own2 = owners(keys, 128, 2)
    cut = 6
    o, _ = run_oracle(oracle_lib, kw, keys, ts, vals, batches)

    def run(ops, own, phase_batches, outs_per_wm):
        for j, (lo, hi, wm) in enumerate(phase_batches):
            for r, op in enumerate(ops):
                sel = np.arange(lo, hi)
                if own is not None:
                    sel = sel[own[lo:hi] == r]
                op.process_batch(keys[sel], ts[sel], vals[sel])
            got = []
            for op in ops:
                op.advance_watermark(wm)
                k, s, e, rr = op.drain()
                got.append((k, s, e, rr.view(np.int64)))
            outs_per_wm.append(tuple(np.concatenate([g[c] for g in got]) for c in range(4)))

    # 2 -> 1
    ops = [W.GpuWindowOperator(W.SlidingEventTimeWindows.of(1000, 250), agg, capacity_hint=4096, parallelism=2,
                               operator_index=r).open() for r in range(2)]
    outs = []
    run(ops, own2, batches[:cut], outs)
    blobs = [op.snapshot_state(W.compute_key_group_range_for_operator_index(128, 2, r)) for r, op in enumerate(ops)]
    for op in ops:
        op.close()
    one = gpu_operator(kw, capacity_hint=4096)
    one.initialize_state(blobs)
    run([one], None, batches[cut:], outs)
    one.advance_watermark(W.LONG_MAX)
    k, s, e, rr = one.drain()
    outs.append((k, s, e, rr.view(np.int64)))
    one.close()
    assert compare(outs, o, False) == []

    # 1 -> 2
    one = gpu_operator(kw, capacity_hint=4096)
    outs = []
    run([one], None, batches[:cut], outs)
    blobs = [one.snapshot_state(W.compute_key_group_range_for_operator_index(128, 2, r)) for r in range(2)]
    one.close()
    ops = [W.GpuWindowOperator(W.SlidingEventTimeWindows.of(1000, 250), agg, capacity_hint=4096, parallelism=2,
                               operator_index=r).open() for r in range(2)]
    for r, op in enumerate(ops):
        op.initialize_state(blobs[r])
    run(ops, own2, batches[cut:], outs)
    last = []
    for op in ops:
        op.advance_watermark(W.LONG_MAX)
        k, s, e, rr = op.drain()
        last.append((k, s, e, rr.view(np.int64)))
        op.close()
    outs.append(tuple(np.concatenate([g[c] for g in last]) for c in range(4)))
    assert compare(outs, o, False) == []


def test_restore_rejects_other_config():
    a = gpu_operator(dict(assigner="tumbling", size=100, slide=100, agg="sum_i64"))
    a.process_batch(np.arange(10, dtype=np.int64), np.arange(10, dtype=np.int64), np.ones(10, np.int64))
    blob = a.snapshot_state()
    a.close()
    b = gpu_operator(dict(assigner="tumbling", size=200, slide=200, agg="sum_i64"))
    with pytest.raises(N.GpuWinError) as ei:
        b.initialize_state(blob)
    assert ei.value.code == -1
    b.close()


# ------------------------------------------------------------------ session windows
# The heap backend snapshots every (key, session window) state entry and the merging
# window set per key group (HeapSnapshotStrategy.java:97-154, MergingWindowSet.java:95-104);
# here every in-flight session is one (key, start, end, accumulator) entry of the blob.
SESSION_AGGS = ["count", "sum_i64", "max_f64", "avg_f64", "avg_i64"]


@pytest.mark.parametrize("agg", SESSION_AGGS)
@pytest.mark.parametrize("gap", [100, 3000])
def test_session_snapshot_restore_mid_stream(oracle_lib, agg, gap):
    kw = dict(assigner="session", gap=gap, agg=agg)
    keys, ts, vals, batches = random_stream(seed=43 + gap, n=20000, num_keys=300, n_batches=16, agg=agg)
    op = gpu_operator(kw)
    outs = []
    for i, (lo, hi, wm) in enumerate(batches):
        op.process_batch(keys[lo:hi], ts[lo:hi], vals[lo:hi])
        if i in (4, 9, 13):  # snapshot after the records, before the watermark
            blob = op.snapshot_state()
            op.close()
            op = gpu_operator(kw)
            op.initialize_state(blob)
        op.advance_watermark(wm)
        _rows(op, outs)
    op.advance_watermark(W.LONG_MAX)
    _rows(op, outs)
    op.close()
    o, _ = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert compare(outs, o, agg in ("sum_f64", "avg_f64")) == []


@pytest.mark.parametrize("agg", ["sum_i64", "avg_f64"])
def test_session_rescale_two_to_one_and_one_to_two(oracle_lib, agg):
    """Session state moves with its key groups (KeyGroupRangeAssignment.java:93-106)."""
    kw = dict(assigner="session", gap=3000, agg=agg)
    keys, ts, vals, batches = random_stream(seed=17, n=20000, num_keys=500, n_batches=12, agg=agg)
    own2 = owners(keys, 128, 2)
    cut = 6
    o, _ = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    dbl = agg == "avg_f64"

    def mk(p, r):
        return W.GpuWindowOperator(W.EventTimeSessionWindows.with_gap(3000), agg, capacity_hint=1024, parallelism=p,
                                   operator_index=r).open()

    def run(ops, own, phase_batches, outs_per_wm):
        for lo, hi, wm in phase_batches:
            for r, op in enumerate(ops):
                sel = np.arange(lo, hi)
                if own is not None:
                    sel = sel[own[lo:hi] == r]
                op.process_batch(keys[sel], ts[sel], vals[sel])
            got = []
            for op in ops:
                op.advance_watermark(wm)
                k, s, e, rr = op.drain()
                got.append((k, s, e, rr.view(np.int64)))
            outs_per_wm.append(tuple(np.concatenate([g[c] for g in got]) for c in range(4)))

    def finish(ops, outs):
        last = []
        for op in ops:
            op.advance_watermark(W.LONG_MAX)
            k, s, e, rr = op.drain()
            last.append((k, s, e, rr.view(np.int64)))
            op.close()
        outs.append(tuple(np.concatenate([g[c] for g in last]) for c in range(4)))

    # 2 -> 1
    ops = [mk(2, r) for r in range(2)]
    outs = []
    run(ops, own2, batches[:cut], outs)
    blobs = [op.snapshot_state(W.compute_key_group_range_for_operator_index(128, 2, r)) for r, op in enumerate(ops)]
    for op in ops:
        op.close()
    one = mk(1, 0)
    one.initialize_state(blobs)
    run([one], None, batches[cut:], outs)
    finish([one], outs)
    assert compare(outs, o, dbl) == []

    # 1 -> 2
    one = mk(1, 0)
    outs = []
    run([one], None, batches[:cut], outs)
    blobs = [one.snapshot_state(W.compute_key_group_range_for_operator_index(128, 2, r)) for r in range(2)]
    one.close()
    ops = [mk(2, r) for r in range(2)]
    for r, op in enumerate(ops):
        op.initialize_state(blobs[r])
    run(ops, own2, batches[cut:], outs)
    finish(ops, outs)
    assert compare(outs, o, dbl) == []


def test_session_restore_widens_for_many_sessions_per_key(oracle_lib):
    """A key with more restored sessions than the slot's inline list goes to the wide table."""
    kw = dict(assigner="session", gap=10, agg="sum_i64")
    keys = np.zeros(20, np.int64)
    ts = np.arange(20, dtype=np.int64) * 1000  # 20 disjoint sessions of one key, none fired
    vals = np.arange(20, dtype=np.int64)
    batches = [(0, 20, -10**9)]
    op = gpu_operator(kw)
    op.process_batch(keys, ts, vals)
    blob = op.snapshot_state()
    op.close()
    op = gpu_operator(kw)
    op.initialize_state(blob)
    outs = []
    op.advance_watermark(-10**9)
    _rows(op, outs)
    op.advance_watermark(W.LONG_MAX)
    _rows(op, outs)
    op.close()
    o, _ = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert compare(outs, o, False) == []


def test_session_and_pane_blobs_do_not_mix():
    s = gpu_operator(dict(assigner="session", gap=100, agg="sum_i64"))
    s.process_batch(np.arange(10, dtype=np.int64), np.arange(10, dtype=np.int64), np.ones(10, np.int64))
    sblob = s.snapshot_state()
    t = gpu_operator(dict(assigner="tumbling", size=100, slide=100, agg="sum_i64"))
    t.process_batch(np.arange(10, dtype=np.int64), np.arange(10, dtype=np.int64), np.ones(10, np.int64))
    tblob = t.snapshot_state()
    for op, blob in ((t, sblob), (s, tblob)):
        with pytest.raises(N.GpuWinError) as ei:
            op.initialize_state(blob)
        assert ei.value.code == -1
    g = gpu_operator(dict(assigner="session", gap=200, agg="sum_i64"))
    with pytest.raises(N.GpuWinError):
        g.initialize_state(sblob)
    for op in (s, t, g):
        op.close()


@pytest.mark.parametrize("trigger", ["event_time", "purging_event_time"])
@pytest.mark.parametrize("agg", ["sum_i64", "avg_f64", "min_f64"])
def test_session_snapshot_with_lateness(oracle_lib, agg, trigger):
    """Under allowed lateness a fired session stays until cleanup; its entry carries the
    fired flag, so a restored handle neither fires it again nor forgets it for late merges."""
    kw = dict(assigner="session", gap=1500, agg=agg, lateness=2000)
    if trigger == "purging_event_time":
        kw["trigger"] = trigger
    keys, ts, vals, batches = random_stream(seed=91, n=20000, num_keys=60, n_batches=30, disorder=4500, wm_lag=200,
                                            agg=agg)
    op = gpu_operator(kw)
    outs = []
    for i, (lo, hi, wm) in enumerate(batches):
        op.process_batch(keys[lo:hi], ts[lo:hi], vals[lo:hi])
        pre = None
        if i in (7, 15, 22):
            pre = op.drain()  # rows late elements fired at once were emitted before the snapshot
            blob = op.snapshot_state()
            op.close()
            op = gpu_operator(kw)
            op.initialize_state(blob)
        op.advance_watermark(wm)
        _rows(op, outs)
        if pre is not None:
            outs[-1] = tuple(np.concatenate([p, q]) for p, q in zip((pre[0], pre[1], pre[2], pre[3].view(np.int64)),
                                                                     outs[-1]))
    op.advance_watermark(W.LONG_MAX)
    _rows(op, outs)
    op.close()
    o, olate = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert olate > 0
    assert compare(outs, o, agg in ("sum_f64", "avg_f64")) == []


# ------------------------------------------------------ per-key-group blobs (JNI slicing)
@pytest.mark.parametrize("kw", [
    dict(assigner="sliding", size=1000, slide=250, agg="sum_i64"),
    dict(assigner="session", gap=300, agg="avg_f64"),
    dict(assigner="count_sliding", size=7, slide=3, agg="max_i64"),
], ids=["pane", "session", "count"])
def test_restore_from_per_key_group_slices(oracle_lib, kw):
    """GpuWindowOperator.snapshotState writes one blob per key group (gw_snapshot_slice,
    what nativeSliceKeyGroup calls); restoring all 128 slices equals restoring the blob."""
    agg = kw["agg"]
    keys, ts, vals, batches = random_stream(seed=29, n=20000, num_keys=700, n_batches=10, agg=agg)
    op = gpu_operator(kw)
    outs = []
    for i, (lo, hi, wm) in enumerate(batches):
        op.process_batch(keys[lo:hi], ts[lo:hi], vals[lo:hi])
        if i == 4:
            if kw["assigner"].startswith("count"):
                _rows(op, outs)  # count windows fire on the element
            blob = op.snapshot_state()
            op.close()
            slices = [N.snapshot_slice(blob, kg) for kg in range(128)]
            assert sum(len(s) - 112 for s in slices) == len(blob) - 96 - 129 * 8
            op = gpu_operator(kw)
            op.initialize_state(slices)
        op.advance_watermark(wm)
        _rows(op, outs)
        if kw["assigner"].startswith("count") and i == 4:
            outs[-2:] = [tuple(np.concatenate([a, b]) for a, b in zip(outs[-2], outs[-1]))]
    op.advance_watermark(W.LONG_MAX)
    _rows(op, outs)
    op.close()
    o, _ = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert compare(outs, o, agg == "avg_f64") == []


def test_foreign_key_hash_files_state_by_that_hash_and_key_group_check():
    """A key_hash column (keys as caller ids for String / Integer / ... keys) files each
    key's state under the key group of that hash (KeyGroupRangeAssignment.java:63-66) and the
    blob carries it; a key arriving with a second, different hash fails the handle;
    GW_FLAG_CHECK_KEY_GROUPS fails a batch holding a key of another subtask
    (StateTable.getMapForKeyGroup, StateTable.java:325-333)."""
    keys = np.arange(100, dtype=np.int64)
    ts = np.arange(100, dtype=np.int64)
    ones = np.ones(100, np.int64)
    op = gpu_operator(dict(assigner="tumbling", size=50, slide=50, agg="sum_i64"))
    lh = np.array([N.lib().gw_java_long_hash(int(k)) for k in keys], np.int32)
    fh = lh * 7 + 1  # not Long.hashCode
    op.process_batch(keys, ts, ones, key_hashes=fh)
    got = parse(op.snapshot_state(), "sum_i64")
    for kg, sec in got.items():
        for s_, e_, k, acc, kh in sec["state"]:
            assert kh == fh[k] and N.lib().gw_key_group_for_hash(int(kh), 128) == kg
    with pytest.raises(N.GpuWinError) as ei:
        op.process_batch(keys, ts, ones, key_hashes=fh + 1)
    assert ei.value.code == -1 and "two different key hashes" in str(ei.value)
    op.close()
    kgr = W.compute_key_group_range_for_operator_index(128, 2, 0)
    mine = np.array([k for k in range(1000) if kgr[0] <= W.assign_to_key_group(k, 128) <= kgr[1]][:50], np.int64)
    other = np.array([k for k in range(1000) if not kgr[0] <= W.assign_to_key_group(k, 128) <= kgr[1]][:1], np.int64)
    op = W.GpuWindowOperator(W.TumblingEventTimeWindows.of(50), "sum_i64", parallelism=2, operator_index=0,
                             flags=N.FLAG_CHECK_KEY_GROUPS, capacity_hint=1024).open()
    op.process_batch(mine, np.arange(50, dtype=np.int64), np.ones(50, np.int64))
    with pytest.raises(N.GpuWinError) as ei:
        op.process_batch(np.concatenate([mine, other]), np.arange(51, dtype=np.int64), np.ones(51, np.int64))
    assert ei.value.code == -1 and "is not in KeyGroupRange" in str(ei.value)
    op.close()

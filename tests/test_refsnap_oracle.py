"""The reference's own snapshot bytes pin the oracle's snapshot and restore for String keys.

Fixtures: tests/golden/ref_snapshots/ -- WindowOperatorMigrationTest's reduce-event-time
snapshots of 16 Flink versions (WindowOperatorMigrationTest.java:364-443), read as data by
tests/refsnap.py.  String keys travel as int64 ids with their String.hashCode (the key_hash
column of gw_ingest); the snapshot files those keys under the key group of that hash and
carries it per entry.  CPU only (the GPU side: tests/test_gpu_refsnap.py)."""
import numpy as np
import pytest

from flink_amd import _native as N
from flink_amd.windowing import java_string_hash
from oracle import oracle as O
from tests import heapsnap, refsnap

FIXTURES = refsnap.migration_fixtures()
IDS = {"key1": 0, "key2": 1}
KEYS = {v: k for k, v in IDS.items()}


def _cfg():
    # TumblingEventTimeWindows.of(3 s), SumReducer on the Int field, EventTimeTrigger; the
    # test harness runs with max parallelism 1 (one key group, the fixtures' range [0, 0])
    return O.make_config("tumbling", size=3000, agg="sum_i32", max_parallelism=1)


def _expected_state():
    return sorted([(3000, 6000, "key2", 2), (0, 3000, "key2", 3), (0, 3000, "key1", 3)])


def _expected_timers():
    return sorted([(2999, "key1", 0, 3000), (5999, "key2", 3000, 6000), (2999, "key2", 0, 3000)])


def test_sixteen_versions_parse_to_the_same_state():
    assert len(FIXTURES) == 16, sorted(FIXTURES)
    for ver, path in FIXTURES.items():
        p = refsnap.parse(open(path, "rb").read())
        assert list(p) == [0], ver
        st = sorted((s, e, k, v[1]) for s, e, k, v in p[0]["state"])
        assert all(v[0] == k for s, e, k, v in p[0]["state"]), ver  # the reduced Tuple2 keeps its key
        assert st == _expected_state(), ver
        assert sorted(p[0]["event"]) == _expected_timers(), ver
        assert p[0]["processing"] == [], ver


def _oracle_after_migration_input():
    op = O.OracleOperator(_cfg())
    keys = np.array([IDS[k] for k, _, _ in refsnap.MIGRATION_INPUT], np.int64)
    op.set_key_hashes(keys, np.array([java_string_hash(k) for k, _, _ in refsnap.MIGRATION_INPUT], np.int32))
    ts = np.array([t for _, _, t in refsnap.MIGRATION_INPUT], np.int64)
    vals = np.array([v for _, v, _ in refsnap.MIGRATION_INPUT], np.int64)
    op.process_batch(keys, ts, vals)
    for wm in refsnap.MIGRATION_WATERMARKS:
        op.process_watermark(wm)
    assert len(op.drain()[0]) == 0  # :428-443: nothing fires before the snapshot
    return op


def test_oracle_snapshot_equals_the_reference_bytes():
    """The oracle's snapshot of the :407-426 input holds the reference file's (window, key,
    state) entries and timers, each entry with String.hashCode(key)."""
    op = _oracle_after_migration_input()
    blob = op.snapshot((0, 0))
    got = heapsnap.parse(blob, "sum_i32")[0]
    st = sorted((s, e, KEYS[k], acc) for s, e, k, acc, kh in got["state"])
    assert st == _expected_state()
    assert all(kh == java_string_hash(KEYS[k]) for s, e, k, acc, kh in got["state"])
    assert sorted((ts, KEYS[k], s, e) for ts, k, s, e in got["timers"]) == _expected_timers()
    ref = refsnap.parse(open(FIXTURES["2.1"], "rb").read())
    conv = refsnap.to_gpuwin_blob(ref, IDS, java_string_hash, N.AGGS["sum_i32"], N.ASSIGNERS["tumbling"], 3000, 3000)
    assert heapsnap.parse(conv, "sum_i32") == heapsnap.parse(blob, "sum_i32")


@pytest.mark.parametrize("ver", sorted(FIXTURES))
def test_oracle_restores_the_reference_snapshot(ver):
    """testRestoreReducingEventTimeWindows (:445-513) on the oracle."""
    ref = refsnap.parse(open(FIXTURES[ver], "rb").read())
    blob = refsnap.to_gpuwin_blob(ref, IDS, java_string_hash, N.AGGS["sum_i32"], N.ASSIGNERS["tumbling"], 3000, 3000)
    op = O.OracleOperator(_cfg())
    op.restore(blob)
    for wm in refsnap.MIGRATION_RESTORE_WATERMARKS:
        op.process_watermark(wm)
        k, s, e, r = op.drain()
        rows = sorted((KEYS[int(k[i])], int(r[i]), int(e[i]) - 1) for i in range(len(k)))
        assert rows == refsnap.MIGRATION_EXPECTED[wm], (ver, wm)


def test_key_table_and_remap_on_cpu():
    """gw_snapshot_keys / gw_snapshot_remap_keys (pure host code of libgpuwin) on a hashed blob."""
    ref = refsnap.parse(open(FIXTURES["2.1"], "rb").read())
    blob = refsnap.to_gpuwin_blob(ref, IDS, java_string_hash, N.AGGS["sum_i32"], N.ASSIGNERS["tumbling"], 3000, 3000)
    assert list(N.snapshot_keys(blob)) == [0, 1]
    moved = N.snapshot_remap_keys(blob, {0: 70, 1: 5})
    assert list(N.snapshot_keys(moved)) == [5, 70]
    p0, p1 = heapsnap.parse(blob, "sum_i32")[0], heapsnap.parse(moved, "sum_i32")[0]
    m = {0: 70, 1: 5}
    assert sorted((s, e, m[k], a, h) for s, e, k, a, h in p0["state"]) == p1["state"]
    assert sorted((t, m[k], s, e) for t, k, s, e in p0["timers"]) == p1["timers"]
    with pytest.raises(N.GpuWinError):
        N.snapshot_remap_keys(blob[:-3], {0: 1})


# ---------------------------------------------------------------- session windows
SESSION_FIXTURES = refsnap.migration_fixtures("session-with-stateful-trigger")


def test_session_fixtures_pin_the_merging_window_set_layout():
    """writeSessionWindowsWithCountTriggerSnapshot (WindowOperatorMigrationTest.java:97-152) for
    16 Flink versions: the heap backend writes the MergingWindowSet as the ListState
    "merging-window-set" (VoidNamespace, key, list of (window, state window)), and a session
    keeps its state under the window it started as: key1's [10, 4000) under [10, 3010), key2's
    [0, 6500) under [0, 3000).  The oracle's MergingWindowSet, fed the same records, holds
    exactly that mapping and the same event-time timers (maxTimestamp = cleanup time at
    lateness 0), and files key1's state (1 + 2) under the same state window.  Key2's contents
    differ by design: the fixture's PurgingTrigger(CountTrigger(4)) purged them on key2's 4th
    element; the oracle runs EventTimeTrigger (the closed set)."""
    assert len(SESSION_FIXTURES) == 16, sorted(SESSION_FIXTURES)
    parsed = {v: refsnap.parse(open(p, "rb").read(), refsnap.list_value) for v, p in SESSION_FIXTURES.items()}
    ref = parsed["2.2"]
    assert all(p == ref for p in parsed.values())
    sec = ref[0]
    op = O.OracleOperator(O.make_config("session", gap=refsnap.SESSION_MIGRATION_GAP, agg="sum_i32",
                                        max_parallelism=1))
    inp = refsnap.SESSION_MIGRATION_INPUT
    keys = np.array([IDS[k] for k, _, _ in inp], np.int64)
    op.set_key_hashes(keys, np.array([java_string_hash(k) for k, _, _ in inp], np.int32))
    op.process_batch(keys, np.array([t for _, _, t in inp], np.int64), np.array([v for _, v, _ in inp], np.int64))
    got = heapsnap.parse(op.snapshot((0, 0)), "sum_i32")[0]
    op.close()
    sets = sorted((KEYS[x[0]], sorted(((a, b), (c, d)) for a, b, c, d in x[1])) for x in got["sets"])
    assert sets == sorted((k, sorted(ws)) for k, ws in sec["sets"])
    for x in got["sets"]:  # the set record carries the key's String.hashCode
        assert x[2] == java_string_hash(KEYS[x[0]])
    assert sorted((t, KEYS[k], s, e) for t, k, s, e in got["timers"]) == sorted(sec["event"])
    st = {(KEYS[k], s, e): v for s, e, k, v, *_ in got["state"]}
    for s, e, k, elems in sec["state"]:
        assert st[(k, s, e)] == sum(v for _, v in elems)  # key1 under [10, 3010): 1 + 2
    assert st[("key2", 0, 3000)] == 10  # key2's state window is the fixture's [0, 3000)

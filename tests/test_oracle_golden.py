"""Pins the CPU oracle (oracle/flink_oracle.c) to the reference's own golden vectors
(tests/golden/, transcribed from Flink's tests — see make_golden.py for file:line)."""
import ctypes

import numpy as np
import pytest

N_FLAG_LATE_SIDE_OUTPUT = 64  # include/gpuwin.h GW_FLAG_LATE_SIDE_OUTPUT
from tests.harness import itcase_expected_sum, itcase_stream, load_golden, replay, config_kwargs


def test_key_groups_kat(oracle_lib):
    o = oracle_lib
    g = load_golden("key_groups.json")
    for key, group in g["string_keys"]:
        h = o.java_string_hash(key)
        assert o.lib().wo_assign_to_key_group(h, g["max_parallelism"]) == group, key


def test_murmur_known_properties(oracle_lib):
    L = oracle_lib.lib()
    # murmurHash is non-negative for every input (MathUtils.java:150-155)
    for x in [0, 1, -1, 2**31 - 1, -(2**31), 123456789, -987654321]:
        assert L.wo_murmur_hash(x) >= 0
    # Long.hashCode (JDK): (int)(v ^ (v >>> 32))
    assert L.wo_long_hash(0) == 0
    assert L.wo_long_hash(1) == 1
    assert L.wo_long_hash(-1) == 0
    assert L.wo_long_hash(1 << 32) == 1
    assert L.wo_long_hash(-(1 << 63)) == -(1 << 31)


def test_key_group_ranges(oracle_lib):
    L = oracle_lib.lib()
    assert L.wo_default_max_parallelism(1) == 128
    assert L.wo_default_max_parallelism(100) == 256
    assert L.wo_default_max_parallelism(30000) == 32768
    for p in [1, 2, 3, 4, 7, 8]:
        covered = []
        for i in range(p):
            s, e = ctypes.c_int32(), ctypes.c_int32()
            L.wo_key_group_range(128, p, i, ctypes.byref(s), ctypes.byref(e))
            covered.extend(range(s.value, e.value + 1))
            for kg in range(s.value, e.value + 1):
                assert L.wo_operator_index_for_key_group(128, p, kg) == i
        assert covered == list(range(128))


def test_window_start_with_offset(oracle_lib):
    L = oracle_lib.lib()
    for ts, off, size, start in load_golden("window_start.json")["cases"]:
        assert L.wo_window_start_with_offset(ts, off, size) == start, (ts, off, size)


def test_assigners(oracle_lib):
    o = oracle_lib
    for kind, size, slide, off, ts, windows in load_golden("assigners.json")["cases"]:
        if kind == "session":
            cfg = o.make_config(assigner="session", gap=size)
        else:
            cfg = o.make_config(assigner=kind, size=size, slide=slide or size, offset=off)
        s = np.zeros(16, np.int64)
        e = np.zeros(16, np.int64)
        P = ctypes.POINTER(ctypes.c_int64)
        n = o.lib().wo_assign_windows(ctypes.byref(cfg), ts, s.ctypes.data_as(P), e.ctypes.data_as(P), 16)
        got = sorted(zip(s[:n].tolist(), e[:n].tolist()))
        assert got == sorted(tuple(w) for w in windows), (kind, ts)


def test_assign_rejects_no_timestamp(oracle_lib):
    o = oracle_lib
    cfg = o.make_config(assigner="tumbling", size=1000, slide=1000)
    s = np.zeros(2, np.int64)
    P = ctypes.POINTER(ctypes.c_int64)
    assert o.lib().wo_assign_windows(ctypes.byref(cfg), -(1 << 63), s.ctypes.data_as(P),
                                     s.ctypes.data_as(P), 2) == -6


def test_config_validation(oracle_lib):
    o = oracle_lib
    L = o.lib()
    bad = [
        o.make_config(assigner="tumbling", size=1000, offset=1000),
        o.make_config(assigner="tumbling", size=0),
        o.make_config(assigner="sliding", size=1000, slide=100, offset=-100),
        o.make_config(assigner="sliding", size=0, slide=100),
        o.make_config(assigner="sliding", size=10**9, slide=1),
        o.make_config(assigner="session", gap=0),
        o.make_config(assigner="tumbling", size=1000, lateness=-1),
    ]
    for c in bad:
        assert L.wo_validate(ctypes.byref(c)) == -1
    assert L.wo_validate(ctypes.byref(o.make_config(assigner="sliding", size=1000, slide=300))) == 0


def test_merge_windows(oracle_lib):
    L = oracle_lib.lib()
    P = ctypes.POINTER(ctypes.c_int64)
    for windows, merges in load_golden("merge_windows.json")["cases"]:
        n = len(windows)
        s = np.array([w[0] for w in windows], np.int64)
        e = np.array([w[1] for w in windows], np.int64)
        grp = np.zeros(n, np.int32)
        gs = np.zeros(n, np.int64)
        ge = np.zeros(n, np.int64)
        ng = L.wo_merge_windows(n, s.ctypes.data_as(P), e.ctypes.data_as(P),
                                grp.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                gs.ctypes.data_as(P), ge.ctypes.data_as(P))
        got = []
        for g in range(ng):
            members = sorted({(int(s[i]), int(e[i])) for i in range(n) if grp[i] == g})
            if len(members) > 1:
                got.append((members, (int(gs[g]), int(ge[g]))))
        exp = [(sorted(tuple(m) for m in mm), tuple(c)) for mm, c in merges]
        assert sorted(got) == sorted(exp)


@pytest.mark.parametrize("test", load_golden("merging_window_set.json")["tests"], ids=lambda t: t["name"])
def test_merging_window_set_vectors(oracle_lib, test):
    """MergingWindowSetTest (MergingWindowSet.java:77-224 driven directly): the result window of
    every addWindow, whether the MergeFunction ran and with which merge result, sources, state
    window and merged state windows, getStateWindow, retireWindow and the persisted list."""
    def w(x):
        return None if x is None else (x[0], x[1])

    m = oracle_lib.MergingWindowSet([(w(a), w(b)) for a, b in test["restore"]])
    try:
        for st in test["steps"]:
            if st[0] == "add":
                res, merge = m.add_window(w(st[1]))
                assert res == w(st[2]), st
                exp = st[3]
                if exp is None:
                    assert merge is None, st
                    continue
                assert merge is not None, st
                assert merge["target"] == w(exp["target"]), st
                assert merge["state_window"] in [w(x) for x in exp["state_window"]], st
                assert sorted(merge["sources"]) == sorted(w(x) for x in exp["sources"]), st
                # mergedStateWindows never holds the merge target (:260, :300)
                assert merge["target"] not in merge["merged_state_windows"]
                if exp["merged_state_windows"] is not None:
                    alts = [sorted(w(x) for x in alt) for alt in exp["merged_state_windows"]]
                    assert sorted(merge["merged_state_windows"]) in alts, st
            elif st[0] == "state":
                got = m.state_window(w(st[1]))
                assert (got is None) if st[2] is None else got in [w(x) for x in st[2]], st
            elif st[0] == "retire":
                m.retire(w(st[1]))
            elif st[0] == "persist":
                assert m.persisted() == sorted((w(a), w(b)) for a, b in st[1]), st
        with pytest.raises(oracle_lib.OracleError):  # retireWindow of a window not in flight (:125-131)
            m.retire((-5, -1))
    finally:
        m.close()


@pytest.mark.parametrize("test", load_golden("operator_harness.json")["tests"], ids=lambda t: t["name"])
def test_operator_harness_vectors(oracle_lib, test):
    o = oracle_lib

    class Backend:
        def __init__(self, cfg, side_output=False):
            self.op = o.OracleOperator(o.make_config(**config_kwargs(cfg),
                                                     flags=N_FLAG_LATE_SIDE_OUTPUT if side_output else 0))

        def process_element(self, k, ts, v):
            self.op.process_element(k, ts, v)

        def process_watermark(self, wm):
            self.op.process_watermark(wm)

        def drain(self):
            return self.op.drain()

        @property
        def late_dropped(self):
            return self.op.late_dropped

        def drain_late(self):
            return self.op.drain_late()

    assert replay(test, Backend) == []
    if "side" in test:  # the reference test's own setting: the late records on the side output
        assert replay(test, Backend, side_output=True) == []


@pytest.mark.parametrize("assigner,size,slide", [("tumbling", 1000, 1000), ("sliding", 1000, 100)])
def test_itcase_closed_form(oracle_lib, assigner, size, slide):
    """EventTimeWindowCheckpointingITCase (flink-tests/.../EventTimeWindowCheckpointingITCase.java:
    314-383 tumbling, 480-552 sliding; generator :798-838, validator :749-771), scaled to
    10 keys x 3000 elements."""
    o = oracle_lib
    nk, n = 10, 3000
    keys, ts, vals, blen, wm = itcase_stream(nk, n, size)
    op = o.OracleOperator(o.make_config(assigner=assigner, size=size, slide=slide, agg="sum_i32"))
    off = 0
    rows = []
    for b in range(n):
        op.process_batch(keys[off:off + blen[b]], ts[off:off + blen[b]], vals[off:off + blen[b]])
        off += blen[b]
        op.process_watermark(int(wm[b]))
        rows.append(op.drain())
    op.process_watermark((1 << 63) - 1)
    rows.append(op.drain())
    k = np.concatenate([r[0] for r in rows]); s = np.concatenate([r[1] for r in rows])
    e = np.concatenate([r[2] for r in rows]); r = np.concatenate([r[3] for r in rows])
    assert op.late_dropped == 0
    for i in range(len(k)):
        assert r[i] == itcase_expected_sum(int(s[i]), int(e[i]), n)
    # every key gets every window that overlaps [0, n)
    n_windows = len({(int(a), int(b)) for a, b in zip(s, e)})
    assert len(k) == nk * n_windows
    expected_windows = (n + size - 1) // slide if assigner == "sliding" else n // size
    assert n_windows == expected_windows


def test_parallel_matches_single(oracle_lib):
    o = oracle_lib
    rng = np.random.default_rng(7)
    n = 20000
    keys = rng.integers(0, 500, n).astype(np.int64)
    ts = np.sort(rng.integers(0, 20000, n)).astype(np.int64)
    vals = rng.integers(-1000, 1000, n).astype(np.int64)
    blen = np.full(20, n // 20, np.int64)
    wm = np.array([ts[(i + 1) * (n // 20) - 1] - 50 for i in range(20)], np.int64)
    cfg = o.make_config(assigner="sliding", size=1000, slide=250, agg="sum_i64")
    r1, c1, _ = o.run_parallel(cfg, 1, blen, wm, keys, ts, vals)
    r4, c4, _ = o.run_parallel(cfg, 4, blen, wm, keys, ts, vals)
    assert r1 == r4 and c1 == c4 and r1 > 0


def test_stagger_vectors(oracle_lib):
    """TumblingEventTimeWindowsTest.testWindowAssignmentWithStagger (tests/golden/stagger.json):
    the offset gw_window_stagger_offset gives for the first element's processing time, used as
    the assigner's offset, reproduces the reference's windows."""
    from flink_amd.windowing import WindowStagger
    o = oracle_lib
    for stagger, size, off, ptime, ts, windows in load_golden("stagger.json")["cases"]:
        woff = WindowStagger.window_offset(getattr(WindowStagger, stagger), ptime, size, off)
        cfg = o.make_config(assigner="tumbling", size=size, slide=size, offset=woff)
        s = np.zeros(4, np.int64)
        e = np.zeros(4, np.int64)
        P = ctypes.POINTER(ctypes.c_int64)
        n = o.lib().wo_assign_windows(ctypes.byref(cfg), ts, s.ctypes.data_as(P), e.ctypes.data_as(P), 4)
        assert sorted(zip(s[:n].tolist(), e[:n].tolist())) == [tuple(w) for w in windows], (stagger, ts)


def test_stagger_offsets():
    """WindowStagger.getStaggerOffset (WindowStagger.java:27-60) + (globalOffset + stagger) % size
    (TumblingEventTimeWindows.java:72-79, Java remainder)."""
    from flink_amd.windowing import WindowStagger as S
    assert S.window_offset(S.ALIGNED, 123, 5000, 100) == 100
    assert S.window_offset(S.ALIGNED, 123, 5000, -100) == -100
    assert S.window_offset(S.RANDOM, 0, 5000, 0, 0.5) == 2500          # (long) (0.5 * 5000)
    assert S.window_offset(S.RANDOM, 0, 5000, 4000, 0.5) == 1500       # (4000 + 2500) % 5000
    assert S.window_offset(S.RANDOM, 0, 7, 0, 0.99999) == 6
    assert S.window_offset(S.NATURAL, 150, 5000, 0) == 150
    assert S.window_offset(S.NATURAL, 12345, 5000, 0) == 2345
    assert S.window_offset(S.NATURAL, -150, 5000, -100) == 4750        # start of -150's window: -5000
    assert S.window_offset(S.NATURAL, 5000, 5000, -100) == -100        # stagger 0: Java % keeps the sign
    from flink_amd import _native as N
    for bad in ((S.RANDOM, 0, 5000, 0, 1.0), (S.ALIGNED, 0, 0, 0, 0.0), (S.ALIGNED, 0, 100, 100, 0.0), (7, 0, 10, 0, 0.0)):
        with pytest.raises(N.GpuWinError):
            S.window_offset(bad[0], bad[1], bad[2], bad[3], bad[4])

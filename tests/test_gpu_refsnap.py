"""String keys through the GPU operator, pinned by the reference's own snapshot bytes.

* testRestoreReducingEventTimeWindows (WindowOperatorMigrationTest.java:445-513) on libgpuwin:
  each of the 16 reference-written snapshots (tests/golden/ref_snapshots/, read as data by
  tests/refsnap.py) restores into the GPU operator -- String keys as dictionary ids with their
  String.hashCode -- and the watermarks 2999 .. 5999 fire exactly (key1, 3)@2999,
  (key2, 3)@2999, (key2, 2)@5999;
* the GPU's own snapshot of that test's input (:407-426) holds the reference file's
  (window, key, state) entries and timers;
* random String-keyed streams: the GPU blob equals the oracle's (entries with key hashes,
  timers), and a keyed snapshot restores into fresh operators with other dictionaries,
  rescaled 1 -> 2 by key groups of String.hashCode, for tumbling / sliding windows,
  sessions and count windows.
"""
import numpy as np
import pytest

from flink_amd import _native as N
from flink_amd import windowing as W
from tests import refsnap
from tests.gpu_helpers import compare
from tests.heapsnap import parse

pytestmark = pytest.mark.gpu

FIXTURES = refsnap.migration_fixtures()
IDS = {"key1": 0, "key2": 1}


def _migration_op(flags=0):
    return W.GpuWindowOperator(W.TumblingEventTimeWindows.of(3000), "sum_i32", max_parallelism=1,
                               capacity_hint=64, flags=flags).open()


@pytest.mark.parametrize("ver", sorted(FIXTURES))
def test_gpu_restores_the_reference_snapshot(ver):
    ref = refsnap.parse(open(FIXTURES[ver], "rb").read())
    blob = refsnap.to_gpuwin_blob(ref, IDS, W.java_string_hash, N.AGGS["sum_i32"], N.ASSIGNERS["tumbling"],
                                  3000, 3000)
    op = _migration_op()
    try:
        op.initialize_state(W.pack_keyed_snapshot(blob, {v: k for k, v in IDS.items()}))
        for wm in refsnap.MIGRATION_RESTORE_WATERMARKS:
            op.process_watermark(wm)
            rows = sorted((r.value[0], int(r.value[3]), r.timestamp) for r in op.get_output()
                          if isinstance(r, W.StreamRecord))
            assert rows == refsnap.MIGRATION_EXPECTED[wm], (ver, wm)
    finally:
        op.close()


@pytest.mark.parametrize("flags", [0, N.FLAG_FORCE_REGION], ids=["direct", "region"])
def test_gpu_snapshot_holds_the_reference_entries(flags):
    op = _migration_op(flags)
    try:
        for k, v, t in refsnap.MIGRATION_INPUT:
            op.process_element(W.StreamRecord((k, v), t))
        for wm in refsnap.MIGRATION_WATERMARKS:
            op.process_watermark(wm)
        assert [r for r in op.get_output() if isinstance(r, W.StreamRecord)] == []
        blob, keys = W.unpack_keyed_snapshot(op.snapshot_state_keyed((0, 0)))
    finally:
        op.close()
    got = parse(blob, "sum_i32")[0]
    ref = refsnap.parse(open(FIXTURES["2.1"], "rb").read())[0]
    assert sorted((s, e, keys[k], a) for s, e, k, a, h in got["state"]) == \
        sorted((s, e, k, v[1]) for s, e, k, v in ref["state"])
    assert all(h == W.java_string_hash(keys[k]) for s, e, k, a, h in got["state"])
    assert sorted((t, keys[k], s, e) for t, k, s, e in got["timers"]) == sorted(ref["event"])


# ---- random String-keyed streams --------------------------------------------------------
def _string_stream(seed, n, nkeys, nb, agg, disorder=200, wm_lag=300, ts_step=3):
    rng = np.random.default_rng(seed)
    words = [f"w{i}-{rng.integers(1 << 30)}" for i in range(nkeys)]
    kidx = rng.integers(0, nkeys, n)
    ts = np.arange(n, dtype=np.int64) * ts_step - rng.integers(0, disorder + 1, n)
    vals = (rng.uniform(0, 1000, n) if agg.endswith("f64") else rng.integers(-10 ** 6, 10 ** 6, n)).astype(
        np.float64 if agg.endswith("f64") else np.int64)
    cuts = np.linspace(0, n, nb + 1).astype(np.int64)
    batches = [(int(cuts[b]), int(cuts[b + 1]), int(ts[:cuts[b + 1]].max()) - wm_lag - 1) for b in range(nb)]
    return words, kidx, ts, vals, batches


def _encode(op, words, kidx):
    ids = np.array([op._encode_key(words[i]) for i in kidx], np.int64)
    return ids, np.asarray(op._hash_out, np.int32)[ids]


def _feed(op, words, kidx, ts, vals, batches, outs, keep=None):
    for lo, hi, wm in batches:
        sel = np.arange(lo, hi) if keep is None else np.arange(lo, hi)[keep[lo:hi]]
        if len(sel):
            ids, hs = _encode(op, words, kidx[sel])
            op.process_batch(ids, ts[sel], vals[sel], key_hashes=hs)
        op.advance_watermark(wm)
        k, s, e, r = op.drain()
        outs.append(([op._decode_key(int(x)) for x in k], s, e, r.view(np.int64)))


def _as_oracle_rows(outs, index):
    """Rows with String keys -> rows keyed by a fixed index of the words (for compare())."""
    return [(np.array([index[w] for w in k], np.int64), s, e, r) for k, s, e, r in outs]


def _merge(a, b):
    return [(np.concatenate([x[0], y[0]]), np.concatenate([x[1], y[1]]), np.concatenate([x[2], y[2]]),
             np.concatenate([x[3], y[3]])) for x, y in zip(a, b)]


def _op(kw, agg, **k):
    a = dict(kw)
    asg = {"tumbling": lambda: W.TumblingEventTimeWindows.of(a["size"]),
           "sliding": lambda: W.SlidingEventTimeWindows.of(a["size"], a["slide"]),
           "session": lambda: W.EventTimeSessionWindows.with_gap(a["gap"]),
           "count_sliding": lambda: W.CountWindows.of(a["size"], a["slide"])}[a["assigner"]]()
    return W.GpuWindowOperator(asg, agg, a.get("lateness", 0), capacity_hint=4096, **k).open()


CFGS = [dict(assigner="tumbling", size=500), dict(assigner="sliding", size=900, slide=300),
        dict(assigner="sliding", size=600, slide=200, lateness=400)]


@pytest.mark.parametrize("kw", CFGS, ids=["tumbling", "sliding", "sliding-lateness"])
@pytest.mark.parametrize("agg", ["sum_i64", "count", "max_i64", "avg_f64"])
def test_string_keys_blob_equals_oracle_and_rescales(oracle_lib, kw, agg):
    O = oracle_lib
    words, kidx, ts, vals, batches = _string_stream(11, 40_000, 700, 16, agg)
    cut = 8
    # uninterrupted oracle over word indices (their String.hashCode as key hashes)
    index = {w: i for i, w in enumerate(words)}
    hashes = np.array([W.java_string_hash(w) for w in words], np.int32)
    oc = O.make_config(kw["assigner"], size=kw["size"], slide=kw.get("slide", kw["size"]),
                       lateness=kw.get("lateness", 0), agg=agg)
    ora = O.OracleOperator(oc)
    ora.set_key_hashes(np.arange(len(words), dtype=np.int64), hashes)
    oouts, oblob = [], None
    vb = vals.view(np.int64) if vals.dtype == np.float64 else vals
    for b, (lo, hi, wm) in enumerate(batches):
        if b == cut:
            oblob = ora.snapshot()
        ora.process_batch(kidx[lo:hi].astype(np.int64), ts[lo:hi], vb[lo:hi])
        ora.process_watermark(wm)
        oouts.append(ora.drain())
    # GPU before the checkpoint; its blob (keys remapped to word indices) equals the oracle's
    g = _op(kw, agg)
    gouts = []
    _feed(g, words, kidx, ts, vals, batches[:cut], gouts)
    blob, keys = W.unpack_keyed_snapshot(g.snapshot_state_keyed())
    g.close()
    gp = parse(N.snapshot_remap_keys(blob, {i: index[w] for i, w in keys.items()}), agg)
    op_ = parse(oblob, agg)
    for kg in op_:
        a, o = gp[kg], op_[kg]
        assert sorted(t for t in a["timers"]) == sorted(o["timers"]), kg
        if agg == "avg_f64":
            assert [x[:3] + x[-1:] for x in a["state"]] == [x[:3] + x[-1:] for x in o["state"]], kg
        else:
            assert a["state"] == o["state"], kg
    # restore into two subtasks with fresh dictionaries (1 -> 2), each fed its key groups
    wrapped = W.pack_keyed_snapshot(blob, keys)
    kgw = np.array([W.assign_to_key_group(w, 128) for w in words])
    halves = []
    for r in range(2):
        lo_, hi_ = W.compute_key_group_range_for_operator_index(128, 2, r)
        sub = _op(kw, agg, parallelism=2, operator_index=r, flags=N.FLAG_CHECK_KEY_GROUPS)
        inner, ks = W.unpack_keyed_snapshot(wrapped)
        sub.initialize_state([W.pack_keyed_snapshot(N.snapshot_slice(inner, kg), ks) for kg in range(lo_, hi_ + 1)])
        mine = (kgw[kidx] >= lo_) & (kgw[kidx] <= hi_)
        outs = []
        _feed(sub, words, kidx, ts, vals, batches[cut:], outs, keep=mine)
        sub.close()
        halves.append(outs)
    got = gouts + _merge(halves[0], halves[1])
    assert compare(_as_oracle_rows(got, index), oouts, agg == "avg_f64") == []


@pytest.mark.parametrize("kw,agg", [(dict(assigner="session", gap=250), "sum_i64"),
                                    (dict(assigner="session", gap=400), "avg_f64"),
                                    (dict(assigner="count_sliding", size=40, slide=15), "sum_i64"),
                                    (dict(assigner="count_sliding", size=25, slide=25), "max_i64")],
                         ids=["session-sum", "session-avg", "count-sliding", "count-tumbling"])
def test_string_keys_slot_path_snapshot_rescale(kw, agg):
    """Sessions and count windows (the per-key slot path): a keyed snapshot of String keys
    restores 1 -> 2 by key groups of String.hashCode and continues exactly like the
    uninterrupted operator."""
    words, kidx, ts, vals, batches = _string_stream(5, 30_000, 300, 12, agg, ts_step=40)
    cut = 6
    full = _op(kw, agg)
    fouts = []
    _feed(full, words, kidx, ts, vals, batches, fouts)
    full.close()
    g = _op(kw, agg)
    gouts = []
    _feed(g, words, kidx, ts, vals, batches[:cut], gouts)
    wrapped = g.snapshot_state_keyed()
    g.close()
    inner, ks = W.unpack_keyed_snapshot(wrapped)
    kgw = np.array([W.assign_to_key_group(w, 128) for w in words])
    halves = []
    for r in range(2):
        lo_, hi_ = W.compute_key_group_range_for_operator_index(128, 2, r)
        sub = _op(kw, agg, parallelism=2, operator_index=r, flags=N.FLAG_CHECK_KEY_GROUPS)
        sub.initialize_state([W.pack_keyed_snapshot(N.snapshot_slice(inner, kg), ks) for kg in range(lo_, hi_ + 1)])
        mine = (kgw[kidx] >= lo_) & (kgw[kidx] <= hi_)
        outs = []
        _feed(sub, words, kidx, ts, vals, batches[cut:], outs, keep=mine)
        sub.close()
        halves.append(outs)
    index = {w: i for i, w in enumerate(words)}
    got = _as_oracle_rows(gouts + _merge(halves[0], halves[1]), index)
    want = _as_oracle_rows(fouts, index)
    assert compare(got, want, agg == "avg_f64") == []

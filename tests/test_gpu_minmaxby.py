"""minBy / maxBy on the GPU (GW_FLAG_BY_FIELD [+ GW_FLAG_BY_LAST]; gw_first.hip fe_by_select):
WindowedStream.minBy / maxBy (WindowedStream.java:725-771) reduce with ComparableAggregator's
byAggregate branch (ComparableAggregator.java:88-95): every row stands for the window's element
whose field is the minimum / maximum, the first of equal ones in arrival order or the last.
Records carry a 64-bit payload (the element's other fields); rows carry the payload of their
element.

Parity: bit-exact against the oracle (oracle/flink_oracle.c by_reduce, itself pinned to
AggregationFunctionTest.minMaxByTest's vectors in tests/test_oracle_minmaxby.py) -- the field and
the element's payload, for tumbling and sliding windows, window classes, lateness re-firings (first
of equal ones), i64 and f64 fields with many equal values, device columns, and a snapshot/restore
round trip."""
import zlib

import numpy as np
import pytest

from flink_amd import _native as N
from flink_amd import windowing as W
from tests.gpu_helpers import corrupt_last_group, gpu_operator, random_stream
from tests.harness import load_golden

pytestmark = pytest.mark.gpu

CONFIGS = [
    dict(assigner="tumbling", size=100),
    dict(assigner="tumbling", size=250, offset=-40, lateness=400),
    dict(assigner="sliding", size=1000, slide=100),
    dict(assigner="sliding", size=1000, slide=10),               # 2 window classes
    dict(assigner="sliding", size=600, slide=200, lateness=900),
]
AGGS = ["max_i64", "min_i64", "max_f64", "min_f64"]


def _flags(first):
    return N.FLAG_BY_FIELD | (0 if first else N.FLAG_BY_LAST)


def _stream(seed, agg, n=20000, num_keys=80, n_batches=25, lateness=0):
    keys, ts, _, batches = random_stream(seed=seed, n=n, num_keys=num_keys, n_batches=n_batches, ts_step=3,
                                         disorder=700 if lateness else 250, wm_lag=250)
    rng = np.random.default_rng(seed + 3)
    vals = rng.integers(-3, 4, n).astype(np.int64)  # 7 distinct fields: ties decide most elements
    if agg.endswith("f64"):
        vals = vals.astype(np.float64)
        vals[rng.random(n) < 0.01] = -0.0
    payload = rng.integers(-(1 << 62), 1 << 62, n).astype(np.int64)
    return keys, ts, vals, payload, batches


def _rows(k, s, e, r, p):
    r = r.view(np.int64)
    i = np.lexsort((p, r, e, s, k))
    return [x[i] for x in (k, s, e, r, p)]


def _expected(oracle_lib, kw, first, keys, ts, vals, payload, batches, cut=None):
    """The oracle's rows; with `cut`, snapshotted after that many batches and restored into a
    fresh operator (the watermark starts over after a restore, as in the reference)."""
    cfg = oracle_lib.make_config(**kw, flags=_flags(first))
    op = oracle_lib.OracleOperator(cfg)
    vb = vals.view(np.int64) if vals.dtype == np.float64 else vals
    outs = []
    try:
        for b, (lo, hi, wm) in enumerate(batches + [(len(keys), len(keys), W.LONG_MAX)]):
            if b == cut:
                blob = op.snapshot()
                op.close()
                op = oracle_lib.OracleOperator(cfg)
                op.restore(blob)
                op.set_arrival(lo)
            op.process_batch(keys[lo:hi], ts[lo:hi], vb[lo:hi])
            op.process_watermark(wm)
            k, s, e, r, q = op.drain_seq()
            outs.append(_rows(k, s, e, r, payload[q]))
        late = op.late_dropped
    finally:
        op.close()
    return outs, late


def _run(op, keys, ts, vals, payload, batches, device=False):
    outs = []
    for lo, hi, wm in batches:
        if hi > lo:
            if device:
                import torch
                cols = [torch.from_numpy(np.ascontiguousarray(x[lo:hi])).cuda()
                        for x in (keys, ts, vals.view(np.int64), payload)]
                op.process_batch_payload_device(*cols)
            else:
                op.process_batch_payload(keys[lo:hi], ts[lo:hi], vals[lo:hi], payload[lo:hi])
        op.advance_watermark(wm)
        outs.append(_rows(*op.drain_payload()))
    return outs


def _check(g, o):
    assert len(g) == len(o)
    for b, (G, O) in enumerate(zip(g, o)):
        assert len(G[0]) == len(O[0]), f"watermark #{b}: {len(G[0])} rows vs {len(O[0])}"
        for c, name in enumerate(["key", "start", "end", "field", "element"]):
            assert np.array_equal(G[c], O[c]), f"watermark #{b}: {name} differs"


@pytest.mark.parametrize("name", ["maxBy_first", "maxBy_last", "minBy_first", "minBy_last"])
def test_golden_running_element(name):
    """AggregationFunctionTest.minMaxByTest's vectors (tests/golden/minmaxby.json): a window
    holding elements 0..p stands for expected[p]; the payload is the element's index."""
    g = load_golden("minmaxby.json")
    inp = np.array(g["input"], dtype=np.int64)
    agg = "max_i64" if name.startswith("max") else "min_i64"
    for p in range(len(inp)):
        op = gpu_operator(dict(assigner="tumbling", size=1000, agg=agg), flags=_flags(name.endswith("first")))
        try:
            op.process_batch_payload(inp[: p + 1, 0].copy(), np.arange(p + 1, dtype=np.int64),
                                     inp[: p + 1, g["by_field"]].copy(), np.arange(p + 1, dtype=np.int64))
            op.advance_watermark(999)
            k, s, e, r, pl = op.drain_payload()
        finally:
            op.close()
        assert len(k) == 1
        assert inp[pl[0]].tolist() == g["expected"][name][p], (name, p)


@pytest.mark.parametrize("first", [True, False], ids=["first", "last"])
@pytest.mark.parametrize("agg", AGGS)
@pytest.mark.parametrize("kw", CONFIGS, ids=lambda c: "-".join(str(v) for v in c.values()))
def test_by_field_vs_oracle(oracle_lib, kw, agg, first):
    lat = kw.get("lateness", 0)
    kw = dict(kw, agg=agg)
    if lat and not first:
        with pytest.raises(N.GpuWinError):
            gpu_operator(kw, flags=_flags(first))
        return
    seed = zlib.crc32(f"by{kw}{first}".encode()) & 0xffff
    keys, ts, vals, payload, batches = _stream(seed, agg, lateness=lat)
    o, olate = _expected(oracle_lib, kw, first, keys, ts, vals, payload, batches)
    op = gpu_operator(kw, flags=_flags(first))
    try:
        g = _run(op, keys, ts, vals, payload, batches + [(len(keys), len(keys), W.LONG_MAX)])
        assert op.num_late_records_dropped == olate
    finally:
        op.close()
    _check(g, o)


@pytest.mark.parametrize("kw", [CONFIGS[0], CONFIGS[4]], ids=["tumbling", "sliding-lateness"])
def test_by_field_device_columns_and_region_path(oracle_lib, kw):
    kw = dict(kw, agg="max_i64")
    keys, ts, vals, payload, batches = _stream(77, "max_i64", n=60000, num_keys=700, n_batches=12,
                                               lateness=kw.get("lateness", 0))
    o, _ = _expected(oracle_lib, kw, True, keys, ts, vals, payload, batches)
    op = gpu_operator(kw, flags=_flags(True) | N.FLAG_FORCE_REGION)
    try:
        g = _run(op, keys, ts, vals, payload, batches + [(len(keys), len(keys), W.LONG_MAX)], device=True)
    finally:
        op.close()
    _check(g, o)


def test_by_field_log_release(oracle_lib):
    """~1.2M records over 60 batches: the log (payload, key, ts, field per record) releases
    what no window can reach and reuses its ring."""
    kw = dict(assigner="sliding", size=2000, slide=500, agg="min_i64")
    keys, ts, vals, payload, batches = _stream(5, "min_i64", n=1_200_000, num_keys=5000, n_batches=60)
    o, _ = _expected(oracle_lib, kw, False, keys, ts, vals, payload, batches)
    op = gpu_operator(kw, flags=_flags(False))
    try:
        g = _run(op, keys, ts, vals, payload, batches + [(len(keys), len(keys), W.LONG_MAX)])
    finally:
        op.close()
    _check(g, o)


@pytest.mark.parametrize("kw,agg,first", [(CONFIGS[0], "max_i64", True), (CONFIGS[2], "min_f64", False),
                                          (CONFIGS[3], "max_i64", False), (CONFIGS[4], "min_i64", True)],
                         ids=["tumbling-max-first", "sliding-min-f64-last", "window-classes-max-last",
                              "sliding-lateness-min-first"])
def test_by_field_snapshot_restore(oracle_lib, kw, agg, first):
    """A minBy / maxBy handle snapshots (window, key, field, element's payload) per (key, window)
    -- the reference's reduced element, HeapReducingState.java:90-97 -- and a fresh handle restored
    from it (through per-key-group slices) continues like the uninterrupted operator: the restored
    element is the state (value1) of every later reduce, so it wins ties when first = true."""
    kw = dict(kw, agg=agg)
    keys, ts, vals, payload, batches = _stream(91, agg, n=24000, num_keys=150, n_batches=24,
                                               lateness=kw.get("lateness", 0))
    cut = 11
    o, _ = _expected(oracle_lib, kw, first, keys, ts, vals, payload, batches, cut=cut)
    a = gpu_operator(kw, flags=_flags(first))
    try:
        outs = _run(a, keys, ts, vals, payload, batches[:cut])
        blob = a.snapshot_state()
    finally:
        a.close()
    b = gpu_operator(kw, flags=_flags(first))
    try:
        b.initialize_state([N.snapshot_slice(blob, kg) for kg in range(128)])
        outs += _run(b, keys, ts, vals, payload, batches[cut:] + [(len(keys), len(keys), W.LONG_MAX)])
    finally:
        b.close()
    _check(outs, o)


def test_by_field_rejections():
    for kw, fl in ((dict(assigner="tumbling", size=100, agg="sum_i64"), N.FLAG_BY_FIELD),
                   (dict(assigner="tumbling", size=100, agg="max_i64"), N.FLAG_BY_LAST),
                   (dict(assigner="tumbling", size=100, agg="max_i64", lateness=50), N.FLAG_BY_FIELD | N.FLAG_BY_LAST),
                   (dict(assigner="session", gap=100, agg="max_i64"), N.FLAG_BY_FIELD)):
        with pytest.raises((N.GpuWinError, ValueError)):
            gpu_operator(kw, flags=fl)


def test_datastream_min_by_emits_elements():
    """env.from_elements(...).key_by(f0).window(tumbling 10).min_by(1, first) emits the elements."""
    els = [("a", 3, "x0"), ("a", 1, "x1"), ("b", 5, "x2"), ("a", 1, "x3"), ("b", 5, "x4"), ("a", 2, "x5")]
    for first, want in ((True, {("a", 1, "x1"), ("b", 5, "x2")}), (False, {("a", 1, "x3"), ("b", 5, "x4")})):
        env = W.StreamExecutionEnvironment()
        stream = env.from_elements([W.StreamRecord(v, t) for t, v in enumerate(els)])
        out = stream.key_by(lambda v: v[0]).window(W.TumblingEventTimeWindows.of(10)).min_by(1, first) \
            .execute_and_collect()
        assert {r.value for r in out} == want


@pytest.mark.parametrize("kw,agg,first", [(CONFIGS[4], "min_i64", True), (CONFIGS[3], "max_i64", False)],
                         ids=["sliding-lateness-min-first", "window-classes-max-last"])
def test_by_field_rejected_restores_leave_the_handle_unchanged(oracle_lib, kw, agg, first):
    """A minBy / maxBy blob rejected part-way (GW_E_INVALID) and a restore after the handle took
    records (GW_E_STATE: initializeState runs before processing) change nothing: no element enters
    the log, no operator keeps restored entries.  The first handle then restores the good blob and
    continues like the oracle restored from it; the second continues like the uninterrupted
    oracle."""
    kw = dict(kw, agg=agg)
    keys, ts, vals, payload, batches = _stream(93, agg, n=24000, num_keys=150, n_batches=24,
                                               lateness=kw.get("lateness", 0))
    cut = 11
    final = [(len(keys), len(keys), W.LONG_MAX)]
    a = gpu_operator(kw, flags=_flags(first))
    try:
        outs = _run(a, keys, ts, vals, payload, batches[:cut])
        blob = a.snapshot_state()
    finally:
        a.close()
    b = gpu_operator(kw, flags=_flags(first))
    try:
        with pytest.raises(N.GpuWinError) as ei:
            b.initialize_state(corrupt_last_group(blob))
        assert ei.value.code == N.GW_E_INVALID
        b.initialize_state(blob)
        outs += _run(b, keys, ts, vals, payload, batches[cut:] + final)
    finally:
        b.close()
    o, _ = _expected(oracle_lib, kw, first, keys, ts, vals, payload, batches, cut=cut)
    _check(outs, o)
    c = gpu_operator(kw, flags=_flags(first))
    try:
        g = _run(c, keys, ts, vals, payload, batches[:2])
        with pytest.raises(N.GpuWinError) as ei:
            c.initialize_state(blob)
        assert ei.value.code == N.GW_E_STATE
        g += _run(c, keys, ts, vals, payload, batches[2:] + final)
    finally:
        c.close()
    o, _ = _expected(oracle_lib, kw, first, keys, ts, vals, payload, batches)
    _check(g, o)

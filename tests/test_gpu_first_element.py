"""Positional aggregations on wider tuples (GW_FLAG_FIRST_ELEMENT): WindowedStream.sum(i) /
min(i) / max(i) on a Tuple3+ emit the window's FIRST element in arrival order with field i
replaced by the aggregate (SumAggregator.reduce copies value1, RS/api/functions/aggregation/
SumAggregator.java:66-76; ComparableAggregator.reduce keeps value1's other fields, :83-104;
the heap ReducingState folds in arrival order, value1 = the state).  Records carry the
non-aggregated fields as a 64-bit payload; every row carries the first element's payload.

Parity: the aggregate column against the oracle's rows for the same stream, the payload column
against the oracle run as MIN over each record's arrival sequence (the same windows, the same
firings, lateness re-firings included), mapped through the payload array."""
import zlib

import numpy as np
import pytest

from flink_amd import _native as N
from flink_amd import windowing as W
from tests.gpu_helpers import corrupt_last_group, gpu_operator, random_stream, run_oracle

pytestmark = pytest.mark.gpu

CONFIGS = [
    dict(assigner="tumbling", size=100),
    dict(assigner="tumbling", size=250, offset=-40, lateness=400),
    dict(assigner="sliding", size=1000, slide=100),
    dict(assigner="sliding", size=1000, slide=10),               # 2 window classes
    dict(assigner="sliding", size=600, slide=200, lateness=900),
]


def _expected(oracle_lib, kw, keys, ts, vals, payload, batches):
    agg_out, late = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    seq = np.arange(len(keys), dtype=np.int64)
    seq_out, _ = run_oracle(oracle_lib, dict(kw, agg="min_i64"), keys, ts, seq, batches)
    out = []
    for a, s in zip(agg_out, seq_out):
        ia = np.lexsort((a[2], a[1], a[0]))
        is_ = np.lexsort((s[2], s[1], s[0]))
        A = [x[ia] for x in a]
        S = [x[is_] for x in s]
        assert all(np.array_equal(A[c], S[c]) for c in range(3))
        out.append((A[0], A[1], A[2], A[3], payload[S[3]]))
    return out, late


def _run_gpu(kw, keys, ts, vals, payload, batches, device=False, flags=0):
    op = gpu_operator(kw, flags=N.FLAG_FIRST_ELEMENT | flags)
    outs = []
    try:
        for lo, hi, wm in batches:
            if device:
                import torch
                cols = [torch.from_numpy(np.ascontiguousarray(x[lo:hi])).cuda()
                        for x in (keys, ts, vals.view(np.int64), payload)]
                op.process_batch_payload_device(*cols)
            else:
                op.process_batch_payload(keys[lo:hi], ts[lo:hi], vals[lo:hi], payload[lo:hi])
            op.advance_watermark(wm)
            outs.append(op.drain_payload())
        op.advance_watermark(W.LONG_MAX)
        outs.append(op.drain_payload())
        late = op.num_late_records_dropped
    finally:
        op.close()
    res = []
    for k, s, e, r, p in outs:
        i = np.lexsort((e, s, k))
        res.append((k[i], s[i], e[i], r.view(np.int64)[i], p[i]))
    return res, late


def _check(g, o, is_double):
    assert len(g) == len(o)
    for b, (G, O) in enumerate(zip(g, o)):
        assert len(G[0]) == len(O[0]), f"watermark #{b}: {len(G[0])} rows vs {len(O[0])}"
        for c in (0, 1, 2, 4):
            assert np.array_equal(G[c], O[c]), f"watermark #{b}: column {c} differs"
        if is_double:
            gv, ov = G[3].view(np.float64), O[3].view(np.float64)
            assert np.allclose(gv, ov, rtol=1e-6, atol=0), f"watermark #{b}: f64 result beyond 1e-6 rel"
        else:
            assert np.array_equal(G[3], O[3]), f"watermark #{b}: result differs"


@pytest.mark.parametrize("agg", ["sum_i64", "min_i64", "max_f64", "sum_f64"])
@pytest.mark.parametrize("kw", CONFIGS, ids=lambda c: "-".join(str(v) for v in c.values()))
def test_first_element_vs_oracle(oracle_lib, kw, agg):
    kw = dict(kw, agg=agg)
    lat = kw.get("lateness", 0)
    seed = zlib.crc32(f"fe{kw}".encode()) & 0xffff
    keys, ts, vals, batches = random_stream(seed=seed, n=20000, num_keys=80, n_batches=25, ts_step=3,
                                            disorder=700 if lat else 250, wm_lag=250, agg=agg)
    payload = np.random.default_rng(seed + 1).integers(-(1 << 62), 1 << 62, len(keys)).astype(np.int64)
    o, olate = _expected(oracle_lib, kw, keys, ts, vals, payload, batches)
    g, glate = _run_gpu(kw, keys, ts, vals, payload, batches)
    assert glate == olate
    _check(g, o, agg.endswith("f64"))


@pytest.mark.parametrize("kw", [CONFIGS[0], CONFIGS[4]], ids=["tumbling", "sliding-lateness"])
def test_first_element_device_columns(oracle_lib, kw):
    kw = dict(kw, agg="max_i64")
    keys, ts, vals, batches = random_stream(seed=77, n=30000, num_keys=500, n_batches=12, ts_step=2,
                                            disorder=900, wm_lag=300, agg="max_i64")
    payload = np.arange(len(keys), dtype=np.int64) * 7919 + 13
    o, olate = _expected(oracle_lib, kw, keys, ts, vals, payload, batches)
    g, glate = _run_gpu(kw, keys, ts, vals, payload, batches, device=True)
    assert glate == olate
    _check(g, o, False)


def test_first_element_log_release(oracle_lib):
    """Many batches: the payload log releases what no window can reach any more and reuses its
    ring (a run over ~1.2M records with a log that stays small)."""
    kw = dict(assigner="sliding", size=2000, slide=500, agg="sum_i64")
    keys, ts, vals, batches = random_stream(seed=5, n=1_200_000, num_keys=5000, n_batches=60, ts_step=1,
                                            disorder=200, wm_lag=200, agg="sum_i64")
    payload = (np.arange(len(keys), dtype=np.int64) << 20) ^ keys
    o, _ = _expected(oracle_lib, kw, keys, ts, vals, payload, batches)
    g, _ = _run_gpu(kw, keys, ts, vals, payload, batches, flags=N.FLAG_FORCE_REGION)
    _check(g, o, False)


def test_first_element_rejections():
    op = gpu_operator(dict(assigner="tumbling", size=100, agg="sum_i64"), flags=N.FLAG_FIRST_ELEMENT)
    try:
        with pytest.raises(N.GpuWinError):
            op.process_batch(np.zeros(4, np.int64), np.zeros(4, np.int64), np.zeros(4, np.int64))
    finally:
        op.close()
    plain = gpu_operator(dict(assigner="tumbling", size=100, agg="sum_i64"))
    try:
        with pytest.raises(N.GpuWinError):
            plain.process_batch_payload(np.zeros(2, np.int64), np.zeros(2, np.int64), np.zeros(2, np.int64),
                                        np.zeros(2, np.int64))
    finally:
        plain.close()
    for kw in (dict(assigner="tumbling", size=100, agg="sum_i64", trigger="purging_event_time"),
               dict(assigner="tumbling", size=100, agg="count"),
               dict(assigner="session", gap=100, agg="sum_i64")):
        with pytest.raises((N.GpuWinError, ValueError)):
            gpu_operator(kw, flags=N.FLAG_FIRST_ELEMENT)


@pytest.mark.parametrize("kw,agg", [(CONFIGS[0], "sum_i64"), (CONFIGS[2], "max_f64"), (CONFIGS[3], "min_i64"),
                                    (CONFIGS[4], "sum_i64")],
                         ids=["tumbling-sum", "sliding-max-f64", "window-classes-min", "sliding-lateness-sum"])
def test_first_element_snapshot_restore(oracle_lib, kw, agg):
    """A first-element handle snapshots (window, key, aggregate, first element's payload) per
    (key, window) -- the reference's reduced Tuple, HeapReducingState.java:90-97 -- and a fresh
    handle restored from it (through per-key-group slices) continues like the uninterrupted
    operator: same rows, same first elements."""
    kw = dict(kw, agg=agg)
    lat = kw.get("lateness", 0)
    keys, ts, vals, batches = random_stream(seed=91, n=24000, num_keys=150, n_batches=24, ts_step=3,
                                            disorder=240, wm_lag=250, agg=agg)
    payload = np.random.default_rng(92).integers(-(1 << 62), 1 << 62, len(keys)).astype(np.int64)
    o, _ = _expected(oracle_lib, kw, keys, ts, vals, payload, batches)
    cut = 11
    a = gpu_operator(kw, flags=N.FLAG_FIRST_ELEMENT)
    outs = []
    try:
        for lo, hi, wm in batches[:cut]:
            a.process_batch_payload(keys[lo:hi], ts[lo:hi], vals[lo:hi], payload[lo:hi])
            a.advance_watermark(wm)
            outs.append(a.drain_payload())
        blob = a.snapshot_state()
    finally:
        a.close()
    b = gpu_operator(kw, flags=N.FLAG_FIRST_ELEMENT)
    try:
        b.initialize_state([N.snapshot_slice(blob, kg) for kg in range(128)])
        for lo, hi, wm in batches[cut:]:
            b.process_batch_payload(keys[lo:hi], ts[lo:hi], vals[lo:hi], payload[lo:hi])
            b.advance_watermark(wm)
            outs.append(b.drain_payload())
        b.advance_watermark(W.LONG_MAX)
        outs.append(b.drain_payload())
    finally:
        b.close()
    g = []
    for k, s, e, r, p in outs:
        i = np.lexsort((e, s, k))
        g.append((k[i], s[i], e[i], r.view(np.int64)[i], p[i]))
    _check(g, o, agg.endswith("f64"))


@pytest.mark.parametrize("kw,agg", [(CONFIGS[4], "sum_i64"), (CONFIGS[3], "min_i64")],
                         ids=["sliding-lateness-sum", "window-classes-min"])
def test_first_element_rejected_restores_leave_the_handle_unchanged(oracle_lib, kw, agg):
    """A first-element blob rejected part-way (GW_E_INVALID) and a restore after the handle took
    records (GW_E_STATE) leave no trace: no payload in the log, no sequence consumed, no entries in
    either operator.  The handle then takes the good blob and continues like a handle that never
    saw the bad one (and, for the refused late restore, like the uninterrupted oracle)."""
    kw = dict(kw, agg=agg)
    keys, ts, vals, batches = random_stream(seed=95, n=24000, num_keys=150, n_batches=24, ts_step=3,
                                            disorder=240, wm_lag=250, agg=agg)
    payload = np.random.default_rng(96).integers(-(1 << 62), 1 << 62, len(keys)).astype(np.int64)
    cut = 11
    a = gpu_operator(kw, flags=N.FLAG_FIRST_ELEMENT)
    try:
        for lo, hi, wm in batches[:cut]:
            a.process_batch_payload(keys[lo:hi], ts[lo:hi], vals[lo:hi], payload[lo:hi])
            a.advance_watermark(wm)
            a.drain_payload()
        blob = a.snapshot_state()
    finally:
        a.close()

    def continue_from(op, blobs):
        for bl in blobs:
            op.initialize_state(bl)
        out = []
        for lo, hi, wm in batches[cut:] + [(len(keys), len(keys), W.LONG_MAX)]:
            op.process_batch_payload(keys[lo:hi], ts[lo:hi], vals[lo:hi], payload[lo:hi])
            op.advance_watermark(wm)
            k, s, e, r, p = op.drain_payload()
            i = np.lexsort((e, s, k))
            out.append((k[i], s[i], e[i], r.view(np.int64)[i], p[i]))
        return out

    b = gpu_operator(kw, flags=N.FLAG_FIRST_ELEMENT)
    c = gpu_operator(kw, flags=N.FLAG_FIRST_ELEMENT)
    try:
        with pytest.raises(N.GpuWinError) as ei:
            b.initialize_state(corrupt_last_group(blob))
        assert ei.value.code == N.GW_E_INVALID
        _check(continue_from(b, [blob]), continue_from(c, [blob]), False)
    finally:
        b.close()
        c.close()
    # restore after processing started: refused, nothing changes
    o, _ = _expected(oracle_lib, kw, keys, ts, vals, payload, batches)
    d = gpu_operator(kw, flags=N.FLAG_FIRST_ELEMENT)
    outs = []
    try:
        for b_, (lo, hi, wm) in enumerate(batches + [(len(keys), len(keys), W.LONG_MAX)]):
            if b_ == 2:
                with pytest.raises(N.GpuWinError) as ei:
                    d.initialize_state(blob)
                assert ei.value.code == N.GW_E_STATE
            d.process_batch_payload(keys[lo:hi], ts[lo:hi], vals[lo:hi], payload[lo:hi])
            d.advance_watermark(wm)
            k, s, e, r, p = d.drain_payload()
            i = np.lexsort((e, s, k))
            outs.append((k[i], s[i], e[i], r.view(np.int64)[i], p[i]))
    finally:
        d.close()
    _check(outs, o, False)

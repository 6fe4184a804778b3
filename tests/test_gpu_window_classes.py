"""Sliding windows whose pane ring exceeds 64 positions (size/gcd + slide/gcd > 64, or allowed
lateness spanning more panes than the ring holds): the handle splits the windows into J
classes k = j (mod J), each an operator with slide J * slide and offset offset + j * slide
(gw_runtime.cpp make_composite), and combines their rows, late counts and side outputs.

Parity against the oracle, which keeps one state per (key, window) as the reference's
WindowOperator does (WindowOperator.java:293-494; SlidingEventTimeWindows.assignWindows
:77-90 assigns size/slide windows per record).  A late record is counted (or side-output)
once: by the class of its last window, the one whose lateness decides the reference's
isSkippedElement && isElementLate (WindowOperator.java:440-446)."""
import ctypes
import zlib

import numpy as np
import pytest

from flink_amd import _native as N
from tests.gpu_helpers import compare, gpu_operator, random_stream, run_gpu, run_oracle

pytestmark = pytest.mark.gpu

DOUBLE = {"sum_f64", "avg_f64", "avg_i64", "min_f64", "max_f64"}

CONFIGS = [
    dict(assigner="sliding", size=1000, slide=10),                 # n = 100: 2 classes
    dict(assigner="sliding", size=7000, slide=60, offset=-25),     # gcd 20, n = 350: 10 classes
    dict(assigner="sliding", size=3000, slide=40),                 # n = 75: 2 classes
    dict(assigner="sliding", size=1000, slide=100, lateness=10_000),  # lateness over 102 panes
    dict(assigner="tumbling", size=100, lateness=10_000),           # 102 windows of lateness: 3 classes
    dict(assigner="tumbling", size=60, offset=-7, lateness=5_000),  # 85 windows: 2 classes
    dict(assigner="sliding", size=300, slide=100, lateness=20_000), # classes of slide >= size (gapped)
]


def _classes(kw):
    size, lat = kw["size"], kw.get("lateness", 0)
    slide = kw.get("slide", size)

    def need(sl):
        g = sl if size < sl else np.gcd(size, sl)  # size < slide: one pane per slide (gapped)
        n, m = (1, 1) if size < sl else (size // g, sl // g)
        r = n + max(m, 1)
        if lat:
            extra = lat // sl + 2
            r += extra * m
        return r

    if need(slide) <= 64:
        return 1
    return next(J for J in range(2, 4097) if need(slide * J) <= 64)


@pytest.mark.parametrize("agg", ["sum_i64", "count", "max_i64", "avg_f64", "sum_f64"])
@pytest.mark.parametrize("kw", CONFIGS, ids=lambda c: "-".join(str(v) for v in c.values()))
@pytest.mark.parametrize("flags", [0, N.FLAG_FORCE_REGION], ids=["auto", "region"])
def test_window_classes_vs_oracle(oracle_lib, kw, agg, flags):
    kw = dict(kw, agg=agg)
    assert _classes(kw) > 1
    lat = kw.get("lateness", 0)
    keys, ts, vals, batches = random_stream(seed=zlib.crc32(f"wc{kw}".encode()) & 0xffff, n=12000, num_keys=60,
                                            n_batches=24, ts_step=3, disorder=600 if lat else 250,
                                            wm_lag=250, agg=agg)
    g, glate, stats = run_gpu(kw, keys, ts, vals, batches, flags=flags)
    o, olate = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert glate == olate
    assert compare(g, o, agg in DOUBLE) == []
    assert stats["events_in"] == len(keys)
    if lat:
        assert glate > 0 or sum(len(x[0]) for x in o) > 0


def test_window_classes_side_output(oracle_lib):
    """Each late record reaches the side output once, from the class of its last window."""
    kw = dict(assigner="sliding", size=1000, slide=10, agg="sum_i64")
    o = oracle_lib
    keys, ts, vals, batches = random_stream(seed=91, n=15000, num_keys=50, n_batches=25, ts_step=3,
                                            disorder=3000, wm_lag=200)
    op = gpu_operator(kw, flags=N.FLAG_LATE_SIDE_OUTPUT)
    ora = o.OracleOperator(o.make_config(**kw, flags=N.FLAG_LATE_SIDE_OUTPUT))
    n_side = 0
    for b, (lo, hi, wm) in enumerate(batches):
        op.process_batch(keys[lo:hi], ts[lo:hi], vals[lo:hi])
        op.advance_watermark(wm)
        ora.process_batch(keys[lo:hi], ts[lo:hi], vals[lo:hi])
        ora.process_watermark(wm)
        k, s, e, r = op.drain()
        assert compare([(k, s, e, r.view(np.int64))], [ora.drain()], False) == [], f"rows at watermark #{b}"
        got = sorted(zip(*[c.tolist() for c in op.drain_late()]))
        exp = sorted(zip(*[c.tolist() for c in ora.drain_late()]))
        assert got == exp, f"side output at watermark #{b}"
        n_side += len(exp)
    assert n_side > 0 and op.num_late_records_dropped == 0
    op.close()
    ora.close()


def _d2h(ptr, n):
    """n int64 words at a device pointer -> numpy (hipMemcpy of the runtime torch loaded)."""
    import torch  # noqa: F401  (one HIP runtime per process: torch's)
    hip = ctypes.CDLL("libamdhip64.so.7")
    out = np.empty(n, np.int64)
    if n:
        assert hip.hipMemcpy(ctypes.c_void_p(out.ctypes.data), ctypes.c_void_p(ptr), ctypes.c_size_t(n * 8), 2) == 0
    return out


def test_window_classes_rows_device_and_stats(oracle_lib):
    """gw_rows_device gathers the classes' rows into one device view (what a device-side
    consumer reads); gw_drain then returns the same rows; stats count each record once."""
    kw = dict(assigner="sliding", size=2000, slide=20, agg="count")
    keys, ts, vals, batches = random_stream(seed=5, n=8000, num_keys=30, n_batches=8, ts_step=5, disorder=100,
                                            wm_lag=150, agg="count")
    op = gpu_operator(kw)
    got = []
    for lo, hi, wm in batches:
        op.process_batch(keys[lo:hi], ts[lo:hi], None)
        op.advance_watermark(wm)
        ptrs, n = op.rows_device()
        op.synchronize()
        view = [_d2h(p, n) for p in ptrs]
        k, s, e, r = op.drain()
        assert len(k) == n
        a = np.lexsort((view[2], view[1], view[0]))
        b = np.lexsort((e, s, k))
        for x, y in zip(view, (k, s, e, r.view(np.int64))):
            assert np.array_equal(x[a], y[b])
        got.append((k, s, e, r.view(np.int64)))
    o, _ = run_oracle(oracle_lib, kw, keys, ts, vals, batches, final_wm=None)
    assert compare(got, o, False) == []
    assert op.stats()["events_in"] == len(keys)
    op.close()


SNAP_CFGS = [
    dict(assigner="sliding", size=1000, slide=10),
    dict(assigner="sliding", size=1000, slide=100, lateness=10_000),
    dict(assigner="tumbling", size=100, lateness=10_000),
]


@pytest.mark.parametrize("agg", ["sum_i64", "avg_f64", "count"])
@pytest.mark.parametrize("cfg", SNAP_CFGS, ids=lambda c: "-".join(str(v) for v in c.values()))
def test_window_classes_snapshot_equals_oracle(oracle_lib, cfg, agg):
    """The classes' blobs merged per key group equal the oracle's heap-layout snapshot of the
    same stream: (window, key) entries, accumulators and timers."""
    from test_gpu_restore import feed_gpu, feed_oracle, same_state
    kw = dict(cfg, agg=agg)
    keys, ts, vals, batches = random_stream(31, 9000, 120, 10, ts_step=3, disorder=1500, wm_lag=300, agg=agg)
    op = gpu_operator(kw, capacity_hint=4096)
    ora = oracle_lib.OracleOperator(oracle_lib.make_config(**kw))
    go, oo = [], []
    feed_gpu(op, keys, ts, vals, batches[:6], go)
    feed_oracle(ora, keys, ts, vals, batches[:6], oo)
    same_state(op.snapshot_state(), ora.snapshot(), agg)
    assert compare(go, oo, agg in DOUBLE) == []
    op.close()
    ora.close()


@pytest.mark.parametrize("agg", ["sum_i64", "avg_f64"])
@pytest.mark.parametrize("cfg", SNAP_CFGS, ids=lambda c: "-".join(str(v) for v in c.values()))
@pytest.mark.parametrize("writer", ["oracle", "gpu"])
def test_window_classes_restore(oracle_lib, cfg, agg, writer):
    """A blob written by either side restores into the classes (split by window class) and
    into the oracle; records of fired windows arriving before the first watermark re-fire
    them (the watermark restarts at Long.MIN_VALUE) and both continue identically."""
    from test_gpu_restore import feed_gpu, feed_oracle, resume
    o = oracle_lib
    kw = dict(cfg, agg=agg)
    keys, ts, vals, batches = random_stream(37, 9000, 120, 10, ts_step=3, disorder=1500, wm_lag=300, agg=agg)
    cut = 5
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
    old = np.arange(0, batches[1][1], 5)
    g, glate, _ = resume("gpu", o, kw, blob, keys, ts, vals, batches[cut:], old)
    r, rlate, _ = resume("oracle", o, kw, blob, keys, ts, vals, batches[cut:], old)
    assert compare(g, r, agg in DOUBLE) == []
    assert glate == rlate


def test_lateness_beyond_4096_classes_is_unsupported():
    # tumbling windows of 1 ms with ~1e9 windows of lateness: no split into <= 4096 classes fits
    with pytest.raises(N.GpuWinError) as ei:
        gpu_operator(dict(assigner="tumbling", size=1, agg="sum_i64", lateness=10 ** 9))
    assert ei.value.code == -2


GAPPED = [
    dict(assigner="sliding", size=30, slide=100),
    dict(assigner="sliding", size=70, slide=250, offset=-40),
    dict(assigner="sliding", size=30, slide=100, lateness=1_500),
]


@pytest.mark.parametrize("agg", ["sum_i64", "count", "min_f64"])
@pytest.mark.parametrize("kw", GAPPED, ids=lambda c: "-".join(str(v) for v in c.values()))
@pytest.mark.parametrize("flags", [0, N.FLAG_FORCE_REGION, N.FLAG_LATE_SIDE_OUTPUT], ids=["auto", "region", "side"])
def test_sliding_with_gaps_vs_oracle(oracle_lib, kw, agg, flags):
    """size < slide (SlidingEventTimeWindows allows it): one pane per slide, the window at its
    start; a record in the gap gets no window (assignWindows returns none) and is dropped
    silently unless it is late (isSkippedElement && isElementLate, WindowOperator.java:440-446)."""
    kw = dict(kw, agg=agg)
    lat = kw.get("lateness", 0)
    keys, ts, vals, batches = random_stream(seed=zlib.crc32(f"gap{kw}".encode()) & 0xffff, n=15000, num_keys=70,
                                            n_batches=20, ts_step=3, disorder=900 if lat else 400, wm_lag=250,
                                            agg=agg)
    if flags == N.FLAG_LATE_SIDE_OUTPUT:
        op = gpu_operator(kw, flags=flags)
        ora = oracle_lib.OracleOperator(oracle_lib.make_config(**kw, flags=flags))
        for b, (lo, hi, wm) in enumerate(batches):
            op.process_batch(keys[lo:hi], ts[lo:hi], vals[lo:hi])
            op.advance_watermark(wm)
            vb = vals.view(np.int64) if vals.dtype == np.float64 else vals
            ora.process_batch(keys[lo:hi], ts[lo:hi], vb[lo:hi])
            ora.process_watermark(wm)
            k, s, e, r = op.drain()
            assert compare([(k, s, e, r.view(np.int64))], [ora.drain()], agg in DOUBLE) == []
            got = sorted(zip(*[c.tolist() for c in op.drain_late()]))
            exp = sorted(zip(*[c.tolist() for c in ora.drain_late()]))
            assert got == exp, f"side output at watermark #{b}"
        op.close()
        ora.close()
        return
    g, glate, stats = run_gpu(kw, keys, ts, vals, batches, flags=flags)
    o, olate = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert glate == olate
    assert compare(g, o, agg in DOUBLE) == []


def test_window_classes_network_buffers(oracle_lib):
    """A window-class handle fed network buffers: every class decodes the channel; the rows
    equal the oracle operator fed the decoded channel."""
    from test_gpu_netbuf import channel_stream, drained, oracle_channel
    from flink_amd import netbuf as NB
    from flink_amd import windowing as W
    kw, types, kf, vf = dict(assigner="sliding", size=1500, slide=15, agg="sum_i64"), "JJ", 0, 1
    data = channel_stream(kw, types, kf, vf, seed=17, n=20000, nb=8, n_keys=200)
    exp = oracle_channel(oracle_lib, kw, data, types, kf, vf)
    op = gpu_operator(kw)
    try:
        op.process_buffers(NB.split_buffers(data, 4093), N.record_layout(types, kf, vf))
        op.advance_watermark(W.LONG_MAX)
        got = drained(op)
    finally:
        op.close()
    assert compare([got], [exp], False) == []


@pytest.mark.parametrize("agg", ["sum_i32", "min_f64"])
def test_window_classes_purging_trigger_with_lateness(oracle_lib, agg):
    kw = dict(assigner="sliding", size=1200, slide=20, lateness=400, trigger="purging_event_time", agg=agg)
    keys, ts, vals, batches = random_stream(seed=23, n=10000, num_keys=40, n_batches=20, ts_step=3, disorder=800,
                                            wm_lag=200, agg=agg)
    g, glate, _ = run_gpu(kw, keys, ts, vals, batches)
    o, olate = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert glate == olate
    assert compare(g, o, agg in DOUBLE) == []

"""gw_clear_rows (a DiscardingSink's consumption of the fired rows) after every other
watermark, drained rows in between, against the oracle.  Since round 6 the call writes no
device status: the host takes the row count as 0 and the next launch that emits rows zeroes
the device cursor first (gw_runtime.cpp rows_reset_now: the fast fire's guard, or a status
write before any other fire, a lateness re-fire included).  Each drained watermark must hold
exactly the oracle's rows of that watermark -- none of a cleared one's -- on the fast fire, the
exact fire (direct path, lateness re-fires) and window-class composites.

Reference: WindowOperator.onEventTime emits each window's result once
(RS/runtime/operators/windowing/WindowOperator.java:439-494); what a sink does with earlier
rows changes nothing after it.
"""
import zlib

import numpy as np
import pytest

from flink_amd import _native as N
from tests.gpu_helpers import compare, gpu_operator, random_stream, run_oracle

pytestmark = pytest.mark.gpu


def _run_alternating(kw, keys, ts, vals, batches, **opkw):
    """Watermark b: rows cleared (after checking the count is reset) when b % 3 == 0, drained
    otherwise (the streams fire every other batch: both kinds meet fires); returns the drained
    watermarks' rows (None for cleared ones)."""
    op = gpu_operator(kw, **opkw)
    outs, cleared = [], 0
    try:
        for b, (lo, hi, wm) in enumerate(batches + [(len(keys), len(keys), 1 << 62)]):
            if hi > lo:
                op.process_batch(keys[lo:hi], ts[lo:hi], vals[lo:hi])
            op.advance_watermark(wm)
            if b % 3 == 0:
                cleared += op.pending_rows()
                op.clear_rows()
                assert op.pending_rows() == 0
                outs.append(None)
            else:
                k, s, e, r = op.drain()
                outs.append((k, s, e, r.view(np.int64)))
        stats = op.stats()
        stats["fast_fires"] = op.kernel_time_ms(3)[1]
    finally:
        op.close()
    return outs, cleared, stats


def _check(oracle_lib, kw, stream, **opkw):
    keys, ts, vals, batches = stream
    g, cleared, stats = _run_alternating(kw, keys, ts, vals, batches, **opkw)
    o, _ = run_oracle(oracle_lib, kw, keys, ts, vals, batches, final_wm=1 << 62)
    assert len(g) == len(o)
    keep = [b for b in range(len(g)) if g[b] is not None]
    assert compare([g[b] for b in keep], [o[b] for b in keep], kw["agg"].endswith("f64")) == []
    assert cleared == sum(len(o[b][0]) for b in range(len(o)) if g[b] is None)
    assert sum(len(o[b][0]) for b in keep) > 0 and cleared > 0
    return stats


@pytest.mark.parametrize("flags,hint", [(N.FLAG_FORCE_REGION, 600_000), (N.FLAG_NO_REGION, 40_000)],
                         ids=["region-buffered", "direct"])
@pytest.mark.parametrize("agg", ["sum_i64", "max_i64", "avg_f64"])
def test_clear_rows_between_fires(oracle_lib, agg, flags, hint):
    kw = dict(assigner="sliding", size=30_000, slide=10_000, agg=agg)
    stream = random_stream(seed=zlib.crc32(f"clr{agg}{flags}".encode()) & 0xffff, n=200_000, num_keys=20_000,
                           n_batches=40, ts_step=1, agg=agg)
    stats = _check(oracle_lib, kw, stream, flags=flags, capacity_hint=hint)
    assert stats["fires"] >= 10


def test_clear_rows_with_lateness_refires(oracle_lib):
    """Lateness > 0: no fast fire; late records re-fire windows (k_refire moves the cursor)."""
    kw = dict(assigner="sliding", size=30_000, slide=10_000, agg="sum_i64", lateness=5_000)
    stream = random_stream(seed=21, n=120_000, num_keys=4_000, n_batches=30, ts_step=1, disorder=8_000)
    stats = _check(oracle_lib, kw, stream, flags=N.FLAG_FORCE_REGION, capacity_hint=10_000)
    assert stats["fast_fires"] == 0


def test_clear_rows_window_classes(oracle_lib):
    """A sliding assigner whose ring exceeds 64 panes: child operators per window class."""
    kw = dict(assigner="sliding", size=70_000, slide=1_000, agg="count")
    stream = random_stream(seed=23, n=150_000, num_keys=3_000, n_batches=24, ts_step=1, agg="count")
    _check(oracle_lib, kw, stream, capacity_hint=5_000)

"""The fire enqueued right behind its flush (gw_runtime.cpp fast_fire, gw_pane.hip
k_fire_guard): one host round trip per watermark instead of two.  Parity with the oracle at
every watermark where it runs, and where the guard must turn it into a no-op so the exact
path takes over: spilled records and a full table after the flush (table growth), a row
buffer too small for the fire, records deferred by the flush.  Lateness > 0 and restored
windows never take it.

Reference: WindowOperator.onEventTime (RS/runtime/operators/windowing/WindowOperator.java:
439-494): the rows of every watermark are the oracle's, whichever way the fire was launched.
"""
import zlib

import numpy as np
import pytest

from flink_amd import _native as N
from tests.gpu_helpers import compare, random_stream, run_gpu, run_oracle

pytestmark = pytest.mark.gpu


def _run(oracle_lib, kw, stream, **opkw):
    keys, ts, vals, batches = stream
    g, glate, stats = run_gpu(kw, keys, ts, vals, batches, **opkw)
    o, olate = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert glate == olate
    assert compare(g, o, kw["agg"].endswith("f64")) == []
    return stats


@pytest.mark.parametrize("agg", ["sum_i64", "max_f64", "avg_f64", "count"])
@pytest.mark.parametrize("flags,hint", [(N.FLAG_FORCE_REGION, 40_000), (N.FLAG_FORCE_REGION, 600_000),
                                        (N.FLAG_NO_REGION, 40_000)],
                         ids=["region-single-pass", "region-buffered", "direct"])
def test_fast_fire_taken_and_exact(oracle_lib, agg, flags, hint):
    kw = dict(assigner="sliding", size=30_000, slide=10_000, agg=agg)
    stream = random_stream(seed=zlib.crc32(f"ff{agg}{flags}{hint}".encode()) & 0xffff, n=200_000, num_keys=20_000,
                           n_batches=60, ts_step=1, agg=agg)
    stats = _run(oracle_lib, kw, stream, flags=flags, capacity_hint=hint)
    assert stats["fires"] >= 10
    assert stats["fast_fires"] >= stats["fires"] // 2, stats


@pytest.mark.parametrize("agg", ["sum_i64", "avg_f64"])
def test_fast_fire_guard_table_growth(oracle_lib, agg):
    """A table sized for 2000 keys gets 300k: flushes end with spills / a full table, the
    guard skips the fire behind them and the exact path grows the table first."""
    kw = dict(assigner="sliding", size=400_000, slide=200_000, agg=agg)
    stream = random_stream(seed=5, n=1_200_000, num_keys=300_000, n_batches=12, ts_step=1, agg=agg)
    stats = _run(oracle_lib, kw, stream, flags=N.FLAG_FORCE_REGION, capacity_hint=2000)
    assert stats["rehashes"] > 0


def test_fast_fire_guard_row_buffer(oracle_lib):
    """The row buffer starts at the capacity hint (1024 rows) while every fire emits ~tens of
    thousands: the guard's room test skips the fire, the exact path grows the buffer."""
    kw = dict(assigner="tumbling", size=20_000, slide=20_000, agg="sum_i64")
    stream = random_stream(seed=7, n=300_000, num_keys=60_000, n_batches=15, ts_step=1)
    _run(oracle_lib, kw, stream, flags=N.FLAG_NO_REGION, capacity_hint=1024)


def test_fast_fire_not_taken_with_lateness(oracle_lib):
    kw = dict(assigner="sliding", size=30_000, slide=10_000, agg="sum_i64", lateness=5_000)
    stream = random_stream(seed=11, n=100_000, num_keys=5_000, n_batches=30, ts_step=1, disorder=8_000)
    stats = _run(oracle_lib, kw, stream, flags=N.FLAG_FORCE_REGION, capacity_hint=10_000)
    assert stats["fast_fires"] == 0


def test_fast_fire_far_future_and_jumps(oracle_lib):
    """Watermark jumps over many windows and records far ahead of the ring: fires whose ring
    does not reach the target, or whose first window is not fired_k, take the exact path."""
    kw = dict(assigner="sliding", size=3_000, slide=1_000, agg="sum_i64")
    rng = np.random.default_rng(3)
    n = 60_000
    keys = rng.integers(0, 3000, n).astype(np.int64)
    ts = np.sort(rng.integers(0, 200_000, n)).astype(np.int64)
    ts[::997] += 1_000_000  # far-future stragglers
    vals = rng.integers(0, 1000, n).astype(np.int64)
    cuts = np.linspace(0, n, 21).astype(np.int64)
    batches, last = [], -(1 << 62)
    for i in range(20):
        lo, hi = int(cuts[i]), int(cuts[i + 1])
        # every fifth watermark jumps to the middle of its batch (a multi-window fire); the
        # others trail the batch; monotone
        wm = int(np.sort(ts[lo:hi])[(hi - lo) // 2]) if i % 5 == 0 else int(ts[lo:hi].min()) - 1
        last = max(last, wm)
        batches.append((lo, hi, last))
    for flags in (N.FLAG_FORCE_REGION, N.FLAG_NO_REGION):
        _run(oracle_lib, kw, (keys, ts, vals, batches), flags=flags, capacity_hint=4096)

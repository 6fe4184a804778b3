"""The headline number's own configuration, checked against the oracle at every watermark.

bench.py's default run (Nexmark Q5 shape: sliding 10 s / 2 s, sum_i64, 10M keys, 100M events
per 2-s pane, 10M-event watermark batches 200 ms of event time apart, the default region path
with narrow records buffered between fires) is replayed here with bench.py's own stream
generator, operator construction and step code (bench.make_stream / make_operator / Steps),
warmup 0 and 12 steps:

* batch 0's watermark fires the windows ending at t0 (the first records jitter below t0);
* batches 1..10 stay buffered and go through ONE 10-batch flush (100M records, the bench's
  steady-state cadence) right before the fire of batch 10's watermark (10M rows);
* batch 11, the closing gw_flush the bench runs before its clock stops, then MAX_WATERMARK.

Every watermark's fired rows are drained and compared with the oracle's
(wo_run_parallel_rows over the same columns and watermarks): row count and the
order-independent row checksum of oracle.rows_hash_sum, bit-exact, then row by row (every
(key, start, end, result) of every watermark, sorted on both sides).  The bench's --checksum reports the same checksum summed over the watermarks.

Reference: WindowOperator.processElement / onEventTime (RS/runtime/operators/windowing/
WindowOperator.java:293-494); parity rule SURVEY.md §8c.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

THREADS = min(16, os.cpu_count() or 1)  # the GPU box's CPU share


@pytest.mark.timeout(900)
def test_headline_bench_cadence_every_watermark(oracle_lib):
    import torch

    import bench
    from flink_amd import _native as N
    from flink_amd import windowing as W

    steps = 12
    args = bench.parse(["--steps", str(steps), "--warmup", "0", "--checksum"])
    E = args.events_per_pane
    nb = E * args.wm_interval_ms // args.slide_ms
    assert nb == 10_000_000 and args.keys == 10_000_000 and args.agg == "sum_i64"
    keys, ts, vals, wms = bench.make_stream(nb, steps, args.keys, E, args.slide_ms, args.disorder_ms, args.agg,
                                            torch.device("cuda", 0))
    op = bench.make_operator(W, N, args, args.keys, nb=nb)
    try:
        op.enable_kernel_timing(True)
        run = bench.Steps(op, N, keys, ts, vals, wms, nb, collect=True, keep_rows=True)
        for b in range(steps):
            run.step(b)
        op.flush()
        op.advance_watermark(W.LONG_MAX)
        run.consume()
        st = op.stats()
        fast = op.kernel_time_ms(3)[1]
    finally:
        op.close()
    assert st["region_format"] == 2, st  # narrow region records: the headline's path
    assert st["applies"] == 3, st  # batch 0, ONE flush of batches 1..10, batch 11
    assert fast >= 1  # batch 10's fire was enqueued right behind its flush (gw_runtime.cpp fast_fire)
    assert st["late_dropped"] == 0
    per_wm = run.per_wm
    assert len(per_wm) == steps + 1
    assert per_wm[10][0] > 0.99 * args.keys  # batch 10's watermark fires ~every key's window

    keys_np, ts_np, vals_np = keys.cpu().numpy(), ts.cpu().numpy(), vals.cpu().numpy()
    del keys, ts, vals
    cfg = oracle_lib.make_config(assigner="sliding", size=args.size_ms, slide=args.slide_ms, agg=args.agg,
                                 max_parallelism=128)
    # the oracle's rows of every watermark (run_parallel_rows; its per-watermark count and
    # order-independent checksum as rows_hash_sum computes them)
    ok, os_, oe, orr, ow, _ = oracle_lib.run_parallel_rows(cfg, THREADS, np.full(steps, nb, np.int64),
                                                           np.array(wms, np.int64), keys_np, ts_np, vals_np,
                                                           int(sum(r for r, _ in per_wm)) + (1 << 20))
    del keys_np, ts_np, vals_np
    ora = []
    for i in range(steps + 1):
        sel = ow == i
        ora.append((int(sel.sum()), bench.rows_checksum((ok[sel], os_[sel], oe[sel], orr[sel]))))
    bad = [(i, per_wm[i], ora[i]) for i in range(len(ora)) if per_wm[i] != ora[i]]
    assert not bad, f"(rows, checksum) differ from the oracle at watermarks {bad[:5]}"
    # bench.py --checksum's figure is the sum of these per-watermark checksums
    assert bench.wrap64(sum(c for _, c in per_wm)) == bench.wrap64(sum(c for _, c in ora))
    # and row by row
    for i, (gk, gs, ge, gr) in enumerate(run.rows):
        sel = ow == i
        o = np.stack([ok[sel], os_[sel], oe[sel], orr[sel]], axis=1)
        g = np.stack([gk, gs, ge, gr.view(np.int64)], axis=1)
        o = o[np.lexsort(o.T[::-1])]
        g = g[np.lexsort(g.T[::-1])]
        assert np.array_equal(g, o), f"watermark {i}: rows differ from the oracle's"


@pytest.mark.timeout(600)
def test_q5_small_batch_cadence_every_watermark(oracle_lib):
    """SURVEY §8(d)'s other sweep point: E = 10M events per 2-s pane, so 1M-record watermark
    batches (bench.py --events-per-pane 10000000), the same sliding 10 s / 2 s sum over 10M
    keys: 25 batches from a cold handle, i.e. two fires of ~10M windows each behind region
    flushes of 1M-record segments, the deferred list grown on the way (the handle starts with
    none) -- every watermark's rows (count and checksum) equal the oracle's."""
    import torch

    import bench
    from flink_amd import _native as N
    from flink_amd import windowing as W

    steps = 25
    args = bench.parse(["--steps", str(steps), "--warmup", "0", "--checksum", "--events-per-pane", "10000000"])
    E = args.events_per_pane
    nb = E * args.wm_interval_ms // args.slide_ms
    assert nb == 1_000_000 and args.keys == 10_000_000
    keys, ts, vals, wms = bench.make_stream(nb, steps, args.keys, E, args.slide_ms, args.disorder_ms, args.agg,
                                            torch.device("cuda", 0))
    op = bench.make_operator(W, N, args, args.keys, nb=nb)
    try:
        run = bench.Steps(op, N, keys, ts, vals, wms, nb, collect=True)
        for b in range(steps):
            run.step(b)
        op.flush()
        op.advance_watermark(W.LONG_MAX)
        run.consume()
        st = op.stats()
    finally:
        op.close()
    assert st["region_format"] == 2, st  # the region path with narrow records, as the bench runs it
    assert st["late_dropped"] == 0
    per_wm = run.per_wm
    assert len(per_wm) == steps + 1
    assert sum(1 for r, _ in per_wm if r > 0.5 * nb) >= 2  # at least two full fires

    keys_np, ts_np, vals_np = keys.cpu().numpy(), ts.cpu().numpy(), vals.cpu().numpy()
    del keys, ts, vals
    cfg = oracle_lib.make_config(assigner="sliding", size=args.size_ms, slide=args.slide_ms, agg=args.agg,
                                 max_parallelism=128)
    rows, cs, _ = oracle_lib.run_parallel_wm(cfg, THREADS, np.full(steps, nb, np.int64), np.array(wms, np.int64),
                                             keys_np, ts_np, vals_np)
    ora = [(int(r), int(c)) for r, c in zip(rows, cs)]
    bad = [(i, per_wm[i], ora[i]) for i in range(len(ora)) if per_wm[i] != ora[i]]
    assert not bad, f"(rows, checksum) differ from the oracle at watermarks {bad[:5]}"

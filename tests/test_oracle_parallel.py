"""The oracle's multi-threaded runner (the full-size parity check and the CPU baseline)
against the single operator: the per-watermark row counts and checksums of
run_parallel_wm equal those of one OracleOperator fed the same stream, at several
simulated parallelisms (keys are independent: KeyGroupRangeAssignment.java:93-127)."""
import numpy as np
import pytest

from gpu_helpers import random_stream


@pytest.mark.parametrize("kw", [
    dict(assigner="sliding", size=1000, slide=200, agg="sum_i64"),
    dict(assigner="tumbling", size=500, agg="max_i64"),
    dict(assigner="session", gap=150, agg="count"),
])
@pytest.mark.parametrize("threads", [1, 3, 8])
def test_run_parallel_wm_matches_single_operator(oracle_lib, kw, threads):
    o = oracle_lib
    keys, ts, vals, batches = random_stream(7, 30_000, 2_000, 12, agg=kw["agg"])
    op = o.OracleOperator(o.make_config(**kw))
    rows, sums = [], []
    for lo, hi, wm in batches:
        op.process_batch(keys[lo:hi], ts[lo:hi], vals[lo:hi])
        op.process_watermark(wm)
        out = op.drain()
        rows.append(len(out[0]))
        sums.append(o.rows_hash_sum(*out))
    op.process_watermark(o.INT64_MAX)
    out = op.drain()
    rows.append(len(out[0]))
    sums.append(o.rows_hash_sum(*out))
    blen = np.array([hi - lo for lo, hi, _ in batches], np.int64)
    wms = np.array([wm for _, _, wm in batches], np.int64)
    prow, pcs, _ = o.run_parallel_wm(o.make_config(**kw), threads, blen, wms, keys, ts, vals)
    assert list(prow) == rows
    assert [int(x) for x in pcs] == sums
    assert sum(rows) > 0

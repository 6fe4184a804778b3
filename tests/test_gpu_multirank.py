"""World-size-2 runs of the product path on the GPU: every rank runs
libgpuwin (its operator subtask owns computeKeyGroupRangeForOperatorIndex(128, 2, rank))
and partitions its share of the stream on the device (gw_partition_device); the exchange
is staged through gloo.  The union of the ranks' fired rows equals the single-operator
oracle's (results independent of parallelism), every record reaches its key group's
owner, and each rank emits only keys of its own key groups."""
import multiprocessing as mp
import random

import numpy as np
import pytest

from flink_amd import _native as N
from tests.dist_worker import owners

pytestmark = pytest.mark.gpu

CASES = [
    (dict(assigner="sliding", size=1000, slide=250, agg="sum_i64"), 0),
    (dict(assigner="tumbling", size=700, slide=700, agg="max_i64"), N.FLAG_FORCE_REGION),
    (dict(assigner="sliding", size=1200, slide=400, agg="avg_f64", lateness=600), 0),
    (dict(assigner="session", gap=100, agg="count"), 0),
]


@pytest.mark.parametrize("cfg,flags", CASES, ids=["sliding_sum", "tumbling_max_region", "sliding_avg_lateness",
                                                  "session_count"])
def test_two_ranks_on_the_gpu_equal_single_operator(oracle_lib, cfg, flags):
    from tests.dist_worker_gpu import worker
    from tests.gpu_helpers import random_stream
    world = 2
    stream_kw = dict(seed=23, n=40000, num_keys=3000, n_batches=10, disorder=400, wm_lag=300)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = random.randint(20000, 40000)
    procs = [ctx.Process(target=worker, args=(r, world, port, cfg, stream_kw, flags, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        gathered = q.get(timeout=150)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert all(bad == 0 for _, bad, _ in gathered)
    o = oracle_lib
    keys, ts, vals, batches = random_stream(**stream_kw, agg=cfg["agg"])
    op = o.OracleOperator(o.make_config(**cfg))
    vb = vals.view(np.int64) if vals.dtype == np.float64 else vals
    single = []
    for lo, hi, wm in batches:
        op.process_batch(keys[lo:hi], ts[lo:hi], vb[lo:hi])
        op.process_watermark(wm)
        single.append(op.drain())
    op.process_watermark((1 << 63) - 1)
    single.append(op.drain())
    ref = sorted(row for r in single for row in zip(*[x.tolist() for x in r]))
    union = sorted(row for rows, _, _ in gathered for row in rows)
    assert sum(late for _, _, late in gathered) == op.late_dropped
    assert len(union) == len(ref) > 0
    if cfg["agg"] in N.DOUBLE_RESULT:
        assert [r[:3] for r in union] == [r[:3] for r in ref]
        a = np.array([r[3] for r in union], np.int64).view(np.float64)
        b = np.array([r[3] for r in ref], np.int64).view(np.float64)
        assert np.allclose(a, b, rtol=1e-6, atol=0)
    else:
        assert union == ref
    for rank, (rows, _, _) in enumerate(gathered):
        if rows:
            ks = np.array([r[0] for r in rows], np.int64)
            assert (owners(ks, 128, world) == rank).all()


PACKED_CASES = [
    (dict(assigner="sliding", size=1000, slide=250, agg="sum_i64"), 0),
    (dict(assigner="tumbling", size=700, slide=700, agg="max_i64", lateness=300), N.FLAG_FORCE_REGION),
]


@pytest.mark.parametrize("cfg,flags", PACKED_CASES, ids=["sliding_sum", "tumbling_max_region_lateness"])
def test_two_ranks_packed_exchange_equal_single_operator(oracle_lib, cfg, flags):
    """The packed protocol (device partition with packing, words + other records over gloo,
    unpack on the receiver) at world size 2: same rows as one operator, most records packed."""
    from tests.dist_worker_gpu import worker_packed
    from tests.gpu_helpers import random_stream
    world = 2
    stream_kw = dict(seed=29, n=40000, num_keys=3000, n_batches=10, ts_step=1, disorder=400, wm_lag=300)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = random.randint(20000, 40000)
    procs = [ctx.Process(target=worker_packed, args=(r, world, port, cfg, stream_kw, flags, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        gathered = q.get(timeout=150)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert all(g[1] == 0 for g in gathered)
    assert sum(g[4] for g in gathered) == 40000 and sum(g[3] for g in gathered) > 0.7 * 40000
    o = oracle_lib
    keys, ts, vals, batches = random_stream(**stream_kw, agg=cfg["agg"])
    op = o.OracleOperator(o.make_config(**cfg))
    single = []
    for lo, hi, wm in batches:
        op.process_batch(keys[lo:hi], ts[lo:hi], vals[lo:hi])
        op.process_watermark(wm)
        single.append(op.drain())
    op.process_watermark((1 << 63) - 1)
    single.append(op.drain())
    ref = sorted(row for r in single for row in zip(*[x.tolist() for x in r]))
    union = sorted(row for g in gathered for row in g[0])
    assert sum(g[2] for g in gathered) == op.late_dropped
    assert len(union) == len(ref) > 0
    assert union == ref

"""World-size-2/3/4 CPU tests (gloo) of the N>1 path: keyBy exchange by key group
(KeyByExchange.exchange_partitioned + combine_watermark), one operator per rank owning
its key groups; the union of the ranks' fired rows must equal a single operator's
(results independent of parallelism)."""
import multiprocessing as mp
import random

import numpy as np
import pytest

from tests.dist_worker import murmur_np, long_hash_np, owners, worker
from tests.gpu_helpers import random_stream


def test_numpy_routing_matches_library(oracle_lib):
    O = oracle_lib.lib()
    rng = np.random.default_rng(4)
    keys = rng.integers(-(1 << 63), (1 << 63) - 1, 3000, dtype=np.int64)
    lh = long_hash_np(keys)
    for i in range(0, 3000, 7):
        assert int(lh[i]) == O.wo_long_hash(int(keys[i]))
        assert int(murmur_np(lh[i:i + 1])[0]) == O.wo_murmur_hash(int(lh[i]))
    own = owners(keys, 128, 4)
    for i in range(0, 3000, 11):
        kg = O.wo_assign_to_key_group(O.wo_long_hash(int(keys[i])), 128)
        assert own[i] == O.wo_operator_index_for_key_group(128, 4, kg)


@pytest.mark.parametrize("world", [2, 3, 4])  # 3: uneven key-group ranges (128 / 3)
@pytest.mark.parametrize("cfg", [dict(assigner="sliding", size=1000, slide=250, agg="sum_i64"),
                                 dict(assigner="session", gap=100, agg="count")],
                         ids=["sliding", "session"])
def test_sharded_job_equals_single_operator(oracle_lib, world, cfg):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = random.randint(20000, 40000)
    procs = [ctx.Process(target=worker, args=(r, world, port, cfg, 17, q)) for r in range(world)]
    for p in procs:
        p.start()
    gathered = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    union = sorted(row for rows, _, _ in gathered for row in rows)
    assert all(bad == 0 for _, bad, _ in gathered)  # every record reached its key group's owner
    assert sum(late for _, _, late in gathered) == 0
    # single operator over the same stream
    o = oracle_lib
    keys, ts, vals, batches = random_stream(seed=17, n=24000, num_keys=500, n_batches=12, agg=cfg["agg"])
    op = o.OracleOperator(o.make_config(**cfg))
    single = []
    for lo, hi, wm in batches:
        op.process_batch(keys[lo:hi], ts[lo:hi], vals[lo:hi])
        op.process_watermark(wm)
        single.append(op.drain())
    op.process_watermark((1 << 63) - 1)
    single.append(op.drain())
    ref = sorted(row for r in single for row in zip(*[x.tolist() for x in r]))
    assert len(union) == len(ref) > 0
    assert union == ref
    # each rank emitted only keys of its own key groups
    for rank, (rows, _, _) in enumerate(gathered):
        if rows:
            ks = np.array([r[0] for r in rows], np.int64)
            assert (owners(ks, 128, world) == rank).all()

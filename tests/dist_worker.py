"""Worker of tests/test_multirank.py (gloo, CPU): a world_size-N keyed window job where
each rank is one parallel source + one window-operator subtask, with the keyBy exchange
done by flink_amd.exchange.KeyByExchange over torch.distributed."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def murmur_np(code):
    """MathUtils.murmurHash vectorised (uint32 arithmetic) — test-side routing oracle."""
    c = code.astype(np.uint32)
    c = (c * np.uint32(0xcc9e2d51)).astype(np.uint32)
    c = ((c << np.uint32(15)) | (c >> np.uint32(17))).astype(np.uint32)
    c = (c * np.uint32(0x1b873593)).astype(np.uint32)
    c = ((c << np.uint32(13)) | (c >> np.uint32(19))).astype(np.uint32)
    c = (c * np.uint32(5) + np.uint32(0xe6546b64)).astype(np.uint32)
    c ^= np.uint32(4)
    c ^= c >> np.uint32(16)
    c = (c * np.uint32(0x85ebca6b)).astype(np.uint32)
    c ^= c >> np.uint32(13)
    c = (c * np.uint32(0xc2b2ae35)).astype(np.uint32)
    c ^= c >> np.uint32(16)
    r = c.view(np.int32).astype(np.int64)
    r = np.where(r >= 0, r, np.where(r == -(1 << 31), 0, -r))
    return r


def long_hash_np(k):
    u = k.view(np.uint64)
    return (u ^ (u >> np.uint64(32))).astype(np.uint32).view(np.int32)


def owners(keys, maxp, p):
    kg = murmur_np(long_hash_np(keys)) % maxp
    return (kg * p) // maxp


def plan_exchange(world, rank, cols, counts, wm):
    """One batch through gw_exchange_plan: the (count, watermark, column mask, 0 packed) message per peer
    goes through one all-to-all, the plan gives every send / receive offset, the columns move
    by point-to-point sends and receives."""
    from flink_amd import _native as N
    msg = torch.zeros(world, N.MSG_WORDS, dtype=torch.int64)
    msg[:, 0] = counts
    msg[:, 1] = wm
    msg[:, 2] = 1
    rmsg = torch.empty_like(msg)
    dist.all_to_all_single(rmsg.view(-1), msg.view(-1))
    (so, sc, ro, rc), total, wmin = N.exchange_plan(msg.view(-1).numpy(), rmsg.view(-1).numpy(), 1, wm)
    out = []
    for c in cols:
        r = torch.empty(total, dtype=c.dtype)
        reqs = []
        for q in range(world):
            if q == rank:
                r[ro[q]:ro[q] + rc[q]] = c[so[q]:so[q] + sc[q]]
                continue
            if sc[q]:
                reqs.append(dist.isend(c[so[q]:so[q] + sc[q]].contiguous(), q))
            if rc[q]:
                reqs.append(dist.irecv(r[ro[q]:ro[q] + rc[q]], q))
        for x in reqs:
            x.wait()
        out.append(r.numpy())
    return out[0], out[1], out[2], wmin


def worker(rank, world, port, cfg_kw, seed, result_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from flink_amd.exchange import KeyByExchange
    from oracle import oracle as O
    from tests.gpu_helpers import random_stream

    keys, ts, vals, batches = random_stream(seed=seed, n=24000, num_keys=500, n_batches=12, agg=cfg_kw["agg"])
    ex = KeyByExchange(world, rank, max_parallelism=128)
    op = O.OracleOperator(O.make_config(**cfg_kw, parallelism=world, operator_index=rank))
    rows = []
    bad_owner = 0
    vbits = vals.view(np.int64) if vals.dtype == np.float64 else vals
    for lo, hi, wm in batches:
        # this rank's source share of the batch (round-robin parallel source)
        idx = np.arange(lo, hi)
        idx = idx[idx % world == rank]
        k, t, v = keys[idx], ts[idx], vbits[idx]
        own = owners(k, 128, world)
        order = np.argsort(own, kind="stable")
        counts = torch.from_numpy(np.bincount(own, minlength=world).astype(np.int64))
        cols = [torch.from_numpy(k[order]), torch.from_numpy(t[order]), torch.from_numpy(v[order])]
        (rk, rt, rv), _ = ex.exchange_partitioned(cols, counts)
        # the native exchange's per-peer plan (gw_exchange_plan), driven over gloo point-to-point
        # sends / receives as gw_exchange_batch drives ncclSend / ncclRecv: same layout
        pk, pt, pv, wmin = plan_exchange(world, rank, cols, counts, wm)
        assert np.array_equal(pk, rk.numpy()) and np.array_equal(pt, rt.numpy()) and np.array_equal(pv, rv.numpy())
        rk, rt, rv = rk.numpy(), rt.numpy(), rv.numpy()
        assert wmin == ex.combine_watermark(wm)
        bad_owner += int((owners(rk, 128, world) != rank).sum())
        op.process_batch(rk, rt, rv)
        op.process_watermark(ex.combine_watermark(wm))
        rows.append(op.drain())
    op.process_watermark(ex.combine_watermark((1 << 63) - 1))
    rows.append(op.drain())
    k = np.concatenate([r[0] for r in rows]); s = np.concatenate([r[1] for r in rows])
    e = np.concatenate([r[2] for r in rows]); r = np.concatenate([r[3] for r in rows])
    mine = list(zip(k.tolist(), s.tolist(), e.tolist(), r.tolist()))
    gathered = [None] * world
    dist.all_gather_object(gathered, (mine, bad_owner, op.late_dropped))
    if rank == 0:
        result_q.put(gathered)
    dist.destroy_process_group()


def worker_packed(rank, world, port, cfg_kw, seed, result_q):
    """The same job through the packed protocol (KeyByExchange.exchange_packed on the host:
    gw_pack_records, gw_exchange_plan / gw_exchange_plan_packed, point-to-point transfers,
    gw_unpack_records); the base pane of a batch is the watermark the ranks combined after the
    previous one."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from flink_amd import _native as N
    from flink_amd.exchange import KeyByExchange
    from oracle import oracle as O
    from tests.gpu_helpers import random_stream

    keys, ts, vals, batches = random_stream(seed=seed, n=24000, num_keys=500, n_batches=12, ts_step=1,
                                            agg=cfg_kw["agg"])
    ex = KeyByExchange(world, rank, max_parallelism=128)
    op = O.OracleOperator(O.make_config(**cfg_kw, parallelism=world, operator_index=rank))
    size, slide = cfg_kw["size"], cfg_kw.get("slide", cfg_kw["size"])
    rows, bad_owner, packed, sent = [], 0, 0, 0
    last = -(1 << 63)
    for lo, hi, wm in batches:
        idx = np.arange(lo, hi)
        idx = idx[idx % world == rank]
        g = N.pack_geom(size, slide, cfg_kw.get("offset", 0), last)
        rk, rt, rv, tp, wmin = ex.exchange_packed(torch.from_numpy(keys[idx]), torch.from_numpy(ts[idx]),
                                                  torch.from_numpy(vals[idx]), g, wm)
        assert wmin == ex.combine_watermark(wm)
        last = wmin
        packed += tp
        sent += rk.size
        bad_owner += int((owners(rk, 128, world) != rank).sum())
        op.process_batch(rk, rt, rv)
        op.process_watermark(wmin)
        rows.append(op.drain())
    op.process_watermark(ex.combine_watermark((1 << 63) - 1))
    rows.append(op.drain())
    k = np.concatenate([r[0] for r in rows]); s = np.concatenate([r[1] for r in rows])
    e = np.concatenate([r[2] for r in rows]); r = np.concatenate([r[3] for r in rows])
    mine = list(zip(k.tolist(), s.tolist(), e.tolist(), r.tolist()))
    gathered = [None] * world
    dist.all_gather_object(gathered, (mine, bad_owner, op.late_dropped, packed, sent))
    if rank == 0:
        result_q.put(gathered)
    dist.destroy_process_group()

"""Worker of tests/test_gpu_multirank.py: one rank of a world_size-N keyed window job on
the GPU -- libgpuwin's operator subtask (parallelism N, operator_index = rank), the keyBy
partition on the device (gw_partition_device via KeyByExchange.partition), the exchange
staged through gloo (every rank shares the box's one GPU, where RCCL refuses two ranks
per device), the watermark combined as the minimum over ranks."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def worker(rank, world, port, cfg_kw, stream_kw, flags, result_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from flink_amd import windowing as W
    from flink_amd.exchange import KeyByExchange
    from tests.dist_worker import owners
    from tests.gpu_helpers import make_assigner, random_stream

    keys, ts, vals, batches = random_stream(**stream_kw, agg=cfg_kw["agg"])
    vbits = vals.view(np.int64) if vals.dtype == np.float64 else vals
    dev = torch.device("cuda", 0)
    ex = KeyByExchange(world, rank, max_parallelism=128, device=dev)
    op = W.GpuWindowOperator(make_assigner(cfg_kw), cfg_kw["agg"], cfg_kw.get("lateness", 0),
                             parallelism=world, operator_index=rank, capacity_hint=4096, flags=flags).open()
    rows, bad_owner = [], 0
    s = torch.cuda.current_stream().cuda_stream
    for lo, hi, wm in batches:
        idx = np.arange(lo, hi)
        idx = idx[idx % world == rank]  # this rank's share of the source (round-robin)
        k = torch.from_numpy(keys[idx]).to(dev)
        t = torch.from_numpy(ts[idx]).to(dev)
        v = torch.from_numpy(vbits[idx]).to(dev)
        pk, pt, pv, counts = ex.partition(k, t, v)
        (rk, rt, rv), n = ex.exchange_partitioned([pk, pt, pv], counts)
        torch.cuda.synchronize()
        bad_owner += int((owners(rk.cpu().numpy(), 128, world) != rank).sum())
        if n:
            op.process_batch_device(rk, rt, rv, stream=s)
        op.advance_watermark(ex.combine_watermark(wm))
        kk, ss, ee, rr = op.drain()
        rows += list(zip(kk.tolist(), ss.tolist(), ee.tolist(), rr.view(np.int64).tolist()))
    op.advance_watermark(ex.combine_watermark(W.LONG_MAX))
    kk, ss, ee, rr = op.drain()
    rows += list(zip(kk.tolist(), ss.tolist(), ee.tolist(), rr.view(np.int64).tolist()))
    late = op.num_late_records_dropped
    op.close()
    gathered = [None] * world
    dist.all_gather_object(gathered, (rows, bad_owner, late))
    if rank == 0:
        result_q.put(gathered)
    dist.destroy_process_group()


def worker_packed(rank, world, port, cfg_kw, stream_kw, flags, result_q):
    """The same job with the packed protocol: the device partition packs the records that fit
    (gw_partition_packed_device, KeyByExchange.exchange_packed), gloo carries the words and the
    other records, the receiver unpacks them (gw_unpack_records) and ingests on the GPU."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from flink_amd import _native as N
    from flink_amd import windowing as W
    from flink_amd.exchange import KeyByExchange
    from tests.dist_worker import owners
    from tests.gpu_helpers import make_assigner, random_stream

    keys, ts, vals, batches = random_stream(**stream_kw, agg=cfg_kw["agg"])
    dev = torch.device("cuda", 0)
    ex = KeyByExchange(world, rank, max_parallelism=128, device=dev)
    op = W.GpuWindowOperator(make_assigner(cfg_kw), cfg_kw["agg"], cfg_kw.get("lateness", 0),
                             parallelism=world, operator_index=rank, capacity_hint=4096, flags=flags).open()
    size, slide = cfg_kw["size"], cfg_kw.get("slide", cfg_kw["size"])
    rows, bad_owner, packed, total = [], 0, 0, 0
    last = W.LONG_MIN
    for lo, hi, wm in batches:
        idx = np.arange(lo, hi)
        idx = idx[idx % world == rank]
        k = torch.from_numpy(keys[idx]).to(dev)
        t = torch.from_numpy(ts[idx]).to(dev)
        v = torch.from_numpy(vals[idx]).to(dev)
        g = N.pack_geom(size, slide, cfg_kw.get("offset", 0), last)
        rk, rt, rv, tp, wmin = ex.exchange_packed(k, t, v, g, wm)
        last = wmin
        packed += tp
        total += rk.size
        bad_owner += int((owners(rk, 128, world) != rank).sum())
        if rk.size:
            op.process_batch(rk, rt, rv)
        op.advance_watermark(wmin)
        kk, ss, ee, rr = op.drain()
        rows += list(zip(kk.tolist(), ss.tolist(), ee.tolist(), rr.view(np.int64).tolist()))
    op.advance_watermark(ex.combine_watermark(W.LONG_MAX))
    kk, ss, ee, rr = op.drain()
    rows += list(zip(kk.tolist(), ss.tolist(), ee.tolist(), rr.view(np.int64).tolist()))
    late = op.num_late_records_dropped
    op.close()
    gathered = [None] * world
    dist.all_gather_object(gathered, (rows, bad_owner, late, packed, total))
    if rank == 0:
        result_q.put(gathered)
    dist.destroy_process_group()

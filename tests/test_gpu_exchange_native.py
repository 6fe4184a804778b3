"""libgpuwin's native keyBy exchange (gw_exchange_*, RCCL) on the box's one GPU: a
world-size-1 communicator (RCCL refuses two ranks on one device), so every record comes
back to rank 0 -- the partition, the count all-to-all, the grouped send/receive of every
column, the receive-set rotation and the watermark all-reduce all run; the ranks > 1 data
path is the same code with more peers (the 2-rank product test uses gloo instead,
tests/test_gpu_multirank.py).  The received batch, fed to the operator, fires what the
oracle fires."""
import numpy as np
import pytest
import torch

from flink_amd import _native as N
from flink_amd import windowing as W
from flink_amd.exchange import NativeKeyByExchange
from gpu_helpers import compare, random_stream

pytestmark = pytest.mark.gpu


class _Dev:
    """__cuda_array_interface__ view of a device pointer (the exchange's receive column)."""

    def __init__(self, ptr, n, typestr):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": typestr, "data": (ptr, False), "version": 2}


def dev_view(ptr, n, typestr="<i8"):
    return torch.as_tensor(_Dev(ptr, n, typestr), device="cuda")


def test_exchange_round_trip_and_watermark():
    ex = NativeKeyByExchange(1, 0)
    ex.set_timeout(30_000)  # bounded waits (gw_wait.h; the CPU tests cover expiry and errors)
    rng = np.random.default_rng(1)
    for n in (0, 1, 1000, 300_000, 17):
        if n == 17:
            ex.set_timeout(0)  # no deadline: only errors end a wait
        k = torch.from_numpy(rng.integers(-(1 << 62), 1 << 62, n).astype(np.int64)).cuda()
        t = torch.from_numpy(rng.integers(0, 1 << 40, n).astype(np.int64)).cuda()
        v = torch.from_numpy(rng.integers(-(1 << 40), 1 << 40, n).astype(np.int64)).cuda()
        h = torch.from_numpy(rng.integers(-(1 << 31), (1 << 31) - 1, n).astype(np.int32)).cuda()
        m, pk, pt, pv, ph, wmo, ist = ex.exchange(k, t, v, key_hashes=h, wm=n * 7)
        assert wmo == n * 7 and ist  # one rank: the watermark comes back; a hand-off stream
        sc, rc = ex.counts()
        assert list(sc) == [n] and list(rc) == [n]
        torch.cuda.synchronize()
        assert m == n
        if n:
            # one destination: the stable partition keeps arrival order
            assert torch.equal(dev_view(pk, n), k)
            assert torch.equal(dev_view(pt, n), t)
            assert torch.equal(dev_view(pv, n), v)
            assert torch.equal(dev_view(ph, n, "<i4"), h)
        m2, qk, qt, qv, qh, _, ist2 = ex.exchange(k, t, None)
        assert m2 == n and qv is None and qh is None
        if n:
            assert qk != pk and ist2 != ist  # the next call uses the other receive set
    assert ex.combine_watermark(12345) == 12345
    assert ex.combine_watermark(W.LONG_MIN) == W.LONG_MIN
    ex.close()


def test_exchanged_batches_fire_like_the_oracle(oracle_lib):
    kw = dict(assigner="sliding", size=1000, slide=250, agg="sum_i64")
    keys, ts, vals, batches = random_stream(31, 60000, 2000, 12)
    ex = NativeKeyByExchange(1, 0)
    op = W.GpuWindowOperator(W.SlidingEventTimeWindows.of(1000, 250), "sum_i64", capacity_hint=4096).open()
    ora = oracle_lib.OracleOperator(oracle_lib.make_config(**kw))
    g, o = [], []
    xs = torch.cuda.Stream()  # the exchange's own stream; the ingest orders through the hand-off
    s = xs.cuda_stream
    for lo, hi, wm in batches:
        k = torch.from_numpy(keys[lo:hi]).cuda()
        t = torch.from_numpy(ts[lo:hi]).cuda()
        v = torch.from_numpy(vals[lo:hi]).cuda()
        torch.cuda.synchronize()
        n, pk, pt, pv, _, wmin, ist = ex.exchange(k, t, v, stream=s, wm=wm)
        op.process_batch_device_ptr(n, pk, pt, pv, stream=ist)
        assert wmin == wm
        op.advance_watermark(wmin)
        kk, ss, ee, rr = op.drain()
        g.append((kk, ss, ee, rr.view(np.int64)))
        ora.process_batch(keys[lo:hi], ts[lo:hi], vals[lo:hi])
        ora.process_watermark(wm)
        o.append(ora.drain())
    op.advance_watermark(W.LONG_MAX)
    kk, ss, ee, rr = op.drain()
    g.append((kk, ss, ee, rr.view(np.int64)))
    ora.process_watermark(W.LONG_MAX)
    o.append(ora.drain())
    assert compare(g, o, False) == []
    op.close()
    ora.close()
    ex.close()


def test_begin_finish_one_batch_ahead(oracle_lib):
    """gw_exchange_begin / gw_exchange_finish pipelined one batch ahead (what bench.py --gpus N
    and the JVM drive): batch b + 1 is partitioned and its counts exchanged before batch b is
    finished; every batch still comes back in order, bit-exact, with packing, and the operator
    fed from it fires what the oracle fires.  Misuse is refused: finishing with nothing begun,
    a third batch begun, gw_exchange_batch with a batch pending."""
    from gpu_helpers import compare, random_stream
    kw = dict(assigner="sliding", size=1000, slide=250, agg="sum_i64")
    keys, ts, vals, batches = random_stream(47, 80_000, 3000, 24, ts_step=1, disorder=300, wm_lag=300)
    ex = NativeKeyByExchange(1, 0)
    ex.enable_packing(1000, 250, 0, with_values=True)
    xs = torch.cuda.Stream()
    with pytest.raises(N.GpuWinError) as e:
        ex.finish(xs.cuda_stream)
    assert e.value.code == N.GW_E_STATE
    op = W.GpuWindowOperator(W.SlidingEventTimeWindows.of(1000, 250), "sum_i64", capacity_hint=4096,
                             flags=N.FLAG_FORCE_REGION).open()
    ora = oracle_lib.OracleOperator(oracle_lib.make_config(**kw))
    cols = [tuple(torch.from_numpy(np.ascontiguousarray(a[lo:hi])).cuda() for a in (keys, ts, vals))
            for lo, hi, _ in batches]
    torch.cuda.synchronize()
    g, o = [], []
    ex.begin(*cols[0], stream=xs.cuda_stream, wm=batches[0][2])
    for b, (lo, hi, wm) in enumerate(batches):
        if b + 1 < len(batches):
            ex.begin(*cols[b + 1], stream=xs.cuda_stream, wm=batches[b + 1][2])
            if b == 3:
                with pytest.raises(N.GpuWinError) as e:  # two pending already
                    ex.begin(*cols[b + 1], stream=xs.cuda_stream, wm=batches[b + 1][2])
                assert e.value.code == N.GW_E_STATE
                with pytest.raises(N.GpuWinError) as e:
                    ex.exchange(*cols[b], stream=xs.cuda_stream, wm=wm)
                assert e.value.code == N.GW_E_STATE
        n, pk, pt, pv, _, wmin, ist = ex.finish(xs.cuda_stream)
        assert wmin == wm and n == hi - lo  # one rank: everything comes back
        op.process_batch_device_ptr(n, pk, pt, pv, stream=ist)
        op.advance_watermark(wmin)
        kk, ss, ee, rr = op.drain()
        g.append((kk, ss, ee, rr.view(np.int64)))
        ora.process_batch(keys[lo:hi], ts[lo:hi], vals[lo:hi])
        ora.process_watermark(wm)
        o.append(ora.drain())
    op.advance_watermark(W.LONG_MAX)
    kk, ss, ee, rr = op.drain()
    g.append((kk, ss, ee, rr.view(np.int64)))
    ora.process_watermark(W.LONG_MAX)
    o.append(ora.drain())
    assert compare(g, o, False) == []
    op.close()
    ora.close()
    ex.close()

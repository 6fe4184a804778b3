"""Packed exchange records on the GPU (include/gpuwin.h gw_pack_geom):

* gw_partition_packed_device against the host: the words (gw_pack_records), the other
  records' columns and the per-bucket counts equal a stable host partition by (owner, does
  not fit), for 1, 2, 5 and 8 subtasks, with records that do not fit for every reason (key
  beyond 32 bits, value beyond 28 bits, pane outside the 16 after the base, no timestamp);
  gw_unpack_device equals gw_unpack_records;
* the native exchange (gw_exchange_batch, world size 1) with packing: from the second batch
  on most records travel packed (gw_exchange_last_packed), arrive unpacked behind the others,
  and the operator fed with them fires exactly what the oracle fires on the original stream
  (sliding sum, tumbling count with allowed lateness)."""
import numpy as np
import pytest
import torch

from flink_amd import _native as N
from flink_amd import windowing as W
from flink_amd.exchange import NativeKeyByExchange, owners_np
from gpu_helpers import compare, random_stream

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("P", [1, 2, 5, 8])
@pytest.mark.parametrize("with_values", [True, False])
def test_device_partition_matches_host(P, with_values):
    rng = np.random.default_rng(P * 10 + with_values)
    n = 200_003
    g = N.pack_geom(1000, 250, -40, 123_456)
    keys = rng.integers(0, 1 << 20, n).astype(np.int64)
    keys[::97] = rng.integers(1 << 32, 1 << 40, keys[::97].size)
    keys[::101] = -rng.integers(1, 1000, keys[::101].size)
    ts = 123_456 - 600 + rng.integers(0, 4600, n).astype(np.int64)
    ts[::89] = W.LONG_MIN
    vals = rng.integers(-(1 << 26), 1 << 26, n).astype(np.int64)
    vals[::83] = 1 << 30
    v = vals if with_values else None
    w, fits = N.pack_records(keys, ts, v, g)
    own = owners_np(keys, 128, P)
    bucket = 2 * own + (~fits).astype(np.int64)
    order = np.argsort(bucket, kind="stable")
    cnt = np.bincount(bucket, minlength=2 * P)
    dk, dt = torch.from_numpy(keys).cuda(), torch.from_numpy(ts).cuda()
    dv = torch.from_numpy(vals).cuda() if with_values else None
    ow = torch.zeros(n, dtype=torch.int64, device="cuda")
    ok, ot = torch.zeros_like(dk), torch.zeros_like(dt)
    ov = torch.zeros_like(dv) if with_values else None
    counts = torch.zeros(2 * P, dtype=torch.int64, device="cuda")
    scratch = torch.empty(N.lib().gw_partition_scratch_bytes(n, 2 * P), dtype=torch.uint8, device="cuda")
    ptr = lambda t: t.data_ptr() if t is not None else None
    N.check(N.lib().gw_partition_packed_device(n, ptr(dk), ptr(dt), ptr(dv), 128, P, g, ptr(ow), ptr(ok), ptr(ot),
                                               ptr(ov), ptr(counts), ptr(scratch),
                                               torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    assert np.array_equal(counts.cpu().numpy(), cnt)
    pos_fit = fits[order]
    assert np.array_equal(ow.cpu().numpy().view(np.uint64)[pos_fit], w[order][pos_fit])
    assert np.array_equal(ok.cpu().numpy()[~pos_fit], keys[order][~pos_fit])
    assert np.array_equal(ot.cpu().numpy()[~pos_fit], ts[order][~pos_fit])
    if with_values:
        assert np.array_equal(ov.cpu().numpy()[~pos_fit], vals[order][~pos_fit])
    assert 0.5 < fits.mean() < 0.99
    # unpack on the device = on the host
    m = int(fits.sum())
    uk, ut = torch.zeros(m, dtype=torch.int64, device="cuda"), torch.zeros(m, dtype=torch.int64, device="cuda")
    uv = torch.zeros(m, dtype=torch.int64, device="cuda") if with_values else None
    words = torch.from_numpy(w[fits].view(np.int64)).cuda()
    N.check(N.lib().gw_unpack_device(m, ptr(words), g, ptr(uk), ptr(ut), ptr(uv),
                                     torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    hk, ht, hv = N.unpack_records(w[fits], g, with_values)
    assert np.array_equal(uk.cpu().numpy(), hk) and np.array_equal(ut.cpu().numpy(), ht)
    if with_values:
        assert np.array_equal(uv.cpu().numpy(), hv)


@pytest.mark.parametrize("P", [1, 2, 5, 8, 16])
@pytest.mark.parametrize("packed", [True, False])
@pytest.mark.parametrize("n", [200_003, 3_000_017])
def test_region_partition_matches_host(P, packed, n):
    """gw_partition_regions_device (the exchange's single-pass partition): region q holds
    owner q's packed words / other records in arrival order, counts per bucket -- the same
    records as the stable host partition, across ~100 and ~1500 tiles of look-back."""
    rng = np.random.default_rng(P * 100 + packed + n % 7)
    g = N.pack_geom(1000, 250, -40, 123_456) if packed else None
    keys = rng.integers(0, 1 << 20, n).astype(np.int64)
    keys[::97] = rng.integers(1 << 32, 1 << 40, keys[::97].size)
    ts = 123_456 - 600 + rng.integers(0, 4600, n).astype(np.int64)
    vals = rng.integers(-(1 << 26), 1 << 26, n).astype(np.int64)
    vals[::83] = 1 << 30
    own = owners_np(keys, 128, P)
    if packed:
        w, fits = N.pack_records(keys, ts, vals, g)
    else:
        w, fits = np.zeros(n, np.uint64), np.zeros(n, bool)
    cap = n + 17
    dk, dt, dv = (torch.from_numpy(a).cuda() for a in (keys, ts, vals))
    ow = torch.full((P * cap,), -1, dtype=torch.int64, device="cuda")
    ok, ot, ov = (torch.full((P * cap,), -1, dtype=torch.int64, device="cuda") for _ in range(3))
    nb = 2 * P if packed else P
    counts = torch.zeros(nb, dtype=torch.int64, device="cuda")
    scratch = torch.empty(N.lib().gw_partition_scratch_bytes(n, 2 * P), dtype=torch.uint8, device="cuda")
    ptr = lambda t: t.data_ptr() if t is not None else None
    N.check(N.lib().gw_partition_regions_device(n, ptr(dk), ptr(dt), ptr(dv), 128, P, g, cap, ptr(ow), ptr(ok),
                                                ptr(ot), ptr(ov), ptr(counts), ptr(scratch),
                                                torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    c = counts.cpu().numpy()
    hw, hk, ht, hv = (t.cpu().numpy() for t in (ow, ok, ot, ov))
    for q in range(P):
        mine = own == q
        pk_idx = np.nonzero(mine & fits)[0]
        ot_idx = np.nonzero(mine & ~fits)[0]
        if packed:
            assert c[2 * q] == pk_idx.size and c[2 * q + 1] == ot_idx.size
            assert np.array_equal(hw[q * cap:q * cap + pk_idx.size].view(np.uint64), w[pk_idx])
        else:
            assert c[q] == ot_idx.size
        r = slice(q * cap, q * cap + ot_idx.size)
        assert np.array_equal(hk[r], keys[ot_idx]) and np.array_equal(ht[r], ts[ot_idx])
        assert np.array_equal(hv[r], vals[ot_idx])


@pytest.mark.parametrize("kw", [dict(assigner="sliding", size=1000, slide=250, agg="sum_i64"),
                                dict(assigner="tumbling", size=600, agg="count", lateness=300)],
                         ids=["sliding_sum", "tumbling_count_lateness"])
def test_packed_native_exchange_fires_like_the_oracle(oracle_lib, kw):
    keys, ts, vals, batches = random_stream(31, 60000, 2000, 30, ts_step=1, disorder=400, wm_lag=300)
    slide = kw.get("slide", kw["size"])
    ex = NativeKeyByExchange(1, 0)
    ex.enable_packing(kw["size"], slide, 0, with_values=kw["agg"] != "count")
    assigner = (W.SlidingEventTimeWindows.of(kw["size"], slide) if kw["assigner"] == "sliding"
                else W.TumblingEventTimeWindows.of(kw["size"]))
    op = W.GpuWindowOperator(assigner, kw["agg"], kw.get("lateness", 0), capacity_hint=4096).open()
    ora = oracle_lib.OracleOperator(oracle_lib.make_config(**kw))
    g, o, packed, total = [], [], 0, 0
    xs = torch.cuda.Stream()
    s = xs.cuda_stream
    for b, (lo, hi, wm) in enumerate(batches):
        k = torch.from_numpy(keys[lo:hi]).cuda()
        t = torch.from_numpy(ts[lo:hi]).cuda()
        v = torch.from_numpy(vals[lo:hi]).cuda() if kw["agg"] != "count" else None
        torch.cuda.synchronize()
        n, pk, pt, pv, _, wmin, ist = ex.exchange(k, t, v, stream=s, wm=wm)
        assert n == hi - lo and wmin == wm
        if b == 0:
            assert ex.last_packed() == 0  # no watermark before the first batch
        packed += ex.last_packed()
        total += n
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
    assert op.num_late_records_dropped == ora.late_dropped
    assert packed > 0.8 * total
    assert compare(g, o, False) == []
    op.close()
    ora.close()
    ex.close()


def _ingest_both(kw, flags, keys, ts, vals, batches, with_values, oracle_lib, classes=False):
    """Operator A ingests each batch as (column records, packed words) through
    gw_ingest_packed_device; the oracle gets the original records.  The words are the records
    that pack against the watermark before the batch (gw_pack_records on the host)."""
    from gpu_helpers import make_assigner
    slide = kw.get("slide", kw["size"])
    op = W.GpuWindowOperator(make_assigner(kw), kw["agg"], kw.get("lateness", 0), capacity_hint=4096,
                             flags=flags).open()
    ora = oracle_lib.OracleOperator(oracle_lib.make_config(**kw))
    g, o, last, packed = [], [], W.LONG_MIN, 0
    s = torch.cuda.current_stream().cuda_stream
    for lo, hi, wm in batches:
        k, t, v = keys[lo:hi], ts[lo:hi], vals[lo:hi]
        geom = N.pack_geom(kw["size"], slide, kw.get("offset", 0), last)
        if geom is None:
            op.process_batch(k, t, v if with_values else None)
        else:
            w, fits = N.pack_records(k, t, v if with_values else None, geom)
            other = ~fits
            dk = torch.from_numpy(np.ascontiguousarray(k[other])).cuda()
            dt = torch.from_numpy(np.ascontiguousarray(t[other])).cuda()
            dv = torch.from_numpy(np.ascontiguousarray(v[other])).cuda() if with_values else None
            dw = torch.from_numpy(np.ascontiguousarray(w[fits]).view(np.int64)).cuda()
            torch.cuda.synchronize()
            op.process_batch_packed_device_ptr(int(other.sum()), dk.data_ptr() if other.any() else None,
                                               dt.data_ptr() if other.any() else None,
                                               dv.data_ptr() if (dv is not None and other.any()) else None,
                                               int(fits.sum()), dw.data_ptr() if fits.any() else None, geom, stream=s)
            torch.cuda.synchronize()
            packed += int(fits.sum())
        op.advance_watermark(wm)
        last = wm
        kk, ss, ee, rr = op.drain()
        g.append((kk, ss, ee, rr.view(np.int64)))
        ora.process_batch(k, t, v)
        ora.process_watermark(wm)
        o.append(ora.drain())
    op.advance_watermark(W.LONG_MAX)
    kk, ss, ee, rr = op.drain()
    g.append((kk, ss, ee, rr.view(np.int64)))
    ora.process_watermark(W.LONG_MAX)
    o.append(ora.drain())
    late = (op.num_late_records_dropped, ora.late_dropped)
    op.close()
    ora.close()
    return g, o, late, packed


@pytest.mark.parametrize("kw,flags", [
    (dict(assigner="sliding", size=1000, slide=250, agg="sum_i64"), N.FLAG_FORCE_REGION),
    (dict(assigner="sliding", size=1000, slide=250, agg="sum_i64"), N.FLAG_NO_REGION),
    (dict(assigner="tumbling", size=500, agg="count", lateness=300), N.FLAG_FORCE_REGION),
    (dict(assigner="tumbling", size=500, agg="max_i64"), N.FLAG_FORCE_LDS_PREAGG),
    (dict(assigner="sliding", size=1200, slide=400, agg="avg_i64", lateness=400), N.FLAG_FORCE_REGION),
    (dict(assigner="sliding", size=40_000, slide=500, agg="min_i64"), 0),  # window classes: staged unpack
], ids=["region_sum", "direct_sum", "region_count_lateness", "preagg_max", "region_avg_lateness", "classes_min"])
def test_packed_ingest_matches_the_oracle(oracle_lib, kw, flags):
    """gw_ingest_packed_device: the region P1 decodes the words itself; the direct and
    pre-aggregation paths and window-class composites unpack them into staging first."""
    keys, ts, vals, batches = random_stream(43, 120_000, 5000, 24, ts_step=1, disorder=300, wm_lag=300,
                                            agg=kw["agg"])
    with_values = kw["agg"] != "count"
    g, o, late, packed = _ingest_both(kw, flags, keys, ts, vals, batches, with_values, oracle_lib)
    assert late[0] == late[1]
    assert packed > 0.5 * keys.size
    assert compare(g, o, kw["agg"].startswith("avg")) == []


@pytest.mark.parametrize("kw", [dict(assigner="sliding", size=1000, slide=250, agg="sum_i64"),
                                dict(assigner="tumbling", size=600, agg="count")], ids=["sliding_sum", "tumbling_count"])
def test_exchange_words_into_packed_ingest(oracle_lib, kw):
    """The native exchange keeping words packed (gw_exchange_set_unpack(0)) feeding
    gw_ingest_packed_device: what the oracle fires."""
    keys, ts, vals, batches = random_stream(37, 60000, 2000, 30, ts_step=1, disorder=400, wm_lag=300)
    slide = kw.get("slide", kw["size"])
    ex = NativeKeyByExchange(1, 0)
    ex.enable_packing(kw["size"], slide, 0, with_values=kw["agg"] != "count")
    ex.keep_words(True)
    assigner = (W.SlidingEventTimeWindows.of(kw["size"], slide) if kw["assigner"] == "sliding"
                else W.TumblingEventTimeWindows.of(kw["size"]))
    op = W.GpuWindowOperator(assigner, kw["agg"], capacity_hint=4096, flags=N.FLAG_FORCE_REGION).open()
    ora = oracle_lib.OracleOperator(oracle_lib.make_config(**kw))
    g, o, words = [], [], 0
    xs = torch.cuda.Stream()
    for lo, hi, wm in batches:
        k = torch.from_numpy(keys[lo:hi]).cuda()
        t = torch.from_numpy(ts[lo:hi]).cuda()
        v = torch.from_numpy(vals[lo:hi]).cuda() if kw["agg"] != "count" else None
        torch.cuda.synchronize()
        n, pk, pt, pv, _, wmin, ist = ex.exchange(k, t, v, stream=xs.cuda_stream, wm=wm)
        nw, pw, geom = ex.last_words()
        assert n + nw == hi - lo
        words += nw
        op.process_batch_packed_device_ptr(n, pk, pt, pv, nw, pw, geom, stream=ist)
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
    assert words > 0.8 * keys.size
    assert op.num_late_records_dropped == ora.late_dropped
    assert compare(g, o, False) == []
    op.close()
    ora.close()
    ex.close()


@pytest.mark.parametrize("case", ["session", "first_element", "side_output", "float", "pane_mismatch",
                                  "offset_mismatch", "count_window"])
def test_packed_ingest_refuses_handles_needing_the_record(case):
    """A word's timestamp is its pane's start: gw_ingest_packed_device refuses (GW_E_UNSUPPORTED,
    the handle unchanged) any handle whose decisions need the record's own timestamp or value,
    and words whose pane grid does not divide the handle's windows."""
    from gpu_helpers import gpu_operator
    size, slide, flags, agg = 1000, 250, 0, "sum_i64"
    geom = N.pack_geom(1000, 250, 0, 10_000)
    kw = dict(assigner="sliding", size=size, slide=slide, agg=agg)
    if case == "session":
        kw = dict(assigner="session", gap=100, agg=agg)
    elif case == "count_window":
        kw = dict(assigner="count_tumbling", size=5, agg=agg)
    elif case == "first_element":
        flags = N.FLAG_FIRST_ELEMENT
    elif case == "side_output":
        flags = N.FLAG_LATE_SIDE_OUTPUT
    elif case == "float":
        kw["agg"] = "sum_f64"
    elif case == "pane_mismatch":
        geom = N.pack_geom(1000, 400, 0, 10_000)  # pane 200 does not divide slide 250
    elif case == "offset_mismatch":
        geom = N.pack_geom(1000, 250, 10, 10_000)
    op = gpu_operator(kw, flags=flags)
    w, fits = N.pack_records(np.arange(64, dtype=np.int64), np.full(64, 10_100, np.int64),
                             np.ones(64, np.int64), geom)
    assert fits.all()
    dw = torch.from_numpy(w.view(np.int64)).cuda()
    torch.cuda.synchronize()
    with pytest.raises(N.GpuWinError) as e:
        op.process_batch_packed_device_ptr(0, None, None, None, 64, dw.data_ptr(), geom,
                                           stream=torch.cuda.current_stream().cuda_stream)
    assert e.value.code == N.GW_E_UNSUPPORTED
    op.close()

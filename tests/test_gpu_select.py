"""gw_select_lookup_device (gw_select.hip): the filter + projection + static-table join a job
chains ahead of keyBy, fused on the device -- against numpy (stable: the survivors in arrival
order), at tile edges, with an index outside the dictionary, and end to end on a YSB-shaped
stream (view events, ad -> campaign, 10-s tumbling count per campaign) against the oracle.

YSB: streaming-benchmarks AdvertisingTopologyNative (filter event_type == "view", project,
join ad_id -> campaign_id, keyBy campaign, 10-s window count); the window semantics are
WindowOperator's (RS/runtime/operators/windowing/WindowOperator.java:293-494).
"""
import numpy as np
import pytest
import torch

from flink_amd import _native as N
from flink_amd import windowing as W
from tests.gpu_helpers import compare, gpu_operator, run_oracle

pytestmark = pytest.mark.gpu


def _select(sel, want, idx, dictionary, ts):
    dev = torch.device("cuda", 0)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    s, i, d, tt = t(sel), t(idx), t(dictionary), t(ts)
    ko = torch.empty(max(len(sel), 1), dtype=torch.int64, device=dev)
    to = torch.empty_like(ko)
    stream = torch.cuda.current_stream(dev).cuda_stream
    n = W.select_lookup_device(s, want, i, d, tt, ko, to, stream)
    return ko[:n].cpu().numpy(), to[:n].cpu().numpy()


@pytest.mark.parametrize("n", [1, 4095, 4096, 4097, 100_003, 1_000_007])
def test_select_lookup_matches_numpy(n):
    rng = np.random.default_rng(n)
    sel = rng.integers(0, 3, n).astype(np.int64)
    idx = rng.integers(0, 1000, n).astype(np.int64)
    dictionary = rng.integers(-(1 << 62), 1 << 62, 1000).astype(np.int64)
    ts = rng.integers(0, 1 << 40, n).astype(np.int64)
    k, t = _select(sel, 0, idx, dictionary, ts)
    m = sel == 0
    assert np.array_equal(k, dictionary[idx[m]])
    assert np.array_equal(t, ts[m])


def test_select_lookup_none_and_all():
    n = 10_000
    idx = np.arange(n, dtype=np.int64) % 7
    dictionary = np.arange(7, dtype=np.int64) * 11
    ts = np.arange(n, dtype=np.int64)
    k, t = _select(np.ones(n, np.int64), 0, idx, dictionary, ts)
    assert len(k) == 0
    k, t = _select(np.zeros(n, np.int64), 0, idx, dictionary, ts)
    assert np.array_equal(k, dictionary[idx]) and np.array_equal(t, ts)


def test_select_lookup_index_outside_dictionary():
    n = 5000
    idx = np.zeros(n, np.int64)
    idx[1234] = 7  # dictionary of 7 entries: 7 is outside
    with pytest.raises(N.GpuWinError) as e:
        _select(np.zeros(n, np.int64), 0, idx, np.arange(7, dtype=np.int64), np.arange(n, dtype=np.int64))
    assert e.value.code == N.GW_E_RANGE


def test_ysb_shaped_stream_end_to_end(oracle_lib):
    """Raw events -> select_lookup_device -> tumbling 10-s count per campaign (the region /
    pre-aggregation paths of a 100-campaign stream) against the oracle over the numpy-filtered
    stream, watermark by watermark."""
    rng = np.random.default_rng(5)
    n, nb = 600_000, 20
    ad = rng.integers(0, 1000, n).astype(np.int64)
    etype = rng.integers(0, 3, n).astype(np.int64)
    ts = (np.arange(n, dtype=np.int64) * 100 // 1000) - rng.integers(0, 51, n).astype(np.int64)
    campaigns = rng.integers(0, 1 << 62, 100).astype(np.int64)
    ad_campaign = np.repeat(campaigns, 10)
    kw = dict(assigner="tumbling", size=10_000, agg="count")
    cut = np.linspace(0, n, nb + 1).astype(np.int64)
    op = gpu_operator(kw, capacity_hint=1024)
    dev = torch.device("cuda", 0)
    t = lambda a: torch.from_numpy(a).to(dev)
    ad_d, et_d, ts_d, dict_d = t(ad), t(etype), t(ts), t(ad_campaign)
    ko = torch.empty(n, dtype=torch.int64, device=dev)
    to = torch.empty_like(ko)
    stream = torch.cuda.current_stream(dev).cuda_stream
    outs, o_batches, wms = [], [], []
    keys_o, ts_o = [], []
    try:
        for b in range(nb):
            lo, hi = cut[b], cut[b + 1]
            m = W.select_lookup_device(et_d[lo:hi], 0, ad_d[lo:hi], dict_d, ts_d[lo:hi], ko, to, stream)
            op.process_batch_device(ko[:m], to[:m], None, stream=stream)
            wm = int(ts[:hi].max()) - 51
            op.advance_watermark(wm)
            k, s, e, r = op.drain()
            outs.append((k, s, e, r.view(np.int64)))
            sel = etype[lo:hi] == 0
            keys_o.append(ad_campaign[ad[lo:hi][sel]])
            ts_o.append(ts[lo:hi][sel])
            wms.append(wm)
        op.advance_watermark(W.LONG_MAX)
        k, s, e, r = op.drain()
        outs.append((k, s, e, r.view(np.int64)))
    finally:
        op.close()
    kk, tt = np.concatenate(keys_o), np.concatenate(ts_o)
    bounds = np.cumsum([0] + [len(x) for x in keys_o])
    batches = [(int(bounds[b]), int(bounds[b + 1]), wms[b]) for b in range(nb)]
    o, _ = run_oracle(oracle_lib, kw, kk, tt, np.zeros(len(kk), np.int64), batches)
    assert compare(outs, o, False) == []
    assert sum(len(x[0]) for x in outs) > 100

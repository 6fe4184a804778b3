"""Full-size parity at the BASELINE.json configurations, on one MI355X.

Each test drives libgpuwin.so through the C ABI over a stream of the config's real size and
compares the rows of EVERY watermark with the CPU oracle (oracle/flink_oracle.c):

* Nexmark Q5 (sliding 10 s / 2 s over 10M keys, 100M events, a watermark every 200 ms of
  event time), sum and count: the oracle runs the whole stream (wo_run_parallel_wm, one
  operator per simulated subtask) and the rows of each watermark are compared by count and
  by an order-independent checksum; a 1/32 key sample is also compared row by row.
* Q7-style tumbling 10 s max over 10M keys, 100M events: the same full per-watermark count
  and checksum, the 1/32 key sample row by row, and the full-stream invariants below.
* Event-time sessions (gap 10 s) with avg over f64 at 12.5M keys (one GPU's share of
  BASELINE's 100M keys over 8 GPUs), ~110M events: every row of every watermark against the
  oracle's (wo_run_parallel_rows): key, start and end exactly, the average within 1e-6
  relative; plus the 1/64 key sample and the invariants.

Keys are independent in the reference (WindowOperator keeps state per key, late drops depend
only on the watermark), so a key sample run through the oracle on the sampled keys' records
is an exact check of those keys' rows.  The full-stream invariants are size-independent:
every record lands in size/slide windows (count), (key, window) pairs are unique per
watermark, and no record is late (the disorder is below the watermark lag).

Reference: WindowOperator.processElement / onEventTime (RS/runtime/operators/windowing/
WindowOperator.java:293-494), parity rule SURVEY.md §8c.
"""
import os

import numpy as np
import pytest

from flink_amd import windowing as W
from gpu_helpers import compare, gpu_operator

pytestmark = pytest.mark.gpu

C1 = -7046029254386353131   # 0x9E3779B97F4A7C15 as int64
C2 = -4658895280553007687   # 0xBF58476D1CE4E5B9
C3 = -7723592293110705685   # 0x94D049BB133111EB
MASK63 = (1 << 63) - 1
T0 = 1_700_000_000_000
THREADS = min(16, os.cpu_count() or 1)  # the GPU box's CPU share


def splitmix64(idx, seed):
    z = (idx + 1) * C1 + seed
    z = (z ^ ((z >> 30) & ((1 << 34) - 1))) * C2
    z = (z ^ ((z >> 27) & ((1 << 37) - 1))) * C3
    return z ^ ((z >> 31) & ((1 << 33) - 1))


def q_stream(n, num_keys, events_per_pane, slide, disorder, seed, value_mod=1_000_000):
    """Nexmark-shaped bids in HBM (bench.py's generator): uniform keys, timestamps advancing
    so each `slide` of event time holds events_per_pane events, jitter <= disorder."""
    import torch
    idx = torch.arange(n, device="cuda", dtype=torch.int64)
    keys = (splitmix64(idx, seed) & MASK63) % num_keys
    jit = (splitmix64(idx, seed ^ 0x77) & MASK63) % (disorder + 1)
    ts = T0 + (idx * slide) // events_per_pane - jit
    vals = (splitmix64(idx, seed ^ 0x1234) & MASK63) % value_mod
    return keys, ts, vals


def bounded_wms(n, nb, events_per_pane, slide, disorder):
    """BoundedOutOfOrdernessWatermarks (maxTs - bound - 1) after each batch of nb events,
    over the un-jittered maximum (flink-core/.../eventtime/BoundedOutOfOrdernessWatermarks.java:57-69)."""
    return [T0 + (((b + 1) * nb - 1) * slide) // events_per_pane - disorder - 1 for b in range(n // nb)]


def row_hash_sum(rows):
    from oracle.oracle import rows_hash_sum
    return rows_hash_sum(*rows)


def run_gpu_rows(kw, keys, ts, vals, nb, wms, capacity_hint, sample, keep_all=False):
    """Drive the GPU operator over device columns in batches of nb records; per watermark
    (the last entry: MAX_WATERMARK) return (rows, checksum, sampled rows -- or every row with
    keep_all) and check that (key, window) is unique."""
    import torch
    op = gpu_operator(kw, capacity_hint=capacity_hint, max_batch=nb)
    stream = torch.cuda.current_stream().cuda_stream
    counts, sums, samp = [], [], []
    total_result = 0
    try:
        for b, wm in enumerate(wms + [W.LONG_MAX]):
            if b < len(wms):
                lo, hi = b * nb, (b + 1) * nb
                op.process_batch_device(keys[lo:hi], ts[lo:hi], vals[lo:hi] if vals is not None else None,
                                        stream=stream)
            op.advance_watermark(wm)
            k, s, e, r = op.drain()
            r = r.view(np.int64)
            counts.append(len(k))
            sums.append(row_hash_sum((k, s, e, r)))
            if len(k):
                order = np.lexsort((s, k))
                ks, ss = k[order], s[order]
                assert not np.any((ks[1:] == ks[:-1]) & (ss[1:] == ss[:-1])), f"duplicate (key, window) at wm #{b}"
            if kw["agg"] == "count":
                total_result += int(r.sum())
            if keep_all:
                samp.append((k, s, e, r))
            else:
                m = sample(k)
                samp.append((k[m], s[m], e[m], r[m]))
        late = op.num_late_records_dropped
    finally:
        op.close()
    return counts, sums, samp, total_result, late


def oracle_sample(o, kw, keys_np, ts_np, vals_np, nb, wms, mask):
    """The oracle over the sampled keys' records, batch by batch, same watermarks."""
    op = o.OracleOperator(o.make_config(**kw))
    outs = []
    for b, wm in enumerate(wms + [W.LONG_MAX]):
        if b < len(wms):
            lo, hi = b * nb, (b + 1) * nb
            mm = mask[lo:hi]
            op.process_batch(keys_np[lo:hi][mm], ts_np[lo:hi][mm], vals_np[lo:hi][mm] if vals_np is not None else None)
        op.process_watermark(wm)
        outs.append(op.drain())
    late = op.late_dropped
    op.close()
    return outs, late


Q5 = dict(assigner="sliding", size=10_000, slide=2_000)
Q7 = dict(assigner="tumbling", size=10_000, slide=10_000)


@pytest.mark.timeout(600)
# sum_i64 at this size runs in tests/test_gpu_headline.py (the bench's own cadence, every row of
# every watermark against the oracle); count here covers the 4-byte narrow records at 2M-record
# batches (the suite stays under ~600 s of the driver's 900-s step)
@pytest.mark.parametrize("agg,full_oracle", [("count", True)])
def test_q5_10m_keys_100m_events(oracle_lib, agg, full_oracle):
    """Nexmark Q5 at its BASELINE size: 10M keys, 100M events (20M per 2-s pane, 50
    watermark batches, 5 windows fire during the stream, the rest at MAX_WATERMARK)."""
    n, K, E, nb, dis = 100_000_000, 10_000_000, 20_000_000, 2_000_000, 100
    kw = dict(Q5, agg=agg)
    keys, ts, vals = q_stream(n, K, E, Q5["slide"], dis, seed=0x5EED0005)
    vals_dev = vals if agg != "count" else None
    wms = bounded_wms(n, nb, E, Q5["slide"], dis)
    sample = lambda k: (k % 32) == 5
    counts, sums, samp, total, late = run_gpu_rows(kw, keys, ts, vals_dev, nb, wms, K, sample)
    assert late == 0
    assert sum(counts) > 5 * K * 0.9  # every key fires in each of its ~5+ windows
    keys_np, ts_np = keys.cpu().numpy(), ts.cpu().numpy()
    vals_np = vals.cpu().numpy() if agg != "count" else None
    del keys, ts, vals, vals_dev
    if agg == "count":
        assert total == 5 * n  # every record counted in size/slide windows
    # row-by-row on the key sample
    mask = sample(keys_np)
    ora, olate = oracle_sample(oracle_lib, kw, keys_np, ts_np, vals_np, nb, wms, mask)
    assert olate == 0
    errs = compare(samp, ora, False)
    assert not errs, errs[:5]
    if full_oracle:  # every watermark's rows over all 10M keys: count + checksum
        cfg = oracle_lib.make_config(**kw)
        rows, cs, sec = oracle_lib.run_parallel_wm(cfg, THREADS, np.full(len(wms), nb), np.array(wms, np.int64),
                                                   keys_np, ts_np, vals_np)
        assert list(rows) == counts
        bad = [b for b in range(len(counts)) if int(cs[b]) != sums[b]]
        assert not bad, f"checksum differs at watermarks {bad[:10]}"


@pytest.mark.timeout(600)
def test_q7_tumbling_max_10m_keys(oracle_lib):
    """Q7/Q8-style tumbling 10 s max(price) over 10M keys, 100M events (one GPU's work after
    the keyBy exchange)."""
    n, K, E, nb, dis = 100_000_000, 10_000_000, 10_000_000, 1_000_000, 100
    kw = dict(Q7, agg="max_i64")
    keys, ts, vals = q_stream(n, K, E, 1_000, dis, seed=0x5EED0007, value_mod=1 << 40)
    wms = bounded_wms(n, nb, E, 1_000, dis)
    sample = lambda k: (k % 32) == 11
    counts, sums, samp, _, late = run_gpu_rows(kw, keys, ts, vals, nb, wms, K, sample)
    assert late == 0
    keys_np, ts_np, vals_np = keys.cpu().numpy(), ts.cpu().numpy(), vals.cpu().numpy()
    del keys, ts, vals
    # rows = distinct (key, tumbling window) pairs
    win = np.floor_divide(ts_np, 10_000)  # TimeWindow.getWindowStartWithOffset, offset 0
    exp_rows = len(np.unique(keys_np.astype(np.int64) * 1_000_003 + (win - win.min())))
    assert sum(counts) == exp_rows
    mask = sample(keys_np)
    ora, olate = oracle_sample(oracle_lib, kw, keys_np, ts_np, vals_np, nb, wms, mask)
    assert olate == 0
    errs = compare(samp, ora, False)
    assert not errs, errs[:5]
    # every watermark's rows over all 10M keys: count + checksum
    rows, cs, sec = oracle_lib.run_parallel_wm(oracle_lib.make_config(**kw), THREADS, np.full(len(wms), nb),
                                               np.array(wms, np.int64), keys_np, ts_np, vals_np)
    assert list(rows) == counts
    bad = [b for b in range(len(counts)) if int(cs[b]) != sums[b]]
    assert not bad, f"checksum differs at watermarks {bad[:10]}"


def session_stream(num_keys, gap, seed):
    """Per key two bursts of 1-8 events: events of a burst 0-3 s apart (< gap), bursts more
    than gap + 1 s apart; the stream in timestamp order, then jittered by <= 100 ms.
    Values f64 uniform in [0, 1000) (SURVEY.md §8d Config 5)."""
    import torch
    k = torch.arange(num_keys, device="cuda", dtype=torch.int64)
    h = splitmix64(k, seed) & MASK63
    L1 = 1 + h % 8
    L2 = 1 + (h >> 3) % 8
    s1 = T0 + (h >> 6) % 60_000
    keys, ts = [], []
    for j in range(8):  # burst 1: event j of every key with L1 > j
        m = L1 > j
        kk = k[m]
        step = (splitmix64(kk * 16 + j, seed ^ 0x33) & MASK63) % 3_000
        keys.append(kk)
        ts.append(s1[m] + j * 3_000 + step)
    e1 = s1 + (L1 - 1) * 3_000 + 3_000
    s2 = e1 + gap + 1_000 + (h >> 20) % 30_000
    for j in range(8):
        m = L2 > j
        kk = k[m]
        step = (splitmix64(kk * 16 + 8 + j, seed ^ 0x33) & MASK63) % 3_000
        keys.append(kk)
        ts.append(s2[m] + j * 3_000 + step)
    keys = torch.cat(keys)
    ts = torch.cat(ts)
    ts, order = torch.sort(ts)
    keys = keys[order]
    n = keys.numel()
    idx = torch.arange(n, device="cuda", dtype=torch.int64)
    ts = ts - (splitmix64(idx, seed ^ 0x55) & MASK63) % 101
    vals = ((splitmix64(idx, seed ^ 0x99) & MASK63) % 1_000_000_000).to(torch.float64) / 1e6
    return keys, ts, vals.view(torch.int64)


@pytest.mark.timeout(600)
def test_sessions_avg_f64_12m_keys(oracle_lib):
    """Event-time sessions (gap 10 s) with avg over f64, 12.5M keys (one GPU's share of
    BASELINE's 100M keys across 8 GPUs), ~112M events, a watermark every 2M events."""
    import torch
    K, gap, nb = 12_500_000, 10_000, 2_000_000
    keys, ts, vals = session_stream(K, gap, seed=0x5EED000A)
    n = keys.numel() // nb * nb
    keys, ts, vals = keys[:n], ts[:n], vals[:n]
    tsh = ts.view(-1, nb).amax(dim=1)
    run_max = torch.cummax(tsh, dim=0).values.cpu().numpy()
    wms = [int(x) - 200 - 1 for x in run_max]  # lag 200 ms > jitter: no record is late
    kw = dict(assigner="session", gap=gap, agg="avg_f64")
    counts, sums, allrows, _, late = run_gpu_rows(kw, keys, ts, vals, nb, wms, K, None, keep_all=True)
    assert late == 0
    keys_np, ts_np, vals_np = keys.cpu().numpy(), ts.cpu().numpy(), vals.cpu().numpy()
    del keys, ts, vals
    assert sum(counts) >= len(np.unique(keys_np))  # at least one session per key
    # every row of every watermark against the full oracle (f64 averages within 1e-6)
    ok_, os_, oe_, or_, ow_, sec = oracle_lib.run_parallel_rows(
        oracle_lib.make_config(**kw), THREADS, np.full(len(wms), nb), np.array(wms, np.int64), keys_np, ts_np,
        vals_np, n + 1024)
    ora = []
    order = np.argsort(ow_, kind="stable")
    bounds = np.searchsorted(ow_[order], np.arange(len(wms) + 2))
    for b in range(len(wms) + 1):
        sel = order[bounds[b]:bounds[b + 1]]
        ora.append((ok_[sel], os_[sel], oe_[sel], or_[sel]))
    errs = compare(allrows, ora, True)
    assert not errs, errs[:5]

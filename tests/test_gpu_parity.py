"""GPU parity tests: libgpuwin.so (through the flink_amd host mirror) against the CPU
oracle and the reference's golden vectors.  Bit-exact for integer/count/min/max and
avg over longs; 1e-6 relative for f64 sums/averages (BASELINE.json north_star)."""
import zlib

import numpy as np
import pytest

from flink_amd import _native as N
from flink_amd import windowing as W
from tests.gpu_helpers import compare, gpu_operator, random_stream, run_gpu, run_oracle
from tests.harness import config_kwargs, itcase_expected_sum, itcase_stream, load_golden, replay

pytestmark = pytest.mark.gpu

TOL_AGGS = {"sum_f64", "avg_f64"}
ALL_AGGS = ["count", "sum_i64", "sum_i32", "sum_f64", "min_i64", "max_i64", "min_f64", "max_f64",
            "avg_i64", "avg_f64"]


def _cmp(gpu, ora, agg):
    if agg in TOL_AGGS:
        return compare(gpu, ora, True)
    return compare(gpu, ora, False)


# ------------------------------------------------------------------ golden vectors
class GpuBackend:
    def __init__(self, cfg, side_output=False):
        self.kw = config_kwargs(cfg)
        self.flags = N.FLAG_LATE_SIDE_OUTPUT if side_output else 0
        self.op = gpu_operator(self.kw, flags=self.flags)
        self.side = []
        self.k, self.t, self.v = [], [], []

    def process_element(self, k, ts, v):
        self.k.append(k); self.t.append(ts); self.v.append(v)

    def process_watermark(self, wm):
        if self.k:
            self.op.process_batch(np.array(self.k, np.int64), np.array(self.t, np.int64),
                                  np.array(self.v, np.int64))
            self.k, self.t, self.v = [], [], []
        self.op.advance_watermark(wm)

    def drain(self):
        k, s, e, r = self.op.drain()
        return k, s, e, r.view(np.int64)

    def snapshot_restore(self):
        if self.k:
            self.op.process_batch(np.array(self.k, np.int64), np.array(self.t, np.int64),
                                  np.array(self.v, np.int64))
            self.k, self.t, self.v = [], [], []
        blob = self.op.snapshot_state()
        self.late_before = getattr(self, "late_before", 0) + self.op.num_late_records_dropped
        if self.flags:
            self.side.append(self.op.drain_late())
        self.op.close()
        self.op = gpu_operator(self.kw, flags=self.flags)
        self.op.initialize_state(blob)

    def drain_late(self):
        parts = self.side + [self.op.drain_late()]
        return tuple(np.concatenate([p[c] for p in parts]) for c in range(3))

    @property
    def late_dropped(self):
        return getattr(self, "late_before", 0) + self.op.num_late_records_dropped


@pytest.mark.parametrize("test", load_golden("operator_harness.json")["tests"], ids=lambda t: t["name"])
def test_golden_harness_vectors(test):
    assert replay(test, GpuBackend) == []
    if "side" in test:  # the reference test's own setting: late records on the side output
        assert replay(test, GpuBackend, side_output=True) == []


@pytest.mark.parametrize("assigner,size,slide", [("tumbling", 1000, 1000), ("sliding", 1000, 100)])
def test_itcase_closed_form(assigner, size, slide):
    """EventTimeWindowCheckpointingITCase generator/validator (see tests/harness.py)."""
    nk, n = 100, 3000
    keys, ts, vals, blen, wm = itcase_stream(nk, n, size)
    op = gpu_operator(dict(assigner=assigner, size=size, slide=slide, agg="sum_i32"))
    rows = []
    off = 0
    for b in range(0, n, 50):  # 50 generator steps per batch, watermark of the last one
        hi = off + int(blen[b:b + 50].sum())
        op.process_batch(keys[off:hi], ts[off:hi], vals[off:hi])
        off = hi
        op.advance_watermark(int(wm[min(b + 49, n - 1)]))
        rows.append(op.drain())
    op.advance_watermark(W.LONG_MAX)
    rows.append(op.drain())
    assert op.num_late_records_dropped == 0
    op.close()
    k = np.concatenate([r[0] for r in rows]); s = np.concatenate([r[1] for r in rows])
    e = np.concatenate([r[2] for r in rows]); r = np.concatenate([r[3] for r in rows])
    exp = np.array([itcase_expected_sum(int(a), int(b), n) for a, b in zip(s, e)], np.int64)
    assert np.array_equal(r, exp)
    n_windows = (n + size - 1) // slide if assigner == "sliding" else n // size
    assert len(k) == nk * n_windows
    assert len(set(zip(k.tolist(), s.tolist()))) == len(k)  # each (key, window) exactly once


# ------------------------------------------------------------------ random streams
CONFIGS = [
    dict(assigner="tumbling", size=1000, slide=1000),
    dict(assigner="tumbling", size=700, slide=700, offset=-300),
    dict(assigner="sliding", size=1000, slide=250),
    dict(assigner="sliding", size=1000, slide=300, offset=-50),  # size % slide != 0 -> pane 100
    dict(assigner="sliding", size=10000, slide=2000),             # Nexmark Q5 shape
    dict(assigner="session", gap=100),
]


@pytest.mark.parametrize("agg", ALL_AGGS)
@pytest.mark.parametrize("cfg", CONFIGS, ids=lambda c: "-".join(str(v) for v in c.values()))
def test_random_stream_vs_oracle(oracle_lib, cfg, agg):
    kw = dict(cfg, agg=agg)
    keys, ts, vals, batches = random_stream(seed=zlib.crc32(f"{agg}{cfg}".encode()) & 0xffff, n=20000, num_keys=300,
                                            n_batches=25, agg=agg)
    g, glate, _ = run_gpu(kw, keys, ts, vals, batches, flags=N.FLAG_NO_REGION)
    o, olate = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert glate == olate == 0
    assert _cmp(g, o, agg) == []


# Region-bucketed ingest (k_rgn_hist/scatter/apply): forced on every batch, with more
# keys than one region holds so several regions and the LDS probe path are exercised.
@pytest.mark.parametrize("agg", ALL_AGGS)
@pytest.mark.parametrize("cfg", CONFIGS[:-1], ids=lambda c: "-".join(str(v) for v in c.values()))
def test_region_path_vs_oracle(oracle_lib, cfg, agg):
    kw = dict(cfg, agg=agg)
    keys, ts, vals, batches = random_stream(seed=zlib.crc32(f"rgn{agg}{cfg}".encode()) & 0xffff, n=60000,
                                            num_keys=20000, n_batches=12, ts_step=1, agg=agg)
    g, glate, _ = run_gpu(kw, keys, ts, vals, batches, flags=N.FLAG_FORCE_REGION, capacity_hint=20000)
    o, olate = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert glate == olate == 0
    assert _cmp(g, o, agg) == []


@pytest.mark.parametrize("size,slide", [(1000, 50), (3000, 100)])
@pytest.mark.parametrize("flags", [N.FLAG_NO_REGION, N.FLAG_FORCE_REGION], ids=["direct", "region"])
@pytest.mark.parametrize("agg", ["sum_i64", "max_f64"])
def test_long_pane_rings(oracle_lib, size, slide, flags, agg):
    """size/slide = 20 and 30: pane rings of 22 and 38 cells, i.e. 4- and 8-byte
    presence masks per slot (Q5's ring of 6 uses 1 byte)."""
    kw = dict(assigner="sliding", size=size, slide=slide, agg=agg)
    keys, ts, vals, batches = random_stream(seed=size + slide, n=30000, num_keys=2000, n_batches=10, ts_step=1,
                                            agg=agg)
    g, glate, _ = run_gpu(kw, keys, ts, vals, batches, flags=flags, capacity_hint=4000)
    o, olate = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert glate == olate == 0
    assert _cmp(g, o, agg) == []


@pytest.mark.parametrize("agg", ["count", "sum_i64", "min_f64", "avg_f64", "avg_i64"])
@pytest.mark.parametrize("cfg", CONFIGS[:-1], ids=lambda c: "-".join(str(v) for v in c.values()))
def test_region_two_pass_partition_vs_oracle(oracle_lib, cfg, agg):
    """A two-pass table (128 pass-1 buckets of 4 regions of 2048 slots, 6 of 1024 for the
    averages): the records are bucketed in two LDS-sorted passes before k_rgn_apply."""
    kw = dict(cfg, agg=agg)
    keys, ts, vals, batches = random_stream(seed=zlib.crc32(f"rgn2{agg}{cfg}".encode()) & 0xffff, n=80000,
                                            num_keys=50000, n_batches=8, ts_step=1, agg=agg)
    g, glate, stats = run_gpu(kw, keys, ts, vals, batches, flags=N.FLAG_FORCE_REGION, capacity_hint=600000)
    assert stats["table_capacity"] >= 750_000  # two-pass: > 128 regions at load 0.8
    o, olate = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert glate == olate == 0
    assert _cmp(g, o, agg) == []


BUFFER_CFGS = [
    dict(assigner="sliding", size=100_000, slide=50_000),    # ~50 batches per fire
    dict(assigner="tumbling", size=200_000, slide=200_000),  # ~100 batches: the 64-segment cap flushes
    dict(assigner="sliding", size=30_000, slide=20_000),     # pane 10 s: buffers span several panes
]


@pytest.mark.parametrize("agg", ["count", "sum_i64", "max_f64", "avg_f64"])
@pytest.mark.parametrize("cfg", BUFFER_CFGS, ids=lambda c: "-".join(str(v) for v in c.values()))
def test_region_buffered_segments_vs_oracle(oracle_lib, cfg, agg):
    """Two-pass region table (512 regions): pass 1 of every watermark batch is buffered
    as a segment and pass 2 + apply run once before the next fire (or when 64 segments
    wait).  Same fired rows as the oracle at every watermark."""
    kw = dict(cfg, agg=agg)
    keys, ts, vals, batches = random_stream(seed=zlib.crc32(f"buf{agg}{cfg}".encode()) & 0xffff, n=150_000,
                                            num_keys=40_000, n_batches=150, ts_step=1, agg=agg)
    g, glate, stats = run_gpu(kw, keys, ts, vals, batches, flags=N.FLAG_FORCE_REGION, capacity_hint=600_000)
    assert stats["table_capacity"] >= 750_000  # two-pass: > 128 regions at load 0.8
    assert 0 < stats["applies"] < 150  # batches were buffered
    o, olate = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert glate == olate == 0
    assert _cmp(g, o, agg) == []


@pytest.mark.parametrize("agg", ["sum_i64", "avg_f64"])
def test_region_two_pass_spills_and_growth(oracle_lib, agg):
    """Far more keys than a two-pass table holds: full regions leave their records in
    the buffer (spills), which are parked, the table grows, and they are merged back."""
    kw = dict(assigner="tumbling", size=1_000_000, slide=1_000_000, agg=agg)
    keys, ts, vals, batches = random_stream(seed=23, n=1_600_000, num_keys=1_200_000, n_batches=4, ts_step=1,
                                            agg=agg)
    g, glate, stats = run_gpu(kw, keys, ts, vals, batches, flags=N.FLAG_FORCE_REGION, capacity_hint=300_000)
    assert stats["rehashes"] > 0
    o, olate = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert glate == olate == 0
    assert _cmp(g, o, agg) == []


def test_region_buffer_limit_flushes(oracle_lib, monkeypatch):
    """A 5000-record buffer (GW_BUFFER_RECORDS) flushes every few 1000-record batches."""
    monkeypatch.setenv("GW_BUFFER_RECORDS", "5000")
    kw = dict(assigner="sliding", size=100_000, slide=50_000, agg="sum_i64")
    keys, ts, vals, batches = random_stream(seed=31, n=100_000, num_keys=30_000, n_batches=100, ts_step=1)
    g, glate, stats = run_gpu(kw, keys, ts, vals, batches, flags=N.FLAG_FORCE_REGION, capacity_hint=600_000)
    assert stats["applies"] >= 20
    o, olate = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert glate == olate == 0
    assert compare(g, o, False) == []


def test_region_buffer_mixed_paths(oracle_lib):
    """Large batches take the buffered region path, small ones the direct path, which
    applies the waiting segments first."""
    kw = dict(assigner="sliding", size=40_000, slide=20_000, agg="sum_i64")
    sizes = [140_000, 900, 140_000, 140_000, 700, 2_000, 140_000, 500] * 2
    n = sum(sizes)
    keys, ts, vals, _ = random_stream(seed=17, n=n, num_keys=200_000, n_batches=1, ts_step=1)
    ts = np.arange(n, dtype=np.int64) // 40 - np.random.default_rng(3).integers(0, 200, n)
    batches, lo = [], 0
    for s in sizes:
        batches.append((lo, lo + s, int(ts[:lo + s].max()) - 201))
        lo += s
    g, glate, stats = run_gpu(kw, keys, ts, vals, batches, capacity_hint=600_000)
    assert stats["table_capacity"] >= 750_000  # two-pass: > 128 regions at load 0.8
    o, olate = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert glate == olate == 0
    assert compare(g, o, False) == []


@pytest.mark.parametrize("cfg", CONFIGS[:-1], ids=lambda c: "-".join(str(v) for v in c.values()))
@pytest.mark.parametrize("flags", [N.FLAG_FORCE_REGION, N.FLAG_FORCE_REGION | N.FLAG_NO_BUFFER],
                         ids=["buffered", "unbuffered"])
def test_region_two_pass_late_and_far_future(oracle_lib, cfg, flags):
    """Late drops and parked far-future records on a two-pass (buffered) region table."""
    kw = dict(cfg, agg="sum_i64")
    keys, ts, vals, batches = random_stream(seed=12, n=30000, num_keys=3000, n_batches=40,
                                            disorder=max(4000, 3 * cfg["size"]), wm_lag=200, agg="sum_i64")
    rng = np.random.default_rng(4)
    far = rng.choice(len(ts), 300, replace=False)
    ts[far] += rng.integers(50_000, 2_000_000, 300)
    g, glate, _ = run_gpu(kw, keys, ts, vals, batches, flags=flags, capacity_hint=600_000)
    o, olate = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert olate > 0
    assert glate == olate
    assert compare(g, o, False) == []


def test_region_partition_eight_bit_digits(oracle_lib):
    """40M expected keys: more than 8192 regions of 2048 slots, so 256 pass-1 buckets (8 hash
    bits), each of nsub regions (pass 2 scales the next 32 hash bits to nsub)."""
    kw = dict(assigner="sliding", size=1000, slide=250, agg="sum_i64")
    keys, ts, vals, batches = random_stream(seed=77, n=50000, num_keys=30000, n_batches=5, ts_step=1,
                                            agg="sum_i64")
    g, glate, stats = run_gpu(kw, keys, ts, vals, batches, flags=N.FLAG_FORCE_REGION, capacity_hint=40_000_000)
    cap = stats["table_capacity"]
    assert cap >= 40_000_000 / 0.88 and cap % (256 * 2048) == 0 and cap // (256 * 2048) > 64
    o, olate = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert glate == olate == 0
    assert compare(g, o, False) == []


@pytest.mark.parametrize("cfg", CONFIGS, ids=lambda c: "-".join(str(v) for v in c.values()))
@pytest.mark.parametrize("flags", [0, N.FLAG_FORCE_REGION], ids=["auto", "region"])
def test_late_records_dropped_like_reference(oracle_lib, cfg, flags):
    """Disorder larger than the watermark lag: some records are late (isWindowLate /
    isElementLate, WindowOperator.java:609-624) and are dropped and counted; sessions
    with late records take the arrival-order replay path."""
    kw = dict(cfg, agg="sum_i64")
    disorder = max(2500, 3 * cfg.get("size", 0))  # late = beyond the oldest unfired window
    keys, ts, vals, batches = random_stream(seed=11, n=20000, num_keys=50, n_batches=40, disorder=disorder,
                                            wm_lag=200, agg="sum_i64")
    g, glate, _ = run_gpu(kw, keys, ts, vals, batches, flags=flags)
    o, olate = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert olate > 0
    assert glate == olate
    assert _cmp(g, o, "sum_i64") == []


@pytest.mark.parametrize("cfg", CONFIGS[:-1], ids=lambda c: "-".join(str(v) for v in c.values()))
@pytest.mark.parametrize("flags", [0, N.FLAG_FORCE_REGION], ids=["auto", "region"])
def test_far_future_records_and_watermark_jumps(oracle_lib, cfg, flags):
    """Records far ahead of the pane ring are parked and merged when their windows
    come up; big watermark jumps fire many windows at once."""
    kw = dict(cfg, agg="count")
    rng = np.random.default_rng(5)
    n = 6000
    keys = rng.integers(0, 40, n).astype(np.int64)
    ts = rng.integers(0, 2_000_000, n).astype(np.int64)  # unordered over a wide span
    vals = np.zeros(n, np.int64)
    batches = [(0, 2000, -1), (2000, 4000, 100_000), (4000, 6000, 1_500_000)]
    g, glate, _ = run_gpu(kw, keys, ts, vals, batches, flags=flags)
    o, olate = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert glate == olate
    assert compare(g, o, False) == []


def test_sessions_many_in_flight_per_key(oracle_lib):
    """Many in-flight sessions per key: keys beyond the slot's inline sessions move to the wide
    table (K2 = 16 -> 32 -> ...) and results stay exact."""
    kw = dict(assigner="session", gap=100, agg="sum_i64")
    rng = np.random.default_rng(8)
    n = 3000
    keys = rng.integers(0, 200, n).astype(np.int64)   # ~15 events per key per batch
    ts = rng.integers(0, 400_000, n).astype(np.int64)  # far apart: mostly separate sessions
    vals = rng.integers(0, 100, n).astype(np.int64)
    batches = [(0, 1000, -1), (1000, 2000, 50_000), (2000, 3000, 300_000)]
    g, glate, stats = run_gpu(kw, keys, ts, vals, batches)
    o, olate = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert glate == olate
    assert compare(g, o, False) == []


@pytest.mark.parametrize("lateness", [0, 5_000_000])
@pytest.mark.parametrize("agg", ["count", "avg_f64"])
def test_sessions_hundreds_in_flight_for_one_key(oracle_lib, lateness, agg):
    """One key with hundreds of in-flight sessions (no per-key limit): 700 disjoint sessions,
    then merges that bridge some of them, fired in steps; with allowed lateness the fired
    sessions stay in the merging window set within the lateness horizon and late elements
    merge into them (EventTimeTrigger.onElement FIRE)."""
    kw = dict(assigner="session", gap=10, agg=agg, lateness=lateness)
    rng = np.random.default_rng(12)
    ts0 = np.arange(700, dtype=np.int64) * 1000
    ts1 = rng.choice(ts0, 200) + 15          # bridge sessions t and t + 1000? no: extend them
    ts2 = rng.integers(0, 700_000, 300).astype(np.int64)
    ts = np.concatenate([ts0, ts1, ts2])
    keys = np.zeros(len(ts), np.int64)
    keys[::9] = 1
    vals = rng.uniform(0, 100, len(ts)) if agg == "avg_f64" else np.zeros(len(ts), np.int64)
    batches = [(0, 700, -1), (700, 900, 200_000), (900, 1200, 400_000)]
    g, glate, _ = run_gpu(kw, keys, ts, vals, batches)
    o, olate = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert glate == olate
    assert compare(g, o, agg == "avg_f64") == []
    assert sum(len(x[0]) for x in o) > 500


@pytest.mark.parametrize("flags", [N.FLAG_NO_REGION, N.FLAG_FORCE_REGION], ids=["direct", "region"])
def test_table_growth(oracle_lib, flags):
    """Far more keys than the capacity hint: probes / regions fill, records are parked,
    the table re-hashes to a larger one and the parked records are merged back."""
    kw = dict(assigner="sliding", size=1000, slide=500, agg="sum_i64")
    keys, ts, vals, batches = random_stream(seed=2, n=200000, num_keys=150000, n_batches=10, agg="sum_i64")
    g, _, stats = run_gpu(kw, keys, ts, vals, batches, capacity_hint=16, flags=flags)
    o, _ = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert stats["rehashes"] > 0
    assert compare(g, o, False) == []


@pytest.mark.parametrize("agg", ["count", "sum_i64", "sum_f64", "min_f64", "max_i64", "avg_f64"])
@pytest.mark.parametrize("flags", [N.FLAG_FORCE_LDS_PREAGG, 0])
def test_lds_preaggregation_low_cardinality(oracle_lib, agg, flags):
    """YSB-like: 100 keys, large batches -> LDS pre-aggregation kernel (forced or auto)."""
    kw = dict(assigner="tumbling", size=10000, slide=10000, agg=agg)
    keys, ts, vals, batches = random_stream(seed=9, n=400000, num_keys=100, n_batches=8, ts_step=1, agg=agg)
    g, _, stats = run_gpu(kw, keys, ts, vals, batches, flags=flags, capacity_hint=100)
    o, _ = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert stats["preagg_batches"] > 0
    assert _cmp(g, o, agg) == []


@pytest.mark.parametrize("agg", ["count", "sum_i64", "avg_f64", "max_i64"])
def test_lds_preaggregation_overflowing_key_cache(oracle_lib, agg):
    """Forced pre-aggregation with 6000 keys (beyond a workgroup's 1024-entry key cache and
    2048 LDS cells: those records go to the table directly), the sentinel key Long.MIN_VALUE,
    and a table that starts at 16 slots (keys without a slot defer; the table grows)."""
    kw = dict(assigner="sliding", size=4000, slide=2000, agg=agg)
    keys, ts, vals, batches = random_stream(seed=19, n=600_000, num_keys=6000, n_batches=6, ts_step=1, agg=agg)
    keys[::101] = W.LONG_MIN
    g, _, stats = run_gpu(kw, keys, ts, vals, batches, flags=N.FLAG_FORCE_LDS_PREAGG, capacity_hint=16)
    o, _ = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert stats["preagg_batches"] > 0
    assert _cmp(g, o, agg) == []


def test_lds_preaggregation_ysb_20m():
    """YSB-shaped, at full batch size: 20M records of 100 campaigns (random 64-bit ids) in
    10-s tumbling windows, one batch, COUNT; every (campaign, window) count checked exactly
    against numpy (the pre-aggregation path is taken automatically)."""
    import torch
    n = 20_000_000
    rng = np.random.default_rng(23)
    campaigns = rng.integers(-(1 << 62), 1 << 62, 100, dtype=np.int64)
    cidx = rng.integers(0, 100, n)
    keys = campaigns[cidx]
    ts = (np.arange(n, dtype=np.int64) // 400) - rng.integers(0, 51, n)
    op = W.GpuWindowOperator(W.TumblingEventTimeWindows.of(10_000), "count", capacity_hint=1024,
                             max_batch=n).open()
    try:
        dk = torch.from_numpy(keys).cuda()
        dt = torch.from_numpy(ts).cuda()
        N.check(N.lib().gw_ingest_device(op.handle, n, dk.data_ptr(), None, dt.data_ptr(), None, op.stream()),
                op.handle)
        op.advance_watermark(W.LONG_MAX)
        k, s, e, r = op.drain()
        stats = op.stats()
    finally:
        op.close()
    assert stats["preagg_batches"] == 1
    win = ts // 10_000  # floor: TimeWindow.getWindowStartWithOffset for negative ts too
    w0 = int(win.min())
    nw = int(win.max()) - w0 + 1
    cnt = np.bincount(cidx * nw + (win - w0), minlength=100 * nw)
    nz = np.nonzero(cnt)[0]
    exp = sorted(zip(campaigns[nz // nw].tolist(), ((nz % nw + w0) * 10_000).tolist(), cnt[nz].tolist()))
    got = sorted(zip(k.tolist(), s.tolist(), r.view(np.int64).tolist()))
    assert len(got) == len(exp)
    assert got == exp
    assert np.all(e - s == 10_000)


@pytest.mark.parametrize("flags", [N.FLAG_NO_REGION, N.FLAG_FORCE_REGION], ids=["direct", "region"])
def test_special_keys_and_timestamps(oracle_lib, flags):
    """Long.MIN_VALUE (the table's empty marker) and Long.MAX_VALUE as keys, negative
    timestamps, duplicates."""
    kw = dict(assigner="sliding", size=300, slide=100, offset=-30, agg="sum_i64")
    keys = np.array([W.LONG_MIN, W.LONG_MAX, 0, -1, W.LONG_MIN, 7, W.LONG_MIN], np.int64)
    ts = np.array([-1000, -999, -1, 0, -950, 5, 1], np.int64)
    vals = np.array([1, 2, 3, 4, 5, 6, 7], np.int64)
    batches = [(0, 4, -2000), (4, 7, -500)]
    g, _, _ = run_gpu(kw, keys, ts, vals, batches, flags=flags)
    o, _ = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert compare(g, o, False) == []


def test_double_ordering_min_max(oracle_lib):
    """Double.compare order: NaN largest, -0.0 < 0.0 (Comparator.java:33-90)."""
    for agg in ["min_f64", "max_f64"]:
        kw = dict(assigner="tumbling", size=100, slide=100, agg=agg)
        vals = np.array([0.0, -0.0, 1.5, np.nan, -np.inf, np.inf, -0.0, 0.0, np.nan, 2.0], np.float64)
        keys = np.array([1, 1, 2, 2, 3, 3, 4, 4, 5, 5], np.int64)
        ts = np.arange(10, dtype=np.int64)
        batches = [(0, 10, 50)]
        g, _, _ = run_gpu(kw, keys, ts, vals, batches)
        o, _ = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
        # compare bit patterns except NaN payloads
        gk = np.concatenate([x[0] for x in g]); gr = np.concatenate([x[3] for x in g]).view(np.float64)
        ok = np.concatenate([x[0] for x in o]); orr = np.concatenate([x[3] for x in o]).view(np.float64)
        gi, oi = np.argsort(gk), np.argsort(ok)
        for a, b in zip(gr[gi], orr[oi]):
            assert (np.isnan(a) and np.isnan(b)) or np.signbit(a) == np.signbit(b) and a == b


def test_no_timestamp_fails_the_operator():
    op = gpu_operator(dict(assigner="tumbling", size=1000, slide=1000, agg="count"))
    with pytest.raises(N.GpuWinError) as ei:
        op.process_batch(np.array([1], np.int64), np.array([W.LONG_MIN], np.int64), None)
    assert ei.value.code == -6
    op.close()


def test_empty_batches_and_idle_watermarks():
    op = gpu_operator(dict(assigner="sliding", size=1000, slide=500, agg="count"))
    op.process_batch(np.zeros(0, np.int64), np.zeros(0, np.int64), None)
    assert op.advance_watermark(10 ** 9) == 0
    op.process_batch(np.array([5], np.int64), np.array([2 * 10 ** 9], np.int64), None)
    assert op.advance_watermark(10 ** 9 + 5) == 0
    assert op.advance_watermark(W.LONG_MAX) == 2
    k, s, e, r = op.drain()
    assert sorted(zip(s.tolist(), r.tolist())) == [(2 * 10 ** 9 - 500, 1), (2 * 10 ** 9, 1)]
    op.close()


def test_partial_drain():
    op = gpu_operator(dict(assigner="tumbling", size=10, slide=10, agg="count"))
    op.process_batch(np.arange(1000, dtype=np.int64), np.zeros(1000, np.int64), None)
    op.advance_watermark(100)
    import ctypes
    got = ctypes.c_int64()
    buf = np.empty(300, np.int64)
    total = 0
    while True:
        rc = N.lib().gw_drain(op.handle, ctypes.c_void_p(buf.ctypes.data), None, None, None, 300, ctypes.byref(got))
        total += got.value
        if rc == 0:
            break
        assert rc == N.GW_E_OUTPUT_FULL
    assert total == 1000
    op.close()


def test_device_ingest_torch():
    import torch
    op = gpu_operator(dict(assigner="tumbling", size=100, slide=100, agg="sum_i64"))
    k = torch.arange(64, dtype=torch.int64, device="cuda") % 8
    t = torch.arange(64, dtype=torch.int64, device="cuda")
    v = torch.ones(64, dtype=torch.int64, device="cuda")
    op.process_batch_device(k, t, v, stream=torch.cuda.current_stream().cuda_stream)
    op.advance_watermark(1000)
    kk, s, e, r = op.drain()
    assert sorted(kk.tolist()) == list(range(8)) and r.tolist() == [8] * 8
    op.close()


def test_key_groups_and_partition_device(oracle_lib):
    import ctypes
    import torch
    L, O = N.lib(), oracle_lib.lib()
    n = 100000
    rng = np.random.default_rng(1)
    keys = rng.integers(-(1 << 62), 1 << 62, n).astype(np.int64)
    ts = np.arange(n, dtype=np.int64)
    vals = rng.integers(0, 100, n).astype(np.int64)
    dk, dt, dv = (torch.from_numpy(x).cuda() for x in (keys, ts, vals))
    kg = torch.empty(n, dtype=torch.int32, device="cuda")
    ow = torch.empty(n, dtype=torch.int32, device="cuda")
    P = lambda x: ctypes.c_void_p(x.data_ptr())
    assert L.gw_key_groups_device(n, P(dk), None, 128, 8, P(kg), P(ow), None) == 0
    torch.cuda.synchronize()
    exp_kg = np.array([O.wo_assign_to_key_group(O.wo_long_hash(int(x)), 128) for x in keys[:5000]])
    assert np.array_equal(kg.cpu().numpy()[:5000], exp_kg)
    assert np.array_equal(ow.cpu().numpy(), kg.cpu().numpy() * 8 // 128)
    for p in [1, 2, 8]:
        ko, to, vo = torch.empty_like(dk), torch.empty_like(dt), torch.empty_like(dv)
        counts = torch.empty(p, dtype=torch.int64, device="cuda")
        scratch = torch.empty(L.gw_partition_scratch_bytes(n, p), dtype=torch.uint8, device="cuda")
        assert L.gw_partition_device(n, P(dk), None, P(dt), P(dv), 128, p, P(ko), P(to), P(vo), P(counts),
                                     P(scratch), None) == 0
        torch.cuda.synchronize()
        owner = kg.cpu().numpy().astype(np.int64) * p // 128
        order = np.argsort(owner, kind="stable")
        assert np.array_equal(counts.cpu().numpy(), np.bincount(owner, minlength=p))
        assert np.array_equal(ko.cpu().numpy(), keys[order])
        assert np.array_equal(to.cpu().numpy(), ts[order])
        assert np.array_equal(vo.cpu().numpy(), vals[order])


def test_q5_shape_size_independent_properties():
    """Nexmark Q5 shape at scale (sliding 10 s / 2 s count over 2M keys, 20M events):
    size-independent properties instead of the oracle — every record is counted in
    exactly size/slide = 5 windows, every fired (key, window) is unique, and each
    window's count equals the records of that key inside [start, end)."""
    import torch
    n, nk = 20_000_000, 2_000_000
    g = torch.Generator(device="cuda").manual_seed(5)
    keys = torch.randint(0, nk, (n,), device="cuda", dtype=torch.int64, generator=g)
    ts = torch.arange(n, device="cuda", dtype=torch.int64) // 1000  # 1000 events / ms -> 2M per pane
    op = gpu_operator(dict(assigner="sliding", size=10000, slide=2000, agg="count"), capacity_hint=nk)
    step = 1_000_000
    total = 0
    kk = int(keys[123].item())
    spot = []
    for lo in range(0, n, step):
        op.process_batch_device(keys[lo:lo + step], ts[lo:lo + step], None,
                                stream=torch.cuda.current_stream().cuda_stream)
        op.advance_watermark(int(ts[lo + step - 1].item()) - 1)
        k, s, e, r = op.drain()
        total += int(r.sum())
        m = k == kk
        spot.append((s[m], e[m], r[m]))
        assert len(np.unique(k * 4096 + (s // 2000) % 4096)) == len(k)  # (key, window) unique
    op.advance_watermark(W.LONG_MAX)
    k, s, e, r = op.drain()
    total += int(r.sum())
    m = k == kk
    spot.append((s[m], e[m], r[m]))
    assert total == 5 * n
    assert op.num_late_records_dropped == 0
    kts = ts[(keys == kk).nonzero().flatten()].cpu().numpy()
    ss = np.concatenate([x[0] for x in spot]); ee = np.concatenate([x[1] for x in spot])
    cc = np.concatenate([x[2] for x in spot])
    assert int(cc.sum()) == 5 * len(kts)
    for st, en, c in zip(ss, ee, cc):
        assert c == int(((kts >= st) & (kts < en)).sum())
    op.close()

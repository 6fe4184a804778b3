"""Staged host ingest (gw_stage_alloc / gw_stage_columns / gw_ingest_stage): the columns a JVM
operator writes straight into library-owned pinned slots, sent over PCIe on a copy stream into
three device buffers used in turn.  Against the oracle on the same stream: slots refilled many
times (each refill waits for the slot's previous transfer), more batches than slots, key hashes
(String-like keys), COUNT without a value column, and the host path gw_ingest on top of it."""
import numpy as np
import pytest

from flink_amd import _native as N
from flink_amd import windowing as W
from tests.gpu_helpers import compare, gpu_operator, random_stream, run_oracle

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("agg,slots", [("sum_i64", 2), ("count", 3), ("max_f64", 5)])
def test_staged_slots_match_oracle(oracle_lib, agg, slots):
    kw = dict(assigner="sliding", size=2000, slide=500, agg=agg)
    keys, ts, vals, batches = random_stream(seed=61, n=300_000, num_keys=20_000, n_batches=24, agg=agg)
    vb = vals.view(np.int64) if vals.dtype == np.float64 else vals
    cap = max(hi - lo for lo, hi, _ in batches)
    op = gpu_operator(kw, capacity_hint=1 << 16)
    outs = []
    try:
        op.stage_alloc(slots, cap)
        for b, (lo, hi, wm) in enumerate(batches):
            k, _, t, v = op.stage_columns(b % slots)
            k[:hi - lo] = keys[lo:hi]
            t[:hi - lo] = ts[lo:hi]
            if agg != "count":
                v[:hi - lo] = vb[lo:hi]
            op.ingest_stage(b % slots, hi - lo, with_value=agg != "count")
            op.advance_watermark(wm)
            k_, s_, e_, r_ = op.drain()
            outs.append((k_, s_, e_, r_.view(np.int64)))
        op.advance_watermark(W.LONG_MAX)
        k_, s_, e_, r_ = op.drain()
        outs.append((k_, s_, e_, r_.view(np.int64)))
    finally:
        op.close()
    o, _ = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert compare(outs, o, agg.endswith("f64")) == []


def test_staged_key_hashes_file_keys_by_their_hash(oracle_lib):
    """Key ids with a caller-given Java hashCode: a snapshot of the staged handle files each key
    under its own key group, as gw_ingest with the same hashes does."""
    kw = dict(assigner="tumbling", size=1000, slide=1000, agg="sum_i64")
    keys, ts, vals, batches = random_stream(seed=62, n=40_000, num_keys=3_000, n_batches=6, agg="sum_i64")
    hashes = ((keys * 1_000_003 + 7) % (1 << 31)).astype(np.int32)
    blobs = []
    for staged in (True, False):
        op = gpu_operator(kw, capacity_hint=1 << 14)
        try:
            if staged:
                op.stage_alloc(2, max(hi - lo for lo, hi, _ in batches))
            for b, (lo, hi, wm) in enumerate(batches):
                if staged:
                    k, h, t, v = op.stage_columns(b % 2)
                    k[:hi - lo], h[:hi - lo], t[:hi - lo], v[:hi - lo] = keys[lo:hi], hashes[lo:hi], ts[lo:hi], vals[lo:hi]
                    op.ingest_stage(b % 2, hi - lo, with_value=True, with_key_hash=True)
                else:
                    op.process_batch(keys[lo:hi], ts[lo:hi], vals[lo:hi], key_hashes=hashes[lo:hi])
                op.advance_watermark(wm)
                op.clear_rows()
            blobs.append(op.snapshot_state())
        finally:
            op.close()
    assert blobs[0] == blobs[1]


def test_staged_rejections():
    op = gpu_operator(dict(assigner="tumbling", size=1000, slide=1000, agg="sum_i64"))
    try:
        op.stage_alloc(2, 100)
        with pytest.raises(N.GpuWinError):
            op.ingest_stage(2, 10)  # no such slot
        with pytest.raises(N.GpuWinError):
            op.ingest_stage(0, 101)  # beyond the slot
        with pytest.raises(N.GpuWinError):
            op.ingest_stage(0, 10, with_value=False)  # SUM needs its values
    finally:
        op.close()


@pytest.mark.parametrize("ahead", [1, 2])
@pytest.mark.parametrize("agg", ["sum_i64", "count"])
def test_sent_ahead_matches_oracle(oracle_lib, agg, ahead):
    """gw_stage_send: batches b+1 (.. b+ahead) go over PCIe while batch b is ingested, fired
    and drained (into pinned host arrays, which the D2H writes directly) -- the host_fed leg's
    loop."""
    import torch

    kw = dict(assigner="sliding", size=2000, slide=500, agg=agg)
    keys, ts, vals, batches = random_stream(seed=63, n=240_000, num_keys=20_000, n_batches=16, agg=agg)
    cap = max(hi - lo for lo, hi, _ in batches)
    slots = 4
    op = gpu_operator(kw, capacity_hint=1 << 16)
    out = [torch.empty(1 << 18, dtype=torch.int64, pin_memory=True).numpy() for _ in range(4)]
    outs = []

    def fill(b):
        lo, hi, _ = batches[b]
        k, _, t, v = op.stage_columns(b % slots)
        k[:hi - lo] = keys[lo:hi]
        t[:hi - lo] = ts[lo:hi]
        if agg != "count":
            v[:hi - lo] = vals[lo:hi]

    try:
        op.stage_alloc(slots, cap)
        for b in range(ahead):
            fill(b)
            op.stage_send(b, batches[b][1] - batches[b][0], with_value=agg != "count")
        for b, (lo, hi, wm) in enumerate(batches):
            op.ingest_stage(b % slots, hi - lo, with_value=agg != "count")
            if b + ahead < len(batches):
                fill(b + ahead)
                nlo, nhi, _ = batches[b + ahead]
                op.stage_send((b + ahead) % slots, nhi - nlo, with_value=agg != "count")
            op.advance_watermark(wm)
            outs.append(tuple(x.copy() for x in op.drain(out)))
        op.advance_watermark(W.LONG_MAX)
        outs.append(tuple(x.copy() for x in op.drain(out)))
    finally:
        op.close()
    o, _ = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert compare(outs, o, False) == []


def test_sent_ahead_order_is_checked():
    op = gpu_operator(dict(assigner="tumbling", size=1000, slide=1000, agg="sum_i64"))
    try:
        op.stage_alloc(4, 100)
        op.stage_send(0, 10)
        with pytest.raises(N.GpuWinError):
            op.ingest_stage(1, 10)  # slot 0 was sent first
        op.stage_send(1, 10)
        op.stage_send(2, 10)
        with pytest.raises(N.GpuWinError):
            op.stage_send(3, 10)  # two batches ahead at most (three device buffers)
    finally:
        op.close()


def test_staging_is_not_reallocated_under_the_caller(oracle_lib):
    """Pinned slots handed out by gw_stage_columns (JVM direct ByteBuffers point into them) and
    batches sent ahead stay valid: a gw_ingest of the same handle (it copies through those slots,
    and a larger batch would reallocate them) is refused with GW_E_STATE, and the sent batch
    still ingests exactly (against the oracle)."""
    kw = dict(assigner="tumbling", size=1000, slide=1000, agg="sum_i64")
    keys, ts, vals, batches = random_stream(seed=64, n=300, num_keys=50, n_batches=1, agg="sum_i64")
    op = gpu_operator(kw)
    try:
        op.stage_alloc(2, 100)
        k, _, t, v = op.stage_columns(0)
        k[:100], t[:100], v[:100] = keys[:100], ts[:100], vals[:100]
        op.stage_send(0, 100)
        with pytest.raises(N.GpuWinError) as ei:
            op.process_batch(keys[100:300], ts[100:300], vals[100:300])  # 200 records: larger slots
        assert ei.value.code == N.GW_E_STATE
        op.ingest_stage(0, 100)
        with pytest.raises(N.GpuWinError) as ei:
            op.process_batch(keys[100:150], ts[100:150], vals[100:150])
        assert ei.value.code == N.GW_E_STATE
        op.advance_watermark(W.LONG_MAX)
        k_, s_, e_, r_ = op.drain()
    finally:
        op.close()
    o, _ = run_oracle(oracle_lib, kw, keys[:100], ts[:100], vals[:100], [(0, 100, W.LONG_MIN)])
    assert compare([(np.empty(0, np.int64),) * 4, (k_, s_, e_, r_)], o, False) == []


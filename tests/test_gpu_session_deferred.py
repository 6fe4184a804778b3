"""The slot sort session path with its tail deferred to the next sync (the default without
allowed lateness and side output): the ingest returns right after the segment launch, and the
migrations, the wide pass and the records whose keys found no slot run at the next call.
Against the oracle:

* keys whose slot hashes agree in their low 14 bits (built by inverting the hash), so that at
  the table sizes the batch starts with more than kMaxProbe (128) of them share one home slot:
  k_sess_prep finds no slot for some, the segment punts them, and the tail regrows the table
  and replays them;
* keys that outgrow their slot mid-batch (the wide pass in the tail) followed at once by a
  watermark whose fire must wait for that tail (the fire launched behind the ingest skips
  itself on the device and runs again after the tail);
* GW_SESSION_SYNC=1 (the tail at once) gives the same rows.
Parity: bit-exact (MergingWindowSet.java:153-224, WindowOperator.java:303-403)."""
import numpy as np
import pytest

from flink_amd import windowing as W
from gpu_helpers import compare, random_stream, run_gpu, run_oracle

pytestmark = pytest.mark.gpu

GOLD = 0x9E3779B97F4A7C15
M64 = (1 << 64) - 1


def key_for_hash(h):
    """The int64 key whose slot hash (x = key * GOLD; x ^ (x >> 32)) is h."""
    hi = h >> 32
    x = (hi << 32) | ((h & 0xFFFFFFFF) ^ hi)
    k = (x * pow(GOLD, -1, 1 << 64)) & M64
    return k - (1 << 64) if k >= 1 << 63 else k


def colliding_keys(n, low_bits=14, low=0x1234):
    return np.array([key_for_hash(((i + 1) << low_bits) | low) for i in range(n)], np.int64)


def test_key_for_hash_inverts_the_slot_hash():
    for h in (1, 0x1234, (7 << 14) | 0x1234, 0xDEADBEEF12345678):
        k = key_for_hash(h) & M64
        x = (k * GOLD) & M64
        assert x ^ (x >> 32) == h


@pytest.mark.parametrize("gap", [5000, 300])
@pytest.mark.parametrize("sync", [False, True])
def test_keys_without_a_slot_replay_after_a_regrow(oracle_lib, monkeypatch, sync, gap):
    """gap 5000: each hot key holds one session per batch; gap 300: hot keys open many and
    move to the wide table, where they collide as well (the wide table then grows too)."""
    if sync:
        monkeypatch.setenv("GW_SESSION_SYNC", "1")
    kw = dict(assigner="session", gap=gap, agg="sum_i64")
    keys, ts, vals, batches = random_stream(seed=71, n=40_000, num_keys=5000, n_batches=4, ts_step=1,
                                            disorder=200, wm_lag=200)
    hot = colliding_keys(300)
    rng = np.random.default_rng(72)
    pick = rng.random(keys.size) < 0.2
    keys[pick] = hot[rng.integers(0, hot.size, int(pick.sum()))]
    g, glate, st = run_gpu(kw, keys, ts, vals, batches, capacity_hint=1024)
    o, olate = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert glate == olate
    assert compare(g, o, False) == []
    assert st["rehashes"] > 0


def test_wide_tail_before_the_fire(oracle_lib):
    """Sparse timestamps: keys open many sessions within a batch (the wide pass runs in the
    deferred tail) and every batch is followed by a watermark that fires some of them."""
    kw = dict(assigner="session", gap=100, agg="count")
    rng = np.random.default_rng(19)
    n = 60_000
    keys = rng.integers(0, 400, n).astype(np.int64)
    ts = np.sort(rng.integers(0, 3_000_000, n)).astype(np.int64)
    vals = np.ones(n, np.int64)
    batches = [(lo, lo + 6000, int(ts[lo + 5999]) - 5000) for lo in range(0, n, 6000)]
    g, glate, st = run_gpu(kw, keys, ts, vals, batches, capacity_hint=1024)
    o, olate = run_oracle(oracle_lib, kw, keys, ts, vals, batches)
    assert glate == olate
    assert compare(g, o, False) == []

"""Corrupt and truncated checkpoint blobs against the host-side blob readers of libgpuwin
(pure host code, CPU): gw_snapshot_slice, gw_snapshot_keys and gw_snapshot_remap_keys must
return GW_E_INVALID (GpuWinError) or a consistent result for ANY bytes, never read or write
outside the blob.  A restore of a damaged checkpoint fails the task with an IOException in
the reference (HeapRestoreOperation / KeyGroupPartitioner reading a truncated stream,
flink-runtime/.../state/heap/HeapRestoreOperation.java); here the same damage must surface
as an error code, not as a crash of the TaskManager process that hosts the library.

Inputs: valid blob version 4 (the heap backend's per-key-group layout) written by the oracle
for pane, session and lateness handles, and v1-v3 entry blobs as test_snapshot_slice builds
them; then seeded truncations, byte flips and extreme header fields (entries, key-group range,
entry width, offsets).  Properties on the valid blobs: the key groups' slices name exactly
the blob's keys, and an invertible key remap round-trips to the same bytes."""
import struct

import numpy as np
import pytest

from flink_amd import _native as N
from gpu_helpers import random_stream
from test_snapshot_slice import HDR, make_blob

CFGS = [
    dict(assigner="tumbling", size=1000, slide=1000, agg="sum_i64"),
    dict(assigner="sliding", size=900, slide=300, agg="min_f64", lateness=700),
    dict(assigner="session", gap=150, agg="sum_i32", lateness=400),
    dict(assigner="count_tumbling", size=7, slide=7, agg="avg_f64"),
]
# header byte offsets (HDR = "<4sIii5q4i3q"): max_parallelism 56, kg_lo 60, kg_hi 64, reserved
# (entry words) 68, entries 88; the (kg_hi - kg_lo + 2) key-group offsets follow at 96
FIELDS = [(4, "<I"), (56, "<i"), (60, "<i"), (64, "<i"), (68, "<i"), (88, "<q")]
EXTREMES = [0, 1, -1, 2**31 - 1, -2**31, 2**62, 2**63 - 1, -2**63]


def oracle_blob(oracle_lib, kw, seed):
    o = oracle_lib
    keys, ts, vals, batches = random_stream(seed, 4000, 200, 6, disorder=600, wm_lag=200, agg=kw["agg"])
    op = o.OracleOperator(o.make_config(**kw))
    for lo, hi, wm in batches[:4]:
        op.process_batch(keys[lo:hi], ts[lo:hi], vals[lo:hi])
        op.process_watermark(wm)
        op.drain()
    return op.snapshot()


def read_all(blob, kgs):
    """Every reader on one (possibly damaged) blob; only GpuWinError may come back."""
    for kg in kgs:
        try:
            part = N.snapshot_slice(blob, kg)
            assert part[:4] == b"GWS1" and len(part) >= HDR.size
        except N.GpuWinError:
            pass
    try:
        ks = N.snapshot_keys(blob)
        assert np.all(np.diff(ks) > 0)
        if len(ks):
            out = N.snapshot_remap_keys(blob, {int(ks[0]): int(ks[0]) ^ 1})
            assert len(out) == len(blob)
    except N.GpuWinError:
        pass


def mutants(blob, seed, n):
    rng = np.random.default_rng(seed)
    L = len(blob)
    kg_lo, kg_hi = struct.unpack_from("<ii", blob, 60)
    head = min(L, HDR.size + 8 * (kg_hi - kg_lo + 2))
    for i in range(n):
        b = bytearray(blob)
        r = i % 4
        if r == 0:  # truncation
            yield bytes(b[:int(rng.integers(0, L))])
            continue
        if r == 1:  # byte flips in the header and offsets
            for _ in range(int(rng.integers(1, 5))):
                b[int(rng.integers(0, head))] ^= int(rng.integers(1, 256))
        elif r == 2:  # one header field at an extreme value
            off, fmt = FIELDS[int(rng.integers(0, len(FIELDS)))]
            v = EXTREMES[int(rng.integers(0, len(EXTREMES)))]
            if fmt == "<I":
                v &= 0xFFFFFFFF
            elif fmt == "<i":
                v = (v + 2**31) % 2**32 - 2**31
            struct.pack_into(fmt, b, off, v)
        else:  # byte flips anywhere (entry bodies: lengths inside v4 key-group records)
            for _ in range(int(rng.integers(1, 9))):
                b[int(rng.integers(0, L))] ^= int(rng.integers(1, 256))
        yield bytes(b)


@pytest.mark.parametrize("kw", CFGS, ids=lambda c: "-".join(str(v) for v in c.values()))
def test_v4_blob_properties(oracle_lib, kw):
    blob = oracle_blob(oracle_lib, kw, 11)
    kg_lo, kg_hi = struct.unpack_from("<ii", blob, 60)
    keys = N.snapshot_keys(blob)
    assert len(keys) > 0
    per_kg = [N.snapshot_keys(N.snapshot_slice(blob, kg)) for kg in range(kg_lo, kg_hi + 1)]
    assert np.array_equal(np.unique(np.concatenate(per_kg)), keys)
    assert sum(len(k) for k in per_kg) == len(keys)  # a key lives in one key group
    there = N.snapshot_remap_keys(blob, {int(k): int(k) + (1 << 40) for k in keys})
    assert there != blob
    assert np.array_equal(N.snapshot_keys(there), keys + (1 << 40))
    assert N.snapshot_remap_keys(there, {int(k) + (1 << 40): int(k) for k in keys}) == blob


@pytest.mark.parametrize("kw", CFGS, ids=lambda c: "-".join(str(v) for v in c.values()))
def test_v4_damaged_blobs(oracle_lib, kw):
    blob = oracle_blob(oracle_lib, kw, 12)
    kg_lo, kg_hi = struct.unpack_from("<ii", blob, 60)
    kgs = sorted({kg_lo, (kg_lo + kg_hi) // 2, kg_hi})
    for m in mutants(blob, 7, 400):
        read_all(m, kgs)


@pytest.mark.parametrize("version,words", [(1, 4), (2, 6), (3, 8)])
def test_entry_blob_damage(version, words):
    blob, _, _ = make_blob(version, words, 8, 23, lambda k: (k * 5) % 4, seed=version)
    for m in mutants(blob, version, 400):
        read_all(m, [8, 15, 23])



@pytest.mark.parametrize("kw", CFGS, ids=lambda c: "-".join(str(v) for v in c.values()))
@pytest.mark.parametrize("count", [-1, -(2**31)])
def test_v4_negative_entry_count_rejected(oracle_lib, kw, count):
    """A key group whose entry count is negative is a damaged blob: the readers that parse the
    key groups refuse it (GW_E_INVALID) instead of reading it as an empty key group.
    (gw_snapshot_slice cuts by the offset table without parsing; the restore that reads the
    slice refuses it the same way -- restore_heap / restore_sessions, GPU handles.)"""
    blob = oracle_blob(oracle_lib, kw, 13)
    kg_lo, kg_hi = struct.unpack_from("<ii", blob, 60)
    nk = kg_hi - kg_lo + 1
    offs = struct.unpack_from(f"<{nk + 1}q", blob, 96)
    pay0 = 96 + 8 * (nk + 1)
    g = next(i for i in range(nk) if offs[i + 1] > offs[i])  # a non-empty key group
    b = bytearray(blob)
    struct.pack_into(">i", b, pay0 + offs[g], count)
    with pytest.raises(N.GpuWinError):
        N.snapshot_keys(bytes(b))
    with pytest.raises(N.GpuWinError):
        N.snapshot_keys(N.snapshot_slice(bytes(b), kg_lo + g))

"""gw_snapshot_slice (pure host code, CPU): cutting a multi-key-group snapshot blob into
per-key-group blobs, as GpuWindowOperator.snapshotState writes them (one blob per key group
into the raw keyed state, like HeapSnapshotStrategy.java:97-154), for every blob version:
pane entries (v1, 32 B), session entries (v2, `reserved` words) and count-window entries
(v3, `reserved` words)."""
import struct

import numpy as np
import pytest

from flink_amd import _native as N

HDR = struct.Struct("<4sIii5q4i3q")  # include/gpuwin.h gw_snapshot / gw_handle::SnapHeader
assert HDR.size == 96


def make_blob(version, words, kg_lo, kg_hi, per_kg, seed=0):
    rng = np.random.default_rng(seed)
    counts = [per_kg(k) for k in range(kg_lo, kg_hi + 1)]
    offs = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    n = int(offs[-1])
    ent = rng.integers(-(1 << 62), 1 << 62, (n, words)).astype(np.int64)
    reserved = 0 if version == 1 else words
    hdr = HDR.pack(b"GWS1", version, 1, 1, 1000, 200, 0, 0, 200, 128, kg_lo, kg_hi, reserved, 5, 0, n)
    return hdr + offs.tobytes() + ent.tobytes(), offs, ent


@pytest.mark.parametrize("version,words", [(1, 4), (2, 6), (3, 2 + 6), (3, 2 + 2 * 5)])
def test_slice_every_key_group(version, words):
    blob, offs, ent = make_blob(version, words, 16, 31, lambda k: (k * 7) % 5, seed=version)
    for i, kg in enumerate(range(16, 32)):
        part = N.snapshot_slice(blob, kg)
        h = HDR.unpack(part[:96])
        assert h[0] == b"GWS1" and h[1] == version
        assert h[10] == kg and h[11] == kg and h[15] == offs[i + 1] - offs[i]
        o = np.frombuffer(part[96:112], np.int64)
        assert o.tolist() == [0, int(offs[i + 1] - offs[i])]
        got = np.frombuffer(part[112:], np.int64).reshape(-1, words)
        assert np.array_equal(got, ent[offs[i]:offs[i + 1]])
        # a slice of a slice is itself
        assert N.snapshot_slice(part, kg) == part


def test_slice_rejects_bad_input():
    blob, _, _ = make_blob(2, 6, 0, 3, lambda k: 2)
    with pytest.raises(N.GpuWinError):
        N.snapshot_slice(blob, 4)  # outside [kg_lo, kg_hi]
    with pytest.raises(N.GpuWinError):
        N.snapshot_slice(blob[:-8], 0)  # truncated
    with pytest.raises(N.GpuWinError):
        N.snapshot_slice(b"XXXX" + blob[4:], 0)
    bad = bytearray(blob)
    bad[96 + 8:96 + 16] = np.int64(99).tobytes()  # offsets beyond the entries
    with pytest.raises(N.GpuWinError):
        N.snapshot_slice(bytes(bad), 0)

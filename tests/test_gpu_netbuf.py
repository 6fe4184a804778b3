"""Network-buffer ingest on the GPU: gw_decode_serialized against the
oracle's sequential decoder (bit-exact columns, watermark positions, consumed bytes), and
gw_ingest_serialized* against the oracle operator fed the same decoded channel.

Parity is pinned by the oracle decoder (tests/test_netbuf_oracle.py: two restatements of
StreamElementSerializer agree) and by the reference's own serializer bytes
(tests/golden/serializer/: StreamElementSerializerUpgradeTest's record, LongSerializer's Long),
decoded here on the device too."""
import ctypes
import struct

import numpy as np
import pytest

from flink_amd import _native as N
from flink_amd import netbuf as NB
from flink_amd import windowing as W
from tests.gpu_helpers import compare, gpu_operator, random_stream
from tests.test_netbuf_oracle import LAYOUTS, random_elements, reference_bytes

pytestmark = pytest.mark.gpu


def gpu_decode(data: bytes, types, kf, vf, rec_cap=None, wm_cap=None):
    import torch
    n = len(data)
    d = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda() if n else torch.zeros(4, dtype=torch.uint8,
                                                                                          device="cuda")
    rc_cap = rec_cap if rec_cap is not None else n // 6 + 1
    w_cap = wm_cap if wm_cap is not None else n // 13 + 1
    k, t, v = (torch.zeros(max(rc_cap, 1), dtype=torch.int64, device="cuda") for _ in range(3))
    wp, wv = (torch.zeros(max(w_cap, 1), dtype=torch.int64, device="cuda") for _ in range(2))
    res = N.GwDecodeResult()
    lay = N.record_layout(types, kf, vf)
    P = lambda x: ctypes.c_void_p(x.data_ptr())
    torch.cuda.synchronize()
    rc = N.lib().gw_decode_serialized(P(d), n, ctypes.byref(lay), P(k), P(t), P(v), rc_cap, P(wp), P(wv), w_cap,
                                      ctypes.byref(res), None)
    r, w = res.records, res.watermarks
    return rc, k[:r].cpu().numpy(), t[:r].cpu().numpy(), v[:r].cpu().numpy(), wp[:w].cpu().numpy(), \
        wv[:w].cpu().numpy(), res


def assert_same_decode(oracle_lib, data, types, kf, vf):
    g = gpu_decode(data, types, kf, vf)
    o = oracle_lib.decode_stream(data, types, kf, vf)
    assert g[0] == o[0] == 0
    assert g[6].records == o[6].records and g[6].watermarks == o[6].watermarks
    assert g[6].consumed == o[6].consumed and g[6].skipped == o[6].skipped
    for i, name in enumerate(["key", "ts", "value", "wm_pos", "wm_val"], start=1):
        if vf < 0 and name == "value":
            continue
        assert np.array_equal(g[i], o[i]), name


@pytest.mark.parametrize("types,kf,vf", LAYOUTS)
def test_decode_matches_oracle(oracle_lib, types, kf, vf):
    rng = np.random.default_rng(11 + kf)
    data = random_elements(rng, 20000, types, kf, vf)
    for cut in (len(data), len(data) - 1, len(data) - 9, 4096 * 3 + 17, 4096, 63, 3, 0):
        assert_same_decode(oracle_lib, data[:cut], types, kf, vf)


def test_decode_payload_mimicking_length_words(oracle_lib):
    # payload bytes that read as valid element lengths keep wrong candidate entries alive
    # across whole chunks: the resolve step must follow the true chain back
    vals = [(25 << 32) | 25, (13 << 32) | 9, 0x0000001d0000001d, (1 << 32) | 2]
    parts = []
    for i in range(30000):
        v = vals[i % len(vals)]
        parts.append(NB.record((v, v ^ 1), "JJ", v & 0xFFFF))
        if i % 997 == 0:
            parts.append(NB.watermark(i))
    data = b"".join(parts)
    for cut in (len(data), len(data) - 5):
        assert_same_decode(oracle_lib, data[:cut], "JJ", 0, 1)


def test_decode_large_stream(oracle_lib):
    rng = np.random.default_rng(5)
    n = 2_000_000
    k = rng.integers(0, 10_000_000, n)
    t = np.arange(n) // 10
    v = rng.integers(0, 1_000_000, n)
    data = NB.serialize_batches("JJ", 0, 1, [(k[i:i + 500_000], t[i:i + 500_000], v[i:i + 500_000])
                                             for i in range(0, n, 500_000)], [1000, 2000, 3000, 4000])
    g = gpu_decode(data, "JJ", 0, 1)
    assert g[0] == 0 and g[6].records == n and g[6].consumed == len(data)
    assert np.array_equal(g[1], k) and np.array_equal(g[2], t) and np.array_equal(g[3], v)
    assert g[4].tolist() == [500_000, 1_000_000, 1_500_000, 2_000_000] and g[5].tolist() == [1000, 2000, 3000, 4000]


def test_decode_reference_serializer_bytes(oracle_lib):
    """The reference's bytes on the device: the record (1234567890L)@123456 built from
    StreamElementSerializerUpgradeTest's tag + timestamp and LongSerializer's Long, repeated across
    several 1-KB chunks with watermarks, decodes bit-exactly like the oracle; the reference's own
    String record under the Long layout fails the task as a corrupt stream (GW_E_INVALID)."""
    rec, lng = reference_bytes()
    element = struct.pack(">i", 17) + rec[:9] + lng
    data = (element * 100 + NB.watermark(123000)) * 7
    g = gpu_decode(data, "J", 0, -1)
    assert g[0] == 0 and g[6].records == 700 and set(g[1].tolist()) == {1234567890} and set(g[2].tolist()) == {123456}
    assert_same_decode(oracle_lib, data, "J", 0, -1)
    assert gpu_decode(data + struct.pack(">i", len(rec)) + rec + data, "J", 0, -1)[0] == -1


def test_decode_errors():
    good = NB.record((1, 2), "JJ", 3) * 500
    bad_tag = struct.pack(">i", 9) + bytes([9]) + b"\0" * 8
    assert gpu_decode(good + bad_tag + good, "JJ", 0, 1)[0] == -1
    assert gpu_decode(good + NB.record((1, 2, 3), "JJJ", 3), "JJ", 0, 1)[0] == -1
    assert gpu_decode(good + NB.record(tuple(range(7)), "JJJJJJJ", 1) + good, "JJ", 0, 1)[0] == -1
    assert gpu_decode(good + NB.record(tuple(range(15)), "J" * 15, 1) + good, "JJ", 0, 1)[0] == -2
    wide = NB.record(tuple(range(8)), "J" * 8, 3) * 300
    assert gpu_decode(wide + NB.record(tuple(range(15)), "J" * 15, 1) + wide, "J" * 8, 0, 1)[0] == -2
    assert gpu_decode(wide + NB.record((1, 2), "JJ", 3) + wide, "J" * 8, 0, 1)[0] == -1
    assert gpu_decode(good, "JJ", 0, 1, rec_cap=100)[0] == -5
    assert gpu_decode(good + NB.watermark(5) * 3, "JJ", 0, 1, wm_cap=2)[0] == -5


CONFIGS = [
    (dict(assigner="tumbling", size=1000, agg="sum_i64"), "JJ", 0, 1),
    (dict(assigner="sliding", size=1000, slide=300, offset=-50, agg="max_i64"), "IJJ", 1, 2),
    (dict(assigner="sliding", size=10000, slide=2000, agg="count"), "JJ", 0, -1),
    (dict(assigner="tumbling", size=700, agg="avg_f64"), "JD", 0, 1),
    (dict(assigner="sliding", size=900, slide=300, agg="sum_f64"), "JFJ", 0, 1),
    (dict(assigner="session", gap=80, agg="sum_i64"), "JJ", 0, 1),
]


def channel_stream(kw, types, kf, vf, seed, n=60000, nb=12, n_keys=500):
    keys, ts, vals, batches = random_stream(seed, n, n_keys, nb, ts_step=3, disorder=200, wm_lag=200,
                                            agg=kw["agg"] if kw["agg"] != "count" else "sum_i64")
    if types[vf if vf >= 0 else 0] == "F":
        vals = vals.astype(np.float32).astype(np.float64)
    data = NB.serialize_batches(types, kf, vf, [(keys[lo:hi], ts[lo:hi], vals[lo:hi]) for lo, hi, _ in batches],
                                [wm for _, _, wm in batches])
    return data


def oracle_channel(oracle_lib, kw, data, types, kf, vf):
    rc, k, t, v, wp, wv, res = oracle_lib.decode_stream(data, types, kf, vf)
    assert rc == 0
    op = oracle_lib.OracleOperator(oracle_lib.make_config(**kw))
    done = 0
    for p, w in list(zip(wp.tolist(), wv.tolist())) + [(len(k), None)]:
        if p > done:
            op.process_batch(k[done:p], t[done:p], v[done:p])
            done = p
        if w is not None:
            op.process_watermark(w)
    op.process_watermark(W.LONG_MAX)
    return op.drain()


def drained(op):
    k, s, e, r = op.drain()
    return k, s, e, r.view(np.int64)


@pytest.mark.parametrize("kw,types,kf,vf", CONFIGS)
def test_operator_network_buffers_match_oracle(oracle_lib, kw, types, kf, vf):
    data = channel_stream(kw, types, kf, vf, seed=31)
    exp = oracle_channel(oracle_lib, kw, data, types, kf, vf)
    lay = N.record_layout(types, kf, vf)
    for bufsize in (32 * 1024, 4093):  # records span buffer boundaries
        op = gpu_operator(kw)
        try:
            op.process_buffers(NB.split_buffers(data, bufsize), lay)
            op.advance_watermark(W.LONG_MAX)
            got = drained(op)
        finally:
            op.close()
        assert compare([got], [exp], kw["agg"] in N.DOUBLE_RESULT) == []


def test_operator_device_bytes_match_oracle(oracle_lib):
    import torch
    kw, types, kf, vf = CONFIGS[1]
    data = channel_stream(kw, types, kf, vf, seed=7, n=200000, nb=20)
    exp = oracle_channel(oracle_lib, kw, data, types, kf, vf)
    op = gpu_operator(kw)
    try:
        d = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
        used, fired = op.process_serialized_device(d, N.record_layout(types, kf, vf))
        assert used == len(data) and fired > 0
        op.advance_watermark(W.LONG_MAX)
        got = drained(op)
    finally:
        op.close()
    assert compare([got], [exp], False) == []


def test_operator_no_timestamp_and_corrupt_fail_the_task():
    lay = N.record_layout("JJ", 0, 1)
    op = gpu_operator(dict(assigner="tumbling", size=100, agg="sum_i64"))
    try:
        with pytest.raises(N.GpuWinError) as e:
            op.process_serialized(NB.record((1, 2), "JJ", 5) + NB.record((1, 2), "JJ") + NB.watermark(500), lay)
            op.advance_watermark(1000)
        assert e.value.code in (-6, -8)
    finally:
        op.close()
    op = gpu_operator(dict(assigner="tumbling", size=100, agg="sum_i64"))
    try:
        with pytest.raises(N.GpuWinError) as e:
            op.process_serialized(NB.record((1, 2), "JJ", 5) + struct.pack(">i", 9) + bytes([7]) + b"\0" * 8, lay)
        assert e.value.code == -1
        with pytest.raises(N.GpuWinError):  # the operator has failed
            op.advance_watermark(1000)
    finally:
        op.close()
    op = gpu_operator(dict(assigner="tumbling", size=100, agg="sum_f64"))
    try:
        with pytest.raises(N.GpuWinError) as e:  # a Long field cannot feed a double sum
            op.process_serialized(NB.record((1, 2), "JJ", 5), lay)
        assert e.value.code == -1
    finally:
        op.close()

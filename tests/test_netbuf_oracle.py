"""Network-buffer decode, CPU side: the oracle's sequential decoder
(oracle/flink_oracle.c wo_decode_stream) against an independent pure-Python restatement of
StreamElementSerializer.deserialize (RS/runtime/streamrecord/StreamElementSerializer.java:
200-225) over streams written by flink_amd.netbuf (the sender side, :163-197).

Parity pinning: the reference's own serializer bytes (tests/golden/serializer/, copied by
tests/golden/make_serializer_fixtures.py): StreamElementSerializerUpgradeTest's StreamRecord
("key", 123456) -- tag 0, big-endian timestamp, String payload -- and LongSerializer's
1234567890L.  A Tuple1<Long> record is its fields' serializer bytes in order
(TupleSerializer.serialize :135-144), so the record (1234567890L)@123456 is exactly the
reference's tag + timestamp followed by the reference's Long bytes: the writer must produce
them and both decoders must read them back; the reference's own String record must be refused
under a Long layout (its length does not match), as a corrupt stream.  Beyond that the byte
format is pinned by the two restatements of the published serializer agreeing, and by the
round trip element -> bytes -> element."""
import struct

import numpy as np
import pytest

from flink_amd import netbuf as NB

LONG_MIN = -(1 << 63)
WIDTH = {"J": 8, "D": 8, "I": 4, "F": 4, "S": 2, "B": 1, "Z": 1}
FMT = {"J": ">q", "D": ">d", "I": ">i", "F": ">f", "S": ">h", "B": ">b", "Z": ">?"}


def py_decode(data, types, key_field, value_field):
    """Element by element, as the reference's deserializer reads a buffer."""
    offs = np.cumsum([0] + [WIDTH[t] for t in types])
    vbytes = int(offs[-1])
    pos, recs, wms = 0, [], []
    while pos + 4 <= len(data):
        (ln,) = struct.unpack_from(">i", data, pos)
        if pos + 4 + ln > len(data):
            break
        tag = data[pos + 4]
        if tag in (0, 1):
            hdr = 9 if tag == 0 else 1
            assert ln == hdr + vbytes
            ts = struct.unpack_from(">q", data, pos + 5)[0] if tag == 0 else LONG_MIN
            v0 = pos + 4 + hdr
            key = struct.unpack_from(">q", data, v0 + offs[key_field])[0]
            val = 0
            if value_field >= 0:
                t = types[value_field]
                x = struct.unpack_from(FMT[t], data, v0 + offs[value_field])[0]
                val = struct.unpack("<q", struct.pack("<d", float(x)))[0] if t in "DF" else int(x)
            recs.append((key, ts, val))
        elif tag == 2:
            wms.append((len(recs), struct.unpack_from(">q", data, pos + 5)[0]))
        elif tag == 6:
            wms.append((len(recs), struct.unpack_from(">q", data, pos + 9)[0]))
        else:
            assert tag in (3, 4, 5)
        pos += 4 + ln
    return recs, wms, pos


def random_elements(rng, n, types, key_field, value_field, p_wm=0.05, p_other=0.05, p_nots=0.02):
    out, recs = [], []
    ts = 1000
    for _ in range(n):
        u = rng.random()
        if u < p_wm:
            out.append(NB.watermark(ts - 50) if rng.random() < 0.7 else NB.internal_watermark(ts - 50, 1))
        elif u < p_wm + p_other:
            c = rng.integers(0, 3)
            out.append([NB.latency_marker(ts, 1, 2, 3), NB.stream_status(True), NB.record_attributes(True)][c])
        else:
            fields = []
            for i, t in enumerate(types):
                if t == "J":
                    fields.append(int(rng.integers(-(1 << 62), 1 << 62)))
                elif t in "DF":
                    fields.append(float(rng.normal() * 1e3))
                elif t == "I":
                    fields.append(int(rng.integers(-(1 << 31), (1 << 31) - 1)))
                elif t == "S":
                    fields.append(int(rng.integers(-(1 << 15), (1 << 15) - 1)))
                elif t == "B":
                    fields.append(int(rng.integers(-128, 127)))
                else:
                    fields.append(bool(rng.integers(0, 2)))
            stamp = None if rng.random() < p_nots else ts + int(rng.integers(-40, 40))
            out.append(NB.record(fields, types, stamp))
            ts += int(rng.integers(0, 5))
    return b"".join(out)


# the last two: elements of 77 and 73 bytes (beyond 64: the two-candidates-per-lane walk)
LAYOUTS = [("JJ", 0, 1), ("JD", 0, 1), ("IJJ", 1, 2), ("JI", 0, 1), ("SJFB", 1, 2), ("JZDJ", 0, 3), ("JJ", 1, -1),
           ("JJJJJJJJ", 3, 7), ("IJJJJJJD", 1, 7)]


@pytest.mark.parametrize("types,kf,vf", LAYOUTS)
def test_oracle_decoder_matches_python_restatement(oracle_lib, types, kf, vf):
    rng = np.random.default_rng(len(types) * 7 + kf)
    data = random_elements(rng, 3000, types, kf, vf)
    for cut in (len(data), len(data) - 3, len(data) - 17):  # tail of a spanning element
        d = data[:cut]
        rc, k, t, v, wp, wv, res = oracle_lib.decode_stream(d, types, kf, vf)
        assert rc == 0
        recs, wms, pos = py_decode(d, types, kf, vf)
        assert res.consumed == pos
        assert [tuple(x) for x in zip(k.tolist(), t.tolist(), v.tolist())] == recs
        assert list(zip(wp.tolist(), wv.tolist())) == wms


def test_round_trip_and_skips(oracle_lib):
    d = (NB.record((5, 7), "JJ", 100) + NB.watermark(99) + NB.record((6, -3), "JJ") +
         NB.latency_marker(1, 2, 3, 4) + NB.stream_status(False) + NB.record_attributes(False) +
         NB.internal_watermark(200, 3) + NB.record((8, 9), "JJ", 150))
    rc, k, t, v, wp, wv, res = oracle_lib.decode_stream(d, "JJ", 0, 1)
    assert rc == 0
    assert k.tolist() == [5, 6, 8] and t.tolist() == [100, LONG_MIN, 150] and v.tolist() == [7, -3, 9]
    assert wp.tolist() == [1, 2] and wv.tolist() == [99, 200]
    assert res.skipped == 3 and res.consumed == len(d)


def test_corrupt_and_unsupported(oracle_lib):
    good = NB.record((1, 2), "JJ", 3)
    bad_tag = struct.pack(">i", 9) + bytes([9]) + b"\0" * 8
    assert oracle_lib.decode_stream(good + bad_tag, "JJ", 0, 1)[0] == -1      # Corrupt stream, found tag
    assert oracle_lib.decode_stream(good + NB.record((1, 2, 3), "JJJ", 3), "JJ", 0, 1)[0] == -1  # length
    too_long = NB.record(tuple(range(15)), "J" * 15, 1)                            # 133 bytes
    assert oracle_lib.decode_stream(too_long, "JJ", 0, 1)[0] == -2            # > GW_MAX_ELEMENT
    wide = NB.record(tuple(range(8)), "J" * 8, 1)                                 # 77 bytes
    assert oracle_lib.decode_stream(wide, "J" * 8, 0, 1)[0] == 0
    assert oracle_lib.decode_stream(wide, "JJ", 0, 1)[0] == -1                # length does not fit the layout
    assert oracle_lib.decode_stream(struct.pack(">i", 0), "JJ", 0, 1)[0] == -1


def test_vectorised_serializer_matches_element_serializer():
    rng = np.random.default_rng(2)
    k = rng.integers(0, 1 << 40, 50)
    t = rng.integers(0, 1 << 40, 50)
    v = rng.normal(size=50)
    fast = NB.serialize_batches("JDI", 0, 1, [(k, t, v)], [123])
    slow = b"".join(NB.record((int(a), float(c), 0), "JDI", int(b)) for a, b, c in zip(k, t, v)) + NB.watermark(123)
    assert fast == slow


def reference_bytes():
    import os
    d = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "serializer")
    rec = open(os.path.join(d, "stream-element-serializer.test-data"), "rb").read()
    lng = open(os.path.join(d, "long-serializer.test-data"), "rb").read()
    assert rec.hex() == "00000000000001e240046b6579" and lng.hex() == "00000000499602d2"
    return rec, lng


def test_reference_serializer_bytes_pin_the_framing(oracle_lib):
    """StreamRecord(Tuple1(1234567890L), 123456) is the reference's tag + timestamp bytes and its
    Long bytes; the writer produces them, the oracle decoder and the Python restatement read them
    back; the reference's String record (13 bytes) under the Long layout is a corrupt stream."""
    rec, lng = reference_bytes()
    element = rec[:9] + lng  # tag 0 + be64 123456, then the Tuple1's only field
    data = struct.pack(">i", len(element)) + element
    assert NB.record([1234567890], "J", timestamp=123456) == data
    rc, k, t, v, wp, wv, res = oracle_lib.decode_stream(data, "J", 0, -1)
    assert rc == 0 and list(k) == [1234567890] and list(t) == [123456] and res.consumed == len(data)
    recs, wms, pos = py_decode(data, "J", 0, -1)
    assert recs == [(1234567890, 123456, 0)] and pos == len(data)
    # the same record followed by a watermark, then the reference's String record: the decoder
    # reads the first two and fails the task on the third (length 13 != 1 + 8 + 8)
    bad = data + NB.watermark(123000) + struct.pack(">i", len(rec)) + rec
    rc, *_ = oracle_lib.decode_stream(bad, "J", 0, -1)
    assert rc == -1  # GW_E_INVALID: "Corrupt stream"

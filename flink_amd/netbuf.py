"""Serialized stream elements of one keyBy input channel (the bytes gw_ingest_serialized
decodes on the GPU).

This is the sender side of the format, as a Flink upstream task writes it into its
network buffers, so a job (or a test) can produce the exact bytes the window operator's
input channel receives:

- every element is a 4-byte big-endian length followed by the element
  (RecordWriter.serializeRecord, flink-runtime/src/main/java/org/apache/flink/runtime/io/
  network/api/writer/RecordWriter.java:144-156);
- the element is StreamElementSerializer.serialize (flink-runtime/src/main/java/org/apache/
  flink/streaming/runtime/streamrecord/StreamElementSerializer.java:163-197): a tag byte,
  then the record's timestamp and value, or the watermark / status / latency marker body;
- a Tuple value is TupleSerializer.serialize (flink-core/src/main/java/org/apache/flink/
  api/java/typeutils/runtime/TupleSerializer.java:135-144): the fields in order, each with
  its big-endian DataOutputView primitive.

Network buffers split the byte stream anywhere, records spanning two buffers included
(SpanningWrapper); `split_buffers` cuts a stream the same way.
"""
from __future__ import annotations

import struct
from typing import Iterable, List, Sequence

import numpy as np

TAG_REC_WITH_TIMESTAMP = 0
TAG_REC_WITHOUT_TIMESTAMP = 1
TAG_WATERMARK = 2
TAG_LATENCY_MARKER = 3
TAG_STREAM_STATUS = 4
TAG_RECORD_ATTRIBUTES = 5
TAG_INTERNAL_WATERMARK = 6

_FMT = {"J": "q", "D": "d", "I": "i", "F": "f", "S": "h", "B": "b", "Z": "?"}
_NP = {"J": ">i8", "D": ">f8", "I": ">i4", "F": ">f4", "S": ">i2", "B": "i1", "Z": "u1"}


def _frame(body: bytes) -> bytes:
    return struct.pack(">i", len(body)) + body


def record(fields: Sequence, types: str, timestamp=None) -> bytes:
    fmt = ">" + "".join(_FMT[t] for t in types)
    value = struct.pack(fmt, *fields)
    if timestamp is None:
        return _frame(bytes([TAG_REC_WITHOUT_TIMESTAMP]) + value)
    return _frame(bytes([TAG_REC_WITH_TIMESTAMP]) + struct.pack(">q", timestamp) + value)


def watermark(ts: int) -> bytes:
    return _frame(bytes([TAG_WATERMARK]) + struct.pack(">q", ts))


def internal_watermark(ts: int, subpartition: int) -> bytes:
    return _frame(bytes([TAG_INTERNAL_WATERMARK]) + struct.pack(">iq", subpartition, ts))


def stream_status(active: bool) -> bytes:
    # WatermarkStatus.ACTIVE_STATUS = 0, IDLE_STATUS = -1
    return _frame(bytes([TAG_STREAM_STATUS]) + struct.pack(">i", 0 if active else -1))


def latency_marker(marked_time: int, op_lo: int, op_hi: int, subtask: int) -> bytes:
    return _frame(bytes([TAG_LATENCY_MARKER]) + struct.pack(">qqqi", marked_time, op_lo, op_hi, subtask))


def record_attributes(backlog: bool) -> bytes:
    return _frame(bytes([TAG_RECORD_ATTRIBUTES, 1 if backlog else 0]))


def serialize_batches(types: str, key_field: int, value_field: int, batches: Iterable,
                      watermarks: Iterable[int]) -> bytes:
    """Vectorised serializer for large streams: batch b = (keys, timestamps, values)
    followed by Watermark(wm[b]).  Every field other than key/value is written as 0."""
    widths = {"J": 8, "D": 8, "I": 4, "F": 4, "S": 2, "B": 1, "Z": 1}
    vbytes = sum(widths[t] for t in types)
    elen = 1 + 8 + vbytes
    out: List[bytes] = []
    for (k, ts, v), wm in zip(batches, watermarks):
        n = len(k)
        rec = np.zeros((n, 4 + elen), dtype=np.uint8)
        rec[:, 0:4] = np.frombuffer(struct.pack(">i", elen), dtype=np.uint8)
        rec[:, 4] = TAG_REC_WITH_TIMESTAMP
        rec[:, 5:13] = np.asarray(ts, dtype=">i8").view(np.uint8).reshape(n, 8)
        off = 13
        for i, t in enumerate(types):
            w = widths[t]
            if i == key_field:
                col = np.asarray(k, dtype=">i8")
            elif i == value_field:
                col = np.asarray(v).astype(_NP[t])
            else:
                col = np.zeros(n, dtype=_NP[t])
            rec[:, off:off + w] = col.view(np.uint8).reshape(n, w)
            off += w
        out.append(rec.tobytes())
        out.append(watermark(int(wm)))
    return b"".join(out)


def split_buffers(stream: bytes, buffer_size: int) -> List[bytes]:
    """Cut a byte stream into network buffers of buffer_size bytes (the last shorter)."""
    return [stream[i:i + buffer_size] for i in range(0, len(stream), buffer_size)]

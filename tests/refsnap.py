"""Data-only reader of the reference's operator-snapshot fixtures (test infrastructure).

The files are what OperatorSnapshotUtil.writeStateHandle writes
(flink-runtime/src/test/java/org/apache/flink/streaming/util/OperatorSnapshotUtil.java:50-124):
a DataOutputStream with the metadata version, a null stream handle, the operator-state
handle lists and the keyed-state handle lists (MetadataV2V3SerializerBase.serializeKeyedStateHandle
:324-345: KEY_GROUPS_HANDLE(_V2) = key-group start, count, one offset per key group, then the
ByteStreamStateHandle holding the heap backend's bytes).  Inside those bytes the heap backend
writes, per key group at its offset (HeapSnapshotStrategy.java:157-174): int key group, then per
state short state id + the state's key-group section:
  * "window-contents" (CopyOnWriteStateMapSnapshot.writeState :127-149): int n, n x (namespace,
    key, state);
  * timers (HeapPriorityQueueSnapshot: int n, n x TimerSerializer.serialize :147-152 =
    flipSignBit(ts), key, namespace).
State ids are the order of the state meta infos in the serialization proxy in front of the key
groups; they are found here by the names the proxy writes (writeUTF), nothing is executed or
deserialized as Java objects.  Keys are Strings (StringValue.writeString: varint length + 1,
then varint chars), namespaces TimeWindow (start, end: TimeWindow.Serializer :159-169).
"""
import struct

STATE_NAMES = ("window-contents", "_timer_state/processing_window-timers", "_timer_state/event_window-timers",
               "merging-window-set", "count")


class Reader:
    def __init__(self, b: bytes, p: int = 0):
        self.b, self.p = b, p

    def u8(self):
        v = self.b[self.p]
        self.p += 1
        return v

    def i16(self):
        v, = struct.unpack_from(">h", self.b, self.p)
        self.p += 2
        return v

    def i32(self):
        v, = struct.unpack_from(">i", self.b, self.p)
        self.p += 4
        return v

    def i64(self):
        v, = struct.unpack_from(">q", self.b, self.p)
        self.p += 8
        return v

    def utf(self):  # DataOutput.writeUTF (modified UTF-8; the names here are ASCII)
        n, = struct.unpack_from(">H", self.b, self.p)
        s = self.b[self.p + 2:self.p + 2 + n].decode("utf-8")
        self.p += 2 + n
        return s

    def varint(self):
        v, sh = 0, 0
        while True:
            c = self.u8()
            if c < 0x80:
                return v | (c << sh)
            v |= (c & 0x7F) << sh
            sh += 7

    def jstring(self):  # StringValue.readString
        n = self.varint()
        if n == 0:
            return None
        return "".join(chr(self.varint()) for _ in range(n - 1))


def _stream_handle(r: Reader) -> bytes:
    t = r.u8()
    if t == 0:
        return b""
    if t != 1:  # BYTE_STREAM_STATE_HANDLE
        raise ValueError(f"stream handle type {t}")
    r.utf()  # handle name
    n = r.i32()
    d = r.b[r.p:r.p + n]
    r.p += n
    return d


def keyed_state(data: bytes):
    """-> (key-group start, key-group count, offsets, backend bytes) of the managed keyed state."""
    r = Reader(data)
    r.i32()  # metadata version
    if r.u8() != 0:
        raise ValueError("expected the null stream handle")
    for _ in range(2):  # raw / managed operator state: none in these fixtures
        if r.i32() > 0:
            raise ValueError("operator state present")
    if r.i32() > 0:
        raise ValueError("raw keyed state present")
    if r.i32() != 1:
        raise ValueError("expected one managed keyed state handle")
    t = r.u8()
    if t not in (3, 12):  # KEY_GROUPS_HANDLE, KEY_GROUPS_HANDLE_V2
        raise ValueError(f"keyed state handle type {t}")
    start, count = r.i32(), r.i32()
    offs = [r.i64() for _ in range(count)]
    return start, count, offs, _stream_handle(r)


def state_ids(backend: bytes):
    """State id -> name: the order in which the serialization proxy names the states."""
    found = []
    for name in STATE_NAMES:
        pat = struct.pack(">H", len(name)) + name.encode()
        at = backend.find(pat)
        if at >= 0:
            found.append((at, name))
    return {i: name for i, (_, name) in enumerate(sorted(found))}


def parse(data: bytes, value_reader=None):
    """-> {key group: {"state": [(start, end, key, value)], "event": [(ts, key, start, end)],
    "processing": [...], "sets": [(key, [((start, end), (state start, state end))])],
    "count": [(start, end, key, count)]}}.  value_reader(Reader) decodes one state value
    (default: the Tuple2<String, Integer> of WindowOperatorMigrationTest's reducing state).
    Session snapshots also hold the MergingWindowSet ListState "merging-window-set"
    (MergingWindowSet.persist :99-106; namespace VoidNamespace = one byte,
    VoidNamespaceSerializer.java:62-70; value ListSerializer :118-128 = int n, then n
    Tuple2<TimeWindow, TimeWindow>) and, under a CountTrigger, its ReducingState<Long> "count"."""
    vr = value_reader or (lambda r: (r.jstring(), r.i32()))
    start, count, offs, be = keyed_state(data)
    ids = state_ids(be)
    out = {}
    for i in range(count):
        r = Reader(be, offs[i])
        end = offs[i + 1] if i + 1 < count else len(be)
        kg = r.i32()
        if kg != start + i:
            raise ValueError(f"key group {kg} at position {i}")
        sec = {"state": [], "event": [], "processing": [], "sets": [], "count": []}
        while r.p < end:
            name = ids[r.i16()]
            n = r.i32()
            for _ in range(n):
                if name == "window-contents":
                    s, e = r.i64(), r.i64()
                    k = r.jstring()
                    sec["state"].append((s, e, k, vr(r)))
                elif name == "merging-window-set":
                    if r.u8() != 0:
                        raise ValueError("VoidNamespace byte")
                    k = r.jstring()
                    sec["sets"].append((k, [((r.i64(), r.i64()), (r.i64(), r.i64())) for _ in range(r.i32())]))
                elif name == "count":
                    s, e = r.i64(), r.i64()
                    k = r.jstring()
                    sec["count"].append((s, e, k, r.i64()))
                else:
                    ts = r.i64() ^ -(1 << 63)
                    k = r.jstring()
                    s, e = r.i64(), r.i64()
                    sec["event" if name.endswith("event_window-timers") else "processing"].append((ts, k, s, e))
        if r.p != end:
            raise ValueError("key-group section overran its offset")
        out[kg] = sec
    return out


def migration_fixtures(kind="reduce-event-time"):
    """Paths of the committed fixtures of one kind ("reduce-event-time",
    "session-with-stateful-trigger"), by Flink version."""
    import glob
    import os
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_snapshots")
    out = {}
    for f in sorted(glob.glob(os.path.join(here, f"win-op-migration-test-{kind}-flink*-snapshot"))):
        out[f.split("-flink")[1].replace("-snapshot", "")] = f
    return out


def list_value(r):
    """ListState<Tuple2<String, Integer>> contents (ListSerializer: int n + the elements)."""
    return [(r.jstring(), r.i32()) for _ in range(r.i32())]


# WindowOperatorMigrationTest.writeSessionWindowsWithCountTriggerSnapshot (:97-152):
# EventTimeSessionWindows.withGap(3 s), PurgingTrigger(CountTrigger(4)), the records below
# (key, value, ts) in arrival order, no watermark, then the snapshot.
SESSION_MIGRATION_GAP = 3000
SESSION_MIGRATION_INPUT = [("key2", 1, 0), ("key2", 2, 1000), ("key2", 3, 2500), ("key2", 4, 3500),
                           ("key1", 1, 10), ("key1", 2, 1000)]


# WindowOperatorMigrationTest.java:407-426 (records, in arrival order) and the watermarks after them
MIGRATION_INPUT = [("key2", 1, 3999), ("key2", 1, 3000), ("key1", 1, 20), ("key1", 1, 0), ("key1", 1, 999),
                   ("key2", 1, 1998), ("key2", 1, 1999), ("key2", 1, 1000)]
MIGRATION_WATERMARKS = [999, 1999]
# :493-505: after the restore, watermarks 2999 .. 5999 fire these (key, sum, timestamp) rows
MIGRATION_RESTORE_WATERMARKS = [2999, 3999, 4999, 5999]
MIGRATION_EXPECTED = {2999: [("key1", 3, 2999), ("key2", 3, 2999)], 3999: [], 4999: [], 5999: [("key2", 2, 5999)]}


def to_gpuwin_blob(parsed, ids, java_hash, agg_code, assigner_code, size, slide, offset=0, max_parallelism=1,
                   acc_of=lambda v: struct.pack(">i", v[1])):
    """A parsed reference snapshot as a gw_snapshot version-4 blob (include/gpuwin.h) with key
    hashes: keys -> ids[key], each entry's key hash = java_hash(key), the accumulator from the
    state value (default: the Int field of the reduced Tuple2, IntSerializer)."""
    kgs = sorted(parsed)
    lo, hi = kgs[0], kgs[-1]
    pay, offs = b"", []
    for kg in range(lo, hi + 1):
        offs.append(len(pay))
        sec = parsed.get(kg, {"state": [], "event": []})
        part = struct.pack(">i", len(sec["state"]))
        for s, e, k, v in sec["state"]:
            part += struct.pack(">qqqi", s, e, ids[k], java_hash(k)) + acc_of(v)
        part += struct.pack(">i", 0)
        part += struct.pack(">i", len(sec["event"]))
        for ts, k, s, e in sec["event"]:
            part += struct.pack(">qqqq", ts ^ -(1 << 63), ids[k], s, e)
        pay += part
    offs.append(len(pay))
    hdr = struct.pack("<4sIii5q4i3q", b"GWS1", 4, agg_code, assigner_code, size, slide, offset, 0, 1,
                      max_parallelism, lo, hi, 0, 0, 0, len(pay))
    return hdr + struct.pack(f"<{len(offs)}q", *offs) + pay


def to_gpuwin_session_blob(parsed, ids, java_hash, agg_code, assigner_code, gap, max_parallelism=1):
    """A parsed reference session snapshot as a gw_snapshot version-4 blob with key hashes:
    "window-contents" entries (state window, key) with the sum of the listed elements' Int
    field as an IntSerializer accumulator, the merging window sets (window -> state window) and
    the event-time timers."""
    kgs = sorted(parsed)
    lo, hi = kgs[0], kgs[-1]
    pay, offs = b"", []
    for kg in range(lo, hi + 1):
        offs.append(len(pay))
        sec = parsed.get(kg, {"state": [], "sets": [], "event": []})
        part = struct.pack(">i", len(sec["state"]))
        for s, e, k, v in sec["state"]:
            part += struct.pack(">qqqii", s, e, ids[k], java_hash(k), sum(x[1] for x in v))
        part += struct.pack(">i", len(sec["sets"]))
        for k, ws in sec["sets"]:
            part += struct.pack(">qii", ids[k], java_hash(k), len(ws))
            for (s, e), (ss, se) in ws:
                part += struct.pack(">qqqq", s, e, ss, se)
        part += struct.pack(">i", len(sec["event"]))
        for ts, k, s, e in sec["event"]:
            part += struct.pack(">qqqq", ts ^ -(1 << 63), ids[k], s, e)
        pay += part
    offs.append(len(pay))
    hdr = struct.pack("<4sIii5q4i3q", b"GWS1", 4, agg_code, assigner_code, 0, 0, 0, gap, 1,
                      max_parallelism, lo, hi, 0, 0, 0, len(pay))
    return hdr + struct.pack(f"<{len(offs)}q", *offs) + pay

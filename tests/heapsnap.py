"""Decoder of snapshot blob version 4 (include/gpuwin.h gw_snapshot): the heap backend's
per-key-group layout of the window operator's keyed state (CopyOnWriteStateMapSnapshot.
writeState, CopyOnWriteStateMapSnapshot.java:127-149; timers as TimerSerializer.serialize
writes them, TimerSerializer.java:147-152).  Test helper: both the oracle and libgpuwin write
it, and the tests compare what they wrote as multisets."""
import struct

HDR = struct.Struct("<4sIii5q4i3q")
ACC_BYTES = {"sum_i32": 4, "avg_i64": 16, "avg_f64": 16}


def parse(blob: bytes, agg: str):
    """-> dict kg -> {"state": [(start, end, key, acc..., [key hash])], "sets": [(key, ((w, sw), ...), [key hash])],
    "timers": [(ts, key, start, end)]}; acc as raw big-endian ints (doubles by their bits)."""
    h = HDR.unpack(blob[:96])
    assert h[0] == b"GWS1" and h[1] == 4, h[:2]
    kg_lo, kg_hi, nbytes = h[10], h[11], h[15]
    hb = 4 if h[8] & 1 else 0  # flags: entries carry the key's hash after the key
    nk = kg_hi - kg_lo + 1
    offs = struct.unpack(f"<{nk + 1}q", blob[96:96 + 8 * (nk + 1)])
    pay = blob[96 + 8 * (nk + 1):]
    assert len(pay) == nbytes == offs[-1]
    ab = ACC_BYTES.get(agg, 8)
    out = {}
    for g in range(nk):
        p = offs[g]
        n, = struct.unpack_from(">i", pay, p); p += 4
        state = []
        for _ in range(n):
            s, e, k = struct.unpack_from(">qqq", pay, p); p += 24
            kh = struct.unpack_from(">i", pay, p) if hb else ()
            p += hb
            acc = struct.unpack_from(">i" if ab == 4 else (">qq" if ab == 16 else ">q"), pay, p); p += ab
            state.append((s, e, k) + acc + kh)
        m, = struct.unpack_from(">i", pay, p); p += 4
        sets = []
        for _ in range(m):  # (key, [be32 key hash,] be32 c, c x (window, state window))
            k, = struct.unpack_from(">q", pay, p); p += 8
            kh = struct.unpack_from(">i", pay, p) if hb else ()
            p += hb
            c, = struct.unpack_from(">i", pay, p); p += 4
            ws = [struct.unpack_from(">qqqq", pay, p + 32 * j) for j in range(c)]
            p += 32 * c
            sets.append((k, tuple(sorted(ws))) + kh)
        t, = struct.unpack_from(">i", pay, p); p += 4
        timers = []
        for _ in range(t):
            ts, k, s, e = struct.unpack_from(">qqqq", pay, p); p += 32
            timers.append((ts ^ -(1 << 63), k, s, e))
        assert p == offs[g + 1]
        out[kg_lo + g] = {"state": sorted(state), "sets": sorted(sets), "timers": sorted(timers)}
    return out


def normalize_sessions(sec):
    """One key group's session state with every entry filed under its window instead of its
    state window (the merging window set maps window -> state window, MergingWindowSet.java:
    116; the reference keeps a merged session's state under one of its original windows,
    :188-201, the GPU under the session itself): -> (state, sets) with sets as (key, windows)."""
    ns = {}
    for x in sec["sets"]:
        for (s, e, ss, se) in x[1]:
            ns[(x[0], ss, se)] = (s, e)
    state = []
    for x in sec["state"]:
        s, e = ns[(x[2], x[0], x[1])]
        state.append((s, e) + x[2:])
    sets = [(x[0], tuple((w[0], w[1]) for w in x[1])) + x[2:] for x in sec["sets"]]
    return sorted(state), sorted(sets)

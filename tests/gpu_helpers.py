"""Helpers for the GPU parity tests: drive libgpuwin.so (through flink_amd) and the CPU
oracle over the same seeded streams and compare the fired multisets.

Parity rule (BASELINE.json north_star): integer / count / min / max
results bit-exact; f64 sums and averages within 1e-6 relative.
"""
import numpy as np

from flink_amd import windowing as W

REL_TOL = 1e-6  # f64 sum/avg tolerance stated by BASELINE.json north_star


def make_assigner(kw):
    if kw["assigner"] == "tumbling":
        return W.TumblingEventTimeWindows.of(kw["size"], kw.get("offset", 0))
    if kw["assigner"] == "sliding":
        return W.SlidingEventTimeWindows.of(kw["size"], kw["slide"], kw.get("offset", 0))
    if kw["assigner"] == "count_tumbling":
        return W.CountWindows.of(kw["size"])
    if kw["assigner"] == "count_sliding":
        return W.CountWindows.of(kw["size"], kw["slide"])
    return W.EventTimeSessionWindows.with_gap(kw["gap"])


def gpu_operator(kw, capacity_hint=1024, flags=0, max_batch=1 << 22):
    trig = W.PurgingTrigger.of(W.EventTimeTrigger.create()) if kw.get("trigger") == "purging_event_time" \
        else W.EventTimeTrigger.create()
    return W.GpuWindowOperator(make_assigner(kw), kw["agg"], kw.get("lateness", 0), trig,
                               capacity_hint=capacity_hint, flags=flags, max_batch=max_batch).open()


def random_stream(seed, n, num_keys, n_batches, ts_step=7, disorder=300, wm_lag=300, agg="sum_i64",
                  key_offset=0, ts0=0):
    """Seeded stream: keys uniform, timestamps advancing with bounded disorder; the
    watermark after each batch is maxTs - wm_lag - 1 (BoundedOutOfOrdernessWatermarks,
    flink-core/.../eventtime/BoundedOutOfOrdernessWatermarks.java:57-69).  With
    disorder <= wm_lag no record is late."""
    rng = np.random.default_rng(seed)
    keys = rng.integers(0, num_keys, n).astype(np.int64) + key_offset
    base = ts0 + np.arange(n, dtype=np.int64) * ts_step
    ts = base - rng.integers(0, disorder + 1, n).astype(np.int64)
    if agg in ("sum_f64", "min_f64", "max_f64", "avg_f64"):
        vals = rng.uniform(0.0, 1000.0, n).astype(np.float64)
    elif agg == "sum_i32":
        vals = rng.integers(-(1 << 31), (1 << 31) - 1, n).astype(np.int64)
    else:
        vals = rng.integers(-(10 ** 6), 10 ** 6, n).astype(np.int64)
    cuts = np.linspace(0, n, n_batches + 1).astype(np.int64)
    batches = []
    for b in range(n_batches):
        lo, hi = cuts[b], cuts[b + 1]
        wm = int(ts[:hi].max()) - wm_lag - 1 if hi > 0 else W.LONG_MIN
        batches.append((lo, hi, wm))
    return keys, ts, vals, batches


def run_oracle(o, kw, keys, ts, vals, batches, final_wm=W.LONG_MAX):
    op = o.OracleOperator(o.make_config(**kw))
    outs = []
    vb = vals.view(np.int64) if vals.dtype == np.float64 else vals
    for lo, hi, wm in batches:
        op.process_batch(keys[lo:hi], ts[lo:hi], vb[lo:hi])
        op.process_watermark(wm)
        outs.append(op.drain())
    if final_wm is not None:
        op.process_watermark(final_wm)
        outs.append(op.drain())
    return outs, op.late_dropped


def run_gpu(kw, keys, ts, vals, batches, final_wm=W.LONG_MAX, **opkw):
    op = gpu_operator(kw, **opkw)
    outs = []
    try:
        for lo, hi, wm in batches:
            op.process_batch(keys[lo:hi], ts[lo:hi], vals[lo:hi])
            op.advance_watermark(wm)
            k, s, e, r = op.drain()
            outs.append((k, s, e, r.view(np.int64)))
        if final_wm is not None:
            op.advance_watermark(final_wm)
            k, s, e, r = op.drain()
            outs.append((k, s, e, r.view(np.int64)))
        late = op.num_late_records_dropped
        stats = op.stats()
        stats["fast_fires"] = op.kernel_time_ms(3)[1]  # fires enqueued behind their flush
    finally:
        op.close()
    return outs, late, stats


def compare(gpu_out, ora_out, is_double):
    """Per-watermark multiset comparison; returns a list of mismatch descriptions."""
    errs = []
    assert len(gpu_out) == len(ora_out)
    for b, (g, o) in enumerate(zip(gpu_out, ora_out)):
        gk = np.lexsort((g[2], g[1], g[0]))
        ok = np.lexsort((o[2], o[1], o[0]))
        G = [x[gk] for x in g]
        O = [x[ok] for x in o]
        if len(G[0]) != len(O[0]):
            errs.append(f"watermark #{b}: {len(G[0])} rows vs oracle {len(O[0])}")
            continue
        for c in range(3):
            if not np.array_equal(G[c], O[c]):
                i = int(np.nonzero(G[c] != O[c])[0][0])
                errs.append(f"watermark #{b}: column {c} differs at row {i}: "
                            f"gpu {[int(x[i]) for x in G[:3]]} oracle {[int(x[i]) for x in O[:3]]}")
                break
        else:
            if is_double:
                gv, ov = G[3].view(np.float64), O[3].view(np.float64)
                both_nan = np.isnan(gv) & np.isnan(ov)
                den = np.maximum(np.abs(gv), np.abs(ov))
                bad = ~both_nan & (np.abs(gv - ov) > REL_TOL * den) & ~(gv == ov)
                if bad.any():
                    i = int(np.nonzero(bad)[0][0])
                    errs.append(f"watermark #{b}: f64 result beyond 1e-6 rel at row {i}: {gv[i]!r} vs {ov[i]!r}")
            elif not np.array_equal(G[3], O[3]):
                i = int(np.nonzero(G[3] != O[3])[0][0])
                errs.append(f"watermark #{b}: result differs at row {i}: {int(G[3][i])} vs {int(O[3][i])} "
                            f"(key {int(G[0][i])} window [{int(G[1][i])},{int(G[2][i])}))")
    return errs


def corrupt_last_group(blob: bytes) -> bytes:
    """The blob with the window start of its last non-empty key group's first entry changed
    (a window of no assigner): the reader rejects it after parsing every earlier group."""
    import struct
    kg_lo, kg_hi = struct.unpack_from("<ii", blob, 60)
    nk = kg_hi - kg_lo + 1
    offs = np.frombuffer(blob[96:96 + 8 * (nk + 1)], np.int64)
    pay0 = 96 + 8 * (nk + 1)
    last = max(g for g in range(nk) if offs[g + 1] - offs[g] > 40)
    assert last > 0
    bad = bytearray(blob)
    bad[pay0 + int(offs[last]) + 4 + 7] ^= 1
    return bytes(bad)

"""minBy / maxBy in the CPU oracle (GW_FLAG_BY_FIELD; oracle/flink_oracle.c by_reduce), pinned to
the reference's own vectors: AggregationFunctionTest.minMaxByTest (flink-runtime/src/test/java/org/
apache/flink/streaming/api/AggregationFunctionTest.java:227-345, tests/golden/minmaxby.json), then
against a direct restatement of ComparableAggregator.reduce's byAggregate branch
(ComparableAggregator.java:88-95) folded per window in arrival order over random streams with many
equal fields (ties decide the element)."""
import numpy as np
import pytest

from tests.harness import load_golden

FLAG_BY_FIELD, FLAG_BY_LAST = 512, 1024  # include/gpuwin.h


def _flags(first):
    return FLAG_BY_FIELD | (0 if first else FLAG_BY_LAST)


@pytest.mark.parametrize("name", ["maxBy_first", "maxBy_last", "minBy_first", "minBy_last"])
@pytest.mark.parametrize("kind", ["i64", "f64"])
def test_golden_running_element(oracle_lib, name, kind):
    """The reference's running outputs: after element p, a window holding elements 0..p stands
    for expected[p]."""
    g = load_golden("minmaxby.json")
    inp = np.array(g["input"], dtype=np.int64)
    f = g["by_field"]
    agg = ("max_" if name.startswith("max") else "min_") + kind
    for p in range(len(inp)):
        op = oracle_lib.OracleOperator(oracle_lib.make_config(assigner="tumbling", size=1000, agg=agg,
                                                              flags=_flags(name.endswith("first"))))
        try:
            vals = inp[: p + 1, f]
            vals = vals.astype(np.float64).view(np.int64) if kind == "f64" else vals
            op.process_batch(inp[: p + 1, 0].copy(), np.arange(p + 1, dtype=np.int64), np.ascontiguousarray(vals))
            op.process_watermark(999)
            k, s, e, r, q = op.drain_seq()
        finally:
            op.close()
        assert len(k) == 1
        assert inp[q[0]].tolist() == g["expected"][name][p], (name, p)
        field = r.view(np.float64)[0] if kind == "f64" else r[0]
        assert field == g["expected"][name][p][f]


def _by_fold(keys, ts, vals, agg, first, size, slide, wm_list, batches):
    """Per (key, window): ComparableAggregator.reduce(byAggregate) in arrival order, fired when the
    watermark passes the window's end - 1 (lateness 0; late records dropped)."""
    is_max = agg.startswith("max")
    f64 = agg.endswith("f64")
    state, rows, wm = {}, [], -(1 << 63)
    for (lo, hi), w in zip(batches, wm_list):
        for i in range(lo, hi):
            t = int(ts[i])
            last_start = t - ((t % slide) + slide) % slide
            st = last_start
            while st > t - size:
                if st + size - 1 > wm:  # not late (cleanup time end - 1 > wm)
                    v = float(vals.view(np.float64)[i]) if f64 else int(vals[i])
                    cur = state.get((int(keys[i]), st))
                    if cur is None:
                        state[(int(keys[i]), st)] = (v, i)
                    else:
                        c = (1 if (v < cur[0] if is_max else v > cur[0]) else 0 if v == cur[0] else -1)
                        if not (c == 1 or (c == 0 and first)):
                            state[(int(keys[i]), st)] = (v, i)
                st -= slide
        wm = max(wm, w)
        for (k, st) in sorted([x for x in state if x[1] + size - 1 <= wm]):
            rows.append((k, st, state.pop((k, st))[1]))
    return sorted(rows)


@pytest.mark.parametrize("agg", ["max_i64", "min_i64", "max_f64", "min_f64"])
@pytest.mark.parametrize("first", [True, False])
@pytest.mark.parametrize("size,slide", [(100, 100), (300, 100)])
def test_oracle_matches_reduce_fold(oracle_lib, agg, first, size, slide):
    rng = np.random.default_rng(size + slide + (7 if first else 0) + len(agg))
    n = 3000
    keys = rng.integers(0, 12, n).astype(np.int64)
    ts = np.arange(n, dtype=np.int64) // 3 + rng.integers(0, 60, n)
    vals = rng.integers(0, 4, n).astype(np.int64)  # many ties
    if agg.endswith("f64"):
        vals = vals.astype(np.float64).view(np.int64)
    cuts = np.linspace(0, n, 11).astype(int)
    batches = [(int(cuts[b]), int(cuts[b + 1])) for b in range(10)]
    wms = [int(ts[: hi].max()) - 40 for _, hi in batches[:-1]] + [(1 << 63) - 1]
    exp = _by_fold(keys, ts, vals, agg, first, size, slide, wms, batches)
    op = oracle_lib.OracleOperator(oracle_lib.make_config(assigner="tumbling" if size == slide else "sliding",
                                                          size=size, slide=slide, agg=agg, flags=_flags(first)))
    got = []
    try:
        for (lo, hi), w in zip(batches, wms):
            op.process_batch(keys[lo:hi], ts[lo:hi], vals[lo:hi])
            op.process_watermark(w)
            k, s, e, r, q = op.drain_seq()
            got += list(zip(k.tolist(), s.tolist(), q.tolist()))
            assert all(r[j] == vals[q[j]] for j in range(len(q)))  # the row's field is its element's
    finally:
        op.close()
    assert sorted(got) == exp


def test_oracle_rejects_by_field_on_sums_and_sessions(oracle_lib):
    L = oracle_lib.lib()
    import ctypes
    for kw in (dict(assigner="tumbling", size=10, agg="sum_i64"), dict(assigner="session", gap=10, agg="max_i64")):
        cfg = oracle_lib.make_config(**kw, flags=FLAG_BY_FIELD)
        assert L.wo_validate(ctypes.byref(cfg)) != 0


@pytest.mark.parametrize("first", [True, False])
def test_oracle_snapshot_keeps_the_element(oracle_lib, first):
    """A minBy / maxBy snapshot holds each window's element (here its arrival number, flags bit 1):
    restored into a fresh operator, the run continues with the same rows and elements."""
    rng = np.random.default_rng(3)
    n = 4000
    keys = rng.integers(0, 20, n).astype(np.int64)
    ts = np.arange(n, dtype=np.int64) // 4
    vals = rng.integers(0, 3, n).astype(np.int64)
    cfg = oracle_lib.make_config(assigner="sliding", size=300, slide=100, agg="max_i64", flags=_flags(first))
    cuts = [(0, 1500, 300), (1500, 3000, 650), (3000, n, (1 << 63) - 1)]

    def run(cut):
        op = oracle_lib.OracleOperator(cfg)
        rows = []
        for b, (lo, hi, wm) in enumerate(cuts):
            if b == cut:
                blob = op.snapshot()
                op.close()
                op = oracle_lib.OracleOperator(cfg)
                op.restore(blob)
                op.set_arrival(lo)
            op.process_batch(keys[lo:hi], ts[lo:hi], vals[lo:hi])
            op.process_watermark(wm)
            k, s, e, r, q = op.drain_seq()
            rows.append(sorted(zip(k.tolist(), s.tolist(), r.tolist(), q.tolist())))
        op.close()
        return rows

    assert run(None) == run(1) == run(2)

"""Localise a restore row-count difference: sliding 600/200, lateness 900, snapshot after 11
batches, restored through per-key-group slices; plain min_i64, first-element min_i64 and minBy."""
import sys

import numpy as np

sys.path.insert(0, ".")
from flink_amd import _native as N  # noqa: E402
from flink_amd import windowing as W  # noqa: E402
from oracle import oracle as O  # noqa: E402
from tests.gpu_helpers import gpu_operator  # noqa: E402
from tests.test_gpu_minmaxby import _stream  # noqa: E402

O.build()
kw = dict(assigner="sliding", size=600, slide=200, lateness=900, agg="min_i64")
keys, ts, vals, payload, batches = _stream(91, "min_i64", n=24000, num_keys=150, n_batches=24, lateness=900)
allb = batches + [(len(keys), len(keys), W.LONG_MAX)]
ora = O.OracleOperator(O.make_config(**kw))
orows = []
for lo, hi, wm in allb:
    ora.process_batch(keys[lo:hi], ts[lo:hi], vals[lo:hi])
    ora.process_watermark(wm)
    k, s, e, r = ora.drain()
    orows.append(sorted(zip(k.tolist(), s.tolist(), r.tolist())))

for name, fl in (("plain", 0), ("first", N.FLAG_FIRST_ELEMENT), ("by", N.FLAG_BY_FIELD)):
    cut = 11
    pay = fl != 0
    a = gpu_operator(kw, flags=fl)
    g = []

    def run(op, bs):
        for lo, hi, wm in bs:
            if hi > lo:
                if pay:
                    op.process_batch_payload(keys[lo:hi], ts[lo:hi], vals[lo:hi], payload[lo:hi])
                else:
                    op.process_batch(keys[lo:hi], ts[lo:hi], vals[lo:hi])
            op.advance_watermark(wm)
            out = op.drain_payload() if pay else op.drain()
            g.append(sorted(zip(out[0].tolist(), out[1].tolist(), out[3].view(np.int64).tolist())))

    run(a, batches[:cut])
    blob = a.snapshot_state()
    a.close()
    b = gpu_operator(kw, flags=fl)
    b.initialize_state([N.snapshot_slice(blob, kg) for kg in range(128)])
    run(b, allb[cut:])
    b.close()
    bad = [i for i in range(len(orows)) if g[i] != orows[i]]
    print(name, "differing watermarks:", bad[:5], flush=True)
    for i in bad[:2]:
        go, oo = set(g[i]), set(orows[i])
        print("  wm", i, "gpu-only", sorted(go - oo)[:6], "oracle-only", sorted(oo - go)[:6], flush=True)

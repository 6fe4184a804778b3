"""Decode throughput of the network-buffer ingest (gw_decode_serialized) on a Q5-shaped
channel: Tuple2<Long, Long> (auction, price) records with timestamps, a watermark every
1M records.  Prints GB/s of serialized bytes; run under rocprofv3 --kernel-trace --stats
for the per-kernel split (k_nb_walk / k_nb_resolve / k_nb_scan / k_nb_decode).

    python scripts/netbuf_bench.py [--records 10000000] [--iters 10]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flink_amd import _native as N  # noqa: E402
from flink_amd import netbuf as NB  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=10_000_000)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--mode", choices=["decode", "operator"], default="decode",
                    help="decode: gw_decode_serialized alone; operator: gw_ingest_serialized_device into a "
                         "sliding 10s/2s sum operator (decode + ingest + fires)")
    a = ap.parse_args()
    import torch
    n = a.records
    rng = np.random.default_rng(1)
    k = rng.integers(0, 10_000_000, n)
    t = np.arange(n) // 50
    v = rng.integers(0, 1_000_000, n)
    step = 1_000_000
    data = NB.serialize_batches("JJ", 0, 1, [(k[i:i + step], t[i:i + step], v[i:i + step]) for i in range(0, n, step)],
                                [int(t[min(i + step, n) - 1]) - 100 for i in range(0, n, step)])
    d = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    cols = torch.empty((3, n), dtype=torch.int64, device="cuda")
    wm = torch.empty((2, n // step + 1), dtype=torch.int64, device="cuda")
    lay = N.record_layout("JJ", 0, 1)
    res = N.GwDecodeResult()
    P = lambda x: ctypes.c_void_p(x.data_ptr())
    L = N.lib()

    def once():
        N.check(L.gw_decode_serialized(P(d), len(data), ctypes.byref(lay), P(cols[0]), P(cols[1]), P(cols[2]), n,
                                       P(wm[0]), P(wm[1]), wm.shape[1], ctypes.byref(res), None))

    if a.mode == "operator":
        from flink_amd import windowing as W
        op = W.GpuWindowOperator(W.SlidingEventTimeWindows.of(10_000, 2_000), "sum_i64",
                                 capacity_hint=10_000_000, max_batch=2_000_000).open()

        def once():  # noqa: F811  (each call: the same bytes, the clock moved on by shifting watermarks)
            used, _ = op.process_serialized_device(d, lay)
            assert used == len(data)
            op.clear_rows()

    once()
    if a.mode == "operator":
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            once()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.iters
        print(json.dumps({"mode": "operator", "records": n, "bytes": len(data), "ms_per_call": dt * 1e3,
                          "records_per_s": n / dt, "stats": {k: v for k, v in op.stats().items()}
                          if isinstance(op.stats(), dict) else None}))
        op.close()
        return
    assert res.records == n and res.consumed == len(data)
    assert torch.equal(cols[0].cpu(), torch.from_numpy(k)) and torch.equal(cols[2].cpu(), torch.from_numpy(v))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        once()
    dt = (time.perf_counter() - t0) / a.iters
    out = {"records": n, "bytes": len(data), "ms_per_call_incl_alloc_sync": dt * 1e3,
           "GBps_serialized_in": len(data) / dt / 1e9, "records_per_s": n / dt,
           "algorithmic_bytes": len(data) + 24 * n}
    print(json.dumps(out))


if __name__ == "__main__":
    main()

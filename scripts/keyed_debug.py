"""Keyed vs slot sort session path on one stream: rows and late counts per watermark."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from gpu_helpers import random_stream, run_gpu  # noqa: E402


def main():
    agg = sys.argv[1] if len(sys.argv) > 1 else "count"
    kw = dict(assigner="session", gap=100, agg=agg)
    keys, ts, vals, batches = random_stream(seed=500, n=1_200_000, num_keys=60_000, n_batches=3, ts_step=1,
                                            disorder=800, wm_lag=400, agg=agg)
    out = {}
    for path, extra in [("sort", {}), ("keyed", {}), ("keyed", {"GW_KSEG_FAST": "0"}),
                        ("keyed", {"GW_SESSION_KEY_BITS": "32"}), ("keyed", {"GW_SESSION_SYNC": "1"})]:
        os.environ["GW_SESSION_PATH"] = path
        for k in ("GW_KSEG_FAST", "GW_SESSION_KEY_BITS", "GW_SESSION_SYNC"):
            os.environ.pop(k, None)
        os.environ.update(extra)
        for cap in (2048, 1 << 22):
            g, late, st = run_gpu(kw, keys, ts, vals, batches, capacity_hint=cap, max_batch=1 << 20)
            tag = f"{path}{extra} cap={cap}"
            print(tag, "late", late, "rows", [len(x[0]) for x in g], "punted", st.get("session_punted"),
                  "rehash", st.get("rehashes"), flush=True)


if __name__ == "__main__":
    main()

"""Host -> device bandwidth on the box for the host-fed leg's transfer shape: one batch of
Q5 columns (10M records x 24 B = 240 MB) from pinned host memory, as one copy, as chunks on
2 / 4 streams, and as a kernel that reads the pinned pages directly (torch's copy of a
mapped host tensor).  Run it under HSA_ENABLE_SDMA=0 as well to time the blit-kernel copy.
Prints one JSON line."""
import json
import os
import time

import torch


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def main():
    nbytes = 240 * 1000 * 1000
    src = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    src.fill_(1)
    dst = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    out = {"bytes": nbytes, "sdma": os.environ.get("HSA_ENABLE_SDMA", "default")}

    def one():
        dst.copy_(src, non_blocking=True)

    out["one_copy_gbs"] = nbytes / timed(one) / 1e9
    for ns in (2, 4, 8):
        streams = [torch.cuda.Stream() for _ in range(ns)]
        chunk = (nbytes + ns - 1) // ns

        def split(streams=streams, chunk=chunk):
            cur = torch.cuda.current_stream()
            for i, s in enumerate(streams):
                s.wait_stream(cur)
                with torch.cuda.stream(s):
                    dst[i * chunk:(i + 1) * chunk].copy_(src[i * chunk:(i + 1) * chunk], non_blocking=True)
            for s in streams:
                cur.wait_stream(s)

        out[f"split{ns}_gbs"] = nbytes / timed(split) / 1e9
    dsrc = torch.empty(nbytes, dtype=torch.uint8, device="cuda")

    def d2h():
        src.copy_(dsrc, non_blocking=True)

    out["d2h_gbs"] = nbytes / timed(d2h) / 1e9
    print(json.dumps(out))


if __name__ == "__main__":
    main()

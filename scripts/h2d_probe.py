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
    # the library's own pinned slots: hipHostMalloc with each flag set, copied as three
    # 80-MB columns with hipMemcpyAsync (what gw_stage_send does)
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    hip.hipHostFree.argtypes = [ctypes.c_void_p]
    stream = torch.cuda.current_stream().cuda_stream
    for name, flags in (("default", 0x0), ("noncoherent", 0x80000000), ("coherent", 0x40000000),
                        ("portable", 0x1)):
        ptr = ctypes.c_void_p()
        if hip.hipHostMalloc(ctypes.byref(ptr), nbytes, flags) != 0:
            out[f"hm_{name}"] = "alloc failed"
            continue
        ctypes.memset(ptr, 1, nbytes)
        col = nbytes // 3

        def three(ptr=ptr, col=col):
            for c in range(3):
                hip.hipMemcpyAsync(ctypes.c_void_p(dst.data_ptr() + c * col), ctypes.c_void_p(ptr.value + c * col),
                                   col, 1, ctypes.c_void_p(stream))

        out[f"hm_{name}_3col_gbs"] = nbytes / timed(three) / 1e9
        hip.hipHostFree(ptr)
    print(json.dumps(out))


if __name__ == "__main__":
    main()

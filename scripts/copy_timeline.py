"""Host<->device copy timeline from a rocprofv3 --memory-copy-trace CSV: the large copies
(>= 16 MB, the host-fed leg's columns and row drains) in time order, their rates, and how
busy the H2D direction is over the span of those copies.
Usage: python scripts/copy_timeline.py RUN_memory_copy_trace.csv"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    big = []
    for r in rows:
        n = int(r.get("Bytes") or r.get("Size") or 0)
        if n < 16 << 20:
            continue
        kind = r.get("Direction") or r.get("Operation") or r.get("Kind") or ""
        big.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n, kind))
    big.sort()
    if not big:
        print("no large copies")
        return
    t0 = big[0][0]
    h2d = [(s, e, n) for s, e, n, k in big if "HOST_TO_DEVICE" in k.upper() or "H2D" in k.upper()]
    for s, e, n, k in big[-60:]:
        print(f"{(s - t0) / 1e6:10.3f} ms  {(e - s) / 1e6:7.3f} ms  {n / 1e6:8.1f} MB  {n / (e - s):6.1f} GB/s  {k}")
    if h2d:
        span = h2d[-1][1] - h2d[0][0]
        busy = 0
        cur_s, cur_e = h2d[0][0], h2d[0][1]
        for s, e, _ in h2d[1:]:
            if s > cur_e:
                busy += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        busy += cur_e - cur_s
        tot = sum(n for _, _, n in h2d)
        print(f"H2D: {len(h2d)} copies, {tot / 1e9:.2f} GB over {span / 1e6:.2f} ms: busy {busy / span:.2%}, "
              f"{tot / span:.1f} GB/s over the span, {tot / busy:.1f} GB/s while busy")


if __name__ == "__main__":
    main()

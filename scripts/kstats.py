"""Readable table of a rocprofv3 `*_kernel_stats.csv` (kernel names shortened to the
function name and template arguments).

    python scripts/kstats.py gpurun_out/prof_x/run_kernel_stats.csv [--top 20]
"""
import argparse
import csv
import re


def short(name: str) -> str:
    name = re.sub(r"rocprim::ROCPRIM_\w+_NS::detail::", "rocprim::", name)
    m = re.match(r"(?:void )?([\w:]+(?:<[^()]*?>)?)\(", name)
    s = m.group(1) if m else name
    if "rocprim" in name:
        k = re.search(r"radix_sort_onesweep_(\w+)", name)
        s = "rocprim::radix_sort_onesweep_" + k.group(1) if k else s[:60]
    elif s.startswith("at::native"):
        s = s[:60]
    return s


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--top", type=int, default=20)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    agg = {}
    for r in rows:
        k = short(r["Name"])
        c, t = agg.get(k, (0, 0))
        agg[k] = (c + int(r["Calls"]), t + int(r["TotalDurationNs"]))
    total = sum(t for _, t in agg.values())
    print(f"{'kernel':64s} {'calls':>6s} {'total ms':>9s} {'avg us':>9s} {'%':>6s}")
    for k, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[: a.top]:
        print(f"{k:64s} {c:6d} {t / 1e6:9.2f} {t / c / 1e3:9.1f} {100 * t / total:6.2f}")


if __name__ == "__main__":
    main()

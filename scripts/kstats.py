"""Summarise a rocprofv3 kernel_stats.csv / kernel_trace.csv: top kernels, and per-grid breakdown of a name filter."""
import collections
import csv
import sys


def top(stats_csv, n=16):
    rows = list(csv.DictReader(open(stats_csv)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"{stats_csv}: total {tot / 1e6:.2f} ms")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
        print(f"{float(r['TotalDurationNs']) / 1e6:8.2f} ms {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:8.1f} us  "
              f"{r['Name'][:100]}")


def by_grid(trace_csv, pat):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(trace_csv)):
        if pat in r["Kernel_Name"]:
            d[(r["Kernel_Name"][:40], int(r["Grid_Size_X"]))].append(
                (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k, v in sorted(d.items()):
        print(f"{k[0]:40s} grid {k[1]:9d} n {len(v):5d} avg {sum(v) / len(v):8.1f} us")


if __name__ == "__main__":
    top(sys.argv[1], int(sys.argv[3]) if len(sys.argv) > 3 else 16)
    if len(sys.argv) > 2:
        by_grid(sys.argv[1].replace("kernel_stats", "kernel_trace"), sys.argv[2])

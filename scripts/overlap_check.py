#!/usr/bin/env python
"""Overlap of the gradient-bucket all-reduce launches with the backward, from a rocprofv3 kernel trace
(``--kernel-trace --output-format csv``): for every all-reduce kernel dispatch, how much of it ran while
a compute kernel of the same device was running, and how many started before the last compute kernel of
their step ended.

    python scripts/overlap_check.py gpurun_out/prof/run_kernel_trace.csv
"""
import csv
import sys


def main(path):
    rows = list(csv.DictReader(open(path)))
    ks = []
    for r in rows:
        name = r.get("Kernel_Name") or r.get("KernelName") or r.get("Name")
        b, e = int(r.get("Start_Timestamp") or r["BeginNs"]), int(r.get("End_Timestamp") or r["EndNs"])
        ks.append((b, e, name))
    ks.sort()
    ar = [k for k in ks if "xgmi" in k[2] or "allreduce" in k[2].lower()]
    comp = [k for k in ks if k not in ar and "optim" not in k[2]]
    over = total = started_inside = 0
    for b, e, n in ar:
        total += e - b
        for cb, ce, cn in comp:
            if ce <= b or cb >= e:
                continue
            over += min(e, ce) - max(b, cb)
        if any(cb < b < ce for cb, ce, _ in comp):
            started_inside += 1
    print(f"all-reduce dispatches: {len(ar)}  total {total / 1e3:.1f} us  overlapped with compute "
          f"{over / 1e3:.1f} us ({100.0 * over / max(total, 1):.1f} %)  started while a compute kernel ran: "
          f"{started_inside}")


if __name__ == "__main__":
    main(sys.argv[1])

"""One training step of a rocprofv3 kernel_trace.csv, split at a kernel that runs once per step (default: the
optimizer, ``optim_apply``): per-kernel-class time of that step, optionally every launch in order.

    python scripts/step_timeline.py gpurun_out/x/resnet18_kernel_trace.csv [--marker optim_apply] [--list]
"""
import argparse
import csv

AKIND = {"0": "dense", "1": "fwd", "2": "dgrad", "3": "colm", "4": "wgrad"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="optim_apply")
    ap.add_argument("--list", action="store_true")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    if len(idx) < 3:
        raise SystemExit(f"fewer than 3 '{a.marker}' launches in {a.trace}")
    step = rows[idx[-3] + 1: idx[-2] + 1]
    cat, tot, prev = {}, 0.0, int(rows[idx[-3]]["End_Timestamp"])
    gaps = 0.0
    for r in step:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        d = (e - s) / 1e3
        tot += d
        gaps += max(s - prev, 0) / 1e3
        prev = e
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("tde::", "")
        key = name.split("<")[0]
        if key == "igemm_kernel":
            key += "_" + AKIND.get(name.split("<")[1].split(",")[0].strip(), "?")
        c = cat.setdefault(key, [0, 0.0])
        c[0] += 1
        c[1] += d
        if a.list:
            print(f"{d:7.1f} us  {name[:70]} grid={r['Grid_Size_X']}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']}")
    print(f"one step: {len(step)} launches, {tot:.1f} us of kernels, {gaps:.1f} us of gaps")
    for k, (n, t) in sorted(cat.items(), key=lambda x: -x[1][1]):
        print(f"{t:8.1f} us {n:4d}x  {k}")


if __name__ == "__main__":
    main()

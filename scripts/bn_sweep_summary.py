"""Per-step BN kernel time of each scripts/sweep_bn.sh configuration (steps = optimizer launches)."""
import csv
import glob
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
for d in sorted(glob.glob(os.path.join(root, "bn_sweep_*")), key=lambda p: int(p.rsplit("_", 1)[1]) if p.rsplit("_", 1)[1].isdigit() else 0):
    f = os.path.join(d, "run_kernel_stats.csv")
    if not os.path.exists(f):
        continue
    rows = list(csv.DictReader(open(f)))
    steps = sum(int(r["Calls"]) for r in rows if "optim_apply" in r["Name"]) or 1
    tot = sum(float(r["TotalDurationNs"]) for r in rows) / steps / 1e3
    per = {}
    for r in rows:
        if "bn_" in r["Name"]:
            k = r["Name"].split("(")[0].split("::")[-1]
            per[k] = per.get(k, 0.0) + float(r["TotalDurationNs"]) / steps / 1e3
    bn = sum(per.values())
    print(f"{os.path.basename(d)}: steps {steps} total {tot:.0f} us/step  BN {bn:.0f} us/step  " +
          "  ".join(f"{k} {v:.0f}" for k, v in sorted(per.items())))

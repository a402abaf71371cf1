"""Print the per-dispatch mean of every counter in rocprofv3 counter_collection CSVs under the given dirs."""
import collections
import csv
import glob
import sys

for d in sys.argv[1:]:
    tot = collections.defaultdict(float)
    n = collections.defaultdict(set)
    dur = {}
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "halo" not in r["Kernel_Name"] and "igemm" not in r["Kernel_Name"]:
                continue
            did = r.get("Dispatch_Id") or r.get("Correlation_Id")
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
            n[r["Counter_Name"]].add(did)
            dur[did] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    print(d, "dispatches", len(dur), "mean dur us", round(sum(dur.values()) / max(len(dur), 1) / 1e3, 2))
    for k in sorted(tot):
        print(f"  {k:32s} {tot[k] / max(len(n[k]), 1):.4g}")

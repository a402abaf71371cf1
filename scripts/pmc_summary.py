"""Summarise the rocprofv3 counter passes of scripts/pmc_models.sh into one markdown table per model.

    python scripts/pmc_summary.py gpurun_out [models...] > profiles/r4_pmc_summary.md

Each pass directory gpurun_out/pmc_<model>_p<i>/ holds a *counter_collection.csv (one row per dispatch and
counter).  Per kernel (summed over its dispatches) the table gives:
  dur        mean dispatch time from the counter rows' timestamps (the counter run serialises dispatches,
             so this is a little longer than in a graph replay)
  MFMA %     SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs * dur * 2.4 GHz).  SQ_VALU_MFMA_BUSY_CYCLES is the sum
             over SIMDs of matrix-core busy cycles: it equals SQ_INSTS_MFMA x 32 for these kernels, whose
             MFMAs are all v_mfma_f32_16x16x4_f32 (8 passes = 32 cycles)
  TF/s       f32 matrix FLOP rate = MFMA busy cycles x 64 FLOP / dur (157 TF/s = every SIMD busy)
  wait %     SQ_WAIT_ANY / SQ_WAVE_CYCLES (waves parked on s_waitcnt / barriers)
  LDS conf.  SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS (bank-conflict cycles per LDS-issue cycle)
  HBM        (FETCH_SIZE + WRITE_SIZE) per dispatch, and that over the dispatch time
"""
import collections
import csv
import glob
import os
import sys

CUS, XCDS, CLK = 256, 8, 2.4   # CUs, XCDs, shader clock in GHz (cycles per ns)


def load(pass_dir):
    """{kernel: {counter: total}}, {kernel: [durations ns]} of one pass directory."""
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    durs = collections.defaultdict(dict)
    for f in glob.glob(os.path.join(pass_dir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
            d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            durs[k][r.get("Dispatch_Id") or r.get("Correlation_Id")] = d
    return tot, durs


def summarise(root, model):
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    durs = collections.defaultdict(dict)
    for p in sorted(glob.glob(os.path.join(root, f"pmc_{model}_p*"))):
        t, d = load(p)
        tag = os.path.basename(p)
        for k, cs in t.items():
            for c, v in cs.items():
                if c == "GRBM_GUI_ACTIVE":
                    c = f"GRBM_GUI_ACTIVE@{tag}"
                tot[k][c] += v
        for k, dd in d.items():
            for i, v in dd.items():
                durs[k][(tag, i)] = v
    rows = []
    for k, cs in tot.items():
        n1 = sum(1 for (tag, _) in durs[k] if tag.endswith("_p1"))
        dl = list(durs[k].values())
        dur = sum(dl) / len(dl) if dl else 0.0
        mb = cs.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / max(n1, 1)        # per dispatch
        mfma = 100.0 * mb / (CUS * 4 * dur * CLK) if dur else 0.0
        busy = mb * 64 / dur / 1e3 if dur else 0.0                       # TFLOP/s (FLOP / ns / 1e3)
        wave = cs.get("SQ_WAVE_CYCLES", 0.0)
        wait = 100.0 * cs.get("SQ_WAIT_ANY", 0.0) / wave if wave else 0.0
        lds_act = cs.get("SQ_ACTIVE_INST_LDS", 0.0)
        conf = cs.get("SQ_LDS_BANK_CONFLICT", 0.0) / lds_act if lds_act else 0.0
        n3 = max(1, sum(1 for (tag, _) in durs[k] if tag.endswith("_p3")))
        n4 = max(1, sum(1 for (tag, _) in durs[k] if tag.endswith("_p4")))
        fetch = cs.get("FETCH_SIZE", 0.0) * 1024 / n3
        write = cs.get("WRITE_SIZE", 0.0) * 1024 / n4
        gbs = (fetch + write) / dur if dur else 0.0   # bytes / ns = GB/s
        rows.append((dur * max(n1, 1), k, n1, dur, mfma, busy, wait, conf, fetch + write, gbs,
                     cs.get("SQ_INSTS_MFMA", 0.0) / max(n1, 1)))
    rows.sort(key=lambda r: -r[0])
    print(f"\n## {model}\n")
    print("| kernel | dispatches | dur µs | MFMA % | TF/s | wait % | LDS conf. | HBM / dispatch | HBM GB/s | MFMA insts / dispatch |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for (_, k, n, dur, mfma, busy, wait, conf, hb, gbs, mi) in rows[:12]:
        name = k if len(k) <= 70 else k[:67] + "..."
        print(f"| `{name}` | {n} | {dur / 1e3:.2f} | {mfma:.1f} | {busy:.1f} | {wait:.0f} | {conf:.2f} | "
              f"{hb / 1e6:.2f} MB | {gbs:.0f} | {mi:.0f} |")


if __name__ == "__main__":
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
    models = sys.argv[2:] or ["mnist_cnn", "mnist_bn_cnn", "lenet5", "mnist_mlp"]
    print("# rocprofv3 counter summary (MI355X)\n")
    print(__doc__.split("\n\n", 1)[1])
    for m in models:
        summarise(root, m)

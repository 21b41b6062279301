"""Average clock of the heaviest kernels from a rocprofv3 run with
``--pmc GRBM_GUI_ACTIVE --kernel-trace -f csv``: GRBM_GUI_ACTIVE cycles over
the dispatch's duration (relative comparison between runs: a lower value in
the sustained training step than in a short isolated bench = the chip runs
slower clocks there).  usage: pmc_clock.py <dir with the csv files>"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(d):
    cc = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not cc or not kt:
        print("csv files not found:", os.listdir(d))
        return
    dur = {}
    for r in csv.DictReader(open(kt[0])):
        dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), r["Kernel_Name"])
    cyc = defaultdict(float)
    for r in csv.DictReader(open(cc[0])):
        if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
            cyc[r["Dispatch_Id"]] += float(r["Counter_Value"])
    agg = defaultdict(lambda: [0.0, 0.0, 0])
    for k, c in cyc.items():
        if k not in dur:
            continue
        ns, name = dur[k]
        name = name.replace("(anonymous namespace)::", "").split("(")[0][:48]
        a = agg[name]
        a[0] += c
        a[1] += ns
        a[2] += 1
    for name, (c, ns, n) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:12]:
        print(f"{name:<48} n={n:<4} time {ns / 1e6:8.2f} ms  GRBM_GUI_ACTIVE/ns = {c / max(ns, 1):.3f}")


if __name__ == "__main__":
    main(sys.argv[1])

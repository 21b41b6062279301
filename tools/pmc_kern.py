"""Per-(kernel, grid) averages of rocprofv3 --pmc counter CSVs:
python tools/pmc_kern.py <dir-with-pN/run_counter_collection.csv> [name-substring]"""
import collections
import csv
import glob
import os
import sys


def main(d, pat=""):
    for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
        agg = collections.defaultdict(lambda: collections.defaultdict(float))
        disp = collections.defaultdict(set)
        for r in csv.DictReader(open(f)):
            if pat not in r["Kernel_Name"]:
                continue
            k = (r["Kernel_Name"].split("(")[0][-48:], r["Grid_Size"], r["Workgroup_Size"])
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
        for k, v in agg.items():
            n = len(disp[k])
            print(os.path.basename(os.path.dirname(f)), k, {c: round(x / n, 1) for c, x in sorted(v.items())})


if __name__ == "__main__":
    main(*sys.argv[1:])

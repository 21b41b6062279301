"""Summarise a rocprofv3 --pmc CSV run: per kernel name, the mean of each
counter over its dispatches plus derived ratios (wave-state split, MFMA busy
share, effective clock from GRBM_GUI_ACTIVE over the dispatch wall time)."""
import collections
import csv
import glob
import sys


def main(d):
    f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    if not f:
        print("no counter_collection.csv under", d)
        return
    rows = list(csv.DictReader(open(f[0])))
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    wall = {}
    for r in rows:
        k = r.get("Kernel_Name", "?")[:70]
        did = r.get("Dispatch_Id")
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        if "Start_Timestamp" in r and "End_Timestamp" in r:
            wall.setdefault(k, {})[did] = (float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
    for k, c in acc.items():
        m = {n: sum(v) / len(v) for n, v in c.items()}
        print(k)
        for n in sorted(m):
            print(f"   {n:28s} {m[n]:.4g}")
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if n in m:
                    print(f"   {n + ' / WAVE_CYCLES':40s} {m[n] / wc:.3f}")
        if k in wall and "GRBM_GUI_ACTIVE" in m:
            w = sum(wall[k].values()) / len(wall[k])
            print(f"   wall ns {w:.0f}   eff clock GHz {m['GRBM_GUI_ACTIVE'] / 8 / w:.2f}")
            if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
                print(f"   MFMA busy share (of 1024 SIMDs x GUI cycles/8) "
                      f"{m['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024 * m['GRBM_GUI_ACTIVE'] / 8):.3f}")


if __name__ == "__main__":
    main(sys.argv[1])

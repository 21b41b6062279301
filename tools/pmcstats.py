#!/usr/bin/env python
"""Summarise a rocprofv3 --pmc counter_collection.csv: per (kernel, grid)
sums of each counter and the wave-cycle breakdown
(WAIT_ANY / WAIT_INST_ANY / ACTIVE_INST_ANY as fractions of WAVE_CYCLES)."""
import csv
import sys
from collections import defaultdict


def main(path, match=""):
    agg = defaultdict(lambda: defaultdict(float))
    n = defaultdict(set)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:60]
        if match and match not in name:
            continue
        key = (name, int(r["Grid_Size"]) // max(int(r["Workgroup_Size"]), 1), r["VGPR_Count"], r["Accum_VGPR_Count"])
        agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
        n[key].add(r["Dispatch_Id"])
    for key, c in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        wc = c.get("SQ_WAVE_CYCLES", 0) or 1
        parts = [f"{k[3:]}={v / wc:.2f}" for k, v in c.items() if k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                                                                           "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS")]
        mf = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(c.get("SQ_BUSY_CYCLES", 1), 1)
        bc = c.get("SQ_LDS_BANK_CONFLICT", 0)
        print(f"{key[0]:<40} wg={key[1]:<7} vgpr={key[2]}/{key[3]} n={len(n[key])} "
              f"mfma/busy={mf:.2f} ldsconf={bc:.3g} " + " ".join(parts))
        print("    " + " ".join(f"{k}={v:.4g}" for k, v in sorted(c.items())))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")

"""Per-kernel hardware counters of the whole training step, from three
rocprofv3 ``--pmc ... --kernel-trace -f csv`` passes over ``bench.py``
(tools/gpu_step_pmc.sh): for every (kernel, grid) that holds >= 0.5 % of the
step's kernel time, the mean dispatch time, the effective clock, the MFMA
utilisation, the LDS bank-conflict share and the HBM-side read / write rate.

  clock   = GRBM_GUI_ACTIVE / 8 XCDs / wall time
  MFMA    = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)

GRBM_GUI_ACTIVE counts over the profiler's counter window, which brackets the
dispatch with a few microseconds of its own: for short dispatches the window
is longer than the kernel and the ratio above reads as an impossible clock
(>2.4 GHz, the part's peak).  Those rows print the clock as "-" and take the
MFMA denominator from the wall time at the peak clock instead (a lower bound
of the utilisation).
  LDS-cf  = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  rd, wr  = 2 x FETCH_SIZE (gfx950 tallies 128-B requests at 64 B), WRITE_SIZE;
            KiB per dispatch over its wall time; L3 (Infinity Cache) hits are
            counted, so this is fabric-side traffic, an upper bound on HBM bytes.

Dispatches are serialised under --pmc, so the times are per kernel without
stream co-residency.  usage: pmc_step_table.py <p1 dir> <p2 dir> <p3 dir>"""
import csv
import glob
import os
import sys
from collections import defaultdict

PEAK_GHZ = 2.4          # MI355X peak engine clock


def load(d):
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    cc = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not kt or not cc:
        return {}, {}
    meta = {}
    for r in csv.DictReader(open(kt[0])):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:44]
        wg = int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"])
        grid = (int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])) // max(wg, 1)
        meta[r["Dispatch_Id"]] = ((name, grid), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    cnt = defaultdict(lambda: defaultdict(float))
    for r in csv.DictReader(open(cc[0])):
        cnt[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    t = defaultdict(lambda: [0, 0.0])
    c = defaultdict(lambda: defaultdict(float))
    for did, (key, ns) in meta.items():
        t[key][0] += 1
        t[key][1] += ns
        for n, v in cnt.get(did, {}).items():
            c[key][n] += v
    return t, c


def main(p1, p2, p3):
    t1, c1 = load(p1)
    _, c2 = load(p2)
    t3, c3 = load(p3)
    t2, _ = load(p2)
    total = sum(v[1] for v in t1.values())
    print(f"{'kernel':<44} {'blocks':>7} {'n':>4} {'us':>8} {'%step':>6} {'GHz':>5} {'MFMA%':>6} {'LDScf%':>6} "
          f"{'rd GB/s':>8} {'wr GB/s':>8}")
    for key, (n, ns) in sorted(t1.items(), key=lambda kv: -kv[1][1]):
        if ns < 0.005 * total:
            continue
        a = c1[key]
        gui = a.get("GRBM_GUI_ACTIVE", 0.0)
        ghz = gui / 8 / ns if ns else 0.0
        if ghz > PEAK_GHZ * 1.02:           # counter window longer than the dispatch (see the module doc)
            ghz_s = "    -"
            cyc = ns * PEAK_GHZ
        else:
            ghz_s = f"{ghz:5.2f}"
            cyc = gui / 8
        mfma = a.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (1024 * cyc) * 100 if cyc else 0.0
        lds = a.get("SQ_LDS_IDX_ACTIVE", 0.0)
        ldscf = a.get("SQ_LDS_BANK_CONFLICT", 0.0) / lds * 100 if lds else 0.0
        rd = wr = float("nan")
        if key in t2 and t2[key][1]:
            rd = 2 * c2[key].get("FETCH_SIZE", 0.0) * 1024 / t2[key][1]
        if key in t3 and t3[key][1]:
            wr = c3[key].get("WRITE_SIZE", 0.0) * 1024 / t3[key][1]
        print(f"{key[0]:<44} {key[1]:>7} {n:>4} {ns / n / 1e3:8.1f} {ns / total * 100:6.1f} {ghz_s} {mfma:6.1f} "
              f"{ldscf:6.2f} {rd:8.0f} {wr:8.0f}")


if __name__ == "__main__":
    main(*sys.argv[1:4])

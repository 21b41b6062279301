"""Idle gaps of a replayed step by queue: for every gap (no kernel running on
any queue) of a rocpd database, the kernel that ended last (and its queue) and
the kernel that started next (and its queue); aggregated by (before, after)
pair.  Shows which cross-queue dependency edges leave the device idle.

usage: python tools/gap_streams.py run_results.db [t0_frac]  (window: two replayed steps)"""
import collections
import sqlite3
import sys


def main():
    db = sqlite3.connect(sys.argv[1])
    frac = float(sys.argv[2]) if len(sys.argv) > 2 else 0.5
    ks = sorted(db.execute("select start, end, name, queue_id from kernels"))
    la = sorted(db.execute("select start, end from regions where name like 'hipGraphLaunch%'"))
    if len(la) >= 4:
        # the replayed steps between the 4th-last and the 2nd-last graph launch
        t0, t1 = la[-4][0], la[-2][0]
    else:
        t0, t1 = ks[0][0] + (ks[-1][1] - ks[0][0]) * frac, ks[-1][1]
    ks = [k for k in ks if t0 <= k[0] < t1]
    qn = collections.Counter(k[3] for k in ks)
    print("kernels per queue:", dict(qn))
    agg = collections.defaultdict(lambda: [0, 0.0])
    busy_end, last = ks[0][1], ks[0]
    tot = 0.0
    for k in ks[1:]:
        if k[0] > busy_end:
            gap = (k[0] - busy_end) / 1e3
            key = (last[2].split("(")[0][-40:], last[3], k[2].split("(")[0][-40:], k[3])
            agg[key][0] += 1
            agg[key][1] += gap
            tot += gap
        if k[1] > busy_end:
            busy_end, last = k[1], k
    span = (ks[-1][1] - ks[0][0]) / 1e3
    print(f"span {span:.0f} us, idle {tot:.0f} us ({100 * tot / span:.1f} %)")
    for key, (n, g) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:25]:
        print(f"{g:9.1f} us {n:5d} x {g / n:7.1f}  q{key[1]} {key[0]:>40s} -> q{key[3]} {key[2]}")


if __name__ == "__main__":
    main()

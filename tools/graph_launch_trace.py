"""Where does the replayed step wait?  Joins the HIP-runtime trace with the
kernel trace of a rocprofv3 database (``--kernel-trace --hip-runtime-trace``):
for the last N hipGraphLaunch calls it prints, relative to the call's start,
when the call returned, when the first kernel of that step started and when
the previous step's last kernel ended -- i.e. whether the device idles at a
step boundary because the host enqueues late (launch returns late / starts
late) or because the launch itself needs long before its first packet.

usage: python tools/graph_launch_trace.py run_results.db [N]"""
import sqlite3
import sys


def main():
    db = sqlite3.connect(sys.argv[1])
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    views = [r[0] for r in db.execute("select name from sqlite_master where type in ('table','view')")]
    reg = "regions" if "regions" in views else None
    if reg is None:
        print("views:", views)
        return
    cols = [r[1] for r in db.execute(f"pragma table_info({reg})")]
    nm = "name" if "name" in cols else cols[0]
    launches = [r for r in db.execute(f"select {nm}, start, end from {reg} where {nm} like 'hipGraphLaunch%' "
                                      "order by start")]
    apis = sorted(db.execute(f"select {nm}, start, end from {reg} order by start"), key=lambda r: r[1])
    kcols = [r[1] for r in db.execute("pragma table_info(kernels)")]
    kn = "kernel_name" if "kernel_name" in kcols else "name"
    ks = sorted((r[1], r[2], r[0]) for r in db.execute(f"select {kn}, start, end from kernels"))
    print(f"{len(launches)} hipGraphLaunch calls, {len(ks)} kernels, {len(apis)} API calls")
    import bisect
    starts = [k[0] for k in ks]
    for name, s, e in launches[-n:]:
        i = bisect.bisect_left(starts, s)
        first_after = ks[i] if i < len(ks) else None
        # the device's last kernel end before this launch's first kernel
        prev_end = max((k[1] for k in ks[max(0, i - 400):i]), default=s)
        # host API calls between the previous launch's return and this launch
        print(f"launch at {s / 1e6:.3f} ms: returns +{(e - s) / 1e3:.1f} us; first kernel after call "
              f"+{(first_after[0] - s) / 1e3:.1f} us ({first_after[2][:40] if first_after else '-'}); "
              f"device busy until +{(prev_end - s) / 1e3:.1f} us when called")
    # host-side API timeline between two consecutive launches
    if len(launches) >= 2:
        a, b = launches[-2], launches[-1]
        between = [r for r in apis if a[2] <= r[1] < b[1]]
        print(f"host calls between the last two launches ({(b[1] - a[2]) / 1e3:.1f} us):")
        for r in between[:40]:
            print(f"   +{(r[1] - a[2]) / 1e3:8.1f} us  {(r[2] - r[1]) / 1e3:8.1f} us  {r[0]}")


if __name__ == "__main__":
    main()

"""Per-queue kernel timeline of one step from a rocpd database: the first and
last ``ms`` milliseconds of the second-to-last step (steps split at the
optimizer's adam kernels), one line per kernel with queue, start, duration.

usage: python tools/step_timeline.py run_results.db [ms]"""
import sqlite3
import sys


def main():
    db = sqlite3.connect(sys.argv[1])
    ms = float(sys.argv[2]) if len(sys.argv) > 2 else 6.0
    ks = sorted(db.execute("select start, end, name, queue_id from kernels"))
    marks = [k[0] for k in ks if "adam" in k[2]]
    # step boundaries: first adam kernel of each update
    bounds = [marks[0]] + [m for a, m in zip(marks, marks[1:]) if m - a > 5e6]
    t0, t1 = bounds[-3], bounds[-2]
    step = [k for k in ks if t0 <= k[0] < t1]
    print(f"step {(t1 - t0) / 1e6:.2f} ms, {len(step)} kernels")
    for lo, hi, tag in ((t0, t0 + ms * 1e6, "start"), (t1 - ms * 1e6, t1, "end")):
        print(f"== {tag}")
        for k in step:
            if lo <= k[0] < hi:
                nm = k[2].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:60]
                print(f"  q{k[3]} {(k[0] - t0) / 1e3:9.1f} us +{(k[1] - k[0]) / 1e3:8.1f}  {nm}")


def idle_report(path, min_us=10.0, top=20):
    """Busy time per queue over the same step, and the main (most-kernel)
    queue's idle intervals: what it ran before and after each one."""
    import collections
    db = sqlite3.connect(path)
    ks = sorted(db.execute("select start, end, name, queue_id from kernels"))
    marks = [k[0] for k in ks if "adam" in k[2]]
    bounds = [marks[0]] + [m for a, m in zip(marks, marks[1:]) if m - a > 5e6]
    t0, t1 = bounds[-3], bounds[-2]
    step = [k for k in ks if t0 <= k[0] < t1]
    per_q = collections.defaultdict(list)
    for k in step:
        per_q[k[3]].append(k)
    main_q = max(per_q, key=lambda q: len(per_q[q]))
    span = (t1 - t0) / 1e3
    for q, lst in sorted(per_q.items()):
        busy = sum(k[1] - k[0] for k in lst) / 1e3
        print(f"queue {q}: {len(lst)} kernels, busy {busy:.0f} us of {span:.0f} ({100 * busy / span:.1f} %)")
    m = per_q[main_q]
    gaps = []
    for a, b in zip(m, m[1:]):
        g = (b[0] - a[1]) / 1e3
        if g >= min_us:
            gaps.append((g, a, b))
    tot = sum(g for g, _, _ in gaps)
    print(f"main queue {main_q}: {len(gaps)} idle intervals >= {min_us} us, {tot:.0f} us in total")
    nm = lambda k: k[2].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:44]
    for g, a, b in sorted(gaps, reverse=True)[:top]:
        print(f"  {g:8.1f} us at {(a[1] - t0) / 1e3:9.1f}: {nm(a):44s} -> {nm(b)}")


if __name__ == "__main__" and len(sys.argv) > 3 and sys.argv[3] == "idle":
    idle_report(sys.argv[1])
elif __name__ == "__main__":
    main()

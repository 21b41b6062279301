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


if __name__ == "__main__":
    main()

#!/usr/bin/env python
"""Summarise a rocprofv3 rocpd database (kernel trace): per-kernel-name total
time, calls, avg, and grid size buckets.  ``python tools/rpstats.py run_results.db [--steps K]``"""
import argparse
import sqlite3
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=0, help="divide totals by K (per-step ms)")
    ap.add_argument("--top", type=int, default=45)
    ap.add_argument("--grid", action="store_true", help="split rows by grid size")
    ap.add_argument("--window", type=float, default=0.0,
                    help="only kernels that start within the last WINDOW ms of the trace (steady-state steps; "
                         "warm-up / capture passes excluded)")
    ap.add_argument("--busy", type=float, default=0.0,
                    help="occupancy of the last BUSY ms of the trace: union of kernel intervals vs span vs the sum "
                         "of kernel times (>1 overlap factor = concurrent kernels)")
    ap.add_argument("--solo", type=float, default=0.0,
                    help="over the last SOLO ms: per kernel, the time it ran ALONE on the device (exposed, on the "
                         "critical path) vs overlapped with another kernel (hidden behind / sharing the chip)")
    ap.add_argument("--gaps", type=float, default=0.0,
                    help="over the last GAPS ms: device-idle gaps (no kernel running) summed by the (kernel before, "
                         "kernel after) pair -- where the replayed step leaves the GPU idle")
    a = ap.parse_args()
    db = sqlite3.connect(a.db)
    cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
    name_col = "kernel_name" if "kernel_name" in cols else "name"
    gx = "grid_x" if "grid_x" in cols else None
    q = f"select {name_col}, start, end" + (f", {gx}, grid_y, grid_z, workgroup_x" if gx else "") + " from kernels"
    if a.busy:
        iv = sorted((r[1], r[2]) for r in db.execute(f"select {name_col}, start, end from kernels"))
        end = max(e for _, e in iv)
        lo = end - a.busy * 1e6
        iv = [(max(s0, lo), e) for s0, e in iv if e > lo]
        tot = sum(e - s0 for s0, e in iv)
        busy, cur_s, cur_e, gaps = 0, None, None, []
        for s0, e in iv:
            if cur_e is None or s0 > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                    gaps.append(s0 - cur_e)
                cur_s, cur_e = s0, e
            else:
                cur_e = max(cur_e, e)
        busy += cur_e - cur_s
        span = end - lo
        gaps.sort()
        print(f"window {span * 1e-6:.2f} ms: busy (union) {busy * 1e-6:.2f} ms = {100 * busy / span:.1f}%, "
              f"kernel sum {tot * 1e-6:.2f} ms (overlap x{tot / max(busy, 1):.2f}), {len(iv)} kernels, "
              f"{len(gaps)} gaps, median gap {gaps[len(gaps) // 2] * 1e-3 if gaps else 0:.2f} us, "
              f"gap sum {sum(gaps) * 1e-6:.2f} ms")
        return
    if a.gaps:
        rows = sorted((r[1], r[2], r[0].replace("(anonymous namespace)::", "").split("(")[0][:60])
                      for r in db.execute(f"select {name_col}, start, end from kernels"))
        end = max(r[1] for r in rows)
        lo = end - a.gaps * 1e6
        rows = [r for r in rows if r[1] > lo]
        pair = defaultdict(lambda: [0.0, 0])
        cur_e, cur_n = None, None
        for s0, e, nm in rows:
            if cur_e is not None and s0 > cur_e:
                k = f"{cur_n}  ->  {nm}"
                pair[k][0] += s0 - cur_e
                pair[k][1] += 1
            if cur_e is None or e > cur_e:
                cur_e, cur_n = e, nm
        div = a.steps or 1
        tot = sum(v[0] for v in pair.values())
        print(f"idle gaps {tot * 1e-6 / div:.3f} ms per {'step' if a.steps else 'window'}")
        for k, (t, n) in sorted(pair.items(), key=lambda kv: -kv[1][0])[: a.top]:
            print(f"{t * 1e-6 / div:8.3f} ms {n / div:7.1f} x {1e-3 * t / n:7.1f} us  {k}")
        return
    if a.solo:
        rows = [(r[0].replace("(anonymous namespace)::", "").split("(")[0][:100], r[1], r[2])
                for r in db.execute(f"select {name_col}, start, end from kernels")]
        end = max(r[2] for r in rows)
        lo = end - a.solo * 1e6
        ev = []
        for i, (nm, s0, e) in enumerate(rows):
            if e <= lo:
                continue
            ev.append((max(s0, lo), 1, i))
            ev.append((e, -1, i))
        ev.sort()
        active, last_t = set(), None
        solo, shared = defaultdict(float), defaultdict(float)
        for t, kind, i in ev:
            if last_t is not None and active and t > last_t:
                dt = t - last_t
                if len(active) == 1:
                    solo[rows[next(iter(active))][0]] += dt
                else:
                    for j in active:
                        shared[rows[j][0]] += dt / len(active)
            if kind == 1:
                active.add(i)
            else:
                active.discard(i)
            last_t = t
        div = a.steps or 1
        ts, tsh = sum(solo.values()), sum(shared.values())
        print(f"solo (exposed) {ts * 1e-6 / div:.2f} ms, overlapped share {tsh * 1e-6 / div:.2f} ms "
              f"(per {'step' if a.steps else 'window'})")
        for k in sorted(solo, key=lambda k: -solo[k])[: a.top]:
            print(f"{solo[k] * 1e-6 / div:9.3f} ms solo  {shared[k] * 1e-6 / div:9.3f} ms shared  {k}")
        return
    agg = defaultdict(lambda: [0.0, 0])
    t0, t1 = None, None
    rows = list(db.execute(q))
    if a.window:
        last = max(r[2] for r in rows)
        rows = [r for r in rows if r[1] >= last - a.window * 1e6]
    for r in rows:
        nm = r[0]
        short = nm.replace("(anonymous namespace)::", "").split("(")[0][:100]
        if a.grid and gx:
            short += f"  grid={r[3] // max(r[6], 1)}x{r[4]}x{r[5]}"
        dur = (r[2] - r[1]) * 1e-6
        agg[short][0] += dur
        agg[short][1] += 1
        t0 = r[1] if t0 is None else min(t0, r[1])
        t1 = r[2] if t1 is None else max(t1, r[2])
    tot = sum(v[0] for v in agg.values())
    div = a.steps or 1
    print(f"kernel time total {tot / div:.2f} ms{'/step' if a.steps else ''}  ({len(agg)} kernels)")
    for k, (t, n) in sorted(agg.items(), key=lambda kv: -kv[1][0])[: a.top]:
        print(f"{t / div:9.3f} ms {100 * t / tot:5.1f}%  {n / div:8.1f} calls  {1e3 * t / n:9.1f} us  {k}")


if __name__ == "__main__":
    main()

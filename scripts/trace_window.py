#!/usr/bin/env python3
"""Per-step kernel breakdown of the LAST ``--steps`` forwards in a rocprofv3 kernel trace.

A forward starts at its embedding gather (``embedding_kernel``); graph-replayed
decode forwards do too.  Kernels are grouped by (name, grid) so the same kernel at
different shapes is split out.  Usage:
    python scripts/trace_window.py gpurun_out/prof62/bench_kernel_trace.csv --steps 20

``--by-pid`` (several rank processes, e.g. TP = 2 on one GPU: one trace file per process, or one
file with a Process_Id column): the window is
taken per process from its own markers; per process it prints its kernel-busy share and
the largest gaps between consecutive kernels of that process (host time the process left
its queue empty), and for the device the time no process had a kernel running.
"""
import argparse
import collections
import csv
import os


def load(paths):
    """Rows of one or more kernel-trace CSVs; with several files (rocprofv3 -o name_%pid%: one
    per process) the process is the file's, else the Process_Id column's."""
    rows = []
    for path in paths:
        tag = os.path.basename(path).replace("_kernel_trace.csv", "") if len(paths) > 1 else None
        with open(path) as f:
            for r in csv.DictReader(f):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                             (int(r["Grid_Size_X"]), int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"])),
                             int(r["Workgroup_Size_X"]), tag or r.get("Process_Id", "0")))
    rows.sort()
    return rows


def window(rows, steps, marker):
    marks = [i for i, r in enumerate(rows) if marker in r[2]]
    lo, hi = marks[-steps - 1], marks[-1]
    return rows[lo:hi]


def union_busy(iv):
    """Total length of the union of [s, e) intervals (ns)."""
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def breakdown(win, steps, top):
    span = (win[-1][1] - win[0][0]) / 1e6
    busy = sum(r[1] - r[0] for r in win) / 1e6
    agg = collections.defaultdict(lambda: [0, 0.0])
    for s, e, n, g, wg, _ in win:
        short = n.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:70]
        k = (short, g[0] // wg, g[1], g[2])
        agg[k][0] += 1
        agg[k][1] += (e - s) / 1e3
    print(f"window: {steps} steps, {span:.1f} ms wall ({span / steps:.2f} ms/step), "
          f"kernel busy {busy:.1f} ms ({100 * busy / span:.1f}%)")
    print(f"{'us/step':>9} {'%':>5} {'calls/step':>10} {'us/call':>8}  kernel [workgroups x gy x gz]")
    for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{t / steps:9.1f} {100 * t / 1e3 / busy:5.1f} {c / steps:10.2f} {t / c:8.1f}  {k[0]} [{k[1]}x{k[2]}x{k[3]}]")


def by_pid(rows, steps, marker, top):
    pids = sorted({r[5] for r in rows})
    lo_all, hi_all = None, None
    for pid in pids:
        mine = [r for r in rows if r[5] == pid]
        if sum(marker in r[2] for r in mine) <= steps:
            print(f"pid {pid}: fewer than {steps + 1} markers, skipped")
            continue
        win = window(mine, steps, marker)
        lo, hi = win[0][0], win[-1][1]
        lo_all = lo if lo_all is None else min(lo_all, lo)
        hi_all = hi if hi_all is None else max(hi_all, hi)
        own = union_busy([(r[0], r[1]) for r in win])
        gaps, end = [], win[0][1]
        for r in win[1:]:
            if r[0] > end:
                gaps.append(r[0] - end)
            end = max(end, r[1])
        gaps.sort(reverse=True)
        print(f"== pid {pid}")
        breakdown(win, steps, top)
        print(f"own kernels busy (union) {100 * own / (hi - lo):.1f}% of its window; largest gaps between its "
              f"kernels (us): {[round(g / 1e3, 1) for g in gaps[:8]]}; gaps > 50 us: "
              f"{sum(g > 50_000 for g in gaps)}, total {sum(gaps) / 1e6:.2f} ms")
    if lo_all is not None:
        dev = [(r[0], r[1]) for r in rows if r[1] > lo_all and r[0] < hi_all]
        busy = union_busy([(max(s, lo_all), min(e, hi_all)) for s, e in dev])
        print(f"== device: {(hi_all - lo_all) / 1e6:.1f} ms window, some kernel running {100 * busy / (hi_all - lo_all):.1f}% "
              f"(idle {(hi_all - lo_all - busy) / 1e6:.2f} ms)")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace", nargs="+")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--marker", default="embedding_kernel")
    ap.add_argument("--by-pid", action="store_true")
    a = ap.parse_args()
    rows = load(a.trace)
    if a.by_pid:
        by_pid(rows, a.steps, a.marker, a.top)
    else:
        breakdown(window(rows, a.steps, a.marker), a.steps, a.top)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Per-step kernel breakdown of the LAST ``--steps`` forwards in a rocprofv3 kernel trace.

A forward starts at its embedding gather (``embedding_kernel``); graph-replayed
decode forwards do too.  Kernels are grouped by (name, grid) so the same kernel at
different shapes is split out.  Usage:
    python scripts/trace_window.py gpurun_out/prof62/bench_kernel_trace.csv --steps 20
"""
import argparse
import csv
import collections

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--top", type=int, default=30)
ap.add_argument("--marker", default="embedding_kernel")
a = ap.parse_args()
rows = []
with open(a.trace) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                     (int(r["Grid_Size_X"]), int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"])),
                     int(r["Workgroup_Size_X"])))
rows.sort()
marks = [i for i, r in enumerate(rows) if a.marker in r[2]]
lo, hi = marks[-a.steps - 1], marks[-1]
win = rows[lo:hi]
span = (win[-1][1] - win[0][0]) / 1e6
busy = sum(r[1] - r[0] for r in win) / 1e6
agg = collections.defaultdict(lambda: [0, 0.0])
for s, e, n, g, wg in win:
    short = n.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:70]
    k = (short, g[0] // wg, g[1], g[2])
    agg[k][0] += 1
    agg[k][1] += (e - s) / 1e3
print(f"window: {a.steps} steps, {span:.1f} ms wall ({span / a.steps:.2f} ms/step), "
      f"kernel busy {busy:.1f} ms ({100 * busy / span:.1f}%)")
print(f"{'us/step':>9} {'%':>5} {'calls/step':>10} {'us/call':>8}  kernel [workgroups x gy x gz]")
for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
    print(f"{t / a.steps:9.1f} {100 * t / 1e3 / busy:5.1f} {c / a.steps:10.2f} {t / c:8.1f}  {k[0]} [{k[1]}x{k[2]}x{k[3]}]")

#!/usr/bin/env python3
"""Busy time and inter-kernel gaps of the last pass in a kernel trace (passes
separated by gaps > --gap-us): python scripts/trace_gaps.py DIR"""
import argparse
import csv
from collections import defaultdict
from pathlib import Path

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("--gap-us", type=float, default=1000)
a = ap.parse_args()
rows = []
for f in Path(a.dir).rglob("*kernel_trace.csv"):
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                     r["Kernel_Name"].replace("(anonymous namespace)", "anon").split("(")[0][:90]))
rows.sort()
wins, cur = [], [rows[0]]
for r in rows[1:]:
    if r[0] - max(x[1] for x in cur[-4:]) > a.gap_us * 1e3:
        wins.append(cur)
        cur = []
    cur.append(r)
wins.append(cur)
for w in wins[-3:]:
    span = (w[-1][1] - w[0][0]) / 1e3
    busy = sum(e - s for s, e, _ in w) / 1e3
    gaps = [(w[i + 1][0] - w[i][1]) / 1e3 for i in range(len(w) - 1)]
    print(f"pass: {len(w)} kernels, span {span:.1f} us, busy {busy:.1f} us, gaps {sum(gaps):.1f} us "
          f"(median {sorted(gaps)[len(gaps) // 2]:.2f}, max {max(gaps):.2f})")
w = wins[-1]
per = defaultdict(float)
for s, e, k in w:
    per[k] += (e - s) / 1e3
for k, us in sorted(per.items(), key=lambda kv: -kv[1])[:15]:
    print(f"   {us:8.1f}  {k}")

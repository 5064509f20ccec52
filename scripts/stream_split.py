#!/usr/bin/env python3
"""Per-stream split of a kernel trace's last window (rocprofv3 csv): for the
kernels after the last gap longer than --gap-us (one backward pass), each
stream's busy time and its top kernels.
  python scripts/stream_split.py DIR [--gap-us 2000] [--top 12]"""
import argparse
import csv
from collections import defaultdict
from pathlib import Path

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("--gap-us", type=float, default=2000)
ap.add_argument("--top", type=int, default=12)
a = ap.parse_args()
rows = []
for f in Path(a.dir).rglob("*kernel_trace.csv"):
    for r in csv.DictReader(open(f)):
        q = r.get("Stream_Id") or r.get("Queue_Id") or "?"
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), q,
                     r["Kernel_Name"].replace("(anonymous namespace)", "anon").split("(")[0][:100]))
rows.sort()
# split into windows at gaps
wins, cur, last_end = [], [], None
for r in rows:
    if last_end is not None and r[0] - last_end > a.gap_us * 1e3:
        wins.append(cur)
        cur = []
    cur.append(r)
    last_end = max(last_end or 0, r[1])
wins.append(cur)
w = wins[-1]
t0, t1 = w[0][0], max(r[1] for r in w)
print(f"windows {len(wins)}; last: {len(w)} kernels, span {(t1 - t0) / 1e3:.1f} us")
by = defaultdict(list)
for r in w:
    by[r[2]].append(r)
for q, rs in by.items():
    busy = sum(e - s for s, e, *_ in rs) / 1e3
    tops = defaultdict(float)
    for s, e, _, k in rs:
        tops[k] += (e - s) / 1e3
    print(f"stream {q}: {len(rs)} kernels, busy {busy:.1f} us")
    for k, us in sorted(tops.items(), key=lambda kv: -kv[1])[:a.top]:
        print(f"   {us:9.1f}  {k}")

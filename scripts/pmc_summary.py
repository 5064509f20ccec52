#!/usr/bin/env python3
"""Per-kernel, per-dispatch mean of each counter from pmc_run.sh output
(rows are summed per (dispatch, counter) first)."""
import csv
import sys
from collections import defaultdict
from pathlib import Path

root = Path(sys.argv[1])
per = defaultdict(float)  # (kernel, counter, dispatch) -> value
for f in root.rglob("*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        key = (r["Kernel_Name"][:100], r["Counter_Name"], f.parent.name + r["Dispatch_Id"])
        per[key] += float(r["Counter_Value"])
agg = defaultdict(lambda: defaultdict(list))
for (k, c, _), v in per.items():
    agg[k][c].append(v)
for k, cs in agg.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} {sum(v) / len(v):14.6g}  (dispatches={len(v)})")

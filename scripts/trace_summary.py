#!/usr/bin/env python3
"""Median kernel duration per (kernel, grid) from rocprofv3 kernel-trace csv
files under a directory: python scripts/trace_summary.py DIR [substr...]"""
import csv
import statistics
import sys
from collections import defaultdict
from pathlib import Path

root = Path(sys.argv[1])
keys = sys.argv[2:]
for f in sorted(root.rglob("*kernel_trace.csv")):
    d = defaultdict(list)
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if keys and not any(k in name for k in keys):
            continue
        d[(name[:90], r.get("Grid_Size_X") or r.get("Grid_Size"))].append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(f.relative_to(root))
    for (n, g), v in sorted(d.items()):
        print(f"  {statistics.median(v):9.2f} us  n={len(v):3d} grid={g}  {n}")

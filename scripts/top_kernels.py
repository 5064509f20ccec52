#!/usr/bin/env python3
"""Top kernels by total time from a rocprofv3 kernel-trace csv directory:
python scripts/top_kernels.py DIR [N]"""
import csv
import sys
from collections import defaultdict
from pathlib import Path

root = Path(sys.argv[1])
top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
d = defaultdict(lambda: [0, 0.0])
for f in root.rglob("*kernel_trace.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("(anonymous namespace)", "anon").split("(")[0][:120]
        d[k][0] += 1
        d[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
tot = sum(v[1] for v in d.values())
print(f"total {tot:.1f} us")
for k, (n, us) in sorted(d.items(), key=lambda kv: -kv[1][1])[:top]:
    print(f"{us:10.1f} us {100 * us / tot:5.1f}% n={n:5d} avg={us / n:8.2f}  {k}")

#!/usr/bin/env python3
"""Per (kernel, grid) summary of a scripts/profile.sh run: median duration
from the kernel trace, and per dispatch FETCH / WRITE bytes and MFMA busy
from the PMC passes (MI355X_MICROARCH.md: FETCH_SIZE / WRITE_SIZE in KB,
gfx950 FETCH_SIZE counts half of a wide streaming read, so the corrected
read bytes are 2 * FETCH_SIZE * 1024; MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES /
(1024 SIMDs * GRBM_GUI_ACTIVE / 8)).

  python scripts/pmc_by_kernel.py gpurun_out/prof_TAG OUT.json [name-substr ...]
"""
import csv
import json
import re
import statistics as st
import sys
from collections import defaultdict
from pathlib import Path


def short(name):
    name = name.replace("(anonymous namespace)", "anon")
    name = re.sub(r"^void ", "", name)
    return name[:160]


def main():
    src = Path(sys.argv[1])
    keys = sys.argv[3:]
    pick = (lambda n: any(k in n for k in keys)) if keys else (lambda n: True)
    dur = defaultdict(list)
    for f in src.rglob("*kernel_trace.csv"):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            if pick(n):
                g = r.get("Grid_Size_X") or r.get("Grid_Size")
                dur[(short(n), str(g))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    ctr = defaultdict(lambda: defaultdict(list))
    for f in src.rglob("*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            if pick(n):
                ctr[(short(n), str(r["Grid_Size"]))][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = []
    for key in sorted(set(dur) | set(ctr), key=lambda k: -sum(dur.get(k, [0]))):
        c = ctr.get(key, {})
        row = {"kernel": key[0], "grid": key[1]}
        if key in dur:
            row.update(n=len(dur[key]), us_median=round(st.median(dur[key]), 2),
                       us_total=round(sum(dur[key]), 1))
        if c.get("FETCH_SIZE"):
            row["fetch_mb_corrected"] = round(2 * st.mean(c["FETCH_SIZE"]) * 1024 / 1e6, 2)
        if c.get("WRITE_SIZE"):
            row["write_mb"] = round(st.mean(c["WRITE_SIZE"]) * 1024 / 1e6, 2)
        b, g = c.get("SQ_VALU_MFMA_BUSY_CYCLES"), c.get("GRBM_GUI_ACTIVE")
        if b and g and len(b) == len(g):
            row["mfma_busy"] = round(st.mean(x / (1024 * y / 8.0) for x, y in zip(b, g) if y), 3)
        out.append(row)
    json.dump(out, open(sys.argv[2], "w"), indent=0)
    print(f"{len(out)} kernels -> {sys.argv[2]}")


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Summarise scripts/profile_elementwise.sh into profiles/<tag>_elementwise_traffic.json.

  python scripts/summarize_elementwise.py gpurun_out/prof_ew <tag>

Dispatches are split into ops at the fill_kernel separators the driver
launches before each op (same order in every pass).  Per op and launch:
duration (kernel trace; an op of several kernels sums them), FETCH_SIZE and
WRITE_SIZE (PMC passes; values in KB as rocprofv3 reports them).  FETCH_SIZE
is corrected by the read factor measured on the calibration kernel of the
same access width (b32: the strided copy, b128: the float4 SGD update;
known bytes / reported bytes), WRITE_SIZE likewise — MI355X_MICROARCH.md
§HBM.  achieved_gbs = algorithmic bytes / duration, against 8 TB/s.
"""
import csv
import json
import statistics as st
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
PEAK = 8000.0
# access width of each op's dominant loads (for the FETCH correction)
WIDTH = {"im2col": "b32", "col2im": "b32", "forward_bias": "b128", "activate_leaky": "b128",
         "means_and_vars": "b32", "means_and_vars_delta": "b32", "add_dots": "b32",
         "add_sums": "b32", "normalize": "b128", "normalize_delta": "b128"}  # (row forms: float4)


def segments(rows, names):
    """rows: (dispatch_id, kernel, value) sorted; -> {op: [[per-launch...]...]}"""
    out, cur = {}, None
    ops = iter(names)
    for did, k, val in rows:
        if "tns::" not in k:  # torch's own allocation / fill kernels
            continue
        if "::fill_kernel" in k:
            cur = next(ops)
            out[cur] = []
            continue
        if cur is not None:
            out[cur].append((did, k, val))
    return out


def load_trace(path):
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"],
                     (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6))
    return sorted(rows)


def load_pmc(path, counter):
    rows = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        did = int(r["Dispatch_Id"])
        rows.setdefault(did, [r["Kernel_Name"], 0.0])
        rows[did][1] += float(r["Counter_Value"])
    return sorted((d, k, v) for d, (k, v) in rows.items())


def per_launch(seg, reps):
    """sum an op's kernels per repetition (equal kernel count per rep)"""
    vals = [v for _, _, v in seg]
    if not vals or len(vals) % reps:
        return None, len(vals)
    per = len(vals) // reps
    return [sum(vals[i * per:(i + 1) * per]) for i in range(reps)], per


def main():
    src, tag = Path(sys.argv[1]), sys.argv[2]
    meta = json.loads([l for l in (src / "trace.log").read_text().splitlines()
                       if l.startswith("{")][-1])
    reps, alg = meta["reps"], meta["algorithmic_bytes"]
    names = list(alg)
    tr = segments(load_trace(next((src / "trace").rglob("*kernel_trace.csv"))), names)
    fe = segments(load_pmc(next((src / "fetch").rglob("*counter_collection.csv")), "FETCH_SIZE"),
                  names)
    wr = segments(load_pmc(next((src / "write").rglob("*counter_collection.csv")), "WRITE_SIZE"),
                  names)
    res = {}
    for op in names:
        d, nk = per_launch(tr.get(op, []), reps)
        f, _ = per_launch(fe.get(op, []), reps)
        w, _ = per_launch(wr.get(op, []), reps)
        kernels = sorted({k.split("(")[0][-80:] for _, k, _ in tr.get(op, [])})
        res[op] = {"kernels": kernels, "kernels_per_launch": nk,
                   "ms_mean": round(st.mean(d), 4) if d else None,
                   "ms_min": round(min(d), 4) if d else None,
                   "fetch_kb_raw": round(st.mean(f), 1) if f else None,
                   "write_kb_raw": round(st.mean(w), 1) if w else None,
                   "alg": alg[op]}
    cal = {}
    for width, op in (("b32", "calib_copy_b32"), ("b128", "calib_sgd_b128")):
        r = res[op]
        cal[width] = {"read": r["alg"]["read"] / (r["fetch_kb_raw"] * 1024.0),
                      "write": r["alg"]["write"] / (r["write_kb_raw"] * 1024.0)}
    out = {"tag": tag, "reps": reps, "peak_gbs": PEAK, "calibration": cal, "ops": {}}
    for op in names:
        r = res[op]
        a = r["alg"]
        ab = a["read"] + a["write"]
        c = cal[WIDTH.get(op, "b32" if op.endswith("b32") else "b128")]
        rd = r["fetch_kb_raw"] * 1024.0 * c["read"] if r["fetch_kb_raw"] is not None else None
        wt = r["write_kb_raw"] * 1024.0 * c["write"] if r["write_kb_raw"] is not None else None
        row = dict(r)
        row.update({"algorithmic_bytes": ab,
                    "traffic_read_bytes": round(rd) if rd is not None else None,
                    "traffic_write_bytes": round(wt) if wt is not None else None})
        if r["ms_mean"]:
            row["achieved_gbs"] = round(ab / (r["ms_mean"] * 1e-3) / 1e9, 1)
            row["frac_of_peak"] = round(row["achieved_gbs"] / PEAK, 4)
            if rd is not None and wt is not None:
                row["traffic_gbs"] = round((rd + wt) / (r["ms_mean"] * 1e-3) / 1e9, 1)
                row["traffic_over_algorithmic"] = round((rd + wt) / ab, 3) if ab else None
        out["ops"][op] = row
    dst = ROOT / "profiles" / f"{tag}_elementwise_traffic.json"
    dst.write_text(json.dumps(out, indent=1))
    print(json.dumps({k: {kk: v.get(kk) for kk in ("ms_mean", "achieved_gbs",
                                                     "traffic_over_algorithmic")}
                      for k, v in out["ops"].items()}, indent=1))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Summarise scripts/gpu_r4_evidence.sh (gpurun_out/pmc_r4) into
profiles/r04_conv_tile4_pmc.json (forward) and profiles/r04_conv_bwd_pmc.json.

Per layer and kernel, the per-dispatch mean of every counter, plus:
  mfma_busy      SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)
                 — the fraction of the launch the average SIMD's matrix pipe
                 was busy (GRBM_GUI_ACTIVE sums the 8 XCDs);
  wait_frac      SQ_WAIT_ANY / SQ_WAVE_CYCLES (waves parked on s_waitcnt /
                 barrier), issue_stall_frac SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES;
  lds_bank_conflict_per_lds_inst;
  fetch_bytes    2 x FETCH_SIZE x 1024 (gfx950 tallies a 128-B request as
                 64 B for 16-B-per-lane streams, MI355X_MICROARCH.md §HBM;
                 the conv B gather's dword loads are uncalibrated — the
                 factor 2 is an upper estimate there), write_bytes WRITE_SIZE
                 x 1024.  Both count Infinity-Cache hits (memory-side of L2).
"""
import csv
import json
import statistics as st
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def per_dispatch(d: Path):
    per = defaultdict(float)
    names = {}
    for f in d.rglob("*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "tns::" not in k:
                continue
            short = k.replace("(anonymous namespace)::", "").split("(")[0][:160]
            did = f.parent.name + ":" + r["Dispatch_Id"]
            names[did] = short
            per[(did, r["Counter_Name"])] += float(r["Counter_Value"])
    out = defaultdict(lambda: defaultdict(list))
    for (did, c), v in per.items():
        out[names[did]][c].append(v)
    return out


def summarise(src: Path, prefix: str, layers):
    res = {}
    for L in layers:
        sq = per_dispatch(src / f"{prefix}{L}_sq")
        fe = per_dispatch(src / f"{prefix}{L}_fetch")
        wr = per_dispatch(src / f"{prefix}{L}_write")
        kern = {}
        for k, cs in sq.items():
            m = {c: st.mean(v) for c, v in cs.items()}
            g = m.get("GRBM_GUI_ACTIVE", 0.0)
            e = {"dispatches": len(next(iter(cs.values()))), "counters": {c: round(v, 1) for c, v in m.items()}}
            if g:
                e["mfma_busy"] = round(m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (1024 * g / 8.0), 4)
                e["gpu_active_us_at_2.4GHz"] = round(g / 8.0 / 2.4e3, 2)
            if m.get("SQ_WAVE_CYCLES"):
                e["wait_frac"] = round(m.get("SQ_WAIT_ANY", 0) / m["SQ_WAVE_CYCLES"], 4)
                e["issue_stall_frac"] = round(m.get("SQ_WAIT_INST_ANY", 0) / m["SQ_WAVE_CYCLES"], 4)
                e["lds_issue_stall_frac"] = round(m.get("SQ_WAIT_INST_LDS", 0) / m["SQ_WAVE_CYCLES"], 4)
            if m.get("SQ_INSTS_LDS"):
                e["lds_bank_conflict_per_lds_inst"] = round(m.get("SQ_LDS_BANK_CONFLICT", 0) / m["SQ_INSTS_LDS"], 4)
            if k in fe and "FETCH_SIZE" in fe[k]:
                e["fetch_bytes"] = round(2 * st.mean(fe[k]["FETCH_SIZE"]) * 1024)
            if k in wr and "WRITE_SIZE" in wr[k]:
                e["write_bytes"] = round(st.mean(wr[k]["WRITE_SIZE"]) * 1024)
            kern[k] = e
        res[str(L)] = kern
    return res


def main():
    src = Path(sys.argv[1]) if len(sys.argv) > 1 else ROOT / "gpurun_out" / "pmc_r4"
    layers = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "11,28,45,10").split(",")]
    note = ("rocprofv3 --pmc passes (one counter group per run) over scripts/conv_one.py / "
            "conv_bwd_one.py at batch 8, scripts/gpu_r4_evidence.sh; see the docstring of "
            "scripts/summarize_pmc_r4.py for the derived fields")
    from tensorium_amd.yolo import yolov3_conv_table
    T = yolov3_conv_table()
    shapes = {str(L): f"{T[L].c}x{T[L].h} k{T[L].size}s{T[L].stride}->{T[L].filters}" for L in layers}
    fwd = {"note": note, "shapes": shapes, "layers": summarise(src, "fwd", layers)}
    bwd = {"note": note, "shapes": shapes, "layers": summarise(src, "bwd", layers)}
    tag = sys.argv[3] if len(sys.argv) > 3 else "r04"
    if tag == "r04":
        (ROOT / "profiles" / "r04_conv_tile4_pmc.json").write_text(json.dumps(fwd, indent=1) + "\n")
        (ROOT / "profiles" / "r04_conv_bwd_pmc.json").write_text(json.dumps(bwd, indent=1) + "\n")
    else:  # later rounds: one file, plus the SQ pass over the 4096^3 SGEMM if present
        out = {"note": note.replace("gpu_r4_evidence", f"gpu_{tag[0]}{tag[2:]}_evidence"),
               "shapes": shapes, "conv_fwd": fwd["layers"], "conv_bwd": bwd["layers"]}
        if (src / "sgemm_sq").exists():
            sg = {}
            for k, cs in per_dispatch(src / "sgemm_sq").items():
                m = {c: st.mean(v) for c, v in cs.items()}
                e = {"dispatches": len(next(iter(cs.values()))),
                     "counters": {c: round(v, 1) for c, v in m.items()}}
                if m.get("GRBM_GUI_ACTIVE"):
                    e["mfma_busy"] = round(m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) /
                                           (1024 * m["GRBM_GUI_ACTIVE"] / 8.0), 4)
                if m.get("SQ_INSTS_LDS"):
                    e["lds_bank_conflict_per_lds_inst"] = round(
                        m.get("SQ_LDS_BANK_CONFLICT", 0) / m["SQ_INSTS_LDS"], 4)
                sg[k] = e
            out["sgemm_4096_sq"] = sg
        (ROOT / "profiles" / f"{tag}_pmc.json").write_text(json.dumps(out, indent=1) + "\n")
    for L in layers:
        for k, e in fwd["layers"][str(L)].items():
            print("fwd", L, k[:70], e.get("mfma_busy"), e.get("fetch_bytes"), e.get("write_bytes"))
        for k, e in bwd["layers"][str(L)].items():
            print("bwd", L, k[:70], e.get("mfma_busy"), e.get("fetch_bytes"), e.get("write_bytes"))


if __name__ == "__main__":
    main()

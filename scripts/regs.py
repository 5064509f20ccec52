#!/usr/bin/env python3
"""Register / LDS / occupancy table of every kernel in one csrc file.

  python scripts/regs.py sgemm_s256 [filter]
"""
import re
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
src = ROOT / "tensorium_amd" / "csrc" / (sys.argv[1] + ".hip")
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off",
       "-x", "hip", "-c", str(src), "-o", "/tmp/_regs.o", "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = []
for line in out.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        cur = {"name": t.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    n = r["name"].replace("_ZN3tns12sgemm_detail17sgemm_mfma_kernelINS0_5ShapeI", "")
    if flt and flt not in n:
        continue
    n = re.sub(r"Li(\d+)E", r"\1,", n)
    print(f"{n[:60]:60s} vgpr={r.get('VGPRs')} agpr={r.get('AGPRs')} "
          f"vspill={r.get('VGPRs Spill')} sspill={r.get('SGPRs Spill')} "
          f"scratch={r.get('ScratchSize [bytes/lane]')} occ={r.get('Occupancy [waves/SIMD]')} "
          f"lds={r.get('LDS Size [bytes/block]')}")

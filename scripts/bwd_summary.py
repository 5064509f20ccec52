#!/usr/bin/env python3
"""Per-class summary of scripts/conv_bwd_layers.py output (one or two files:
the second is compared against the first).

  python scripts/bwd_summary.py gpurun_out/bwd_layers.json [gpurun_out/bwd_layers2.json]
"""
import json
import re
import sys
from collections import defaultdict


def load(path):
    d = json.loads(open(path).read().strip().splitlines()[-1])
    rows = d if isinstance(d, list) else d.get("layers", d)
    agg = defaultdict(lambda: [0, 0.0, 0.0, 0.0, 0.0, 0.0])
    for r in rows:
        C, H, k, s, F = map(int, re.match(r"(\d+)x(\d+) k(\d)s(\d)->(\d+)", r["shape"]).groups())
        a = agg[(H, k, s, F)]
        a[0] += 1
        for i, key in enumerate(("call_ms", "dw_ms", "dx_ms", "im2col_ms", "col2im_ms")):
            a[1 + i] += r[key]
    return agg


paths = sys.argv[1:]
aggs = [load(p) for p in paths]
tot = [sum(v[1] for v in a.values()) for a in aggs]
print("total call ms", [round(t, 3) for t in tot])
for key, v in sorted(aggs[0].items(), key=lambda kv: -kv[1][1]):
    line = f"{key} x{v[0]}: call {v[1]:.3f} dw {v[2]:.3f} dx {v[3]:.3f} im2col {v[4]:.3f} col2im {v[5]:.3f}"
    if len(aggs) > 1:
        w = aggs[1][key]
        line += f" | call {w[1]:.3f} dw {w[2]:.3f} dx {w[3]:.3f}"
    print(line)

#!/usr/bin/env python3
"""Compare two scripts/conv_bwd_layers.py records per layer (call_ms)."""
import json
import sys

a = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
b = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print("sum call_ms", round(sum(r["call_ms"] for r in a), 3), round(sum(r["call_ms"] for r in b), 3),
      "dw_ms", round(sum(r["dw_ms"] for r in a), 3), round(sum(r["dw_ms"] for r in b), 3))
for x, y in zip(a, b):
    if abs(x["call_ms"] - y["call_ms"]) > 0.005:
        print(x["layer"], x["shape"], x["call_ms"], y["call_ms"], x["dw_ms"], y["dw_ms"])

#!/usr/bin/env python3
"""Summarise gpurun_out/fwdsweep.jsonl (scripts/gpu_r5.sh fwdsweep): per
(layer, variant) the per-pass ms."""
import collections
import json
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/fwdsweep.jsonl"
d = collections.defaultdict(list)
for part in open(path).read().split('{"round": ')[1:]:
    head, rest = part.split(', "res": ', 1)
    _, v = head.split(', "variant": ')
    res = json.loads(rest.strip()[:-1].strip())
    for x in res["layers"]:
        d[(x["layer"], int(v))].append(x["ms"])
for k in sorted(d):
    print(k, d[k], round(min(d[k]), 4))

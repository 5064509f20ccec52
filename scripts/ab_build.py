#!/usr/bin/env python3
"""Side build for A/B timing: ab/<name>/libtensorium_hip.so with extra
compile flags on the listed sources only (every other object is taken from
the main build, so a variant links in seconds).

  python scripts/ab_build.py <name> "<flags>" sgemm_nn_big.hip [more.hip ...]
"""
import os
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from tensorium_amd import build  # noqa: E402

name, flags, *srcs = sys.argv[1:]
out = ROOT / "ab" / name
(out / "_build").mkdir(parents=True, exist_ok=True)
build.build_hip()  # main objects current
for o in build.BUILD.glob("*.o"):
    if o.name[:-2] not in srcs:
        shutil.copy2(o, out / "_build" / o.name)
for s in srcs:
    (out / "_build" / (s + ".o")).unlink(missing_ok=True)
os.environ["TNS_EXTRA_CFLAGS"] = flags
print(build.build_hip(out=out))

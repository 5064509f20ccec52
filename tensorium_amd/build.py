"""Build libtensorium_hip.so (gfx950) and the CPU oracle in-tree.

The HIP library is compiled with plain ``hipcc --offload-arch=gfx950`` — no
torch extension, no JIT cache — so the ``.so`` lives in the package directory
and travels with the repo snapshot to the GPU box.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
BUILD = PKG / "_build"
LIB = PKG / "libtensorium_hip.so"
ORACLE_DIR = ROOT / "oracle"
ORACLE_LIB = ORACLE_DIR / "libtns_oracle.so"

ARCH = "gfx950"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CXXFLAGS = [
    "-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}",
    # no implicit FMA contraction: the reference rounds mul and add separately
    # wherever it does not issue an FMA itself (numerics)
    "-ffp-contract=off",
    "-Wall", "-Wno-unused-function", "-Wno-unused-value", "-Wno-unused-result",
]


def _sources() -> list[Path]:
    return sorted(CSRC.glob("*.hip")) + sorted(CSRC.glob("*.cpp"))


def _newer(target: Path, deps: list[Path]) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def _run(cmd: list[str], verbose: bool) -> None:
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError(f"command failed ({r.returncode}): {' '.join(cmd[:3])} ...")
    if verbose and (r.stdout or r.stderr):
        sys.stderr.write(r.stdout + r.stderr)


def build_hip(verbose: bool = False, force: bool = False, out: Path | None = None) -> Path:
    """Compile csrc/ into LIB (or into out/libtensorium_hip.so, objects under
    out/_build — side builds for A/B perf runs)."""
    build = (out / "_build") if out else BUILD
    lib_path = (out / "libtensorium_hip.so") if out else LIB
    build.mkdir(parents=True, exist_ok=True)
    headers = sorted(CSRC.glob("*.hpp")) + [ROOT / "include" / "tns.h"]
    extra = os.environ.get("TNS_EXTRA_CFLAGS", "").split()  # A/B side builds
    if os.environ.get("TNS_DIAG") == "1":   # + the measured, not picked forms
        extra.append("-DTNS_DIAG_KERNELS")
    # the flag set the objects were compiled with: a different set (e.g.
    # TNS_DIAG toggled) rebuilds everything, never a mix of the two
    stamp = build / "flags.stamp"
    flags = " ".join([*CXXFLAGS, *extra])
    if not stamp.exists() or stamp.read_text() != flags:
        force = True
    objs: list[Path] = []
    jobs = []
    for src in _sources():
        obj = build / (src.name + ".o")
        objs.append(obj)
        if force or _newer(obj, [src, *headers]):
            lang = ["-x", "hip"] if src.suffix == ".hip" else []
            jobs.append([HIPCC, *CXXFLAGS, *extra, *lang, "-c", str(src), "-o", str(obj)])
    if jobs:
        stamp.unlink(missing_ok=True)  # (a failed build leaves no stamp)
        with ThreadPoolExecutor(max_workers=min(len(jobs), 8)) as ex:
            list(ex.map(lambda c: _run(c, verbose), jobs))
        stamp.write_text(flags)
    if force or jobs or _newer(lib_path, objs):
        tmp = lib_path.with_suffix(".so.tmp")
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o",
              str(tmp)], verbose)
        os.replace(tmp, lib_path)
    return lib_path


def build_oracle(verbose: bool = False) -> Path:
    if shutil.which("make") is None:
        raise RuntimeError("make not found")
    _run(["make", "-s", "-C", str(ORACLE_DIR)], verbose)
    return ORACLE_LIB


def build_all(verbose: bool = False, force: bool = False) -> None:
    build_oracle(verbose)
    build_hip(verbose, force)


if __name__ == "__main__":
    if "--out" in sys.argv:
        print(build_hip(True, "--force" in sys.argv, Path(sys.argv[sys.argv.index("--out") + 1])))
    else:
        build_all(verbose=True, force="--force" in sys.argv)
        print(LIB)

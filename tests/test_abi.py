"""The C-ABI library builds, loads and exports every symbol include/tns.h
declares (no compute without a GPU).  Also checks that the product package
never imports the oracle."""
import ctypes
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def test_header_symbols_exported(hiplib):
    from tensorium_amd import _abi
    names = _abi.header_symbols()
    assert len(names) >= 40
    missing = [n for n in names if not hasattr(hiplib, n)]
    assert not missing, missing
    # every exported tns_ symbol has a ctypes prototype
    assert set(names) == set(_abi.PROTOTYPES), set(names) ^ set(_abi.PROTOTYPES)


def test_exports_are_plain_c(hiplib):
    out = subprocess.run(["nm", "-D", "--defined-only", str(ROOT / "tensorium_amd" /
                                                              "libtensorium_hip.so")],
                         capture_output=True, text=True, check=True).stdout
    syms = {l.split()[-1] for l in out.splitlines() if " T " in l}
    from tensorium_amd import _abi
    for n in _abi.header_symbols():
        assert n in syms, f"{n} not exported unmangled"


def test_abi_version_and_error_channel_without_gpu(hiplib):
    assert hiplib.tns_abi_version() == 1
    hiplib.tns_clear_error()
    assert hiplib.tns_last_error() == b""
    assert hiplib.tns_set_option(99, 1) != 0
    assert b"unknown option" in hiplib.tns_last_error()
    assert hiplib.tns_set_option(0, 1) == 0


def test_error_hook_called(hiplib):
    seen = []
    HOOK = ctypes.CFUNCTYPE(None, ctypes.c_int, ctypes.c_char_p)
    cb = HOOK(lambda code, msg: seen.append((code, msg)))
    hiplib.tns_set_error_hook(ctypes.cast(cb, ctypes.c_void_p))
    try:
        hiplib.tns_set_option(123, 0)
    finally:
        hiplib.tns_set_error_hook(None)
    assert seen and seen[0][0] == 1


def test_null_ctx_rejected(hiplib):
    assert hiplib.tns_hip_finish(None) == 1
    assert hiplib.tns_hip_gemm(None, 0, 0, 1, 1, 1, 1.0, None, 0, 1, None, 0, 1, 0.0, None, 0,
                               1) == 1


def test_gfx950_code_object_present():
    data = (ROOT / "tensorium_amd" / "libtensorium_hip.so").read_bytes()
    assert b"amdgcn-amd-amdhsa--gfx950" in data


def test_product_does_not_import_oracle():
    for p in (ROOT / "tensorium_amd").rglob("*.py"):
        txt = p.read_text()
        assert "from oracle" not in txt and "import oracle" not in txt, p
    for p in (ROOT / "tensorium_amd" / "csrc").iterdir():
        for line in p.read_text().splitlines():
            if line.lstrip().startswith("#include"):
                assert "oracle" not in line, (p, line)
    # the shipped library neither defines nor imports any oracle symbol
    out = subprocess.run(["nm", "-D", str(ROOT / "tensorium_amd" / "libtensorium_hip.so")],
                         capture_output=True, text=True, check=True).stdout
    assert " ora_" not in out

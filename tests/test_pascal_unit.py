"""pascal/nnHip.pas against include/tns.h and TNNCuda<T>'s method list.

No Pascal compiler exists in this image (no fpc / lazbuild), so the unit
cannot be compiled here; this mechanical cross-check is the evidence that a
maintainer's binding is complete and ABI-correct:
  * every function include/tns.h declares has exactly one `cdecl; external`
    declaration in the unit, and nothing else is declared external;
  * same parameter count, and each parameter's width matches (int64_t <->
    int64/SizeInt, int32_t <-> longint, uint8_t <-> boolean/byte, float <->
    single, double <-> double, any pointer <-> a pointer type), and the same
    result width (void <-> procedure);
  * TNNHip<T> declares every public method of TNNCuda<T> (nncuda.pas:100-157,
    list transcribed below) plus initHIP / useHipOpTable, and useHipOpTable
    states the TNS_OPT_SRSS_QUIRK choice.
"""
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
HDR = ROOT / "include" / "tns.h"
PAS = ROOT / "pascal" / "nnHip.pas"

# TNNCuda<T> public methods, nncuda.pas:100-157
TNNCUDA_METHODS = [
    "deviceCount", "Create", "Destroy", "CompileLog", "createDeviceBuffer", "freeDeviceBuffer",
    "readBuffer", "writeBuffer", "ActivateArray", "activateArraySWISH", "DeriveArray",
    "forwardBias", "backwardBias", "gemm", "gemmBatched", "gemmStridedBatched", "addvv",
    "subvv", "mulvv", "fmavv", "axpy", "power", "scale", "crossEntropyLogistic", "fill", "copy",
    "softmaxBatch", "crossEntropySoftmax", "forwardMaxPool", "backwardMaxPool", "im2col",
    "col2im", "upSample", "fmavss", "meansAndVars", "means", "variances", "normalize",
    "meansAndVarsDelta", "normalizeDelta", "addDots", "forwardScale", "forwardScaleAdd",
    "forwardDropout", "backwardDropout", "costL2", "clamp", "inverseSqrt", "finish",
    "compileToCUBIN", "loadCUBIN", "compileFile", "loadCUBinFile",
]


def _c_width(t: str) -> str:
    t = t.replace("const", "").strip()
    if "*" in t or t.endswith("_t") and t == "tns_error_hook_t":
        return "ptr"
    return {"int64_t": "i64", "int32_t": "i32", "int": "i32", "uint8_t": "u8", "float": "f32",
            "double": "f64", "void": "void", "size_t": "i64"}[t]


def parse_header():
    src = re.sub(r"/\*.*?\*/", " ", HDR.read_text(), flags=re.S)
    src = re.sub(r"//[^\n]*", " ", src)
    src = re.sub(r"#[^\n]*", " ", src)
    src = re.sub(r"typedef[^;]*;", " ", src)
    src = re.sub(r"enum\s*\{[^}]*\}\s*;", " ", src)
    src = src.replace('extern "C" {', " ").replace("}", " ")
    protos = {}
    for m in re.finditer(r"([A-Za-z_][\w\s\*]*?)\b(tns_\w+)\s*\(([^;]*?)\)\s*;", src):
        ret, name, args = m.group(1).strip(), m.group(2), m.group(3).strip()
        params = []
        if args and args != "void":
            for a in args.split(","):
                a = a.strip()
                mm = re.match(r"(.*?)(\w+)$", a)
                ty = mm.group(1).strip()
                params.append(_c_width(ty))
        protos[name] = (_c_width(ret), params)
    return protos


PAS_WIDTH = {"int64": "i64", "sizeint": "i64", "longint": "i32", "boolean": "u8", "byte": "u8",
             "single": "f32", "double": "f64"}
PAS_PTRS = {"pointer", "psingle", "thipmem", "ptnsctx", "pptnsctx", "phipmem", "pint64",
            "plongint", "pansichar", "ttnserrorhook"}


def _pas_width(t: str) -> str:
    t = t.strip().lower()
    if t in PAS_WIDTH:
        return PAS_WIDTH[t]
    if t in PAS_PTRS:
        return "ptr"
    raise AssertionError(f"unknown Pascal parameter type {t!r}")


def parse_pascal_externals():
    src = re.sub(r"\{[^}]*\}", " ", PAS.read_text())
    src = re.sub(r"//[^\n]*", " ", src)
    decls = {}
    pat = re.compile(r"\b(function|procedure)\s+(tns_\w+)\s*\(([^)]*)\)\s*(?::\s*(\w+))?\s*;"
                     r"\s*cdecl\s*;\s*external\s+libtns\s*;", re.S | re.I)
    for m in pat.finditer(src):
        kind, name, args, ret = m.group(1).lower(), m.group(2), m.group(3), m.group(4)
        params = []
        for grp in [g for g in args.split(";") if g.strip()]:
            names, ty = grp.rsplit(":", 1)
            mod = names.strip().split()[0].lower() if names.strip() else ""
            count = len([n for n in names.replace("const ", " ").replace("var ", " ")
                         .replace("out ", " ").split(",") if n.strip()])
            w = "ptr" if mod in ("var", "out") else _pas_width(ty)
            params += [w] * count
        rw = "void" if kind == "procedure" else _pas_width(ret)
        assert name not in decls, f"{name} declared twice"
        decls[name] = (rw, params)
    # functions declared without a parameter list: `function f(): T; cdecl; ...`
    return decls


def test_every_header_function_bound_with_matching_widths():
    protos = parse_header()
    decls = parse_pascal_externals()
    assert len(protos) > 60, sorted(protos)
    missing = sorted(set(protos) - set(decls))
    extra = sorted(set(decls) - set(protos))
    assert not missing, f"tns.h functions without a Pascal declaration: {missing}"
    assert not extra, f"Pascal externals not in tns.h: {extra}"
    for name, (ret, params) in protos.items():
        pret, pparams = decls[name]
        assert pret == ret, f"{name}: result {pret} vs {ret}"
        assert len(pparams) == len(params), f"{name}: {len(pparams)} params vs {len(params)}"
        for i, (a, b) in enumerate(zip(pparams, params)):
            assert a == b, f"{name}: parameter {i} is {a} in Pascal, {b} in C"


def test_header_parse_sanity():
    protos = parse_header()
    assert protos["tns_cblas_sgemm"] == ("void", ["i32", "i32", "i32", "i64", "i64", "i64",
                                                  "f32", "ptr", "i64", "ptr", "i64", "f32",
                                                  "ptr", "i64"])
    assert protos["tns_im2col"][1][-1] == "u8"
    assert protos["tns_hip_op_ms"] == ("f64", ["ptr", "i32"])


def test_tnnhip_has_tnncuda_method_list():
    src = PAS.read_text()
    cls = src[src.index("TNNHip<T> = class"):src.index("property ctx")]
    declared = set(re.findall(r"(?:procedure|function|constructor|destructor)\s+(\w+)", cls))
    missing = [m for m in TNNCUDA_METHODS if m not in declared]
    assert not missing, missing
    for m in TNNCUDA_METHODS:   # every declared method has an implementation
        assert re.search(rf"TNNHip<T>\.{m}\b", src), m


def test_init_and_op_table_binding():
    src = PAS.read_text()
    assert re.search(r"procedure initHIP\(const deviceIndex: SizeInt; const srssQuirk: boolean = true;"
                     r"\s+const pipelineBackward: boolean = true\);", src)
    i = src.index("procedure initHIP(const deviceIndex: SizeInt; const srssQuirk: boolean;")
    body = src[i:src.index("end;", i)]
    assert "tns_set_option(TNS_OPT_SRSS_QUIRK, 1)" in body   # initHIP applies the drop
    # ... and, by default, the pipelined conv backward the bench headlines
    assert re.search(r"if pipelineBackward then\s+tns_set_option\(TNS_OPT_BWD_OVERLAP, 2\)", body)
    assert "procedure useHipOpTable(const srssQuirk: boolean = true);" in src
    assert "tns_set_option(TNS_OPT_SRSS_QUIRK, 1)" in src
    for slot, fn in [("gemm", "tns_cblas_sgemm"), ("gemmStridedBatched",
                                                   "tns_cblas_sgemm_batch_strided"),
                     ("im2Colvv", "tns_im2col"), ("col2imvv", "tns_col2im"),
                     ("im2colStridedBatchedvv", "tns_im2col_strided_batched"),
                     ("col2imStridedBatchedvv", "tns_col2im_strided_batched")]:
        assert re.search(rf"TSingleTensor\.{slot}\s*:= @{fn};", src), slot


@pytest.mark.parametrize("name", ["tns_hip_gemm", "tns_hip_conv_backward_bn",
                                  "tns_hip_sgemm_strided_batched_multi", "tns_hip_means",
                                  "tns_hip_variances", "tns_hip_gemm_batched"])
def test_spot_widths(name):
    decls = parse_pascal_externals()
    protos = parse_header()
    assert decls[name] == protos[name]

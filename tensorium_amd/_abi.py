"""ctypes prototypes for libtensorium_hip.so (mirror of include/tns.h).

The library is the product: this module only declares argument types.  It
never substitutes a CPU implementation — if the ``.so`` is missing or a HIP
device is absent, calls fail loudly (``TnsError``).
"""
from __future__ import annotations

import ctypes as C
import os
import re
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
LIB_PATH = PKG / "libtensorium_hip.so"
HEADER = ROOT / "include" / "tns.h"

i32, i64, u8, f32 = C.c_int32, C.c_int64, C.c_uint8, C.c_float
fptr = C.c_void_p  # float* (host or device)
vp = C.c_void_p

# enum values (ntensors.pas:106-128, ntypes.pas:66-71)
CblasRowMajor, CblasColMajor = 101, 102
CblasNoTrans, CblasTrans = 111, 112
ACT = dict(LOGISTIC=0, RELU=1, RELU6=2, RELIE=3, LINEAR=4, RAMP=5, TANH=6, PLSE=7,
           REVLEAKY=8, LEAKY=9, ELU=10, LOGGY=11, STAIR=12, HARDTAN=13, LHTAN=14, SELU=15)
TNS_OK = 0
TNS_OP_GEMM, TNS_OP_IM2COL, TNS_OP_COL2IM, TNS_OP_BIAS, TNS_OP_ACTIVATE = range(5)
TNS_OPT_STRICT_BETA0 = 0
TNS_OPT_CONV_VARIANT, TNS_OPT_CONV_PAD, TNS_OPT_NT_SDOT, TNS_OPT_SRSS_QUIRK = 1, 2, 3, 4
TNS_OPT_TT_EXACT = 5
TNS_OPT_SDOT_FORM = 6
TNS_OPT_DX_FUSED = 7
TNS_OPT_DX_TILE = 8
TNS_OPT_DW_TILE = 9
TNS_OPT_BWD_OVERLAP = 10
TNS_OPT_DX_CONV = 11
TNS_OPT_DW_RES = 12
TNS_OPT_DERIVE_SUMS = 13
TNS_OPT_SCRATCH_CAP = 14

_CONV = [i64] * 11  # aChannels .. dilationX

PROTOTYPES: dict[str, tuple] = {
    "tns_abi_version": (C.c_int, []),
    "tns_last_error": (C.c_char_p, []),
    "tns_clear_error": (None, []),
    "tns_set_error_hook": (None, [vp]),
    "tns_device_count": (C.c_int, []),
    "tns_set_option": (C.c_int, [i32, i64]),
    # boundary A
    "tns_cblas_sgemm": (None, [i32, i32, i32, i64, i64, i64, f32, fptr, i64, fptr, i64, f32,
                               fptr, i64]),
    "tns_cblas_sgemm_batch_strided": (None, [i32, i32, i32, i64, i64, i64, f32, fptr, i64, i64,
                                             fptr, i64, i64, f32, fptr, i64, i64, i64]),
    "tns_im2col": (None, [*_CONV, fptr, i64, fptr, i64, u8]),
    "tns_col2im": (None, [*_CONV, fptr, i64, fptr, i64, i64, u8]),
    "tns_im2col_strided_batched": (None, [*_CONV, fptr, i64, i64, fptr, i64, i64, i64]),
    "tns_col2im_strided_batched": (None, [*_CONV, fptr, i64, i64, fptr, i64, i64, i64]),
    # boundary B
    "tns_hip_create": (C.c_int, [i32, C.POINTER(vp)]),
    "tns_hip_destroy": (C.c_int, [vp]),
    "tns_hip_set_stream": (C.c_int, [vp, vp]),
    "tns_hip_get_stream": (vp, [vp]),
    "tns_hip_pending_dw": (C.c_int, [vp]),
    "tns_hip_finish": (C.c_int, [vp]),
    "tns_hip_malloc": (C.c_int, [vp, i64, C.POINTER(vp)]),
    "tns_hip_free": (C.c_int, [vp, vp]),
    "tns_hip_write_buffer": (C.c_int, [vp, fptr, i64, vp]),
    "tns_hip_read_buffer": (C.c_int, [vp, fptr, i64, vp]),
    "tns_hip_gemm": (C.c_int, [vp, u8, u8, i64, i64, i64, f32, fptr, i64, i64, fptr, i64, i64,
                               f32, fptr, i64, i64]),
    "tns_hip_gemm_strided_batched": (C.c_int, [vp, u8, u8, i64, i64, i64, f32, fptr, i64, i64,
                                               i64, fptr, i64, i64, i64, f32, fptr, i64, i64,
                                               i64, i64]),
    "tns_hip_im2col": (C.c_int, [vp, *_CONV, fptr, i64, fptr, i64]),
    "tns_hip_im2col_strided_batched": (C.c_int, [vp, *_CONV, fptr, i64, i64, fptr, i64, i64,
                                                 i64]),
    "tns_hip_col2im": (C.c_int, [vp, *_CONV, fptr, i64, fptr, i64]),
    "tns_hip_col2im_strided_batched": (C.c_int, [vp, *_CONV, fptr, i64, i64, fptr, i64, i64,
                                                 i64]),
    "tns_hip_forward_bias": (C.c_int, [vp, i64, fptr, i64, i64, fptr, i64, i64]),
    "tns_hip_backward_bias": (C.c_int, [vp, i64, fptr, i64, fptr, i64, i64, i64]),
    "tns_hip_activate_array": (C.c_int, [vp, i64, fptr, i64, i32]),
    "tns_hip_derive_array": (C.c_int, [vp, i64, fptr, i64, i32, fptr]),
    "tns_hip_axpy": (C.c_int, [vp, i64, f32, fptr, i64, i64, fptr, i64, i64]),
    "tns_hip_sgd_update": (C.c_int, [vp, i64, fptr, fptr, i64, fptr, fptr, fptr, fptr, f32, f32,
                                     f32]),
    "tns_hip_scale": (C.c_int, [vp, i64, f32, fptr, i64]),
    "tns_hip_fill": (C.c_int, [vp, i64, fptr, i64, f32, i64]),
    "tns_hip_copy": (C.c_int, [vp, i64, fptr, i64, i64, fptr, i64, i64]),
    "tns_hip_clamp": (C.c_int, [vp, i64, f32, fptr, fptr, i64, i64]),
    "tns_hip_conv2d": (C.c_int, [vp, i64, i64, i64, i64, fptr, fptr, i64, i64, i64, i64, i64,
                                 i64, i64, i64, i64, fptr, fptr]),
    "tns_hip_conv_forward": (C.c_int, [vp, i64, i64, i64, i64, fptr, fptr, fptr, i64, i64, i64,
                                       i64, i64, i32, fptr, fptr, i32]),
    "tns_hip_conv_backward": (C.c_int, [vp, i64, i64, i64, i64, fptr, fptr, i64, i64, i64, i64,
                                        i64, i32, fptr, fptr, fptr, fptr, fptr, fptr]),
    "tns_hip_conv_forward_train": (C.c_int, [vp, i64, i64, i64, i64, fptr, fptr, i64, i64, i64,
                                             i64, i64, i32, fptr, fptr, fptr, fptr, f32, i32,
                                             fptr, fptr, fptr, fptr, fptr, fptr]),
    "tns_hip_conv_backward_bn": (C.c_int, [vp, i64, i64, i64, i64, fptr, fptr, i64, i64, i64,
                                           i64, i64, i32, fptr, fptr, fptr, fptr, fptr, fptr,
                                           fptr, fptr, fptr, fptr, fptr, fptr, fptr]),
    "tns_hip_set_telemetry": (C.c_int, [vp, i32]),
    "tns_gemm_variant_count": (C.c_int, []),
    "tns_sdot_chains_variant_count": (C.c_int, []),
    "tns_sdot_rc_variant_count": (C.c_int, []),
    "tns_conv_tile_variant_count": (C.c_int, []),
    "tns_conv_dx_tile_count": (C.c_int, []),
    "tns_conv_dx_conv_count": (C.c_int, []),
    "tns_conv_dw_res_count": (C.c_int, []),
    "tns_conv_dw_tile_count": (C.c_int, []),
    "tns_conv_tile_variant_name": (C.c_char_p, [C.c_int32]),
    "tns_conv_slab_count": (C.c_int, []),
    "tns_conv1x1_count": (C.c_int, []),
    "tns_conv1x1_name": (C.c_char_p, [C.c_int32]),
    "tns_conv_slab_name": (C.c_char_p, [C.c_int32]),
    "tns_conv_pp_variant_count": (C.c_int, []),
    "tns_conv_pp_variant_name": (C.c_char_p, [C.c_int32]),
    "tns_conv_dma_variant_count": (C.c_int, []),
    "tns_conv_dma_variant_name": (C.c_char_p, [C.c_int32]),
    "tns_conv_patch_variant_count": (C.c_int, []),
    "tns_conv_patch_variant_name": (C.c_char_p, [C.c_int32]),
    "tns_sdot_chains_variant_name": (C.c_char_p, [C.c_int32]),
    "tns_sdot_rc_variant_name": (C.c_char_p, [C.c_int32]),
    "tns_gemm_variant_name": (C.c_char_p, [i32]),
    "tns_hip_gemm_variant": (C.c_int, [vp, i32, u8, u8, i64, i64, i64, f32, fptr, i64, i64, i64,
                                       fptr, i64, i64, i64, f32, fptr, i64, i64, i64, i64]),
    "tns_hip_op_ms": (C.c_double, [vp, i32]),
}


class TnsError(RuntimeError):
    pass


_lib = None


def header_symbols() -> list[str]:
    """Function names declared in include/tns.h (the exported C ABI)."""
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"\b(tns_[a-z0-9_]+)\s*\(", text)
    seen: list[str] = []
    for n in names:
        if n not in seen and not n.endswith("_t"):
            seen.append(n)
    return seen


def load(path: str | os.PathLike | None = None) -> C.CDLL:
    """Load libtensorium_hip.so (in-tree) and attach prototypes.  Raises
    TnsError if the library has not been built — there is no fallback."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    # TNS_LIB: an alternative build of the same library (A/B perf runs)
    p = Path(path) if path else Path(os.environ.get("TNS_LIB") or LIB_PATH)
    if not p.exists():
        raise TnsError(f"{p} not built — run `python -m tensorium_amd.build` "
                       "(the HIP backend has no CPU fallback)")
    lib = C.CDLL(str(p), mode=C.RTLD_GLOBAL)
    # (an A/B build of an older revision may lack entry points added since;
    # only the in-tree library must export every one)
    older = bool(os.environ.get("TNS_LIB")) and path is None
    for name, (res, args) in PROTOTYPES.items():
        if older and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


def check(rc: int) -> None:
    if rc != TNS_OK:
        lib = load()
        msg = lib.tns_last_error().decode(errors="replace")
        lib.tns_clear_error()  # consumed: a later op-table call starts clean
        raise TnsError(f"tns status {rc}: {msg}")


PROTOTYPES.update({
    "tns_hip_shortcut": (C.c_int, [vp, i64, fptr, i64, fptr, i64, fptr, i64, i32]),
    "tns_hip_upsample": (C.c_int, [vp, i64, i64, i64, i64, fptr, i64, i32, f32, fptr, i32]),
    "tns_hip_addvv": (C.c_int, [vp, i64, fptr, i64, i64, fptr, i64, i64, fptr, i64, i64]),
    "tns_hip_subvv": (C.c_int, [vp, i64, fptr, i64, i64, fptr, i64, i64, fptr, i64, i64]),
    "tns_hip_mulvv": (C.c_int, [vp, i64, fptr, i64, i64, fptr, i64, i64, fptr, i64, i64]),
    "tns_hip_fmavv": (C.c_int, [vp, i64, fptr, i64, i64, fptr, i64, i64, fptr, i64, i64, fptr,
                                i64, i64]),
    "tns_hip_fmavss": (C.c_int, [vp, i64, fptr, i64, f32, f32, fptr]),
    "tns_hip_inverse_sqrt": (C.c_int, [vp, i64, f32, fptr, fptr, i64, i64]),
    "tns_hip_sgemm_strided_batched_multi": (C.c_int, [C.POINTER(i32), i32, u8, u8, i64, i64, i64,
                                                      f32, fptr, i64, i64, fptr, i64, i64, f32,
                                                      fptr, i64, i64, i64]),
    "tns_set_op_devices": (C.c_int, [C.POINTER(i32), i32]),
    "tns_hip_yolo_forward": (C.c_int, [vp, i64, i64, i64, i64, fptr, fptr]),
    "tns_hip_means_and_vars": (C.c_int, [vp, i64, i64, i64, fptr, i64, fptr, fptr]),
    "tns_hip_means": (C.c_int, [vp, i64, i64, i64, fptr, i64, fptr]),
    "tns_hip_variances": (C.c_int, [vp, i64, i64, i64, fptr, i64, fptr, fptr]),
    "tns_hip_gemm_batched": (C.c_int, [vp, u8, u8, i64, i64, i64, f32, vp, i64, i64, vp, i64, i64,
                                       f32, vp, i64, i64, i64]),
    "tns_hip_normalize": (C.c_int, [vp, i64, i64, i64, fptr, i64, fptr, i64, fptr, i64]),
    "tns_hip_forward_scale": (C.c_int, [vp, i64, fptr, i64, i64, fptr, i64, i64]),
    "tns_hip_forward_scale_add": (C.c_int, [vp, i64, fptr, i64, i64, fptr, fptr, i64, i64]),
    "tns_hip_means_and_vars_delta": (C.c_int, [vp, i64, i64, i64, fptr, fptr, i64, fptr, fptr,
                                               fptr, fptr]),
    "tns_hip_normalize_delta": (C.c_int, [vp, i64, i64, i64, fptr, fptr, i64, fptr, fptr, fptr,
                                          fptr]),
    "tns_hip_add_dots": (C.c_int, [vp, i64, i64, i64, fptr, fptr, i64, fptr]),
    "tns_hip_softmax_batch": (C.c_int, [vp, i64, fptr, i64, i64, i64, i64, i64, i64, f32, fptr,
                                        i64]),
    "tns_hip_cross_entropy_softmax": (C.c_int, [vp, i64, fptr, fptr, fptr, fptr]),
    "tns_hip_sum": (C.c_int, [vp, i64, fptr, i64, fptr]),
    "tns_mlp_buffer_floats": (i64, [i32, C.POINTER(i64), i32, i64]),
    "tns_hip_mlp_train_step": (C.c_int, [vp, i32, C.POINTER(i64), C.POINTER(i32), i32, i64, fptr,
                                         fptr, f32, f32, f32, fptr, fptr]),
})

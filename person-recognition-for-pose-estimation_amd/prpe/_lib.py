"""ctypes binding of libprpe.so (the C ABI declared in include/prpe.h).

This is the only way the product reaches the device kernels: there is no CPU or
PyTorch fallback. ``lib()`` raises if the library is missing, was built for another ABI
version, or was built from other sources than the ones beside it (``prpe_source_hash``
against prpe/_srchash.py), and every call raises ``PrpeError`` on a non-zero status.
"""
from __future__ import annotations

import ctypes as C
import os

from ._srchash import source_hash

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libprpe.so")
ABI_VERSION = 10


class PrpeError(RuntimeError):
    pass


class View(C.Structure):
    _fields_ = [("ptr", C.c_void_p),
                ("n", C.c_int32), ("h", C.c_int32), ("w", C.c_int32), ("c", C.c_int32),
                ("sn", C.c_int64), ("sh", C.c_int64), ("sw", C.c_int64), ("sc", C.c_int64)]


class ConvDesc(C.Structure):
    _fields_ = [("x", View), ("y", View), ("res", View),
                ("kh", C.c_int32), ("kw", C.c_int32), ("stride", C.c_int32), ("pad", C.c_int32),
                ("w_hi", C.c_void_p), ("w_lo", C.c_void_p), ("w_lo2", C.c_void_p),
                ("k_pad", C.c_int32), ("co_pad", C.c_int32),
                ("scale", C.c_void_p), ("bias", C.c_void_p), ("slope", C.c_void_p),
                ("in_scale", C.c_void_p), ("in_bias", C.c_void_p),
                ("act", C.c_int32), ("res_mode", C.c_int32), ("precision", C.c_int32), ("tile", C.c_int32),
                ("k_order", C.c_int32),
                ("w_h16", C.c_void_p), ("w_l16", C.c_void_p), ("scale16", C.c_void_p),
                ("x_amax", C.c_void_p), ("y_amax", C.c_void_p),
                ("x2", View), ("x2_amax", C.c_void_p), ("x_planes", C.c_int32), ("y_planes", C.c_int32),
                ("w2", C.c_void_p), ("y2", View),
                ("w3", C.c_void_p), ("scale2", C.c_void_p), ("bias2", C.c_void_p), ("act2", C.c_int32),
                ("n2", C.c_int32), ("workspace", C.c_void_p), ("workspace_bytes", C.c_int64)]


class BneckDesc(C.Structure):
    _fields_ = [("x", View), ("y", View), ("x_amax", C.c_void_p), ("y_amax", C.c_void_p), ("mid", C.c_int32),
                ("w_h16", C.c_void_p * 3), ("w_l16", C.c_void_p * 3), ("k_pad", C.c_int32 * 3),
                ("scale16", C.c_void_p * 3), ("bias", C.c_void_p * 3)]


class StemDesc(C.Structure):
    _fields_ = [("x", C.c_void_p), ("xsn", C.c_int64), ("xsh", C.c_int64), ("n", C.c_int32), ("h", C.c_int32),
                ("w", C.c_int32), ("x_amax", C.c_void_p), ("w_h16", C.c_void_p), ("w_l16", C.c_void_p),
                ("k_pad", C.c_int32), ("scale16", C.c_void_p), ("bias", C.c_void_p), ("y", View),
                ("y_amax", C.c_void_p)]


ACT = {"none": 0, "relu": 1, "silu": 2, "prelu": 3, "gelu": 4, "sigmoid": 5}
RES_NONE, RES_PRE, RES_POST = 0, 1, 2

# symbol -> (restype, argtypes); exactly the entry points of include/prpe.h
_P = C.c_void_p
_I = C.c_int32
_L = C.c_int64
_F = C.c_float
_VP = C.POINTER(View)
SIGNATURES = {
    "prpe_conv2d_workspace_bytes": (C.c_int64, [C.POINTER(ConvDesc)]),
    "prpe_conv2d": (C.c_int, [C.POINTER(ConvDesc), _P]),
    "prpe_bottleneck": (C.c_int, [C.POINTER(BneckDesc), _P]),
    "prpe_stem_maxpool": (C.c_int, [C.POINTER(StemDesc), _P]),
    "prpe_upconv3x3_workspace_bytes": (C.c_int64, [_VP, _VP]),
    "prpe_upconv3x3": (C.c_int, [_VP, _VP, _I, _P, _P, _P, _I, _I, _P, _P, _L, _P]),
    "prpe_dwconv": (C.c_int, [_VP, _VP, _VP, _P, _I, _I, _I, _P, _P, _I, _P]),
    "prpe_maxpool": (C.c_int, [_VP, _VP, _I, _I, _I, _P]),
    "prpe_upsample_nearest2x": (C.c_int, [_VP, _VP, _P]),
    "prpe_copy_pad": (C.c_int, [_VP, _VP, _P, _P]),
    "prpe_norm_sigmoid": (C.c_int, [_VP, _VP, _P]),
    "prpe_layernorm": (C.c_int, [_P, _L, _P, _L, _L, _I, _P, _P, _F, _I, _P]),
    "prpe_attention": (C.c_int, [_P, _P, _I, _I, _I, _I, _F, _P]),
    "prpe_attention_strided": (C.c_int, [_P, _L, _L, _L, _L, _P, _I, _I, _I, _I, _F, _I, _P]),
    "prpe_psa_attention": (C.c_int, [_VP, _VP, _VP, _I, _I, _I, _F, _P]),
    "prpe_dfl_decode": (C.c_int, [_P, _P, _I, _I, _I, C.POINTER(C.c_int32), C.POINTER(C.c_float), _P]),
    "prpe_l2norm": (C.c_int, [_P, _P, _P, _I, _I, C.c_float, _P]),
    "prpe_nms_workspace_bytes": (C.c_int64, [_I, _I, _I, _I]),
    "prpe_nms": (C.c_int, [_P, _I, _I, _I, _I, _F, _F, _I, _I, _P, _P, _P, _L, _P]),
    "prpe_softargmax": (C.c_int, [_P, _I, _I, _I, _I, _P, _P, _P, _P, _P]),
    "prpe_flip_average": (C.c_int, [_P, _P, _P, _I, _I, _I, _I, C.POINTER(C.c_int32), _I, _P]),
    "prpe_ce_argmax": (C.c_int, [_P, _L, _I, _I, _P, _P, _P, _P, _P]),
    "prpe_det_metrics_update_workspace_bytes": (C.c_int64, [_I]),
    "prpe_det_metrics_update": (C.c_int, [_P, _P, _I, _I, _P, _P, _I, _P, _P, _L, _P, _L, _P]),
    "prpe_det_metrics_compute_workspace_bytes": (C.c_int64, [_L]),
    "prpe_det_metrics_compute": (C.c_int, [_P, _P, _L, _P, _P, _P, _L, _P]),
    "prpe_det_eval_loss": (C.c_int, [_P, _P, _P, _P, _I, _I, _I, _P, _P, _P, _I, _P, _P, _P]),
    "prpe_abi_version": (C.c_int, []),
    "prpe_build_info": (C.c_char_p, []),
    "prpe_source_hash": (C.c_char_p, []),
}

_lib = None


def lib():
    """Load libprpe.so once; raise loudly when it is missing (no fallback path exists)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise PrpeError(f"{LIB_PATH} not found: build it with "
                            "`python person-recognition-for-pose-estimation_amd/build.py` "
                            "(the HIP path has no CPU fallback)")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        if L.prpe_abi_version() != ABI_VERSION:
            raise PrpeError("libprpe.so ABI version mismatch; rebuild")
        check_source_hash(L.prpe_source_hash().decode())
        _lib = L
    return _lib


def check_source_hash(built: str, present: str | None = None):
    """Refuse a library built from other sources than the ones beside it (a stale prebuilt
    .so would otherwise load silently). ``present`` defaults to the hash of the sources on disk."""
    present = source_hash() if present is None else present
    if present is None:
        raise PrpeError("prpe sources (csrc/, include/prpe.h) not found beside libprpe.so: cannot verify the build")
    if built != present:
        raise PrpeError(f"{LIB_PATH} is stale: built from sources {built[:16]}, the sources here hash to "
                        f"{present[:16]}; rebuild with `python person-recognition-for-pose-estimation_amd/build.py`")


def check(status: int, what: str):
    if status != 0:
        raise PrpeError(f"{what} failed with status {status}")

"""ctypes binding of libvissm.so (include/vissm.h).

The product path calls the HIP kernels only through this module.  There is no
CPU or PyTorch fallback: if the library is missing or a call fails, an error is
raised.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

_HERE = os.path.dirname(os.path.abspath(__file__))
# VISSM_LIB selects an alternative build of the same library (A/B timing of kernel variants)
LIB_PATH = os.environ.get("VISSM_LIB", os.path.join(_HERE, "libvissm.so"))

VISSM_PREC_FP32 = 0
VISSM_PREC_BF16 = 1
VISSM_PREC_BF16X3 = 2
VISSM_PREC_BF16X2 = 3   # split-bf16 weights, bf16 activations in every weight product (forward and backward)
VISSM_PREC_BF16X2_BF16 = 4   # vissm_flow_ar_elbo_fused only: split-weight recompute, bf16 backward products
# host-level modes (not C-ABI precisions): forward products at the first precision (the values that reach
# the ELBO: ELBO within 1e-4 of the float64 oracle), backward products bf16 (gradients at bf16 accuracy)
VISSM_PREC_BF16X3F = 16   # forward bf16x3
VISSM_PREC_BF16X2F = 17   # forward bf16x2 (the weights' rounding removed: two MFMAs per product instead of three)
HOST_MODES = {VISSM_PREC_BF16X3F: (VISSM_PREC_BF16X3, VISSM_PREC_BF16),
              VISSM_PREC_BF16X2F: (VISSM_PREC_BF16X2, VISSM_PREC_BF16)}
# training-step precision modes by name (main.py / bench.py --precision, tests)
TRAIN_PRECISIONS = {"fp32": VISSM_PREC_FP32, "bf16": VISSM_PREC_BF16, "bf16x3": VISSM_PREC_BF16X3,
                    "bf16x2": VISSM_PREC_BF16X2, "bf16x3f": VISSM_PREC_BF16X3F, "bf16x2f": VISSM_PREC_BF16X2F}

MODEL_AR, MODEL_LV, MODEL_SV, MODEL_FHN = 0, 1, 2, 3

_c_void_p = ctypes.c_void_p
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_u64 = ctypes.c_uint64
_f32 = ctypes.c_float
_size_t = ctypes.c_size_t


class FlowDesc(ctypes.Structure):
    _fields_ = [(n, _i32) for n in ("B", "L", "k", "H", "n_hidden", "bn", "stride2", "swap_out",
                                    "n_logsig", "n_win", "precision", "chunk_tiles", "u_pitch",
                                    "out_pitch")]


class FlowParams(ctypes.Structure):
    _fields_ = ([(n, _c_void_p) for n in ("w_eps", "w_hid", "b_hid", "bn_g", "bn_b", "w_head", "b_head",
                                          "theta_x", "w_theta", "b_theta")] + [("theta_rank", _i32)])


class FlowGrads(ctypes.Structure):
    _fields_ = [(n, _c_void_p) for n in ("w_eps", "w_hid", "b_hid", "bn_g", "bn_b", "w_head", "b_head")]


class ElboDesc(ctypes.Structure):
    _fields_ = [("model", _i32), ("B", _i32), ("M", _i32), ("n_win", _i32), ("dt", _f32), ("obs_std", _f32)]


class GatherDesc(ctypes.Structure):
    _fields_ = [("n", _i32), ("len", _i32), ("C", _i32), ("stride", _i32), ("offset", _i64), ("j_step", _i64),
                ("c_pitch", _i64), ("os_r", _i64), ("os_j", _i64), ("os_c", _i64)]


class FeatDesc(ctypes.Structure):
    _fields_ = [(n, _i32) for n in ("n_win", "Lf", "Cin", "H", "k", "stride", "Lh")] + [("in_win_stride", _i64)]


class FeatParams(ctypes.Structure):
    _fields_ = [("w", _c_void_p * 4), ("b", _c_void_p * 4), ("conv_w", _c_void_p), ("conv_b", _c_void_p)]


class FeatGrads(ctypes.Structure):
    _fields_ = [("w", _c_void_p * 4), ("b", _c_void_p * 4), ("conv_w", _c_void_p), ("conv_b", _c_void_p)]


class LvFeatDesc(ctypes.Structure):
    _fields_ = ([(n, _i32) for n in ("n_win", "R", "Cin", "H")] + [("in_win_stride", _i64)] +
                [("n_layers", _i32), ("sv_diff", _i32)])


GEMM_F32, GEMM_ELU_BF16, GEMM_DELU_BF16 = 0, 1, 2


class GemmDesc(ctypes.Structure):
    _fields_ = ([(n, _i64) for n in ("M", "N", "K", "lda", "ldb", "ldc")] +
                [(n, _i32) for n in ("a_kmajor", "b_kmajor", "epilogue", "split_k")])


THETA_MAX_P, THETA_MAX_BIJ = 5, 8


class ThetaDesc(ctypes.Structure):
    _fields_ = [("B", _i32), ("P", _i32), ("n_bij", _i32), ("relu", _i32), ("base_loc", _f32), ("base_scale", _f32),
                ("perm", (_i32 * THETA_MAX_P) * (THETA_MAX_BIJ - 1))]


class ElboData(ctypes.Structure):
    _fields_ = [(n, _c_void_p) for n in ("win", "obs", "obs_bin", "mask", "shift", "dim_one", "plain_from",
                                        "obs_list")] + [("obs_stride", ctypes.c_int32)]


# exported symbol -> (restype, argtypes); tests check that every symbol of include/vissm.h is here
SIGNATURES = {
    "vissm_last_error": (ctypes.c_char_p, []),
    "vissm_version": (_i32, []),
    "vissm_source_hash": (ctypes.c_char_p, []),
    "vissm_build_flags": (ctypes.c_char_p, []),
    "vissm_normal_base": (_i32, [_u64, _u64, _c_void_p, _c_void_p, _i32, _i32, _i32, _c_void_p]),
    "vissm_normal_base_dev": (_i32, [_u64, _c_void_p, _c_void_p, _c_void_p, _i32, _i32, _i32, _c_void_p]),
    "vissm_base_logprob": (_i32, [_c_void_p, _c_void_p, _i32, _i32, _i32, _c_void_p]),
    "vissm_flow_workspace_size": (_size_t, [ctypes.POINTER(FlowDesc), _i32]),
    "vissm_flow_geometry": (_i32, [ctypes.POINTER(FlowDesc), _i32, ctypes.POINTER(_i32)]),
    "vissm_flow_fwd": (_i32, [ctypes.POINTER(FlowDesc), ctypes.POINTER(FlowParams), _c_void_p, _c_void_p,
                              _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _size_t, _c_void_p]),
    "vissm_flow_bwd": (_i32, [ctypes.POINTER(FlowDesc), ctypes.POINTER(FlowParams), _c_void_p, _c_void_p,
                              _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                              ctypes.POINTER(FlowGrads), _c_void_p, _size_t, _c_void_p]),
    "vissm_flow_kernel_precision": (_i32, [ctypes.POINTER(FlowDesc)]),
    "vissm_flow_ar_elbo_fused_supported": (_i32, [ctypes.POINTER(FlowDesc)]),
    "vissm_flow_ar_elbo_fused_workspace_size": (_size_t, [ctypes.POINTER(FlowDesc)]),
    "vissm_flow_ar_elbo_fused": (_i32, [ctypes.POINTER(FlowDesc), ctypes.POINTER(FlowParams), _c_void_p, _c_void_p,
                                        _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _f32, _f32,
                                        _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                                        ctypes.POINTER(FlowGrads), _c_void_p, _size_t, _c_void_p]),
    "vissm_feat_workspace_size": (_size_t, [ctypes.POINTER(FeatDesc)]),
    "vissm_feat_fwd": (_i32, [ctypes.POINTER(FeatDesc), ctypes.POINTER(FeatParams), _c_void_p, _c_void_p, _c_void_p,
                              _c_void_p]),
    "vissm_feat_bwd": (_i32, [ctypes.POINTER(FeatDesc), ctypes.POINTER(FeatParams), _c_void_p, _c_void_p, _c_void_p,
                              ctypes.POINTER(FeatGrads), _c_void_p, _size_t, _c_void_p]),
    "vissm_lv_mlp_workspace_size": (_size_t, [ctypes.POINTER(LvFeatDesc)]),
    "vissm_lv_mlp_fwd": (_i32, [ctypes.POINTER(LvFeatDesc), ctypes.POINTER(FeatParams), _c_void_p, _c_void_p,
                                _c_void_p, _c_void_p, _c_void_p]),
    "vissm_lv_mlp_bwd": (_i32, [ctypes.POINTER(LvFeatDesc), ctypes.POINTER(FeatParams), _c_void_p, _c_void_p,
                                _c_void_p, _i32, ctypes.POINTER(FeatGrads), _c_void_p, _size_t, _c_void_p]),
    "vissm_lv_pack": (_i32, [_c_void_p, _c_void_p, _i32, _i32, _i32, _c_void_p, _c_void_p, _c_void_p, _i32, _i32,
                             _i32, _c_void_p, _c_void_p, _c_void_p]),
    "vissm_lv_conv_diag": (_i32, [_c_void_p, _i32, _c_void_p, _i32, _i32, _i32, _i32, _c_void_p, _c_void_p]),
    "vissm_lv_conv_diag_bwd": (_i32, [_c_void_p, _i32, _i32, _i32, _i32, _i32, _i32, _c_void_p, _c_void_p,
                                      _c_void_p, _c_void_p]),
    "vissm_lv_conv_wscatter": (_i32, [_c_void_p, _i32, _i32, _i32, _i32, _c_void_p, _c_void_p]),
    "vissm_gemm_workspace_size": (_size_t, [ctypes.POINTER(GemmDesc)]),
    "vissm_gemm_bf16": (_i32, [ctypes.POINTER(GemmDesc), _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                               _size_t, _c_void_p]),
    "vissm_gemm_bf16x3_workspace_size": (_size_t, [ctypes.POINTER(GemmDesc)]),
    "vissm_gemm_bf16x3": (_i32, [ctypes.POINTER(GemmDesc)] + [_c_void_p] * 7 + [_size_t, _c_void_p]),
    "vissm_elbo_fwd": (_i32, [ctypes.POINTER(ElboDesc), ctypes.POINTER(ElboData), _c_void_p, _c_void_p,
                              _c_void_p, _c_void_p, _c_void_p, _c_void_p]),
    "vissm_elbo_bwd": (_i32, [ctypes.POINTER(ElboDesc), ctypes.POINTER(ElboData), _c_void_p, _c_void_p,
                              _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p]),
    "vissm_elbo_fwd_theta_grad": (_i32, [ctypes.POINTER(ElboDesc), ctypes.POINTER(ElboData)] + [_c_void_p] * 10),
    "vissm_elbo_fwd_grad": (_i32, [ctypes.POINTER(ElboDesc), ctypes.POINTER(ElboData)] + [_c_void_p] * 11),
    "vissm_adamax_workspace_size": (_size_t, [_i64]),
    "vissm_adamax_step": (_i32, [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _i64, _f32, _f32, _f32, _f32,
                                 _f32, _c_void_p, _c_void_p, _size_t, _c_void_p]),
    "vissm_adamax_step_guarded": (_i32, [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _i64, _f32, _f32, _f32, _f32,
                                         _f32, _c_void_p, _c_void_p, _c_void_p, _size_t, _c_void_p]),
    "vissm_sqnorm": (_i32, [_c_void_p, _i64, _c_void_p, _c_void_p, _size_t, _c_void_p]),
    "vissm_reduce_rows": (_i32, [_c_void_p, _c_void_p, _i64, _i64, _c_void_p]),
    "vissm_reduce_rows_bf16": (_i32, [_c_void_p, _c_void_p, _i64, _i64, _c_void_p]),
    "vissm_split_bf16": (_i32, [_c_void_p, _c_void_p, _c_void_p, _i64, _c_void_p]),
    "vissm_gather_windows": (_i32, [ctypes.POINTER(GatherDesc), _c_void_p, _c_void_p, _c_void_p, _c_void_p]),
    "vissm_theta_num_params": (_i32, [_i32, _i32]),
    "vissm_theta_workspace_size": (_size_t, [ctypes.POINTER(ThetaDesc)]),
    "vissm_theta_fwd": (_i32, [ctypes.POINTER(ThetaDesc), _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                               _c_void_p]),
    "vissm_theta_branch_fwd": (_i32, [_i32] * 5 + [_c_void_p] * 10 + [_c_void_p]),
    "vissm_theta_branch_bwd_workspace_size": (_size_t, [_i32, _i32]),
    "vissm_theta_branch_bwd": (_i32, [_i32] * 5 + [_c_void_p] * 15 + [_size_t, _c_void_p]),
    "vissm_theta_bwd": (_i32, [ctypes.POINTER(ThetaDesc), _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                               _c_void_p, _c_void_p, _size_t, _c_void_p]),
    "vissm_profile_enable": (None, [_i32]),
    "vissm_profile_read": (_i32, [_i32, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_i64)]),
    "vissm_profile_reset": (None, []),
    "vissm_profile_bytes": (_i32, [_i32, ctypes.POINTER(ctypes.c_double)]),
}

PROF_FLOW_FWD, PROF_FLOW_BWD, PROF_ELBO_FWD, PROF_ELBO_BWD, PROF_NORMAL = 0, 1, 2, 3, 4
PROF_FLOW_BWD_NODU, PROF_FLOW_BWD_DU, PROF_FLOW_FUSED = 5, 6, 7


class VissmError(RuntimeError):
    pass


_lib: Optional[ctypes.CDLL] = None


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libvissm.so (raises if it is missing: there is no fallback path)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise VissmError(
            f"libvissm.so not found at {path}; build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "or `make -C viforssms_amd/csrc`")
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    check_source_hash(lib, path)
    _lib = lib
    return lib


def check_source_hash(lib: ctypes.CDLL, path: str = LIB_PATH) -> str:
    """Refuse a library that was not built from this tree's sources (a stale or foreign `.so`): the hash compiled
    into it (vissm_source_hash, Makefile) must equal srchash.source_hash() of the sources next to this module."""
    from . import srchash
    built = lib.vissm_source_hash().decode()
    want = srchash.source_hash()
    if built != want:
        raise VissmError(
            f"{path} was built from other sources (library {built[:16]}, tree {want[:16]}): rebuild it with "
            "`make -C viforssms_amd/csrc` or `python -c 'import __graft_entry__ as g; g.build()'`")
    return built


def check(rc: int, what: str):
    if rc != 0:
        msg = load().vissm_last_error()
        raise VissmError(f"{what} failed (rc={rc}): {msg.decode() if msg else ''}")


def flow_geometry(desc: FlowDesc, which: int) -> dict:
    """vissm_flow_geometry: the launch geometry the kernels pick for `desc` (which: 0 forward, 1 backward,
    2 the fused last AR flow).  Host arithmetic only, callable without a GPU."""
    out = (_i32 * 4)()
    check(load().vissm_flow_geometry(ctypes.byref(desc), which, out), "vissm_flow_geometry")
    return {"tile": out[0], "chunk_tiles": out[1], "n_chunks": out[2], "n_groups": out[3]}


def ptr(t) -> Optional[int]:
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()


def stream_handle(device=None) -> int:
    import torch
    return torch.cuda.current_stream(device).cuda_stream

"""torch.autograd wrappers around the libvissm HIP kernels.

Each Function's forward and backward is exactly one C-ABI call (plus
caller-allocated workspace from torch's caching allocator, so no hipMalloc
happens on the step path).  Tensors must be contiguous fp32 on the current
HIP device.
"""
from __future__ import annotations

import ctypes
import os
import dataclasses
from dataclasses import dataclass
from typing import Optional

import torch

from . import _lib
from ._lib import FlowDesc, FlowParams, FlowGrads, ElboDesc, ElboData, GatherDesc, check, ptr


_FORCE_DU = os.environ.get("VISSM_FORCE_DU") == "1"  # A/B timing hook: always compute the flows' du


def _require_gpu(*ts):
    for t in ts:
        if t is None:
            continue
        if not t.is_cuda:
            raise _lib.VissmError("libvissm kernels run on the GPU only; got a CPU tensor "
                                  "(there is deliberately no CPU fallback)")
        if t.dtype not in (torch.float32, torch.int32):
            raise _lib.VissmError(f"expected fp32/int32 tensors, got {t.dtype}")
        if not t.is_contiguous():
            raise _lib.VissmError("expected contiguous tensors")


def _require_rows(*ts):
    """As _require_gpu for [B, n] row tensors that may lie a pitch apart (VissmFlowDesc.u_pitch / out_pitch)."""
    for t in ts:
        _require_gpu(t[0] if t.dim() == 2 and t.stride(1) == 1 else t)   # one row: unit stride


def _workspace(nbytes: int, device) -> torch.Tensor:
    return torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=device)


# ---------------------------------------------------------------------------------------
# base noise
# ---------------------------------------------------------------------------------------
def normal_base(seed: int, offset: int, B: int, L: int, n_last: int, device) -> (torch.Tensor, torch.Tensor):
    """init_dist.slp (AR.py:31-35): eps ~ N(0,1) [B, L] and the base log-prob over the last n_last entries."""
    lib = _lib.load()
    eps = torch.empty(B, L, dtype=torch.float32, device=device)
    lp = torch.empty(B, dtype=torch.float32, device=device)
    check(lib.vissm_normal_base(ctypes.c_uint64(seed & (2 ** 64 - 1)), ctypes.c_uint64(offset), ptr(eps), ptr(lp),
                                B, L, n_last, _lib.stream_handle(device)), "vissm_normal_base")
    return eps, lp


def normal_base_dev(seed: int, offset_dev: torch.Tensor, B: int, L: int, n_last: int):
    """normal_base with the Philox row offset in a device uint64 (int64 storage) tensor."""
    lib = _lib.load()
    if not (offset_dev.is_cuda and offset_dev.dtype == torch.int64 and offset_dev.numel() == 1):
        raise _lib.VissmError("normal_base_dev: offset must be one int64 on the GPU")
    dev = offset_dev.device
    eps = torch.empty(B, L, dtype=torch.float32, device=dev)
    lp = torch.empty(B, dtype=torch.float32, device=dev)
    check(lib.vissm_normal_base_dev(ctypes.c_uint64(seed & (2 ** 64 - 1)), ptr(offset_dev), ptr(eps), ptr(lp),
                                    B, L, n_last, _lib.stream_handle(dev)), "vissm_normal_base_dev")
    return eps, lp


def base_logprob(eps: torch.Tensor, n_last: int) -> torch.Tensor:
    lib = _lib.load()
    _require_gpu(eps)
    B, L = eps.shape
    lp = torch.empty(B, dtype=torch.float32, device=eps.device)
    check(lib.vissm_base_logprob(ptr(eps), ptr(lp), B, L, n_last, _lib.stream_handle(eps.device)),
          "vissm_base_logprob")
    return lp


# ---------------------------------------------------------------------------------------
# split-bf16 operand planes
# ---------------------------------------------------------------------------------------
def _dense_layout(t: torch.Tensor) -> bool:
    """t covers its storage span densely in some dimension order (a contiguous tensor or a permuted view of one)."""
    dims = sorted((st, sz) for st, sz in zip(t.stride(), t.shape) if sz > 1)
    expect = 1
    for st, sz in dims:
        if st != expect:
            return False
        expect *= sz
    return True


def theta_branch_fwd(theta, W0, b0, W1, b1, W2, b2, term: bool = True):
    """The flows' theta-branch forward (include/vissm.h vissm_theta_branch_fwd; nma._ThetaBranchK): the collapsed
    weights (Wc, bc) and, if term, theta_term = theta Wc + bc -- (theta_term or None, Wc, bc)."""
    lib = _lib.load()
    _require_gpu(W0, b0, W1, b1, W2, b2)
    P, n0 = W0.shape
    n1, H = W1.shape[1], W2.shape[1]
    dev = W0.device
    ws = [t.contiguous().float() for t in (W0, b0, W1, b1, W2, b2)]
    Wc, bc = torch.empty(P, H, device=dev), torch.empty(H, device=dev)
    tt, th, B = None, None, 0
    if term:
        th = theta.contiguous().float()
        B = th.shape[0]
        tt = torch.empty(B, H, device=dev)
    check(lib.vissm_theta_branch_fwd(B, P, n0, n1, H, ptr(th), *[ptr(t) for t in ws], ptr(Wc), ptr(bc), ptr(tt),
                                     _lib.stream_handle(dev)), "vissm_theta_branch_fwd")
    return tt, Wc, bc


def theta_branch_bwd(theta, d, W0, b0, W1, b1, W2):
    """The flows' theta-branch backward (include/vissm.h vissm_theta_branch_bwd; nma._ThetaBranch): dtheta and the
    gradients of (W0, b0, W1, b1, W2, b2) from d = d loss / d theta_term, in three launches."""
    lib = _lib.load()
    _require_gpu(theta, d, W0, b0, W1, b1, W2)
    B, P = theta.shape
    n0, n1, H = W0.shape[1], W1.shape[1], W2.shape[1]
    dev = d.device
    args = [t.contiguous().float() for t in (theta, d, W0, b0, W1, b1, W2)]
    outs = [torch.empty(sh, device=dev) for sh in ((B, P), (P, n0), (n0,), (n0, n1), (n1,), (n1, H), (H,))]
    nb = lib.vissm_theta_branch_bwd_workspace_size(B, P)
    ws = _workspace(nb, dev)
    check(lib.vissm_theta_branch_bwd(B, P, n0, n1, H, *[ptr(t) for t in args], *[ptr(t) for t in outs], ptr(ws), nb,
                                     _lib.stream_handle(dev)), "vissm_theta_branch_bwd")
    return tuple(outs)


def split_bf16(x: torch.Tensor):
    """(hi, lo) bf16 planes with x = hi + lo to ~2^-16 relative (vissm_split_bf16, one pass over x), laid out with
    x's strides: x may be a transposed view (LV's time-mixing features)."""
    if not x.is_cuda or x.dtype != torch.float32:
        raise _lib.VissmError("split_bf16: fp32 GPU tensor expected (there is deliberately no CPU fallback)")
    if not _dense_layout(x):
        x = x.contiguous()
    hi = torch.empty_strided(x.shape, x.stride(), dtype=torch.bfloat16, device=x.device)
    lo = torch.empty_strided(x.shape, x.stride(), dtype=torch.bfloat16, device=x.device)
    if x.data_ptr() % 16:
        x = x.clone(memory_format=torch.preserve_format)
    check(_lib.load().vissm_split_bf16(ptr(x), ptr(hi), ptr(lo), x.numel(), _lib.stream_handle(x.device)),
          "vissm_split_bf16")
    return hi, lo


# ---------------------------------------------------------------------------------------
# window gather
# ---------------------------------------------------------------------------------------
def gather_windows(src: torch.Tensor, starts: torch.Tensor, out: torch.Tensor, n: int, length: int, C: int,
                   stride: int = 1, offset: int = 0, j_step: int = 1, c_pitch: int = 0, os=None) -> torch.Tensor:
    """out[r*os_r + j*os_j + c*os_c] = src.flat[c*c_pitch + stride*starts[r] + offset + j*j_step]
    (vissm_gather_windows: the train loop's window gather, AR.py:267-288, from a device-resident table)."""
    _require_gpu(src, starts, out)
    if starts.dtype != torch.int32 or src.dtype != torch.float32:
        raise _lib.VissmError("gather_windows: int32 starts and fp32 tables expected")
    os_r, os_j, os_c = os
    d = GatherDesc(n, length, C, stride, offset, j_step, c_pitch, os_r, os_j, os_c)
    check(_lib.load().vissm_gather_windows(ctypes.byref(d), ptr(src), ptr(starts), ptr(out),
                                           _lib.stream_handle(src.device)), "vissm_gather_windows")
    return out


# ---------------------------------------------------------------------------------------
# IAF flow
# ---------------------------------------------------------------------------------------
@dataclass(frozen=True)
class FlowShape:
    B: int
    L: int
    k: int
    H: int
    n_hidden: int
    bn: bool
    stride2: bool
    swap_out: bool
    n_logsig: int
    n_win: int
    precision: int = _lib.VISSM_PREC_FP32
    bwd_precision: Optional[int] = None   # the backward kernel's precision when it differs (VISSM_PREC_BF16X3F)
    chunk_tiles: int = 0                  # VissmFlowDesc.chunk_tiles: 0 = automatic launch geometry
    pad_out: bool = False                 # u_next rows padded to 16 floats (it feeds another flow, whose du stores
                                          # are then 64-byte aligned)

    def desc(self, u_pitch: int = 0, out_pitch: int = 0) -> FlowDesc:
        return FlowDesc(self.B, self.L, self.k, self.H, self.n_hidden, int(self.bn), int(self.stride2),
                        int(self.swap_out), self.n_logsig, self.n_win, self.precision, int(self.chunk_tiles),
                        int(u_pitch), int(out_pitch))

    @property
    def Lout(self):
        return self.L - self.k

    @property
    def Lh(self):
        return self.Lout // (2 if self.stride2 else 1)


def kernel_precision(shape: FlowShape) -> int:
    """vissm_flow_kernel_precision: the precision the flow kernels compute `shape` in (its own, or fp32 where the
    matrix-core kernels do not cover it)."""
    rc = _lib.load().vissm_flow_kernel_precision(ctypes.byref(shape.desc()))
    if rc < 0:
        check(rc, "vissm_flow_kernel_precision")
    return rc


def _flow_params(w_eps, w_hid, b_hid, bn_g, bn_b, w_head, b_head, tf=None) -> FlowParams:
    """VissmFlowParams; tf = (theta [B, R], w_theta [R, H], b_theta [H]) is the theta branch's factorization
    (theta_term = theta w_theta + b_theta), which the two-sample AR kernels fold into their layer-0 product."""
    if tf is None:
        return FlowParams(ptr(w_eps), ptr(w_hid), ptr(b_hid), ptr(bn_g), ptr(bn_b), ptr(w_head), ptr(b_head))
    th, wt, bt = tf
    _require_gpu(th, wt, bt)
    if not (th.is_contiguous() and wt.is_contiguous() and bt.is_contiguous()) or th.shape[1] != wt.shape[0]:
        raise _lib.VissmError("theta factors: contiguous theta [B, R], w_theta [R, H], b_theta [H] expected")
    return FlowParams(ptr(w_eps), ptr(w_hid), ptr(b_hid), ptr(bn_g), ptr(bn_b), ptr(w_head), ptr(b_head),
                      ptr(th), ptr(wt), ptr(bt), int(th.shape[1]))


# ---------------------------------------------------------------------------------------
# window-shared feature branch + the first conv's feature channels (vissm_feat_fwd / _bwd)
# ---------------------------------------------------------------------------------------
class FeatConvFn(torch.autograd.Function):
    """C [n_win, Lh, H] = conv_b + the feature channels of the first conv over F = the four dense + ELU layers
    of the window's time features h0 [n_win, Lf, Cin] (AR.py:53-62; SV_dense.py:53-62; fitz_nag_NVP.py:71-79), one
    HIP launch each way (the torch form is ~40 small launches per flow).  The gradient reaches the four dense
    layers and the conv kernel (its sample channel 0 gets zero here: that part is the flow kernel's w_eps) and
    bias; h0 is data."""

    @staticmethod
    def forward(ctx, h0, s, Lh, W0, b0, W1, b1, W2, b2, W3, b3, conv_w, conv_b):
        ws = (W0, b0, W1, b1, W2, b2, W3, b3, conv_w, conv_b)
        _require_gpu(*ws)
        n_win, Lf, Cin = h0.shape
        if not h0.is_cuda or h0.dtype != torch.float32 or h0.stride(2) != 1 or h0.stride(1) != Cin:
            h0 = h0.contiguous()
            _require_gpu(h0)
        H, k = W3.shape[1], conv_w.shape[0]
        d = _lib.FeatDesc(n_win, Lf, Cin, H, k, s, Lh, h0.stride(0) if n_win > 1 else Lf * Cin)
        p = _feat_params(ws)
        C = torch.empty(n_win, Lh, H, dtype=torch.float32, device=h0.device)
        act = torch.empty(4, n_win, Lf, H, dtype=torch.float32, device=h0.device)
        check(_lib.load().vissm_feat_fwd(ctypes.byref(d), ctypes.byref(p), ptr(h0), ptr(C), ptr(act),
                                         _lib.stream_handle(h0.device)), "vissm_feat_fwd")
        ctx.save_for_backward(h0, act, *ws)
        ctx.desc = d
        return C

    @staticmethod
    def backward(ctx, dC):
        h0, act, *ws = ctx.saved_tensors
        d = ctx.desc
        dC = dC.contiguous()
        gr = [torch.empty_like(t) for t in ws]
        g = _lib.FeatGrads((ctypes.c_void_p * 4)(*[ptr(t) for t in gr[0:8:2]]),
                           (ctypes.c_void_p * 4)(*[ptr(t) for t in gr[1:8:2]]), ptr(gr[8]), ptr(gr[9]))
        lib = _lib.load()
        nb = lib.vissm_feat_workspace_size(ctypes.byref(d))
        if nb == 0:
            raise _lib.VissmError(f"vissm_feat_workspace_size failed: {lib.vissm_last_error().decode()}")
        wsb = _workspace(nb, dC.device)
        check(lib.vissm_feat_bwd(ctypes.byref(d), ctypes.byref(_feat_params(ws)), ptr(h0), ptr(act), ptr(dC),
                                 ctypes.byref(g), ptr(wsb), nb, _lib.stream_handle(dC.device)), "vissm_feat_bwd")
        return (None, None, None, *gr)


def _feat_params(ws) -> "_lib.FeatParams":
    return _lib.FeatParams((ctypes.c_void_p * 4)(*[ptr(t) for t in ws[0:8:2]]),
                           (ctypes.c_void_p * 4)(*[ptr(t) for t in ws[1:8:2]]), ptr(ws[8]), ptr(ws[9]))


def feat_conv(h0, s: int, Lh: int, W0, b0, W1, b1, W2, b2, W3, b3, conv_w, conv_b):
    return FeatConvFn.apply(h0, s, Lh, W0, b0, W1, b1, W2, b2, W3, b3, conv_w, conv_b)


# ---------------------------------------------------------------------------------------
# bf16 matrix-core GEMM (vissm_gemm_bf16) and Lotka-Volterra's feature branch built on it (vissm_lv_*)
# ---------------------------------------------------------------------------------------
def gemm_bf16(M: int, N: int, K: int, A, lda: int, a_kmajor: bool, B, ldb: int, b_kmajor: bool, C, ldc: int,
              epilogue: int = 0, aux=None, split_k: int = 1):
    """C[m][n] = sum_k A[m][k] B[k][n] on bf16 operands (layouts: include/vissm.h VissmGemmDesc); C fp32 or, for the
    ELU / elu' epilogues, bf16."""
    lib = _lib.load()
    d = _lib.GemmDesc(M, N, K, lda, ldb, ldc, int(a_kmajor), int(b_kmajor), epilogue, split_k)
    nb = lib.vissm_gemm_workspace_size(ctypes.byref(d))
    ws = _workspace(nb, C.device) if nb else None
    check(lib.vissm_gemm_bf16(ctypes.byref(d), ptr(A), ptr(B), ptr(C), ptr(aux) if aux is not None else None,
                              ptr(ws) if ws is not None else None, nb, _lib.stream_handle(C.device)), "vissm_gemm_bf16")


def gemm_bf16x3(M: int, N: int, K: int, A, A_lo, lda: int, a_kmajor: bool, B, B_lo, ldb: int, b_kmajor: bool, C,
                ldc: int, epilogue: int = 0, aux=None, split_k: int = 1):
    """C = A_hi B_hi + A_hi B_lo + A_lo B_hi: the split-bf16 form of gemm_bf16, fp32-class products (fp32 C, or for
    the ELU / elu' epilogues a [2][M][ldc] bf16 hi / lo plane pair, aux the same)"""
    lib = _lib.load()
    d = _lib.GemmDesc(M, N, K, lda, ldb, ldc, int(a_kmajor), int(b_kmajor), epilogue, split_k)
    nb = lib.vissm_gemm_bf16x3_workspace_size(ctypes.byref(d))
    ws = _workspace(nb, C.device) if nb else None
    check(lib.vissm_gemm_bf16x3(ctypes.byref(d), ptr(A), ptr(A_lo), ptr(B), ptr(B_lo), ptr(C),
                                ptr(aux) if aux is not None else None, ptr(ws) if ws is not None else None, nb,
                                _lib.stream_handle(C.device)), "vissm_gemm_bf16x3")


def _r8(n: int) -> int:
    return (n + 7) // 8 * 8


class LvFeatConvFn(torch.autograd.Function):
    """Lotka-Volterra's window-shared conv input C [n_win, Lh, H] (lotka_volterra_partial.py:71-82): the three dense +
    ELU layers of the window's time features h0 [n_win, R, Cin] (fp32, vissm_lv_mlp_*), the time-mixing layer
    D = elu(H3 W3 + b3) [R, U] and the conv over D's R channels (transposed by the reference, U its time axis) as
    matrix-core GEMMs (vissm_gemm_bf16: the layer with its ELU in the epilogue, then G = D^T Wc [U, k H] and the
    conv's diagonal sum), and the backward the same way (dD with elu' in the epilogue, dWc = D dG, dW3 = H3^T dP and
    dH3 = dP W3^T split over K).  x3 = False: the bf16 precision's arithmetic (the torch form: fp32 layers,
    linear_bf16 conv) plus bf16 operands in the time-mixing layer.  x3 = True (the parity precisions): every product
    in the split-bf16 form (vissm_gemm_bf16x3, fp32-class; D and dP kept as hi / lo plane pairs).  The gradient
    reaches the four dense layers and the conv kernel (its sample channel 0 gets zero: the flow kernel's w_eps) and
    bias."""

    @staticmethod
    def _mm(x3, M, N, K, A, lda, akm, B, ldb, bkm, C, ldc, epi=0, aux=None, split=1):
        """C = A B with A / B (hi, lo) pairs: one bf16 product (x3 False: the hi planes) or the split-bf16 form"""
        if x3:
            gemm_bf16x3(M, N, K, A[0], A[1], lda, akm, B[0], B[1], ldb, bkm, C, ldc, epi, aux, split)
        else:
            gemm_bf16(M, N, K, A[0], lda, akm, B[0], ldb, bkm, C, ldc, epi, aux, split)

    @staticmethod
    def forward(ctx, h0, s, Lh, x3, W0, b0, W1, b1, W2, b2, W3, b3, conv_w, conv_b):
        ws = (W0, b0, W1, b1, W2, b2, W3, b3, conv_w, conv_b)
        _require_gpu(*ws)
        n_win, R, Cin = h0.shape
        if h0.dtype != torch.float32 or h0.stride(2) != 1 or h0.stride(1) != Cin:
            h0 = h0.contiguous()
        _require_gpu(h0)
        H, U, k = W0.shape[1], W3.shape[1], conv_w.shape[0]
        if tuple(conv_w.shape) != (k, 1 + R, H) or s * (Lh - 1) + k > U or H >= 64:
            raise _lib.VissmError(f"lv_feat: conv_w {tuple(conv_w.shape)}, R {R}, U {U}, Lh {Lh}, s {s}: shapes "
                                  "do not match")
        dev = h0.device
        Up, NC = _r8(U), _r8(k * H)
        npl = 2 if x3 else 1   # bf16 planes per operand
        lib, st = _lib.load(), _lib.stream_handle(dev)
        d = _lib.LvFeatDesc(n_win, R, Cin, H, h0.stride(0) if n_win > 1 else R * Cin, 3, 0)
        p = _feat_params(ws)
        act = torch.empty(3, n_win, R, H, dtype=torch.float32, device=dev)
        H3b = torch.empty(npl, n_win, R, 64, dtype=torch.bfloat16, device=dev)
        check(lib.vissm_lv_mlp_fwd(ctypes.byref(d), ctypes.byref(p), ptr(h0), ptr(act), ptr(H3b[0]),
                                   ptr(H3b[1]) if x3 else None, st), "vissm_lv_mlp_fwd")
        W3b = torch.empty(npl, 64, Up, dtype=torch.bfloat16, device=dev)
        Wc = torch.empty(npl, R, NC, dtype=torch.bfloat16, device=dev)
        check(lib.vissm_lv_pack(ptr(W3), ptr(b3), H, U, Up, ptr(W3b[0]), ptr(W3b[1]) if x3 else None, ptr(conv_w), R,
                                k, NC, ptr(Wc[0]), ptr(Wc[1]) if x3 else None, st), "vissm_lv_pack")
        D = torch.empty(n_win, npl, R, Up, dtype=torch.bfloat16, device=dev)   # hi (/ lo) planes per window
        G = torch.empty(U, NC, dtype=torch.float32, device=dev)
        C = torch.empty(n_win, Lh, H, dtype=torch.float32, device=dev)
        sk = int(os.environ.get("VISSM_LV_SPLIT", "5"))
        mm = LvFeatConvFn._mm
        for w in range(n_win):
            mm(x3, R, U, 64, H3b[:, w], 64, False, W3b, Up, True, D[w], Up, _lib.GEMM_ELU_BF16)
            mm(x3, U, NC, R, D[w], Up, True, Wc, NC, True, G, NC, split=sk)
            check(lib.vissm_lv_conv_diag(ptr(G), NC, ptr(conv_b), H, k, s, Lh, ptr(C[w]), st), "vissm_lv_conv_diag")
        ctx.save_for_backward(h0, act, H3b, D, W3b, Wc, *ws)
        ctx.dims = (d, n_win, R, H, U, k, s, Lh, Up, NC, x3)
        return C

    @staticmethod
    def backward(ctx, dC):
        h0, act, H3b, D, W3b, Wc, *ws = ctx.saved_tensors
        d, n_win, R, H, U, k, s, Lh, Up, NC, x3 = ctx.dims
        dev = dC.device
        dC = dC.contiguous()
        npl = 2 if x3 else 1
        lib, st = _lib.load(), _lib.stream_handle(dev)
        dG = torch.empty(npl, U, NC, dtype=torch.bfloat16, device=dev)
        dP = torch.empty(npl, R, Up, dtype=torch.bfloat16, device=dev)
        dWc = torch.empty(n_win, R, NC, dtype=torch.float32, device=dev)
        dW3b = torch.empty(n_win, 64, U, dtype=torch.float32, device=dev)
        dH3 = torch.empty(n_win, R, 64, dtype=torch.float32, device=dev)
        dcb = torch.empty(n_win, H, dtype=torch.float32, device=dev)
        sk = int(os.environ.get("VISSM_LV_SPLIT", "5"))
        sw = int(os.environ.get("VISSM_LV_SPLIT_W3", "8"))
        mm = LvFeatConvFn._mm
        for w in range(n_win):
            check(lib.vissm_lv_conv_diag_bwd(ptr(dC[w]), H, k, s, Lh, U, NC, ptr(dG[0]), ptr(dG[1]) if x3 else None,
                                             ptr(dcb[w]), st), "vissm_lv_conv_diag_bwd")
            mm(x3, R, U, NC, Wc, NC, False, dG, NC, False, dP, Up, _lib.GEMM_DELU_BF16, aux=D[w])
            mm(x3, R, NC, U, D[w], Up, False, dG, NC, True, dWc[w], NC, split=sk)
            mm(x3, 64, U, R, H3b[:, w], 64, True, dP, Up, True, dW3b[w], U, split=sw)
            mm(x3, R, 64, U, dP, Up, False, W3b, Up, False, dH3[w], 64, split=sw)
        if n_win > 1:   # (the reference's LV windows: one per step at the benchmark shapes)
            dWc, dW3b, dcb = dWc.sum(0, keepdim=True), dW3b.sum(0, keepdim=True), dcb.sum(0, keepdim=True)
        gr = [torch.empty_like(t) for t in ws[:6]]
        dconv_w = torch.empty_like(ws[8])
        check(lib.vissm_lv_conv_wscatter(ptr(dWc[0]), NC, R, k, H, ptr(dconv_w), st), "vissm_lv_conv_wscatter")
        g = _lib.FeatGrads((ctypes.c_void_p * 4)(ptr(gr[0]), ptr(gr[2]), ptr(gr[4]), None),
                           (ctypes.c_void_p * 4)(ptr(gr[1]), ptr(gr[3]), ptr(gr[5]), None), None, None)
        nb = lib.vissm_lv_mlp_workspace_size(ctypes.byref(d))
        if nb == 0:
            raise _lib.VissmError(f"vissm_lv_mlp_workspace_size failed: {lib.vissm_last_error().decode()}")
        wsb = _workspace(nb, dev)
        check(lib.vissm_lv_mlp_bwd(ctypes.byref(d), ctypes.byref(_feat_params(ws)), ptr(h0), ptr(act), ptr(dH3), 64,
                                   ctypes.byref(g), ptr(wsb), nb, st), "vissm_lv_mlp_bwd")
        return (None, None, None, None, *gr, dW3b[0, :H], dW3b[0, H], dconv_w, dcb[0])


def lv_feat_conv(h0, s: int, Lh: int, W0, b0, W1, b1, W2, b2, W3, b3, conv_w, conv_b, x3: bool = False):
    return LvFeatConvFn.apply(h0, s, Lh, bool(x3), W0, b0, W1, b1, W2, b2, W3, b3, conv_w, conv_b)


class SvFeatConvFn(torch.autograd.Function):
    """Stochastic volatility's window-shared conv input C [n_win, Lh, H] (SV_dense.py:50-62): the four dense + ELU
    layers over the window's time features with their first differences (the input assembly inside the kernel:
    vissm_lv_mlp_* at n_layers = 4, sv_diff = 1; fp32), then the conv over the 50 feature channels at kernel_len 50
    as one split-bf16 matrix-core GEMM G = F [Wc_0 | .. | Wc_{k-1}] (vissm_gemm_bf16x3: fp32-class products, the
    torch form's fp32 arithmetic to ~1e-6) and its diagonal sum; backward: dG (hi / lo planes), dF = dG Wc^T and
    dWc = F^T dG the same way, then the four layers' gradients.  ts [n_win, L, Cr] gets no gradient (data)."""

    @staticmethod
    def forward(ctx, ts, s, Lh, W0, b0, W1, b1, W2, b2, W3, b3, conv_w, conv_b):
        ws = (W0, b0, W1, b1, W2, b2, W3, b3, conv_w, conv_b)
        _require_gpu(*ws)
        n_win, L, Cr = ts.shape
        if ts.dtype != torch.float32 or ts.stride(2) != 1 or ts.stride(1) != Cr:
            ts = ts.contiguous()
        _require_gpu(ts)
        R, Cin = L - 1, 2 * Cr - 2
        H, k = W0.shape[1], conv_w.shape[0]
        if (tuple(W0.shape) != (Cin, H) or tuple(W3.shape) != (H, H) or tuple(conv_w.shape) != (k, 1 + H, H)
                or s * (Lh - 1) + k > R or H >= 64):
            raise _lib.VissmError(f"sv_feat: ts {tuple(ts.shape)}, W0 {tuple(W0.shape)}, conv_w {tuple(conv_w.shape)}, "
                                  f"Lh {Lh}, s {s}: shapes do not match")
        dev = ts.device
        NC = k * H
        NCp = _r8(NC)
        lib, st = _lib.load(), _lib.stream_handle(dev)
        d = _lib.LvFeatDesc(n_win, R, Cin, H, ts.stride(0) if n_win > 1 else L * Cr, 4, 1)
        act = torch.empty(4, n_win, R, H, dtype=torch.float32, device=dev)
        Fh = torch.empty(n_win, R, 64, dtype=torch.bfloat16, device=dev)
        Fl = torch.empty_like(Fh)
        check(lib.vissm_lv_mlp_fwd(ctypes.byref(d), ctypes.byref(_feat_params(ws)), ptr(ts), ptr(act), ptr(Fh),
                                   ptr(Fl), st), "vissm_lv_mlp_fwd")
        Wch = torch.empty(H, NCp, dtype=torch.bfloat16, device=dev)
        Wcl = torch.empty_like(Wch)
        check(lib.vissm_lv_pack(None, None, H, 0, 0, None, None, ptr(conv_w), H, k, NCp, ptr(Wch), ptr(Wcl), st),
              "vissm_lv_pack")
        G = torch.empty(R, NCp, dtype=torch.float32, device=dev)
        C = torch.empty(n_win, Lh, H, dtype=torch.float32, device=dev)
        for w in range(n_win):
            gemm_bf16x3(R, NC, H, Fh[w], Fl[w], 64, False, Wch, Wcl, NCp, True, G, NCp)
            check(lib.vissm_lv_conv_diag(ptr(G), NCp, ptr(conv_b), H, k, s, Lh, ptr(C[w]), st), "vissm_lv_conv_diag")
        ctx.save_for_backward(ts, act, Fh, Fl, Wch, Wcl, *ws)
        ctx.dims = (d, n_win, R, H, k, s, Lh, NC, NCp)
        return C

    @staticmethod
    def backward(ctx, dC):
        ts, act, Fh, Fl, Wch, Wcl, *ws = ctx.saved_tensors
        d, n_win, R, H, k, s, Lh, NC, NCp = ctx.dims
        dev = dC.device
        dC = dC.contiguous()
        lib, st = _lib.load(), _lib.stream_handle(dev)
        dGh = torch.empty(R, NCp, dtype=torch.bfloat16, device=dev)
        dGl = torch.empty_like(dGh)
        dF = torch.empty(n_win, R, H, dtype=torch.float32, device=dev)
        dWc = torch.empty(n_win, H, NC, dtype=torch.float32, device=dev)
        dcb = torch.empty(n_win, H, dtype=torch.float32, device=dev)
        for w in range(n_win):
            check(lib.vissm_lv_conv_diag_bwd(ptr(dC[w]), H, k, s, Lh, R, NCp, ptr(dGh), ptr(dGl), ptr(dcb[w]), st),
                  "vissm_lv_conv_diag_bwd")
            # dF = dG Wc^T (K = k H, split over it: R / 128 row tiles alone would leave the chip empty)
            gemm_bf16x3(R, H, NC, dGh, dGl, NCp, False, Wch, Wcl, NCp, False, dF[w], H, split_k=16)
            # dWc = F^T dG (K = R)
            gemm_bf16x3(H, NC, R, Fh[w], Fl[w], 64, True, dGh, dGl, NCp, True, dWc[w], NC, split_k=8)
        if n_win > 1:
            dWc, dcb = dWc.sum(0, keepdim=True), dcb.sum(0, keepdim=True)
        gr = [torch.empty_like(t) for t in ws[:8]]
        dconv_w = torch.empty_like(ws[8])
        check(lib.vissm_lv_conv_wscatter(ptr(dWc[0]), NC, H, k, H, ptr(dconv_w), st), "vissm_lv_conv_wscatter")
        g = _lib.FeatGrads((ctypes.c_void_p * 4)(ptr(gr[0]), ptr(gr[2]), ptr(gr[4]), ptr(gr[6])),
                           (ctypes.c_void_p * 4)(ptr(gr[1]), ptr(gr[3]), ptr(gr[5]), ptr(gr[7])), None, None)
        nb = lib.vissm_lv_mlp_workspace_size(ctypes.byref(d))
        if nb == 0:
            raise _lib.VissmError(f"vissm_lv_mlp_workspace_size failed: {lib.vissm_last_error().decode()}")
        wsb = _workspace(nb, dev)
        check(lib.vissm_lv_mlp_bwd(ctypes.byref(d), ctypes.byref(_feat_params(ws)), ptr(ts), ptr(act), ptr(dF), H,
                                   ctypes.byref(g), ptr(wsb), nb, st), "vissm_lv_mlp_bwd")
        return (None, None, None, *gr, dconv_w, dcb[0])


def sv_feat_conv(ts, s: int, Lh: int, W0, b0, W1, b1, W2, b2, W3, b3, conv_w, conv_b):
    return SvFeatConvFn.apply(ts, s, Lh, W0, b0, W1, b1, W2, b2, W3, b3, conv_w, conv_b)


class MAFlowFn(torch.autograd.Function):
    """One IAF flow (IAF._create_flow, AR.py:50-85) -> (u_next, logsig)."""

    @staticmethod
    def forward(ctx, shape: FlowShape, win, u, C, theta_term, w_eps, w_hid, b_hid, bn_g, bn_b, w_head, b_head,
                tf=None):
        lib = _lib.load()
        u = _rows(u, shape.L)
        _require_rows(u)
        _require_gpu(C, theta_term, w_eps, w_hid, b_hid, bn_g, bn_b, w_head, b_head, win)
        dev = u.device
        pout = (shape.Lout + 15) // 16 * 16 if shape.pad_out else shape.Lout
        d = shape.desc(_pitch(u, shape.L), pout)
        u_next = _rows_empty(shape.B, shape.Lout, pout, dev)
        logsig = torch.empty(shape.B, dtype=torch.float32, device=dev)
        wsz = lib.vissm_flow_workspace_size(ctypes.byref(d), 0)
        if wsz == 0:
            check(-1, "vissm_flow_workspace_size")
        ws = _workspace(wsz, dev)
        prm = _flow_params(w_eps, w_hid, b_hid, bn_g, bn_b, w_head, b_head, tf)
        check(lib.vissm_flow_fwd(ctypes.byref(d), ctypes.byref(prm), ptr(u), ptr(C), ptr(win), ptr(theta_term),
                                 ptr(u_next), ptr(logsig), ptr(ws), wsz, _lib.stream_handle(dev)),
              "vissm_flow_fwd")
        ctx.shape = shape
        # the theta-fold factors are constants here (theta_term carries their gradient) but are saved like the
        # rest, so autograd's version check catches an in-place change between forward and backward
        tf = tuple(tf) if tf is not None else ()
        ctx.n_tf = len(tf)
        ctx.save_for_backward(win, u, C, theta_term, w_eps, w_hid, b_hid, bn_g, bn_b, w_head, b_head, *tf)
        return u_next, logsig

    @staticmethod
    def backward(ctx, g_next, g_ls):
        lib = _lib.load()
        shape: FlowShape = ctx.shape
        saved = ctx.saved_tensors
        win, u, C, theta_term, w_eps, w_hid, b_hid, bn_g, bn_b, w_head, b_head = saved[:11]
        tf = tuple(saved[11:]) if ctx.n_tf else None
        dev = u.device
        if g_next is None:
            g_next = torch.zeros(shape.B, shape.Lout, dtype=torch.float32, device=dev)
        if g_ls is None:
            g_ls = torch.zeros(shape.B, dtype=torch.float32, device=dev)
        g_next = _rows(g_next, shape.Lout)
        g_ls = g_ls.contiguous()
        if shape.bwd_precision is not None:
            shape = dataclasses.replace(shape, precision=shape.bwd_precision, bwd_precision=None)
        u = _rows(u, shape.L)
        pu = _pitch(u, shape.L)
        d = shape.desc(pu, _pitch(g_next, shape.Lout))
        # the base noise needs no gradient: the bf16 kernels then skip the transposed convolution (the exact-fp32
        # kernels a shape beyond flow5 falls back to always write du)
        need_du = ctx.needs_input_grad[2] or kernel_precision(shape) == _lib.VISSM_PREC_FP32 or _FORCE_DU
        du = _rows_empty(shape.B, shape.L, pu, dev) if need_du else None   # du rows at u's pitch
        dC = torch.empty_like(C)
        dth = torch.empty_like(theta_term)
        gw = [torch.empty_like(t) if t is not None else None for t in (w_eps, w_hid, b_hid, bn_g, bn_b, w_head, b_head)]
        grads = FlowGrads(*[ptr(t) for t in gw])
        wsz = lib.vissm_flow_workspace_size(ctypes.byref(d), 1)
        ws = _workspace(wsz, dev)
        prm = _flow_params(w_eps, w_hid, b_hid, bn_g, bn_b, w_head, b_head, tf)
        check(lib.vissm_flow_bwd(ctypes.byref(d), ctypes.byref(prm), ptr(u), ptr(C), ptr(win), ptr(theta_term),
                                 ptr(g_next), ptr(g_ls), ptr(du), ptr(dC), ptr(dth), ctypes.byref(grads), ptr(ws),
                                 wsz, _lib.stream_handle(dev)), "vissm_flow_bwd")
        return (None, None, du, dC, dth, *gw, None)


def _rows(t: torch.Tensor, n: int) -> torch.Tensor:
    """t as rows of n unit-stride floats at some pitch >= n (VissmFlowDesc.u_pitch / out_pitch); copied only when it
    is not (a transposed or sliced-column view)."""
    if t.stride(1) != 1 or (t.shape[0] > 1 and t.stride(0) < n):
        t = t.contiguous()
    return t


def _pitch(t: torch.Tensor, n: int) -> int:
    return t.stride(0) if t.shape[0] > 1 else n


def _rows_empty(B: int, n: int, pitch: int, device) -> torch.Tensor:
    """[B, n] float32 rows `pitch` floats apart (a column slice of a [B, pitch] buffer)."""
    buf = torch.empty(B, pitch, dtype=torch.float32, device=device)
    return buf if pitch == n else buf[:, :n]


def ma_flow(shape: FlowShape, win, u, C, theta_term, w_eps, w_hid, b_hid, bn_g, bn_b, w_head, b_head, tf=None):
    return MAFlowFn.apply(shape, win, u, C, theta_term, w_eps, w_hid, b_hid, bn_g, bn_b, w_head, b_head, tf)


def ar_fused_supported(shape: FlowShape) -> bool:
    d = shape.desc()
    return bool(_lib.load().vissm_flow_ar_elbo_fused_supported(ctypes.byref(d)))


def ar_last_flow_fused(shape: FlowShape, win, u, C, theta_term, theta, obs, obs_bin, obs_std: float, scale: float,
                       w_eps, w_hid, b_hid, w_head, b_head, tf=None):
    """The last AR(1) flow fused with its ELBO terms (vissm_flow_ar_elbo_fused): one backward-style pass that
    recomputes the flow's output x and differentiates loss = -scale sum_b (sde + obs + logsig) w.r.t. u, C,
    theta_term and the flow's weights (no autograd: the caller routes them; the theta dependence of sde goes
    through vissm_elbo_bwd on x).  Returns (x [B, Lout], logsig [B], du, dC, dtheta_term,
    [g_w_eps, g_w_hid, g_b_hid, g_w_head, g_b_head])."""
    lib = _lib.load()
    u = _rows(u, shape.L)
    _require_rows(u)
    _require_gpu(C, theta_term, theta, obs, obs_bin, w_eps, w_hid, b_hid, w_head, b_head, win)
    dev = u.device
    pu = _pitch(u, shape.L)
    d = shape.desc(pu, 0)
    wsz = lib.vissm_flow_ar_elbo_fused_workspace_size(ctypes.byref(d))
    if wsz == 0:
        raise _lib.VissmError("vissm_flow_ar_elbo_fused: unsupported flow shape")
    ws = _workspace(wsz, dev)
    x = torch.empty(shape.B, shape.Lout, dtype=torch.float32, device=dev)
    logsig = torch.empty(shape.B, dtype=torch.float32, device=dev)
    du = _rows_empty(shape.B, shape.L, pu, dev)
    dC = torch.empty_like(C)
    dth = torch.empty_like(theta_term)
    gw = [torch.empty_like(t) for t in (w_eps, w_hid, b_hid, w_head, b_head)]
    grads = FlowGrads(ptr(gw[0]), ptr(gw[1]), ptr(gw[2]), None, None, ptr(gw[3]), ptr(gw[4]))
    prm = _flow_params(w_eps, w_hid, b_hid, None, None, w_head, b_head, tf)
    check(lib.vissm_flow_ar_elbo_fused(ctypes.byref(d), ctypes.byref(prm), ptr(u), ptr(C), ptr(win), ptr(theta_term),
                                       ptr(theta), ptr(obs), ptr(obs_bin), float(obs_std), float(scale), ptr(x),
                                       ptr(logsig), ptr(du), ptr(dC), ptr(dth), ctypes.byref(grads), ptr(ws), wsz,
                                       _lib.stream_handle(dev)), "vissm_flow_ar_elbo_fused")
    return x, logsig, du, dC, dth, gw


# ---------------------------------------------------------------------------------------
# ELBO log-densities
# ---------------------------------------------------------------------------------------
@dataclass
class ElboFeeds:
    """Per-window observation feeds (device tensors, fp32; win int32 [B] or None)."""
    obs: Optional[torch.Tensor] = None
    obs_bin: Optional[torch.Tensor] = None
    mask: Optional[torch.Tensor] = None
    shift: Optional[torch.Tensor] = None
    dim_one: Optional[torch.Tensor] = None
    win: Optional[torch.Tensor] = None
    n_win: int = 1
    plain_from: Optional[torch.Tensor] = None   # int32 [n_win]: VissmElboData.plain_from (None: NULL)
    obs_list: Optional[torch.Tensor] = None     # int32 [n_win, stride]: VissmElboData.obs_list (None: NULL)

    def cdata(self) -> ElboData:
        ol = self.obs_list
        if ol is not None and (ol.dtype != torch.int32 or ol.dim() != 2 or not ol.is_contiguous()
                               or ol.shape[0] != self.n_win or ol.shape[1] < 1):
            raise ValueError("obs_list must be a contiguous int32 [n_win, stride >= 1] tensor")
        return ElboData(ptr(self.win), ptr(self.obs), ptr(self.obs_bin), ptr(self.mask), ptr(self.shift),
                        ptr(self.dim_one), ptr(self.plain_from), ptr(ol), int(ol.shape[1]) if ol is not None else 0)


class ElboFn(torch.autograd.Function):
    """Path log-densities per sample -> (sde, obs, extra)."""

    @staticmethod
    def forward(ctx, model: int, M: int, dt: float, obs_std: float, feeds: ElboFeeds, z, theta):
        lib = _lib.load()
        _require_gpu(z, theta, feeds.obs, feeds.obs_bin, feeds.mask, feeds.shift, feeds.dim_one, feeds.win)
        B = z.shape[0]
        d = ElboDesc(model, B, M, feeds.n_win, float(dt), float(obs_std))
        data = feeds.cdata()
        sde = torch.empty(B, dtype=torch.float32, device=z.device)
        obs = torch.empty_like(sde)
        extra = torch.empty_like(sde)
        check(lib.vissm_elbo_fwd(ctypes.byref(d), ctypes.byref(data), ptr(z), ptr(theta), ptr(sde), ptr(obs),
                                 ptr(extra), _lib.stream_handle(z.device)), "vissm_elbo_fwd")
        ctx.args = (model, M, dt, obs_std, feeds)
        ctx.save_for_backward(z, theta)
        return sde, obs, extra

    @staticmethod
    def backward(ctx, g_sde, g_obs, g_extra):
        lib = _lib.load()
        model, M, dt, obs_std, feeds = ctx.args
        z, theta = ctx.saved_tensors
        B = z.shape[0]
        zero = None

        def fix(g):
            nonlocal zero
            if g is None:
                if zero is None:
                    zero = torch.zeros(B, dtype=torch.float32, device=z.device)
                return zero
            return g.contiguous()

        g_sde, g_obs, g_extra = fix(g_sde), fix(g_obs), fix(g_extra)
        d = ElboDesc(model, B, M, feeds.n_win, float(dt), float(obs_std))
        data = feeds.cdata()
        dz = torch.empty_like(z)
        dth = torch.empty_like(theta)
        check(lib.vissm_elbo_bwd(ctypes.byref(d), ctypes.byref(data), ptr(z), ptr(theta), ptr(g_sde), ptr(g_obs),
                                 ptr(g_extra), ptr(dz), ptr(dth), _lib.stream_handle(z.device)), "vissm_elbo_bwd")
        return None, None, None, None, None, dz, dth


def elbo_terms(model: int, M: int, dt: float, obs_std: float, feeds: ElboFeeds, z, theta):
    return ElboFn.apply(model, M, dt, obs_std, feeds, z, theta)


def elbo_values_and_theta_grad(model: int, M: int, dt: float, obs_std: float, feeds: ElboFeeds, z, theta,
                               g_sde: torch.Tensor, g_obs: torch.Tensor):
    """(sde, obs) per sample and d(g_sde . sde + g_obs . obs)/d theta for a path z that is a constant (no dz:
    vissm_elbo_bwd with dz = NULL); no autograd."""
    lib = _lib.load()
    _require_gpu(z, theta, g_sde, g_obs, feeds.obs, feeds.obs_bin, feeds.mask, feeds.shift, feeds.dim_one, feeds.win)
    B = z.shape[0]
    d = ElboDesc(model, B, M, feeds.n_win, float(dt), float(obs_std))
    data = feeds.cdata()
    sde = torch.empty(B, dtype=torch.float32, device=z.device)
    obs = torch.empty_like(sde)
    extra = torch.empty_like(sde)
    dth = torch.empty_like(theta)
    st = _lib.stream_handle(z.device)
    if os.environ.get("VISSM_ELBO_TWO_PASS") == "1":   # A/B hook: the two calls, z read twice
        check(lib.vissm_elbo_fwd(ctypes.byref(d), ctypes.byref(data), ptr(z), ptr(theta), ptr(sde), ptr(obs),
                                 ptr(extra), st), "vissm_elbo_fwd")
        check(lib.vissm_elbo_bwd(ctypes.byref(d), ctypes.byref(data), ptr(z), ptr(theta), ptr(g_sde), ptr(g_obs),
                                 ptr(extra), None, ptr(dth), st), "vissm_elbo_bwd")
        return sde, obs, dth
    # one pass over z for AR(1) (vissm_elbo_fwd then vissm_elbo_bwd with dz = NULL for the other models)
    check(lib.vissm_elbo_fwd_theta_grad(ctypes.byref(d), ctypes.byref(data), ptr(z), ptr(theta), ptr(g_sde),
                                        ptr(g_obs), ptr(extra), ptr(sde), ptr(obs), ptr(extra), ptr(dth), st),
          "vissm_elbo_fwd_theta_grad")
    return sde, obs, dth


def elbo_values_grad(model: int, M: int, dt: float, obs_std: float, feeds: ElboFeeds, z, theta,
                     g_sde: torch.Tensor, g_obs: Optional[torch.Tensor], g_extra: Optional[torch.Tensor]):
    """(sde, obs, extra) per sample, dz and dtheta of g_sde . sde + g_obs . obs + g_extra . extra in ONE pass over z
    (vissm_elbo_fwd_grad): the training step knows these upstream gradients before the forward.  No autograd: the
    caller feeds dz / dtheta into a multi-root backward (Engine.forward_onepass)."""
    lib = _lib.load()
    _require_gpu(z, theta, g_sde, feeds.obs, feeds.obs_bin, feeds.mask, feeds.shift, feeds.dim_one, feeds.win,
                 feeds.plain_from, feeds.obs_list)
    B = z.shape[0]
    d = ElboDesc(model, B, M, feeds.n_win, float(dt), float(obs_std))
    data = feeds.cdata()
    sde = torch.empty(B, dtype=torch.float32, device=z.device)
    obs = torch.empty_like(sde)
    extra = torch.empty_like(sde)
    z = z.contiguous()
    dz = torch.empty_like(z)
    dth = torch.empty_like(theta)
    check(lib.vissm_elbo_fwd_grad(ctypes.byref(d), ctypes.byref(data), ptr(z), ptr(theta), ptr(g_sde), ptr(g_obs),
                                  ptr(g_extra), ptr(sde), ptr(obs), ptr(extra), ptr(dz), ptr(dth),
                                  _lib.stream_handle(z.device)), "vissm_elbo_fwd_grad")
    return sde, obs, extra, dz, dth


# ---------------------------------------------------------------------------------------
# optimiser
# ---------------------------------------------------------------------------------------
class AdamaxKernel:
    """Fused global-norm clip + Adamax over flat fp32 buffers (optimisers/adamax.py:42-58)."""

    def __init__(self, n: int, device):
        lib = _lib.load()
        self.n = n
        self.wsz = lib.vissm_adamax_workspace_size(n)
        self.ws = _workspace(self.wsz, device)
        self.gnorm = torch.zeros(1, dtype=torch.float32, device=device)
        self.skipped = torch.zeros(1, dtype=torch.int32, device=device)  # guarded steps skipped so far

    def step(self, params, grads, v, m, lr, beta1, beta2, eps=1e-8, clip=0.0, guard=False):
        """guard: skip the update (params and slots untouched, self.skipped += 1) when the global norm
        is not finite, instead of the reference's NaN-everything (vissm_adamax_step_guarded)."""
        lib = _lib.load()
        _require_gpu(params, grads, v, m)
        if guard:
            check(lib.vissm_adamax_step_guarded(ptr(params), ptr(grads), ptr(v), ptr(m), self.n, float(lr),
                                                float(beta1), float(beta2), float(eps), float(clip), ptr(self.gnorm),
                                                ptr(self.skipped), ptr(self.ws), self.wsz,
                                                _lib.stream_handle(params.device)), "vissm_adamax_step_guarded")
        else:
            check(lib.vissm_adamax_step(ptr(params), ptr(grads), ptr(v), ptr(m), self.n, float(lr), float(beta1),
                                        float(beta2), float(eps), float(clip), ptr(self.gnorm), ptr(self.ws), self.wsz,
                                        _lib.stream_handle(params.device)), "vissm_adamax_step")
        return self.gnorm


def sqnorm(x: torch.Tensor) -> torch.Tensor:
    lib = _lib.load()
    _require_gpu(x)
    n = x.numel()
    wsz = lib.vissm_adamax_workspace_size(n)
    ws = _workspace(wsz, x.device)
    out = torch.empty(1, dtype=torch.float32, device=x.device)
    check(lib.vissm_sqnorm(ptr(x), n, ptr(out), ptr(ws), wsz, _lib.stream_handle(x.device)), "vissm_sqnorm")
    return out


# ---------------------------------------------------------------------------------------
# q(theta) (AR.py:376-391): MAF bijectors over the base draw, one HIP launch each way
# ---------------------------------------------------------------------------------------
def theta_desc(B: int, P: int, n_bij: int, relu: bool, base_loc: float, base_scale: float, perms) -> "_lib.ThetaDesc":
    if not (1 <= P <= _lib.THETA_MAX_P and 1 <= n_bij <= _lib.THETA_MAX_BIJ):
        raise _lib.VissmError(f"q(theta): P={P}, n_bij={n_bij} outside the kernel's range")
    d = _lib.ThetaDesc()
    d.B, d.P, d.n_bij, d.relu = B, P, n_bij, int(bool(relu))
    d.base_loc, d.base_scale = float(base_loc), float(base_scale)
    for i, p in enumerate(perms):
        for q, v in enumerate(p):
            d.perm[i][q] = int(v)
    return d


class ThetaFlowFn(torch.autograd.Function):
    """theta, log q(theta) = q(theta) sample from the base draw x0 (vissm_theta_fwd).  The backward
    (vissm_theta_bwd) adds the MAF variables' gradient straight into `grad_slice` (the flat gradient
    buffer's view of those variables); `anchor` is one of them, an input only so that autograd runs this
    backward (its own gradient is part of grad_slice, so None is returned for it).

    Supported use: loss.backward() into the parameter store (every VI_SSM step and pre-training minimize).
    Under torch.autograd.grad (e.g. optimisers.AdamaxOptimizer.compute_gradients on a loss that reaches theta)
    the q(theta) variables would come back as None while their gradient is still added into the store's flat
    gradient; the model classes never take that route, and INTEGRATION.md states the restriction."""

    @staticmethod
    def forward(ctx, desc_args, w, mask, grad_slice, x0, anchor):
        _require_gpu(w, mask, x0)
        lib = _lib.load()
        B, P = x0.shape
        d = theta_desc(B, P, *desc_args)
        theta = torch.empty(B, P, dtype=torch.float32, device=x0.device)
        logq = torch.empty(B, dtype=torch.float32, device=x0.device)
        check(lib.vissm_theta_fwd(ctypes.byref(d), ptr(w), ptr(mask), ptr(x0), ptr(theta), ptr(logq),
                                  _lib.stream_handle(x0.device)), "vissm_theta_fwd")
        ctx.desc_args, ctx.grad_slice = desc_args, grad_slice
        ctx.save_for_backward(w, mask, x0)
        return theta, logq

    @staticmethod
    def backward(ctx, g_theta, g_logq):
        w, mask, x0 = ctx.saved_tensors
        lib = _lib.load()
        B, P = x0.shape
        d = theta_desc(B, P, *ctx.desc_args)
        g_theta = g_theta.contiguous() if g_theta is not None else None
        g_logq = g_logq.contiguous() if g_logq is not None else None
        ws = _workspace(lib.vissm_theta_workspace_size(ctypes.byref(d)), x0.device)
        check(lib.vissm_theta_bwd(ctypes.byref(d), ptr(w), ptr(mask), ptr(x0), ptr(g_theta), ptr(g_logq),
                                  ptr(ctx.grad_slice), ptr(ws), ws.numel(), _lib.stream_handle(x0.device)),
              "vissm_theta_bwd")
        return None, None, None, None, None, None

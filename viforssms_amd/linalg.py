"""Small dense products of the window-shared and q(theta) parts (host torch): a linear layer
whose weight gradient is a split-K product.  Their weight gradients reduce over tens of
thousands of rows (trajectories, or positions of a window) into tiny [in, out] outputs, which a
library GEMM maps onto a handful of tiles; chunking K into a batched product summed in a fixed
order fills the chip and stays deterministic."""
from __future__ import annotations

from typing import Optional

import torch


def tn_split_k(a: torch.Tensor, b: torch.Tensor, chunk: int = 1024) -> torch.Tensor:
    """a^T b over a long row axis (K = batch or positions) as a batched product of K-chunks summed
    in a fixed order: a library GEMM with a small [m, n] output and K ~ 1e4-1e5 runs on a handful
    of tiles."""
    K = a.shape[0]
    n = K // chunk
    if n < 4 or a.shape[1] * b.shape[1] > (1 << 16):  # a large output fills the chip by itself
        return a.t() @ b
    out = torch.bmm(a[:n * chunk].reshape(n, chunk, -1).transpose(1, 2), b[:n * chunk].reshape(n, chunk, -1)).sum(0)
    if K > n * chunk:
        out = out + a[n * chunk:].t() @ b[n * chunk:]
    return out


class _LinearSK(torch.autograd.Function):
    """y = x W (+ b) over the last axis of x, with the weight gradient as a split-K product."""

    @staticmethod
    def forward(ctx, x, W, b):
        ctx.save_for_backward(x, W)
        ctx.has_b = b is not None
        y = x @ W
        return y + b if b is not None else y

    @staticmethod
    def backward(ctx, dy):
        x, W = ctx.saved_tensors
        d2 = dy.reshape(-1, dy.shape[-1])
        if x.dim() == 3 and x.shape[-1] * W.shape[-1] > (1 << 16):
            dW = (x.transpose(1, 2) @ dy).sum(0)  # x may be a transposed view (LV): no copy
        else:
            dW = tn_split_k(x.reshape(-1, x.shape[-1]), d2.contiguous())
        db = d2.sum(0) if ctx.has_b else None
        return dy @ W.t(), dW, db


def linear(x: torch.Tensor, W: torch.Tensor, b: Optional[torch.Tensor] = None) -> torch.Tensor:
    return _LinearSK.apply(x, W, b)


# ---------------------------------------------------------------------------------------
# split-bf16 products for the large window-shared GEMMs at the bf16 training precisions
# ---------------------------------------------------------------------------------------
def _mm(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """bf16 a [.., M, K] @ b [.., K, N] on the matrix cores with fp32 accumulation and output (b may be 2-D
    against a batched a)."""
    if a.dim() == 2 and b.dim() == 2:
        return torch.mm(a, b, out_dtype=torch.float32)
    if b.dim() == 2:
        b = b.expand(a.shape[0], *b.shape)
    if a.dim() == 2:
        a = a.expand(b.shape[0], *a.shape)
    return torch.bmm(a, b, out_dtype=torch.float32)


def _t(a: torch.Tensor) -> torch.Tensor:
    return a.transpose(-1, -2)


def mm_bf16x3(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """a @ b for fp32 a [.., M, K] (any dense layout) and b [K, N] as split-bf16 products with fp32 accumulation
    and output, a_hi b_hi + a_hi b_lo + a_lo b_hi (~2^-16 relative per product: fp32-class at the bf16 GEMM
    rate).  The two products against a_hi share one GEMM over [b_hi | b_lo]."""
    from .ops import split_bf16
    ah, al = split_bf16(a)
    bh, bl = split_bf16(b.contiguous())
    N = b.shape[-1]
    y2 = _mm(ah, torch.cat([bh, bl], -1))
    return y2[..., :N] + y2[..., N:] + _mm(al, bh)


class _LinearX3(torch.autograd.Function):
    """y = x W (+ b) with every product (forward, dx, dW) on split-bf16 operands (the LV time-mixing conv over
    features: [10061 x 10061] x [10061 x k H] per flow at LV-cfg, 1.8e12 FLOP per step in fp32).  x is split once
    (vissm_split_bf16) and its planes are what the backward keeps; dx is one GEMM over the concatenated inner
    dimension, [dy_hi | dy_hi | dy_lo] [W_hi | W_lo | W_hi]^T, so its [M, K] output is written once."""

    @staticmethod
    def forward(ctx, x, W, b):
        from .ops import split_bf16
        xh, xl = split_bf16(x)
        Wh, Wl = split_bf16(W.contiguous())
        N = W.shape[-1]
        y2 = _mm(xh, torch.cat([Wh, Wl], -1))
        y = y2[..., :N] + y2[..., N:] + _mm(xl, Wh)
        ctx.save_for_backward(xh, xl, Wh, Wl)
        ctx.has_b = b is not None
        return y + b if b is not None else y

    @staticmethod
    def backward(ctx, dy):
        from .ops import split_bf16
        xh, xl, Wh, Wl = ctx.saved_tensors
        N = Wh.shape[-1]
        dyh, dyl = split_bf16(dy.contiguous())
        dx = dW = None
        if ctx.needs_input_grad[0]:
            A, Wc = torch.cat([dyh, dyh, dyl], -1), torch.cat([Wh, Wl, Wh], -1)
            if xh.stride(-2) == 1 and xh.shape[-2] > 1:
                # x is a transposed view (LV: F = h^T): dx in h's layout, so the ELU backward it feeds stays a
                # contiguous elementwise pass
                dx = _t(_mm(Wc, _t(A)))
            else:
                dx = _mm(A, _t(Wc))
        if ctx.needs_input_grad[1]:
            g2 = _mm(_t(xh), torch.cat([dyh, dyl], -1))
            g = g2[..., :N] + g2[..., N:] + _mm(_t(xl), dyh)
            dW = g.sum(0) if g.dim() == 3 else g
        db = dy.reshape(-1, dy.shape[-1]).sum(0) if ctx.has_b else None
        return dx, dW, db


class _LinearB1(torch.autograd.Function):
    """y = x W (+ b) with every product on single bf16 operands and fp32 accumulation / output (the flow kernels'
    own precision class; A/B alternative to _LinearX3)."""

    @staticmethod
    def forward(ctx, x, W, b):
        xb, Wb = x.to(torch.bfloat16), W.to(torch.bfloat16)
        ctx.save_for_backward(xb, Wb)
        ctx.has_b = b is not None
        y = _mm(xb, Wb)
        return y + b if b is not None else y

    @staticmethod
    def backward(ctx, dy):
        xb, Wb = ctx.saved_tensors
        dyb = dy.to(torch.bfloat16)
        dx = dW = None
        if ctx.needs_input_grad[0]:
            dx = _t(_mm(Wb, _t(dyb))) if (xb.stride(-2) == 1 and xb.shape[-2] > 1) else _mm(dyb, _t(Wb))
        if ctx.needs_input_grad[1]:
            g = _mm(_t(xb), dyb)
            dW = g.sum(0) if g.dim() == 3 else g
        db = dy.reshape(-1, dy.shape[-1]).sum(0) if ctx.has_b else None
        return dx, dW, db


def linear_bf16(x: torch.Tensor, W: torch.Tensor, b: Optional[torch.Tensor] = None) -> torch.Tensor:
    """linear() with single-bf16 matrix-core products; CPU tensors (host tests) take linear()."""
    if not x.is_cuda:
        return linear(x, W, b)
    return _LinearB1.apply(x, W, b)


def linear_x3(x: torch.Tensor, W: torch.Tensor, b: Optional[torch.Tensor] = None) -> torch.Tensor:
    """linear() with split-bf16 (bf16x3) matrix-core products; CPU tensors (host tests) take linear()."""
    if not x.is_cuda:
        return linear(x, W, b)
    return _LinearX3.apply(x, W, b)

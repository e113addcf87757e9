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

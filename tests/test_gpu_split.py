"""Split-bf16 planes (vissm_split_bf16) and the split-bf16 linear layer of LV's window-shared conv over its
time-mixing features (linalg.linear_x3) against float64 products of the same operands.

The reference runs that conv in fp32 (lotka_volterra_partial.py:78-82); the bf16 training precisions run it as
a_hi b_hi + a_hi b_lo + a_lo b_hi, held here to the fp32-class bound the LV parity tests assume (1e-5 relative
L2 error of every product: forward, input gradient, weight gradient)."""
import pytest
import torch

from viforssms_amd.linalg import linear_bf16, linear_x3
from viforssms_amd.ops import split_bf16

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("n", [0, 1, 3, 4, 7, 1 << 20, (1 << 20) + 5])
def test_split_planes_match_torch_rounding(n):
    g = torch.Generator(device=DEV).manual_seed(n)
    x = torch.randn(n, device=DEV, generator=g) * torch.exp(torch.randn(n, device=DEV, generator=g) * 8)
    if n > 4:
        x[:4] = torch.tensor([0.0, -0.0, 3.0e38, 1.0e-40], device=DEV)
    hi, lo = split_bf16(x)
    rh = x.to(torch.bfloat16)
    rl = (x - rh.float()).to(torch.bfloat16)
    assert torch.equal(hi.view(torch.int16), rh.view(torch.int16))
    assert torch.equal(lo.view(torch.int16), rl.view(torch.int16))


def test_split_keeps_a_transposed_layout():
    x = torch.randn(300, 257, device=DEV).t()          # the LV features are a transposed view
    hi, lo = split_bf16(x)
    assert hi.stride() == x.stride() and lo.stride() == x.stride()
    assert torch.equal(hi, x.to(torch.bfloat16))
    assert torch.equal(lo, (x - x.to(torch.bfloat16).float()).to(torch.bfloat16))


def _rel(a, b):
    return ((a.double() - b).norm() / b.norm()).item()


@pytest.mark.parametrize("batched,transposed", [(False, False), (False, True), (True, True), (True, False)])
def test_linear_x3_products_against_float64(batched, transposed):
    g = torch.Generator(device=DEV).manual_seed(7)
    nw, Lf, CF, N = (3 if batched else 1), 515, 1031, 200
    if transposed:
        x = torch.randn(nw, CF, Lf, device=DEV, generator=g).transpose(1, 2)
    else:
        x = torch.randn(nw, Lf, CF, device=DEV, generator=g)
    if not batched:
        x = x[0]
    x = x.detach().requires_grad_(True)
    W = (torch.randn(CF, N, device=DEV, generator=g) * 0.03).requires_grad_(True)
    b = torch.randn(N, device=DEV, generator=g).requires_grad_(True)
    dy = torch.randn(*x.shape[:-1], N, device=DEV, generator=g)
    y = linear_x3(x, W, b)
    y.backward(dy)
    x64, W64, dy64 = x.detach().double(), W.detach().double(), dy.double()
    y64 = x64 @ W64 + b.detach().double()
    dx64 = dy64 @ W64.t()
    dW64 = (x64.transpose(-1, -2) @ dy64)
    if batched:
        dW64 = dW64.sum(0)
    assert _rel(y, y64) < 1e-5
    assert _rel(x.grad, dx64) < 1e-5
    assert _rel(W.grad, dW64) < 1e-5
    assert torch.allclose(b.grad.double(), dy64.reshape(-1, N).sum(0), rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("transposed", [False, True])
def test_linear_bf16_products_at_bf16_accuracy(transposed):
    """The single-bf16 alternative (VISSM_FEATURE_GEMM=bf16): every product within the bf16 operand rounding
    (~2^-9 relative per operand; 1e-2 relative L2 over the products' 1031-term sums), gradients in the layout of x."""
    g = torch.Generator(device=DEV).manual_seed(3)
    Lf, CF, N = 515, 1031, 200
    x = torch.randn(CF, Lf, device=DEV, generator=g).t() if transposed else torch.randn(Lf, CF, device=DEV, generator=g)
    x = x.detach().requires_grad_(True)
    W = (torch.randn(CF, N, device=DEV, generator=g) * 0.03).requires_grad_(True)
    dy = torch.randn(Lf, N, device=DEV, generator=g)
    y = linear_bf16(x, W)
    y.backward(dy)
    x64, W64, dy64 = x.detach().double(), W.detach().double(), dy.double()
    assert _rel(y, x64 @ W64) < 1e-2
    assert _rel(x.grad, dy64 @ W64.t()) < 1e-2
    assert _rel(W.grad, x64.t() @ dy64) < 1e-2
    assert x.grad.stride() == x.stride()

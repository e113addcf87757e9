"""Host-side products of the window-shared / q(theta) parts against plain autograd (float64):
the collapsed theta branch with closed-form gradients, the split-K linear layer, the diagonal
gather of the window conv, the MAF permutation as a one-hot product."""
import numpy as np
import pytest
import torch

from viforssms_amd.linalg import linear, tn_split_k
from viforssms_amd.nma import _DiagSum, _ThetaBranch


def _grads(f, inputs, d):
    out = f(*inputs)
    return out, torch.autograd.grad(out, inputs, d)


def test_theta_branch_matches_three_linear_layers():
    g = torch.Generator().manual_seed(0)
    B, P, H = 5000, 3, 50
    mk = lambda *s: torch.randn(*s, generator=g, dtype=torch.float64).requires_grad_(True)
    ins = [mk(B, P), mk(P, H), mk(H), mk(H, H), mk(H), mk(H, H), mk(H)]
    d = torch.randn(B, H, generator=g, dtype=torch.float64)
    o1, g1 = _grads(_ThetaBranch.apply, ins, d)
    o2, g2 = _grads(lambda t, W0, b0, W1, b1, W2, b2: ((t @ W0 + b0) @ W1 + b1) @ W2 + b2, ins, d)
    assert torch.allclose(o1, o2, rtol=1e-12, atol=1e-10)
    for a, b in zip(g1, g2):
        assert torch.allclose(a, b, rtol=1e-10, atol=1e-9)


@pytest.mark.parametrize("shape", [(65536, 5), (2, 5025, 14), (5024, 50), (100, 7)])
def test_split_k_linear(shape):
    g = torch.Generator().manual_seed(1)
    x = torch.randn(*shape, generator=g, dtype=torch.float64).requires_grad_(True)
    W = torch.randn(shape[-1], 9, generator=g, dtype=torch.float64).requires_grad_(True)
    b = torch.randn(9, generator=g, dtype=torch.float64).requires_grad_(True)
    d = torch.randn(*shape[:-1], 9, generator=g, dtype=torch.float64)
    o1, g1 = _grads(linear, [x, W, b], d)
    o2, g2 = _grads(lambda x, W, b: x @ W + b, [x, W, b], d)
    assert torch.allclose(o1, o2)
    for a, c in zip(g1, g2):
        assert torch.allclose(a, c, rtol=1e-10, atol=1e-8)
    a = torch.randn(70000, 3, generator=g, dtype=torch.float64)
    c = torch.randn(70000, 4, generator=g, dtype=torch.float64)
    assert torch.allclose(tn_split_k(a, c), a.t() @ c, rtol=1e-12, atol=1e-9)


@pytest.mark.parametrize("s", [1, 2])
def test_diag_sum_backward_is_the_scatter(s):
    g = torch.Generator().manual_seed(2)
    nw, Lf, k, H = 2, 41, 5, 6
    Lh = (Lf - k) // s + 1
    G = torch.randn(nw, Lf, k, H, generator=g, dtype=torch.float64).requires_grad_(True)
    view = lambda G: G.as_strided((nw, Lh, k, H), (Lf * k * H, s * k * H, k * H + H, 1)).sum(2)
    d = torch.randn(nw, Lh, H, generator=g, dtype=torch.float64)
    o1, g1 = _grads(lambda G: _DiagSum.apply(G, Lh, s), [G], d)
    o2, g2 = _grads(view, [G], d)
    assert torch.equal(o1, o2) and torch.equal(g1[0], g2[0])


def test_maf_permutation_product_is_exact():
    from viforssms_amd.params import ParamStore
    from viforssms_amd.theta_flow import ThetaFlow
    st = ParamStore()
    tf = ThetaFlow(st, 3, 3, [[2, 0, 1], [1, 2, 0]], 0.0, 1.0, "elu")
    z = torch.randn(10, 3, dtype=torch.float32)
    for i in range(2):
        assert torch.equal(z @ tf._perm_matrix(i, z), z[..., tf.perms[i]])
